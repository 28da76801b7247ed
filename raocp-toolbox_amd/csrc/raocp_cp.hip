// raocp_cp.hip — the two node-block kernels of one Chambolle–Pock iteration
// (included by raocp_kernels.hip, inside namespace raocp).
//
//   k_cpd: dual half step + prox of g* + xi2 (solver.py:44-61, cache.py:321-393, 63-95)
//   k_cpp: next primal half step + AVaR kernel projection + the finished iteration's
//          xi0, xi1, delta0, delta1 (solver.py:27-39, cache.py:248-317, 63-95)
//
// Block decomposition. A FAMILY block owns parents [i0, i1) (FB consecutive nonleaf
// nodes) together with all their children [cb, ce): everything the L / L^T rows of a
// family touch is inside the family (a child's eta3/eta4 use its parent's x, u; the
// parent's x, u under L^T sum over its children; the kernel projection couples y_i with
// the children's tau, s). A LEAF block owns leaves [l0, l1). Each block first stages
// every input range it reads into LDS by LDS-DMA (one memory round trip; ranges are
// contiguous by the BFS numbering), then computes from LDS with the lanes-over-rows
// mapping of raocp_kernels.hip, and stores its rows coalesced. A few hundred fat
// blocks instead of thousands of thin ones: the per-block dispatch cost and the
// dependent global loads were what bounded the previous kernels (TA-busy ~75 %).
//
// Arithmetic (operation order included) is that of k_cp_dual / k_cp_primal, which the
// GPU parity tests pin against the reference.

// LDS-DMA staging of a T array (Stg: 16-B chunk slots from the 16-B boundary below the
// source; doubles keep Stg::dbl's footprint, which the host sizes blocks by; a float region
// needs no more slots)
template <class T, class PT>
__device__ __forceinline__ ldsp<T> stg_arr(Stg& st, PT src, int count) {
    if constexpr (sizeof(T) == 8) {
        return (ldsp<T>)st.dbl(src, count);
    } else {
        const uintptr_t a = (uintptr_t)src;
        const int sh = (int)(a & 15), nb = count > 0 ? sh + (int)sizeof(T) * count : 0;
        ldsd* d = st.region((const char*)(a - sh), nb, (nb + 15) >> 4);
        return (ldsp<T>)((__attribute__((address_space(3))) char*)d + sh);
    }
}

// block tables (host): family block {cb, ce, y0, y1}, {e7a, e7b, i0, i1}; leaf block {e14a, e14b, l0, l1}.
// The table, not the block index, says which nodes a block owns (a shard launches only its blocks).

// ==============================================================================
// k_cpd — dual. Roles: blocks [0, nbF) families, [nbF, nbF + nbL) leaves.
// ==============================================================================
template <class T, int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_cpd(Dev p, Ctl* __restrict__ ctl, Bufs bf, double* __restrict__ xi2_,
                                                double* __restrict__ part, int nbF) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ T s_x[kBlock];
    __shared__ double s_red[2][kBlock / 64];
    int done;      // read once the staging loads are in flight (ctl_done, raocp_dyn.hip)
    T alpha;
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    cglbp<T> pz = (cglbp<T>)bf.z0;   // p
    cglbp<T> zp = (cglbp<T>)bf.z1;   // z+
    cglbp<T> d = (cglbp<T>)bf.e0;    // eta (this iteration's dual)
    glbp<T> eo = (glbp<T>)bf.e1;               // eta+
    glbp<T> xi2 = (glbp<T>)xi2_;
    const int bid = blockIdx.x;
    Stg st{(ldsd*)smem_, 0, stg_table()};
    double m2 = 0.0, m5 = 0.0;
    auto finish = [&](int e, T dv, T v, T pv, T b) {
        const T ep = alpha * (v - pv);
        eo[e] = ep;
        const T x2 = (dv - ep) / alpha + b;
        xi2[e] = x2;
        m2 = nmax(m2, fabs(x2));
        m5 = nmax(m5, fabs(ep - dv));
    };
    if (bid < nbF) {
        const Rec t0 = ((crec4*)p.cpd_tab)[2 * bid], t1 = ((crec4*)p.cpd_tab)[2 * bid + 1];
        const int i0 = t1.z, i1 = t1.w, P = i1 - i0;
        const int cb = t0.x, ce = t0.y, C = ce - cb, y0 = t0.z, Y = t0.w - t0.z, e7a = t1.x, E7n = t1.y - t1.x;
        // stage
        const auto Xz = stg_arr<T>(st, zp + p.X0 + (size_t)i0 * nx, P * nx);
        const auto Xp = stg_arr<T>(st, pz + p.X0 + (size_t)i0 * nx, P * nx);
        const auto Uz = stg_arr<T>(st, zp + p.U0 + (size_t)i0 * nu, P * nu);
        const auto Up = stg_arr<T>(st, pz + p.U0 + (size_t)i0 * nu, P * nu);
        const auto Yz = stg_arr<T>(st, zp + p.Y0 + y0, Y);
        const auto Yp = stg_arr<T>(st, pz + p.Y0 + y0, Y);
        const auto Sz = stg_arr<T>(st, zp + p.S0 + i0, P);
        const auto Sp = stg_arr<T>(st, pz + p.S0 + i0, P);
        const auto Tz = stg_arr<T>(st, zp + p.T0 + cb, C);
        const auto Tp = stg_arr<T>(st, pz + p.T0 + cb, C);
        const auto CD = stg_arr<T>(st, (cglbp<T>)p.cond + cb, C);
        const auto D1 = stg_arr<T>(st, d + p.E1 + y0, Y);
        const auto D2 = stg_arr<T>(st, d + p.E2 + i0, P);
        const auto D7 = stg_arr<T>(st, d + e7a, E7n);
        const auto D3 = stg_arr<T>(st, d + e3(p, cb), C * nx);
        const auto D4 = stg_arr<T>(st, d + e4(p, cb), C * nu);
        const auto D5 = stg_arr<T>(st, d + p.E5 + cb, C);
        const auto D6 = stg_arr<T>(st, d + p.E6 + cb, C);
        const ldsrec* FR = st.rec(p.frec + i0, P);   // {yrel, nch, ch_start, e7off}
        const ldsrec* CR = st.rec(p.crec + cb, C);   // {anc, iSQ, iSR, 0}
        const auto BI = st.ints(p.iBnl + i0, P);
        const int nQ = p.nSQ * nx * nx, nR = p.nSR * nu * nu, nBx = p.nBnl * (nx + nu);
        const auto SQ = stg_arr<T>(st, (cglbp<T>)p.SQ, nQ);
        const auto SR = stg_arr<T>(st, (cglbp<T>)p.SR, nR);
        const auto BL = stg_arr<T>(st, (cglbp<T>)p.blo_nl, nBx);
        const auto BH = stg_arr<T>(st, (cglbp<T>)p.bhi_nl, nBx);
        st.issue();
        done = ctl->done;
        alpha = ctl->alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        // children rows eta3 (nx), eta4 (nu), eta5, eta6 -> one SOC of dim nx+nu+2 per child
        {
            const int G = nx + nu + 2, per = blockDim.x / G;
            const int gl = threadIdx.x / G, r = threadIdx.x - gl * G, base = gl * G;
            for (int c0 = 0; c0 < C; c0 += per) {
                const int jj = c0 + gl, j = cb + jj;
                const bool live = gl < per && jj < C;
                T v = T(0), bb = T(0), dv = T(0);
                int e = -1;
                if (live) {
                    const Rec cr = CR[jj];
                    const int ai = cr.x - i0;
                    T av = T(0);
                    if (r < nx) {
                        e = e3(p, j) + r;
                        dv = D3[jj * nx + r];
                        ldsp<T> M = SQ + (size_t)cr.y * nx * nx + r;
                        ldsp<T> xz = Xz + ai * nx;
                        ldsp<T> xp = Xp + ai * nx;
                        T sa = T(0), sb = T(0);
                        _Pragma("unroll 4") for (int k = 0; k < nx; ++k) {
                            const T mk = M[k * nx], zk = xz[k], pk = xp[k];
                            sa = fma(mk, T(2) * zk - pk, sa);
                            sb = fma(mk, zk - pk, sb);
                        }
                        av = sa;
                        bb = sb;
                    } else if (r < nx + nu) {
                        const int rr = r - nx;
                        e = e4(p, j) + rr;
                        dv = D4[jj * nu + rr];
                        ldsp<T> M = SR + (size_t)cr.z * nu * nu + rr;
                        ldsp<T> uz = Uz + ai * nu;
                        ldsp<T> up = Up + ai * nu;
                        T sa = T(0), sb = T(0);
                        _Pragma("unroll 4") for (int k = 0; k < nu; ++k) {
                            const T mk = M[k * nu], zk = uz[k], pk = up[k];
                            sa = fma(mk, T(2) * zk - pk, sa);
                            sb = fma(mk, zk - pk, sb);
                        }
                        av = sa;
                        bb = sb;
                    } else {
                        const bool five = r == nx + nu;
                        e = (five ? p.E5 : p.E6) + j;
                        dv = five ? D5[jj] : D6[jj];
                        const T zt = Tz[jj], pt = Tp[jj];
                        av = T(0.5) * (T(2) * zt - pt);
                        bb = T(0.5) * (zt - pt);
                    }
                    v = (dv + alpha * av) / alpha;
                    if (r == nx + nu) v += T(-0.5);
                    if (r == nx + nu + 1) v += T(0.5);
                }
                s_x[threadIdx.x] = (live && r < G - 1) ? v * v : T(0);
                if (live && r == G - 1) s_x[threadIdx.x] = v;
                __syncthreads();
                if (live) {
                    T ss = T(0);
                    for (int q = 0; q < G - 1; ++q) ss += s_x[base + q];
                    const T nf = sqrt(ss), t = s_x[base + G - 1];
                    finish(e, dv, v, soc_apply_t<T>(v, r == G - 1, nf, t), bb);
                }
                __syncthreads();
            }
        }
        // parent rows eta1 (2c+1), eta2, eta7 (nx+nu)
        {
            const int G = 2 * p.cmax + 2 + nx + nu, per = blockDim.x / G;
            const int gl = threadIdx.x / G, r = threadIdx.x - gl * G;
            for (int q0 = 0; q0 < P; q0 += per) {
                const int ii = q0 + gl, i = i0 + ii;
                if (!(gl < per && ii < P)) continue;
                const Rec fr = FR[ii];
                const int c = fr.y, yo = fr.x - y0, cl = fr.z - cb;
                if (r < 2 * c + 1) {
                    const int e = p.E1 + fr.x + r;
                    const T zy = Yz[yo + r], py = Yp[yo + r];
                    const T av = T(2) * zy - py, bb = zy - py;
                    const T dv = D1[yo + r];
                    const T v = (dv + alpha * av) / alpha;
                    finish(e, dv, v, r < 2 * c ? fmax(v, T(0)) : v, bb);
                } else if (r == 2 * p.cmax + 1) {
                    const int e = p.E2 + i;
                    T bya = T(0), byb = T(0);
                    for (int k = 0; k < c; ++k) {
                        const T cp = CD[cl + k];
                        bya = fma(cp, T(2) * Yz[yo + k] - Yp[yo + k], bya);
                        byb = fma(cp, Yz[yo + k] - Yp[yo + k], byb);
                    }
                    bya += T(2) * Yz[yo + 2 * c] - Yp[yo + 2 * c];
                    byb += Yz[yo + 2 * c] - Yp[yo + 2 * c];
                    const T zs = Sz[ii], ps = Sp[ii];
                    const T av = (T(2) * zs - ps) - bya, bb = (zs - ps) - byb;
                    const T dv = D2[ii];
                    const T v = (dv + alpha * av) / alpha;
                    finish(e, dv, v, fmax(v, T(0)), bb);
                } else if (r >= 2 * p.cmax + 2 && fr.w >= 0) {
                    const int rr = r - (2 * p.cmax + 2);
                    const int e = fr.w + rr;
                    const T zv = rr < nx ? Xz[ii * nx + rr] : Uz[ii * nu + rr - nx];
                    const T pv_ = rr < nx ? Xp[ii * nx + rr] : Up[ii * nu + rr - nx];
                    const T av = T(2) * zv - pv_, bb = zv - pv_;
                    const T dv = D7[fr.w - e7a + rr];
                    const T v = (dv + alpha * av) / alpha;
                    const int bi = BI[ii];
                    finish(e, dv, v, box_apply_t<T>(v, BL[bi * (nx + nu) + rr], BH[bi * (nx + nu) + rr], ctl), bb);
                }
            }
        }
    } else {
        // leaves [l0, l1): eta11 (nx), eta12, eta13 -> SOC of dim nx+2 ; eta14 (nx) box
        const int lb = bid - nbF;
        const Rec t0 = ((crec4*)p.cpd_tab)[2 * nbF + lb];
        const int l0 = t0.z, l1 = t0.w, Lc = l1 - l0;
        const int e14a = t0.x, E14n = t0.y - t0.x;
        const auto Xz = stg_arr<T>(st, zp + p.X0 + (size_t)l0 * nx, Lc * nx);
        const auto Xp = stg_arr<T>(st, pz + p.X0 + (size_t)l0 * nx, Lc * nx);
        const auto Sz = stg_arr<T>(st, zp + p.S0 + l0, Lc);
        const auto Sp = stg_arr<T>(st, pz + p.S0 + l0, Lc);
        const auto D11 = stg_arr<T>(st, d + e11(p, l0), Lc * nx);
        const auto D12 = stg_arr<T>(st, d + p.E12 + l0, Lc);
        const auto D13 = stg_arr<T>(st, d + p.E13 + l0, Lc);
        const auto D14 = stg_arr<T>(st, d + e14a, E14n);
        const ldsrec* LR = st.rec(p.lrec + (l0 - p.m), Lc);  // {iSP, iBl, e14off, 0}
        const int nP = p.nSP * nx * nx, nBx = p.nBl * nx;
        const auto SP = stg_arr<T>(st, (cglbp<T>)p.SP, nP);
        const auto BL = stg_arr<T>(st, (cglbp<T>)p.blo_l, nBx);
        const auto BH = stg_arr<T>(st, (cglbp<T>)p.bhi_l, nBx);
        st.issue();
        done = ctl->done;
        alpha = ctl->alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        const int G = 2 * nx + 2, per = blockDim.x / G;
        const int gl = threadIdx.x / G, r = threadIdx.x - gl * G, base = gl * G;
        for (int q0 = 0; q0 < Lc; q0 += per) {
            const int ll = q0 + gl, l = l0 + ll;
            const bool live = gl < per && ll < Lc;
            T v = T(0), bb = T(0), dv = T(0);
            int e = -1;
            Rec lr = {0, 0, -1, 0};
            if (live) {
                lr = LR[ll];
                T av = T(0);
                if (r < nx) {
                    e = e11(p, l) + r;
                    dv = D11[ll * nx + r];
                    ldsp<T> M = SP + (size_t)lr.x * nx * nx + r;
                    ldsp<T> xz = Xz + ll * nx;
                    ldsp<T> xp = Xp + ll * nx;
                    T sa = T(0), sb = T(0);
                    _Pragma("unroll 4") for (int k = 0; k < nx; ++k) {
                        const T mk = M[k * nx], zk = xz[k], pk = xp[k];
                        sa = fma(mk, T(2) * zk - pk, sa);
                        sb = fma(mk, zk - pk, sb);
                    }
                    av = sa;
                    bb = sb;
                } else if (r < nx + 2) {
                    e = (r == nx ? p.E12 : p.E13) + l;
                    dv = r == nx ? D12[ll] : D13[ll];
                    const T zs = Sz[ll], ps = Sp[ll];
                    av = T(0.5) * (T(2) * zs - ps);
                    bb = T(0.5) * (zs - ps);
                } else if (lr.z >= 0) {
                    const int rr = r - nx - 2;
                    e = lr.z + rr;
                    dv = D14[lr.z - e14a + rr];
                    const T zv = Xz[ll * nx + rr], pv_ = Xp[ll * nx + rr];
                    av = T(2) * zv - pv_;
                    bb = zv - pv_;
                }
                if (e >= 0) {
                    v = (dv + alpha * av) / alpha;
                    if (r == nx) v += T(-0.5);
                    if (r == nx + 1) v += T(0.5);
                }
            }
            s_x[threadIdx.x] = (live && r < nx + 1) ? v * v : T(0);
            if (live && r == nx + 1) s_x[threadIdx.x] = v;
            __syncthreads();
            if (live && e >= 0) {
                if (r < nx + 2) {
                    T ss = T(0);
                    for (int q = 0; q < nx + 1; ++q) ss += s_x[base + q];
                    finish(e, dv, v, soc_apply_t<T>(v, r == nx + 1, sqrt(ss), s_x[base + nx + 1]), bb);
                } else {
                    const int rr = r - nx - 2;
                    finish(e, dv, v, box_apply_t<T>(v, BL[lr.y * nx + rr], BH[lr.y * nx + rr], ctl), bb);
                }
            }
            __syncthreads();
        }
    }
    double* prow = part + (size_t)bid * 6;
    block_max_store(m2, prow + 2, s_red[0]);
    block_max_store(m5, prow + 5, s_red[1]);
}

// ==============================================================================
// k_cpp — next primal half step from eta+ (FULL form of k_cp_primal):
//   out = z+ - alpha L^T(eta+), s_0 -= alpha, kernel projection of (y, tau, s);
//   xi1 = (p - z+)/alpha - L^T(d - eta+), xi0 = xi1 + L^T xi2, delta1 = z+ - p,
//   delta0 = delta1 + L^T(d - eta+)
// Buffers: p = z0, z+ = z1, out = z2, d = e0, eta+ = e1.
// ==============================================================================
template <class T, int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_cpp(Dev p, Ctl* __restrict__ ctl, Bufs bf, const double* __restrict__ xi2_,
                                                double* __restrict__ part, int nbF) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ T s_x[kBlock];
    __shared__ double s_red[4][kBlock / 64];
    int done;      // read once the staging loads are in flight (ctl_done, raocp_dyn.hip)
    T alpha;
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    cglbp<T> pz = (cglbp<T>)bf.z0;   // p_prev
    cglbp<T> zp = (cglbp<T>)bf.z1;   // z+ (also where the half step starts)
    glbp<T> out = (glbp<T>)bf.z2;
    cglbp<T> dP = (cglbp<T>)bf.e0;   // d_prev
    cglbp<T> dA = (cglbp<T>)bf.e1;   // eta+
    cglbp<T> xg = (cglbp<T>)xi2_;
    const int bid = blockIdx.x;
    Stg st{(ldsd*)smem_, 0, stg_table()};
    double m0 = 0.0, m1 = 0.0, m3 = 0.0, m4 = 0.0;
    stamp(p, 0);
    // residual terms of one primal entry: pp = p, zz = z+, w = L^T(d - eta+), lc = L^T xi2
    auto account = [&](T pp, T zz, T w, T lc) {
        const T x1 = (pp - zz) / alpha - w;
        const T x0v = x1 + lc;
        const T dl1 = zz - pp;
        const T dl0 = dl1 + w;
        m0 = nmax(m0, fabs(x0v)); m1 = nmax(m1, fabs(x1)); m3 = nmax(m3, fabs(dl0)); m4 = nmax(m4, fabs(dl1));
    };
    if (bid < nbF) {
        const Rec t0 = ((crec4*)p.cpd_tab)[2 * bid], t1 = ((crec4*)p.cpd_tab)[2 * bid + 1];
        const int i0 = t1.z, i1 = t1.w, P = i1 - i0;
        const int cb = t0.x, ce = t0.y, C = ce - cb, y0 = t0.z, Y = t0.w - t0.z, e7a = t1.x, E7n = t1.y - t1.x;
        // a family may straddle a stage boundary: leaf and nonleaf children are told apart per child
        // stage: three duals (A = eta+, P = d_prev, X = xi2) over the family's ranges
        cglbp<T> dsrc[3] = {dA, dP, xg};
        ldsp<T> D1[3], D2[3], D2c[3], D3[3], D4[3], D5[3], D6[3], D7[3], Dc12[3], Dc13[3];
        _Pragma("unroll") for (int a = 0; a < 3; ++a) {
            cglbp<T> s = dsrc[a];
            D1[a] = stg_arr<T>(st, s + p.E1 + y0, Y);
            D2[a] = stg_arr<T>(st, s + p.E2 + i0, P);
            D3[a] = stg_arr<T>(st, s + e3(p, cb), C * nx);
            D4[a] = stg_arr<T>(st, s + e4(p, cb), C * nu);
            D5[a] = stg_arr<T>(st, s + p.E5 + cb, C);
            D6[a] = stg_arr<T>(st, s + p.E6 + cb, C);
            D7[a] = stg_arr<T>(st, s + e7a, E7n);
            D2c[a] = stg_arr<T>(st, s + p.E2 + cb, C);    // s_j of nonleaf children: eta2_j
            Dc12[a] = stg_arr<T>(st, s + p.E12 + cb, C);  // s_j of leaf children: (eta12_j + eta13_j) / 2
            Dc13[a] = stg_arr<T>(st, s + p.E13 + cb, C);
        }
        const auto Xz = stg_arr<T>(st, zp + p.X0 + (size_t)i0 * nx, P * nx);
        const auto Xp = stg_arr<T>(st, pz + p.X0 + (size_t)i0 * nx, P * nx);
        const auto Uz = stg_arr<T>(st, zp + p.U0 + (size_t)i0 * nu, P * nu);
        const auto Up = stg_arr<T>(st, pz + p.U0 + (size_t)i0 * nu, P * nu);
        const auto Yz = stg_arr<T>(st, zp + p.Y0 + y0, Y);
        const auto Yp = stg_arr<T>(st, pz + p.Y0 + y0, Y);
        const auto Tz = stg_arr<T>(st, zp + p.T0 + cb, C);
        const auto Tp = stg_arr<T>(st, pz + p.T0 + cb, C);
        const auto Scz = stg_arr<T>(st, zp + p.S0 + cb, C);
        const auto Scp = stg_arr<T>(st, pz + p.S0 + cb, C);
        const auto CD = stg_arr<T>(st, (cglbp<T>)p.cond + cb, C);
        const auto AR = stg_arr<T>(st, (cglbp<T>)p.alpha_r + i0, P);
        const ldsrec* FR = st.rec(p.frec + i0, P);   // {yrel, nch, ch_start, e7off}
        const ldsrec* CR = st.rec(p.crec + cb, C);   // {anc, iSQ, iSR, 0}
        const int nQ = p.nSQ * nx * nx, nR = p.nSR * nu * nu;
        const auto SQ = stg_arr<T>(st, (cglbp<T>)p.SQ, nQ);
        const auto SR = stg_arr<T>(st, (cglbp<T>)p.SR, nR);
        stamp(p, 1);
        st.issue();
        done = ctl->done;
        alpha = ctl->alpha;
        dma_wait();
        lds_sync();
        stamp(p, 2);
        if (done) return;
        const int G = nx + nu + p.cmax + 1, per = blockDim.x / G;
        const int gl = threadIdx.x / G, r = threadIdx.x - gl * G, base = gl * G;
        for (int q0 = 0; q0 < P; q0 += per) {
            const int ii = q0 + gl, i = i0 + ii;
            const bool live = gl < per && ii < P;
            Rec fr = {0, 0, 0, -1};
            if (live) fr = FR[ii];
            const int c = fr.y, cl = fr.z - cb;
            if (live && r < nx + nu) {
                // x / u rows: sum over children of sqrtQ_j eta3_j (sqrtR_j eta4_j) + Gamma' eta7
                const bool isx = r < nx;
                const int rr = isx ? r : r - nx;
                T accA = T(0), accW = T(0), accC = T(0);
                if (fr.w >= 0) {
                    const int o = fr.w - e7a + (isx ? rr : nx + rr);
                    accA = D7[0][o];
                    accW = D7[1][o] - D7[0][o];
                    accC = D7[2][o];
                }
                for (int q = 0; q < c; ++q) {
                    const int jj = cl + q;
                    const Rec cr = CR[jj];
                    T sA = T(0), sW = T(0), sC = T(0);
                    if (isx) {
                        ldsp<T> M = SQ + (size_t)cr.y * nx * nx + rr;
                        const int o = jj * nx;
                        _Pragma("unroll 4") for (int k = 0; k < nx; ++k) {
                            const T mk = M[k * nx], va = D3[0][o + k];
                            sA = fma(mk, va, sA);
                            sW = fma(mk, D3[1][o + k] - va, sW);
                            sC = fma(mk, D3[2][o + k], sC);
                        }
                    } else {
                        ldsp<T> M = SR + (size_t)cr.z * nu * nu + rr;
                        const int o = jj * nu;
                        _Pragma("unroll 4") for (int k = 0; k < nu; ++k) {
                            const T mk = M[k * nu], va = D4[0][o + k];
                            sA = fma(mk, va, sA);
                            sW = fma(mk, D4[1][o + k] - va, sW);
                            sC = fma(mk, D4[2][o + k], sC);
                        }
                    }
                    accA += sA;
                    accW += sW;
                    accC += sC;
                }
                const int e = isx ? p.X0 + i * nx + rr : p.U0 + i * nu + rr;
                const T zz = isx ? Xz[ii * nx + rr] : Uz[ii * nu + rr];
                const T pp = isx ? Xp[ii * nx + rr] : Up[ii * nu + rr];
                out[e] = zz - alpha * accA;
                account(pp, zz, accW, accC);
            }
            // AVaR kernel block: lane rk < cmax -> child; == cmax -> y_2c (and root s_0)
            const int rk = r - (nx + nu);
            T vals[4] = {0, 0, 0, 0};
            T y2c = T(0);
            const int yo = fr.x - y0;
            const T e2A = live ? D2[0][ii] : T(0);
            T e2W = T(0), e2C = T(0);
            if (live) { e2W = D2[1][ii] - D2[0][ii]; e2C = D2[2][ii]; }
            if (live && rk >= 0 && rk < c) {
                const int jj = cl + rk, j = cb + jj;
                const T b = CD[jj];
                const int f0 = yo + rk, f1 = yo + c + rk;
                const T lt0 = D1[0][f0] - b * e2A, lt1 = D1[0][f1] - T(0) * e2A;
                vals[0] = Yz[f0] - alpha * lt0;
                vals[1] = Yz[f1] - alpha * lt1;
                const T ltt = T(0.5) * (D5[0][jj] + D6[0][jj]);
                vals[2] = Tz[jj] - alpha * ltt;
                const T lts = j < p.m ? D2c[0][jj] : T(0.5) * (Dc12[0][jj] + Dc13[0][jj]);
                vals[3] = Scz[jj] - alpha * lts;
                const T w0 = (D1[1][f0] - D1[0][f0]) - b * e2W, c0 = D1[2][f0] - b * e2C;
                const T w1 = (D1[1][f1] - D1[0][f1]) - T(0) * e2W, c1 = D1[2][f1] - T(0) * e2C;
                const T wt = T(0.5) * ((D5[1][jj] - D5[0][jj]) + (D6[1][jj] - D6[0][jj]));
                const T ct = T(0.5) * (D5[2][jj] + D6[2][jj]);
                T ws, cs2;
                if (j < p.m) { ws = D2c[1][jj] - D2c[0][jj]; cs2 = D2c[2][jj]; }
                else {
                    ws = T(0.5) * ((Dc12[1][jj] - Dc12[0][jj]) + (Dc13[1][jj] - Dc13[0][jj]));
                    cs2 = T(0.5) * (Dc12[2][jj] + Dc13[2][jj]);
                }
                account(Yp[f0], Yz[f0], w0, c0);
                account(Yp[f1], Yz[f1], w1, c1);
                account(Tp[jj], Tz[jj], wt, ct);
                account(Scp[jj], Scz[jj], ws, cs2);
            }
            if (live && rk == p.cmax) {
                const int f2 = yo + 2 * c;
                y2c = Yz[f2] - alpha * (D1[0][f2] - T(1) * e2A);
                account(Yp[f2], Yz[f2], (D1[1][f2] - D1[0][f2]) - T(1) * e2W, D1[2][f2] - T(1) * e2C);
                if (i == 0) {
                    // root s_0: L^T -> eta2_0 ; then the relaxation prox s_0 -= alpha (cache.py:253-257)
                    const T z0s = zp[p.S0], p0s = pz[p.S0];
                    out[p.S0] = (z0s - alpha * e2A) - alpha;
                    account(p0s, z0s, e2W, e2C);
                }
            }
            // kernel projection (kernel_proj_group with staged alpha_r)
            {
                const int cmax = p.cmax;
                const bool mine = live && rk >= 0 && rk <= cmax;
                const T al = live ? AR[ii] : T(0);
                const int kb = base + nx + nu;
                if (mine && rk == cmax) s_x[kb + cmax] = y2c;
                __syncthreads();
                T rkv = T(0);
                if (live && rk >= 0 && rk < c) rkv = al * vals[0] - vals[1] + s_x[kb + cmax] - vals[2] - vals[3];
                __syncthreads();
                if (mine && rk < cmax) s_x[kb + rk] = rkv;
                __syncthreads();
                T sr = T(0);
                if (mine) for (int q = 0; q < c; ++q) sr += s_x[kb + q];
                const T a = al * al + T(3);
                T w = T(0);
                if (live && rk >= 0 && rk < c) w = (rkv - sr / (a + T(c))) / a;
                __syncthreads();
                if (mine && rk < cmax) s_x[kb + rk] = w;
                __syncthreads();
                if (live && rk >= 0 && rk < c) {
                    vals[0] -= al * w;
                    vals[1] += w;
                    vals[2] += w;
                    vals[3] += w;
                }
                if (live && rk == cmax) {
                    T sw = T(0);
                    for (int q = 0; q < c; ++q) sw += s_x[kb + q];
                    y2c -= sw;
                }
                __syncthreads();
            }
            if (live && rk >= 0 && rk < c) {
                const int j = cb + cl + rk;
                out[p.Y0 + fr.x + rk] = vals[0];
                out[p.Y0 + fr.x + c + rk] = vals[1];
                out[p.T0 + j] = vals[2];
                out[p.S0 + j] = vals[3];
            }
            if (live && rk == p.cmax) out[p.Y0 + fr.x + 2 * c] = y2c;
            stamp(p, 3 + q0 / per);
        }
    } else {
        // leaves: x = sqrtPf eta11 + eta14
        const int lb = bid - nbF;
        const Rec t0 = ((crec4*)p.cpd_tab)[2 * nbF + lb];
        const int l0 = t0.z, l1 = t0.w, Lc = l1 - l0;
        const int e14a = t0.x, E14n = t0.y - t0.x;
        cglbp<T> dsrc[3] = {dA, dP, xg};
        ldsp<T> D11[3], D14[3];
        _Pragma("unroll") for (int a = 0; a < 3; ++a) {
            D11[a] = stg_arr<T>(st, dsrc[a] + e11(p, l0), Lc * nx);
            D14[a] = stg_arr<T>(st, dsrc[a] + e14a, E14n);
        }
        const auto Xz = stg_arr<T>(st, zp + p.X0 + (size_t)l0 * nx, Lc * nx);
        const auto Xp = stg_arr<T>(st, pz + p.X0 + (size_t)l0 * nx, Lc * nx);
        const ldsrec* LR = st.rec(p.lrec + (l0 - p.m), Lc);
        const int nP = p.nSP * nx * nx;
        const auto SP = stg_arr<T>(st, (cglbp<T>)p.SP, nP);
        st.issue();
        done = ctl->done;
        alpha = ctl->alpha;
        dma_wait();
        lds_sync();
        if (done) return;
        const int per = blockDim.x / nx;
        const int gl = threadIdx.x / nx, r = threadIdx.x - gl * nx;
        for (int q0 = 0; q0 < Lc; q0 += per) {
            const int ll = q0 + gl, l = l0 + ll;
            if (!(gl < per && ll < Lc)) continue;
            const Rec lr = LR[ll];
            ldsp<T> M = SP + (size_t)lr.x * nx * nx + r;
            const int o = ll * nx;
            T sA = T(0), sW = T(0), sC = T(0);
            _Pragma("unroll 4") for (int k = 0; k < nx; ++k) {
                const T mk = M[k * nx], va = D11[0][o + k];
                sA = fma(mk, va, sA);
                sW = fma(mk, D11[1][o + k] - va, sW);
                sC = fma(mk, D11[2][o + k], sC);
            }
            if (lr.z >= 0) {
                const int q = lr.z - e14a + r;
                sA += D14[0][q];
                sW += D14[1][q] - D14[0][q];
                sC += D14[2][q];
            }
            const int e = p.X0 + l * nx + r;
            const T zz = Xz[o + r], pp = Xp[o + r];
            out[e] = zz - alpha * sA;
            account(pp, zz, sW, sC);
        }
    }
    double* prow = part + (size_t)bid * 6;
    block_max_store(m0, prow + 0, s_red[0]);
    block_max_store(m1, prow + 1, s_red[1]);
    block_max_store(m3, prow + 3, s_red[2]);
    block_max_store(m4, prow + 4, s_red[3]);
    stamp(p, 10);
}
