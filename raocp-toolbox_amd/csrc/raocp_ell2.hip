// raocp_ell2.hip — L and L^T (operators.py:19-53, 55-94) in any scalar type T on the
// node blocks of the CP kernels (Dev::cp2_tab, raocp_cp2.hip): the operators of an fp32
// context (BASELINE configs[4]) and, in fp64, of contexts that run the MFMA CP kernels.
// Included by raocp_kernels.hip after raocp_cp2.hip (namespace raocp).
//
// L, family block (parents [i0, i1), children [cb, ce)):
//   eta3_j = sqrtQ_j x_anc(j), eta4_j = sqrtR_j u_anc(j)   16-child MFMA tiles
//   eta5_j = eta6_j = tau_j / 2
//   eta1_i = y_i, eta2_i = s_i - b_i' y_i, eta7_i = [x_i; u_i] (boxed nodes)
// L, leaf block: eta11_l = sqrtPf_l x_l (tiles), eta12_l = eta13_l = s_l / 2, eta14_l = x_l.
// L^T, family block: x_i = [eta7_i]_x + sum_j sqrtQ_j eta3_j, u_i likewise (per-parent
//   tiles on regular blocks, else products through LDS), y_i = eta1_i - b_i eta2_i,
//   s_i = eta2_i, tau_j = (eta5_j + eta6_j) / 2;
// L^T, leaf block: x_l = sqrtPf_l eta11_l + eta14_l, s_l = (eta12_l + eta13_l) / 2.
// Slots an operator does not write keep their value (the reference's output template).
// Algorithmic bytes per launch: w (|P| + |D|) over active entries.

template <class T, int RTX, int RTU>
__global__ void __launch_bounds__(256) k_ell2(Dev p, const double* __restrict__ z_, double* __restrict__ eta_,
                                              int nbF) {
    typedef typename MF<T>::v4 v4;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    const int nx = p.nx, nu = p.nu;
    const T* z = (const T*)z_;
    glbp<T> eg = (glbp<T>)eta_;
    const int bid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const int lo = lane & 15, h = lane >> 4;
    const crec4* tab = (const crec4*)p.cp2_tab;
    StgB st{(ldsd*)smem_, 0, stg_table()};
    if (bid < nbF) {
        const Rec t0 = tab[kCpFamRecs * bid], t1 = tab[kCpFamRecs * bid + 1], t2 = tab[kCpFamRecs * bid + 2];
        const int i0 = t1.z, i1 = t1.w, P = i1 - i0;
        const int cb = t0.x, ce = t0.y, C = ce - cb, y0 = t0.z, Y = t0.w - t0.z;
        const ldsp<T> X = st.arr(z + p.X0 + (size_t)i0 * nx, P * nx);
        const ldsp<T> U = st.arr(z + p.U0 + (size_t)i0 * nu, P * nu);
        const ldsp<T> Yv = st.arr(z + p.Y0 + y0, Y);
        const ldsp<T> S = st.arr(z + p.S0 + i0, P);
        const ldsp<T> Tc = st.arr(z + p.T0 + cb, C);
        const ldsp<T> CD = st.arr((const T*)p.cond + cb, C);
        const ldsp<Rec> FR = st.arr(p.frec + i0, P);
        const ldsp<Rec> CR = st.arr(p.crec + cb, C);
        st.issue();
        WFr<T, RTX> wq;
        WFr<T, RTU> wr;
        wq.load((const T*)p.SQ, t2.x, nx);
        wr.load((const T*)p.SR, t2.y, nu);
        dma_wait();
        lds_sync();
        const int ntc = (C + 15) >> 4;
        for (int t = wv; t < ntc; t += nw) {
            const int j0 = 16 * t, ja = j0 + lo;
            const bool la = ja < C;
            const int ai = la ? CR[ja].x - i0 : 0;
            v4 ax[RTX], au[RTU];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) ax[r] = v4{0, 0, 0, 0};
            _Pragma("unroll") for (int r = 0; r < RTU; ++r) au[r] = v4{0, 0, 0, 0};
            tile1<T, RTX, 4 * RTX>(wq, nx, [&](int k, T& a) { if (la) a = X[ai * nx + k]; }, ax);
            tile1<T, RTU, 4 * RTU>(wr, nu, [&](int k, T& a) { if (la) a = U[ai * nu + k]; }, au);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int jn = j0 + MF<T>::row(h, e);
                if (jn >= C) continue;
                const int j = cb + jn;
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r < nx) eg[e3(p, j) + r] = ax[rt][e];
                }
                _Pragma("unroll") for (int rt = 0; rt < RTU; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r < nu) eg[e4(p, j) + r] = au[rt][e];
                }
                if (lo == 0) {
                    const T hv = T(0.5) * Tc[jn];
                    eg[p.E5 + j] = hv;
                    eg[p.E6 + j] = hv;
                }
            }
        }
        // eta7 = [x; u] (boxed) | eta1 = y | eta2 = s - b'y, b = [p; 0; 1]: one flat task list
        const int nD = P * (nx + nu), nF = nD + Y, nG = nF + P;
        for (int q = tid; q < nG; q += blockDim.x) {
            if (q < nD) {
                const int ii = q / (nx + nu), rr = q - ii * (nx + nu);
                const int o7 = FR[ii].w;
                if (o7 >= 0) eg[o7 + rr] = rr < nx ? X[ii * nx + rr] : U[ii * nu + rr - nx];
            } else if (q < nF) {
                const int e = q - nD;
                eg[p.E1 + y0 + e] = Yv[e];
            } else {
                const int ii = q - nF;
                const Rec fr = FR[ii];
                const int c = fr.y, yo = fr.x - y0, cl = fr.z - cb;
                T by = T(0);
                for (int k = 0; k < c; ++k) by = fma(CD[cl + k], Yv[yo + k], by);
                for (int k = c; k < 2 * c; ++k) by += T(0) * Yv[yo + k];
                by += Yv[yo + 2 * c];
                eg[p.E2 + i0 + ii] = S[ii] - by;
            }
        }
    } else {
        const int lb = bid - nbF;
        const Rec t0 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb], t1 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb + 1];
        const int l0 = t0.z, l1 = t0.w, Lc = l1 - l0;
        const ldsp<T> X = st.arr(z + p.X0 + (size_t)l0 * nx, Lc * nx);
        const ldsp<T> S = st.arr(z + p.S0 + l0, Lc);
        const ldsp<Rec> LR = st.arr(p.lrec + (l0 - p.m), Lc);
        st.issue();
        WFr<T, RTX> wp;
        wp.load((const T*)p.SP, t1.x, nx);
        dma_wait();
        lds_sync();
        const int ntl = (Lc + 15) >> 4;
        for (int t = wv; t < ntl; t += nw) {
            const int q0 = 16 * t, qa = q0 + lo;
            const bool la = qa < Lc;
            v4 ax[RTX];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) ax[r] = v4{0, 0, 0, 0};
            tile1<T, RTX, 4 * RTX>(wp, nx, [&](int k, T& a) { if (la) a = X[qa * nx + k]; }, ax);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int qn = q0 + MF<T>::row(h, e);
                if (qn >= Lc) continue;
                const int l = l0 + qn;
                const Rec lr = LR[qn];
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r < nx) {
                        eg[e11(p, l) + r] = ax[rt][e];
                        if (lr.z >= 0) eg[lr.z + r] = X[qn * nx + r];
                    }
                }
                if (lo == 0) {
                    const T hv = T(0.5) * S[qn];
                    eg[p.E12 + l] = hv;
                    eg[p.E13 + l] = hv;
                }
            }
        }
    }
}

template <class T, int RTX, int RTU>
__global__ void __launch_bounds__(256) k_ellt2(Dev p, const double* __restrict__ eta_, double* __restrict__ z_,
                                               int nbF) {
    typedef typename MF<T>::v4 v4;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    const int nx = p.nx, nu = p.nu;
    const T* d = (const T*)eta_;
    glbp<T> zg = (glbp<T>)z_;
    const int bid = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, nw = blockDim.x >> 6;
    const int lo = lane & 15, h = lane >> 4;
    const crec4* tab = (const crec4*)p.cp2_tab;
    StgB st{(ldsd*)smem_, 0, stg_table()};
    if (bid < nbF) {
        const Rec t0 = tab[kCpFamRecs * bid], t1 = tab[kCpFamRecs * bid + 1], t2 = tab[kCpFamRecs * bid + 2];
        const int i0 = t1.z, i1 = t1.w, P = i1 - i0;
        const int cb = t0.x, ce = t0.y, C = ce - cb, y0 = t0.z, Y = t0.w - t0.z, e7a = t1.x, E7n = t1.y - t1.x;
        const ldsp<T> D1 = st.arr(d + p.E1 + y0, Y);
        const ldsp<T> D2 = st.arr(d + p.E2 + i0, P);
        const ldsp<T> D3 = st.arr(d + e3(p, cb), C * nx);
        const ldsp<T> D4 = st.arr(d + e4(p, cb), C * nu);
        const ldsp<T> D5 = st.arr(d + p.E5 + cb, C);
        const ldsp<T> D6 = st.arr(d + p.E6 + cb, C);
        const ldsp<T> D7 = st.arr(d + e7a, E7n);
        const ldsp<T> CD = st.arr((const T*)p.cond + cb, C);
        const ldsp<Rec> FR = st.arr(p.frec + i0, P);
        st.issue();
        const int creg = t2.z;
        WFr<T, RTX> wq;
        WFr<T, RTU> wr;
        wq.load((const T*)p.SQ, t2.x, nx);
        wr.load((const T*)p.SR, t2.y, nu);
        dma_wait();
        lds_sync();
        auto row_out = [&](int q, bool isx, int r, T sum) {
            const int o7 = FR[q].w;
            T acc = o7 >= 0 ? D7[o7 - e7a + (isx ? r : nx + r)] : T(0);
            acc += sum;
            if (isx) zg[p.X0 + (size_t)(i0 + q) * nx + r] = acc;
            else zg[p.U0 + (size_t)(i0 + q) * nu + r] = acc;
        };
        if (creg > 0) {
            // per-parent tiles: element e of this lane is child e % c of parent h + 4 (e / c)
            const int Q = 4 / creg, PT = 4 * Q;
            const int hA = MF<T>::h_of(lo), eA = MF<T>::e_of(lo);
            const int pA = hA + 4 * (eA / creg), kA = eA % creg;
            const int ntp = (P + PT - 1) / PT;
            auto pass = [&](auto rtc, const auto& wf, int n, ldsp<T> DD, bool isx) {
                constexpr int RT = decltype(rtc)::value;
                for (int t = wv; t < ntp; t += nw) {
                    const int pb = t * PT;
                    const bool la = eA < Q * creg && pb + pA < P;
                    const int ja = la ? (pb + pA) * creg + kA : 0;
                    v4 acc[RT];
                    _Pragma("unroll") for (int r = 0; r < RT; ++r) acc[r] = v4{0, 0, 0, 0};
                    tile1<T, RT, 4 * RT>(wf, n, [&](int k, T& a) { if (la) a = DD[ja * n + k]; }, acc);
                    _Pragma("unroll") for (int sl = 0; sl < 4; ++sl) {
                        const int q = pb + h + 4 * sl;
                        if (sl >= Q || q >= P) continue;
                        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                            const int r = 16 * rt + lo;
                            if (r >= n) continue;
                            T sum = T(0);
                            _Pragma("unroll") for (int e = 0; e < 4; ++e)
                                if (e / creg == sl && e < Q * creg) sum += acc[rt][e];
                            row_out(q, isx, r, sum);
                        }
                    }
                }
            };
            pass(std::integral_constant<int, RTX>{}, wq, nx, D3, true);
            pass(std::integral_constant<int, RTU>{}, wr, nu, D4, false);
        } else {
            // irregular block: child products into LDS, then per-parent sums in child order
            typedef __attribute__((address_space(3))) T lT;
            lT* PX = (lT*)((__attribute__((address_space(3))) char*)smem_ + st.o);
            lT* PU = PX + C * nx;
            const int ntc = (C + 15) >> 4;
            auto prod = [&](auto rtc, const auto& wf, int n, ldsp<T> DD, lT* PO) {
                constexpr int RT = decltype(rtc)::value;
                for (int t = wv; t < ntc; t += nw) {
                    const int j0 = 16 * t, ja = j0 + lo;
                    const bool la = ja < C;
                    v4 acc[RT];
                    _Pragma("unroll") for (int r = 0; r < RT; ++r) acc[r] = v4{0, 0, 0, 0};
                    tile1<T, RT, 4 * RT>(wf, n, [&](int k, T& a) { if (la) a = DD[ja * n + k]; }, acc);
                    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                        const int jn = j0 + MF<T>::row(h, e);
                        if (jn >= C) continue;
                        _Pragma("unroll") for (int rt = 0; rt < RT; ++rt) {
                            const int r = 16 * rt + lo;
                            if (r < n) PO[jn * n + r] = acc[rt][e];
                        }
                    }
                }
            };
            prod(std::integral_constant<int, RTX>{}, wq, nx, D3, PX);
            prod(std::integral_constant<int, RTU>{}, wr, nu, D4, PU);
            lds_sync();
            for (int e = tid; e < P * (nx + nu); e += blockDim.x) {
                const int q = e / (nx + nu), rr = e - q * (nx + nu);
                const bool isx = rr < nx;
                const int r = isx ? rr : rr - nx, n_ = isx ? nx : nu;
                const lT* PP = isx ? PX : PU;
                const Rec fr = FR[q];
                T sum = T(0);
                for (int jj = fr.z - cb; jj < fr.z - cb + fr.y; ++jj) sum += PP[jj * n_ + r];
                row_out(q, isx, r, sum);
            }
        }
        // y = eta1 - b eta2 | s = eta2 | tau_j = (eta5 + eta6) / 2
        const int G = 2 * p.cmax + 1;
        const int nD = P * G, nE = nD + P, nF = nE + C;
        for (int q = tid; q < nF; q += blockDim.x) {
            if (q < nD) {
                const int ii = q / G, k = q - ii * G;
                const Rec fr = FR[ii];
                const int c = fr.y;
                if (k < 2 * c + 1) {
                    const T b = k < c ? CD[fr.z - cb + k] : (k < 2 * c ? T(0) : T(1));
                    zg[p.Y0 + fr.x + k] = D1[fr.x - y0 + k] - b * D2[ii];
                }
            } else if (q < nE) {
                const int ii = q - nD;
                zg[p.S0 + i0 + ii] = D2[ii];
            } else {
                const int jj = q - nE;
                zg[p.T0 + cb + jj] = T(0.5) * (D5[jj] + D6[jj]);
            }
        }
    } else {
        const int lb = bid - nbF;
        const Rec t0 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb], t1 = tab[kCpFamRecs * nbF + kCpLeafRecs * lb + 1];
        const int l0 = t0.z, l1 = t0.w, Lc = l1 - l0;
        const int e14a = t0.x, E14n = t0.y - t0.x;
        const ldsp<T> D11 = st.arr(d + e11(p, l0), Lc * nx);
        const ldsp<T> D14 = st.arr(d + e14a, E14n);
        const ldsp<T> D12 = st.arr(d + p.E12 + l0, Lc);
        const ldsp<T> D13 = st.arr(d + p.E13 + l0, Lc);
        const ldsp<Rec> LR = st.arr(p.lrec + (l0 - p.m), Lc);
        st.issue();
        WFr<T, RTX> wp;
        wp.load((const T*)p.SP, t1.x, nx);
        dma_wait();
        lds_sync();
        const int ntl = (Lc + 15) >> 4;
        for (int t = wv; t < ntl; t += nw) {
            const int q0 = 16 * t, qa = q0 + lo;
            const bool la = qa < Lc;
            v4 ax[RTX];
            _Pragma("unroll") for (int r = 0; r < RTX; ++r) ax[r] = v4{0, 0, 0, 0};
            tile1<T, RTX, 4 * RTX>(wp, nx, [&](int k, T& a) { if (la) a = D11[qa * nx + k]; }, ax);
            _Pragma("unroll") for (int e = 0; e < 4; ++e) {
                const int qn = q0 + MF<T>::row(h, e);
                if (qn >= Lc) continue;
                const int l = l0 + qn;
                const int o14 = LR[qn].z;
                _Pragma("unroll") for (int rt = 0; rt < RTX; ++rt) {
                    const int r = 16 * rt + lo;
                    if (r < nx) zg[p.X0 + (size_t)l * nx + r] = o14 >= 0 ? ax[rt][e] + D14[o14 - e14a + r] : ax[rt][e];
                }
                if (lo == 0) zg[p.S0 + l] = T(0.5) * (D12[qn] + D13[qn]);
            }
        }
    }
}
