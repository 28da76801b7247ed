// raocp_ells.hip — L and L^T (operators.py:19-53, 55-94) as streaming wave-task kernels
// (included by raocp_kernels.hip after raocp_ell.hip, inside namespace raocp).
//
// One wave = one independent task: no LDS, no barriers, few registers, so occupancy (up to
// 8 waves per SIMD) keeps the loads of many tasks in flight per CU and hides the HBM
// latency that bounds the node-range block kernels of raocp_ell.hip.
//   L   product tasks (16 consecutive nodes x 16 weight rows, one v_mfma_f64_16x16x4 chain):
//         Q  eta3_j = sqrtQ_j x_anc(j)   (children j >= 1)
//         R  eta4_j = sqrtR_j u_anc(j)
//         P  eta11_l = sqrtPf_l x_l      (leaves)
//       copy tasks (64 lanes x kEllsE elements of one flat list):
//         eta1 = y | eta2_i = s_i - b_i'y_i | eta5_j = eta6_j = tau_j / 2 | eta7_i = [x_i; u_i]
//         | eta12_l = eta13_l = s_l / 2 | eta14_l = x_l          (boxes where active)
//   L^T product tasks over 16 consecutive PARENTS, accumulating child slot q = 0 .. cmax-1:
//         X  x_i = sum_q sqrtQ_j eta3_j + [eta7_i]_x      (j = ch_start_i + q)
//         U  u_i = sum_q sqrtR_j eta4_j + [eta7_i]_u
//         P  x_l = sqrtPf_l eta11_l + eta14_l
//       copy tasks: y_i = eta1_i - b_i eta2_i, s_i = eta2_i | tau_j = (eta5_j + eta6_j) / 2
//         | s_l = (eta12_l + eta13_l) / 2                          (tau_0 is never written)
// MFMA operands: lane (lo, hi) takes the contiguous k slice [hi ks, hi ks + ks), ks = ceil(n/4):
// A = the node's vector (one run of ks doubles straight from HBM), B = the matching weights
// M[k n + r0 + lo] (column-major tables, L2-resident). Result lane (lo, hi), element e:
// node hi + 4e, row r0 + lo. A tile whose nodes use different tables takes a per-lane path.
// Only the summation order differs from the reference (k slices, then the children).
//
// Algorithmic bytes per launch: 8 (|P| + |D|) over active entries, as for raocp_ell.hip.

constexpr int kEllsE = 4;  // copy elements per lane per task

struct EllsPlan {
    int nQ, nR, nP;  // product tasks: node tiles x row tiles
    int rtx, rtu;    // row tiles of nx / nu rows
    int ncopy;       // copy tasks
};

typedef __attribute__((address_space(1))) const int gint;

// acc += 16 nodes x 16 rows of M_tab(node) v(node) for nodes [first, first + cnt); ar(node):
// the node's vector, tab(node): its table (-1 = no contribution)
template <int NC, class AR, class TAB>
__device__ __forceinline__ d4 ells_tile(const double* T, int nr, int first, int cnt, int r0, AR ar, TAB tab, d4 acc) {
    const int n = NC ? NC : nr;
    constexpr int KSC = NC ? (NC + 3) / 4 : 16;
    const int ks = NC ? KSC : (n + 3) / 4;
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
    const bool live = lo < cnt;
    const int node = first + (live ? lo : 0);
    const int ta = live ? tab(node) : -1;
    const unsigned long long bal = __ballot(ta >= 0);
    if (!bal) return acc;
    const int t0 = __shfl(ta, (int)__builtin_ctzll(bal), 64);
    const int r = r0 + lo;
    if (__all(ta < 0 || ta == t0)) {
        const glbd* M = (const glbd*)(T + (size_t)t0 * n * n);
        const glbd* va = ta >= 0 ? (const glbd*)ar(node) : nullptr;
        double a[KSC], b[KSC];
        _Pragma("unroll") for (int s = 0; s < KSC; ++s) {
            const int k = hi * ks + s;
            const bool ok = s < ks && k < n;
            a[s] = (va && ok) ? va[k] : 0.0;
            b[s] = (ok && r < n) ? M[k * n + r] : 0.0;
        }
        _Pragma("unroll") for (int s = 0; s < KSC; ++s)
            if (s < ks) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a[s], b[s], acc, 0, 0, 0);
    } else {
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e;
            if (nd < cnt && r < n) {
                const int t = tab(first + nd);
                if (t >= 0) {
                    const glbd* M = (const glbd*)(T + (size_t)t * n * n) + r;
                    const glbd* x = (const glbd*)ar(first + nd);
                    double s0 = 0.0, s1 = 0.0;
                    int k = 0;
                    for (; k + 1 < n; k += 2) {
                        s0 = fma(M[k * n], x[k], s0);
                        s1 = fma(M[(k + 1) * n], x[k + 1], s1);
                    }
                    if (k < n) s0 = fma(M[k * n], x[k], s0);
                    acc[e] += s0 + s1;
                }
            }
        }
    }
    return acc;
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(256) k_ells(Dev p, EllsPlan pl, const double* __restrict__ z,
                                              double* __restrict__ eta) {
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    int w = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
    const glbd* zg = (const glbd*)z;
    glbd* eg = (glbd*)eta;
    gint* anc = (gint*)p.anc;
    const d4 zero = {0.0, 0.0, 0.0, 0.0};
    if (w < pl.nQ) {  // eta3_j = sqrtQ_j x_anc(j)
        const int tile = w / pl.rtx, r0 = (w - tile * pl.rtx) * 16;
        const int first = 1 + tile * 16, cnt = min(16, p.n - first);
        const d4 d = ells_tile<NXc>(
            p.SQ, nx, first, cnt, r0, [&](int j) { return zg + p.X0 + (size_t)anc[j] * nx; },
            [&](int j) { return ((gint*)p.iSQ)[j]; }, zero);
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e, r = r0 + lo;
            if (nd < cnt && r < nx) eg[e3(p, first + nd) + r] = d[e];
        }
        return;
    }
    w -= pl.nQ;
    if (w < pl.nR) {  // eta4_j = sqrtR_j u_anc(j)
        const int tile = w / pl.rtu, r0 = (w - tile * pl.rtu) * 16;
        const int first = 1 + tile * 16, cnt = min(16, p.n - first);
        const d4 d = ells_tile<NUc>(
            p.SR, nu, first, cnt, r0, [&](int j) { return zg + p.U0 + (size_t)anc[j] * nu; },
            [&](int j) { return ((gint*)p.iSR)[j]; }, zero);
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e, r = r0 + lo;
            if (nd < cnt && r < nu) eg[e4(p, first + nd) + r] = d[e];
        }
        return;
    }
    w -= pl.nR;
    if (w < pl.nP) {  // eta11_l = sqrtPf_l x_l
        const int tile = w / pl.rtx, r0 = (w - tile * pl.rtx) * 16;
        const int first = p.m + tile * 16, cnt = min(16, p.n - first);
        const d4 d = ells_tile<NXc>(
            p.SP, nx, first, cnt, r0, [&](int q) { return zg + p.X0 + (size_t)q * nx; },
            [&](int q) { return ((gint*)p.iSP)[q]; }, zero);
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e, r = r0 + lo;
            if (nd < cnt && r < nx) eg[e11(p, first + nd) + r] = d[e];
        }
        return;
    }
    w -= pl.nP;
    // copies: flat list [eta1 (ny) | eta2 (m) | eta5,6 (n-1) | eta7 (m (nx+nu)) | eta12,13 (n-m) |
    // eta14 ((n-m) nx)]; all loads of a task before its stores
    const int n = p.n, m = p.m, R = nx + nu;
    const int ny = p.T0 - p.Y0;
    const int sB = ny, sC = sB + m, sD = sC + (n - 1), sE = sD + m * R, sF = sE + (n - m), tot = sF + (n - m) * nx;
    double v[kEllsE];
    int d0[kEllsE], d1[kEllsE];
    _Pragma("unroll") for (int u = 0; u < kEllsE; ++u) {
        const int t = (w * kEllsE + u) * 64 + l;
        d0[u] = d1[u] = -1;
        v[u] = 0.0;
        if (t >= tot) continue;
        if (t < sB) {  // eta1 = y
            d0[u] = p.E1 + t;
            v[u] = zg[p.Y0 + t];
        } else if (t < sC) {  // eta2_i = s_i - b'y_i, b = [p; 0; 1]
            const int i = t - sB;
            const int c = ((gint*)p.nch)[i], cs = ((gint*)p.ch_start)[i], yo = ((gint*)p.yrel)[i];
            const glbd* y = zg + p.Y0 + yo;
            double by = 0.0;
            for (int k = 0; k < c; ++k) by = fma(((const glbd*)p.cond)[cs + k], y[k], by);
            for (int k = c; k < 2 * c; ++k) by += 0.0 * y[k];
            by += y[2 * c];
            d0[u] = p.E2 + i;
            v[u] = zg[p.S0 + i] - by;
        } else if (t < sD) {  // eta5 = eta6 = tau_j / 2
            const int j = 1 + t - sC;
            d0[u] = p.E5 + j;
            d1[u] = p.E6 + j;
            v[u] = 0.5 * zg[p.T0 + j];
        } else if (t < sE) {  // eta7_i = [x_i; u_i] (boxed nonleaf)
            const int e = t - sD, i = e / R, rr = e - i * R;
            const int o7 = ((gint*)p.e7off)[i];
            if (o7 >= 0) {
                d0[u] = o7 + rr;
                v[u] = rr < nx ? zg[p.X0 + (size_t)i * nx + rr] : zg[p.U0 + (size_t)i * nu + rr - nx];
            }
        } else if (t < sF) {  // eta12 = eta13 = s_l / 2
            const int q = m + t - sE;
            d0[u] = p.E12 + q;
            d1[u] = p.E13 + q;
            v[u] = 0.5 * zg[p.S0 + q];
        } else {  // eta14_l = x_l (boxed leaves)
            const int e = t - sF, q = e / nx, r = e - q * nx;
            const int o14 = ((gint*)p.e14off)[q];
            if (o14 >= 0) {
                d0[u] = o14 + r;
                v[u] = zg[p.X0 + (size_t)(m + q) * nx + r];
            }
        }
    }
    _Pragma("unroll") for (int u = 0; u < kEllsE; ++u) {
        if (d0[u] >= 0) eg[d0[u]] = v[u];
        if (d1[u] >= 0) eg[d1[u]] = v[u];
    }
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(256) k_ellts(Dev p, EllsPlan pl, const double* __restrict__ eta,
                                               double* __restrict__ z) {
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    int w = __builtin_amdgcn_readfirstlane((int)((blockIdx.x * blockDim.x + threadIdx.x) >> 6));
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
    const glbd* eg = (const glbd*)eta;
    glbd* zg = (glbd*)z;
    gint* chs = (gint*)p.ch_start;
    gint* nch = (gint*)p.nch;
    gint* e7o = (gint*)p.e7off;
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    if (w < pl.nQ + pl.nR) {  // x_i (Q rows) / u_i (R rows) of parents [first, first + 16)
        const bool isx = w < pl.nQ;
        const int ww = isx ? w : w - pl.nQ, rt = isx ? pl.rtx : pl.rtu, n = isx ? nx : nu;
        const int tile = ww / rt, r0 = (ww - tile * rt) * 16;
        const int first = tile * 16, cnt = min(16, p.m - first);
        for (int q = 0; q < p.cmax; ++q) {
            if (isx)
                acc = ells_tile<NXc>(
                    p.SQ, nx, first, cnt, r0, [&](int i) { return eg + e3(p, chs[i] + q); },
                    [&](int i) { return q < nch[i] ? ((gint*)p.iSQ)[chs[i] + q] : -1; }, acc);
            else
                acc = ells_tile<NUc>(
                    p.SR, nu, first, cnt, r0, [&](int i) { return eg + e4(p, chs[i] + q); },
                    [&](int i) { return q < nch[i] ? ((gint*)p.iSR)[chs[i] + q] : -1; }, acc);
        }
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e, r = r0 + lo;
            if (nd < cnt && r < n) {
                const int i = first + nd, o7 = e7o[i];
                const double g7 = o7 >= 0 ? (double)eg[o7 + (isx ? 0 : nx) + r] : 0.0;
                if (isx) zg[p.X0 + (size_t)i * nx + r] = acc[e] + g7;
                else zg[p.U0 + (size_t)i * nu + r] = acc[e] + g7;
            }
        }
        return;
    }
    w -= pl.nQ + pl.nR;
    if (w < pl.nP) {  // x_l = sqrtPf_l eta11_l + eta14_l
        const int tile = w / pl.rtx, r0 = (w - tile * pl.rtx) * 16;
        const int first = p.m + tile * 16, cnt = min(16, p.n - first);
        acc = ells_tile<NXc>(
            p.SP, nx, first, cnt, r0, [&](int q) { return eg + e11(p, q); }, [&](int q) { return ((gint*)p.iSP)[q]; },
            acc);
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e, r = r0 + lo;
            if (nd < cnt && r < nx) {
                const int q = first + nd, o14 = ((gint*)p.e14off)[q - p.m];
                zg[p.X0 + (size_t)q * nx + r] = acc[e] + (o14 >= 0 ? (double)eg[o14 + r] : 0.0);
            }
        }
        return;
    }
    w -= pl.nP;
    // copies: [nonleaf i: y_i = eta1_i - b eta2_i, s_i = eta2_i (m) | tau_j (n-1) | leaf s_l (n-m)]
    const int n = p.n, m = p.m;
    const int sB = m, sC = sB + (n - 1), tot = sC + (n - m);
    _Pragma("unroll") for (int u = 0; u < kEllsE; ++u) {
        const int t = (w * kEllsE + u) * 64 + l;
        if (t >= tot) continue;
        if (t < sB) {
            const int i = t, c = nch[i], cs = chs[i], yo = ((gint*)p.yrel)[i];
            const double e2 = eg[p.E2 + i];
            for (int k = 0; k < 2 * c + 1; ++k) {
                const double b = k < c ? (double)((const glbd*)p.cond)[cs + k] : (k < 2 * c ? 0.0 : 1.0);
                zg[p.Y0 + yo + k] = eg[p.E1 + yo + k] - b * e2;
            }
            zg[p.S0 + i] = e2;
        } else if (t < sC) {
            const int j = 1 + t - sB;
            zg[p.T0 + j] = 0.5 * (eg[p.E5 + j] + eg[p.E6 + j]);
        } else {
            const int q = m + t - sC;
            zg[p.S0 + q] = 0.5 * (eg[p.E12 + q] + eg[p.E13 + q]);
        }
    }
}
