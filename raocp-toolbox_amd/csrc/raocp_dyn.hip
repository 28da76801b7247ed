// raocp_dyn.hip — projection of (x, u) onto the tree dynamics (cache.py:259-288).
// Included by raocp_kernels.hip (inside namespace raocp).
//
// Reference recursion (offline P, K, Abar = A + BK, R~ = I + sum B'PB per node):
//   backward, stage N-1 .. 0, nonleaf i (a leaf child j has q_j = -x_j):
//     d_i = R~^-1 (u_i - sum_j B_j' q_j)
//     q_i = (-x_i + K_i'(d_i - u_i)) + sum_j Abar_j' (P_j B_j d_i + q_j)
//   forward, stage 0 .. N-1:  x_0 = x0bar ; u_i = K_i x_i + d_i ; x_j = Abar_j x_i + B_j d_i.
// Device form. With h = sum_j B_j' q_j, a = sum_j A_j' q_j, v = u - h and the per-class
// M = K' + sum_j Abar_j' P_j B_j, G = M R~^-1 - K' (host, raocp_capi.hip):
//     d = R~^-1 v ,  q = (-x + a) + G v                      (backward, 2 phases)
//     u = K x + d ,  x_j = [Abar_j | B_j] [x; d]              (forward, 1 phase)
// so a backward level is two phases and a forward level one, each ending in one
// workgroup barrier. Tables (row-major, zero-padded, 16-B aligned rows):
//   W [kind][nu+nx][KP]   rows B' then A' of the child's (A, B) pair
//   RG[cls ][nu+nx][NUP]  rows R~^-1 then G
//   KM[cls ][nu   ][KP]   K
//   F [pair][nx   ][KF]   [Abar | B | 0] of (child kind, parent class)
// KP = nx rounded up to 8, KF = nx + nu rounded up to 8, NUP = nu rounded up to 2.
//
// Lane mapping ("split-k"): every output row of a dot product of length KP (or KF) is
// produced by KS = 4 consecutive lanes, each reading one 16-B-aligned slice of the
// matrix row (global, L1/L2-resident) and of the vector row (LDS) with 16-byte loads,
// then reduced with two xor-shuffles. A child's rows are R = nu + nx consecutive
// groups. This keeps each lane's dependent chain to KP/4 (KF/4) FMAs, which is what a
// level costs when the tree is narrow (the top stages), and spreads wide levels over
// all lanes of the workgroup.
//
// Launch structure (the recursion is sequential in the stage): the tree is cut at
// stage s;
//   k_dyn_bottom_back — one workgroup per subtree rooted at stage s, levels N-1..s;
//   k_dyn_top        — ONE workgroup: stages s-1..0 backward, then 0..s-1 forward;
//   k_dyn_bottom_fwd — one workgroup per subtree, levels s..N-1 forward.
// Vectors of the nodes a kernel covers are staged into LDS in its prologue (padded
// rows with zero tails), so the dependent steps only touch LDS for vectors.
// Trees that do not fit run one launch per phase and stage on padded global rows
// (k_dyn_gather, k_dyn_stage_a / _b / _f).

constexpr int kKS = 4;
constexpr int kDynBlock = 1024;

typedef double d2v __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2v lds2;
typedef __attribute__((address_space(1))) d2v glb2;

__device__ __forceinline__ d2v ld2(const ldsd* p) { return *(const lds2*)p; }
__device__ __forceinline__ d2v ld2(const glbd* p) { return *(const glb2*)p; }

constexpr __host__ __device__ int rup(int a, int b) { return (a + b - 1) / b * b; }
// row stride of a matrix table whose rows hold k (even) doubles: an odd number of 16-B
// units, so the ds_read_b128 of lanes reading different rows spread over the banks
constexpr __host__ __device__ int tstride(int k) { return (k / 2) % 2 == 0 ? k + 2 : k; }

template <int NXc, int NUc>
struct Geo {
    int nx, nu, R, KP, KF, NUP, PH, PS, SKP, SKF, SNU;  // S*: table row strides
    __device__ __forceinline__ Geo(const Dev& p) {
        nx = NXc ? NXc : p.nx;
        nu = NUc ? NUc : p.nu;
        R = nu + nx;
        KP = rup(nx, 2 * kKS);
        KF = rup(nx + nu, 2 * kKS);
        NUP = rup(nu, 2);
        PH = NUP;                   // child product row: [h (NUP) | a (nx, even-padded)]
        PS = NUP + rup(nx, 2);
        SKP = tstride(KP);
        SKF = tstride(KF);
        SNU = tstride(NUP);
    }
    // compile-time padded lengths (0: runtime)
    static constexpr int cKP = NXc ? rup(NXc, 2 * kKS) : 0;
    static constexpr int cKF = NXc ? rup(NXc + NUc, 2 * kKS) : 0;
    static constexpr int cNUP = NUc ? rup(NUc, 2) : 0;
};

// sum_k m[k] v[k] over kc (even) elements, both 16-B aligned; all loads issued first
template <int KC, class PM, class PV>
__device__ __forceinline__ double dot_slice(PM m, PV v, int kc) {
    if constexpr (KC == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (int k = 0; k < kc; k += 2) {
            const d2v a = ld2(m + k), b = ld2(v + k);
            s0 = fma(a.x, b.x, s0);
            s1 = fma(a.y, b.y, s1);
        }
        return s0 + s1;
    } else if constexpr (KC > 12) {
        // long slices (KS = 1 on wide levels) in batches of 8 doubles: loading a whole
        // 24 / 32-element slice of matrix and vector at once needs 2 KC VGPRs, which at 1024
        // threads (128 VGPRs) spilled the whole kernel to scratch
        double s0 = 0.0, s1 = 0.0;
        _Pragma("unroll") for (int k0 = 0; k0 < KC; k0 += 8) {
            constexpr int B = 4;
            d2v a[B], b[B];
            _Pragma("unroll") for (int t = 0; t < B; ++t) {
                if (k0 + 2 * t < KC) {
                    a[t] = ld2(m + k0 + 2 * t);
                    b[t] = ld2(v + k0 + 2 * t);
                }
            }
            _Pragma("unroll") for (int t = 0; t < B; ++t) {
                if (k0 + 2 * t < KC) {
                    s0 = fma(a[t].x, b[t].x, s0);
                    s1 = fma(a[t].y, b[t].y, s1);
                }
            }
        }
        return s0 + s1;
    } else {
        d2v a[KC / 2], b[KC / 2];
        _Pragma("unroll") for (int t = 0; t < KC / 2; ++t) {
            a[t] = ld2(m + 2 * t);
            b[t] = ld2(v + 2 * t);
        }
        __builtin_amdgcn_sched_barrier(0);
        double s0 = 0.0, s1 = 0.0;
        _Pragma("unroll") for (int t = 0; t < KC / 2; ++t) {
            s0 = fma(a[t].x, b[t].x, s0);
            s1 = fma(a[t].y, b[t].y, s1);
        }
        return s0 + s1;
    }
}

// xor-exchange within lane quads by DPP (VALU, no LDS round trip)
template <int CTRL>
__device__ __forceinline__ double dpp_quad(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

// reduce over the KS consecutive lanes of a split-k group (all live or all idle)
template <int KS>
__device__ __forceinline__ double ks_reduce(double v) {
    if constexpr (KS >= 2) v += dpp_quad<0xB1>(v);  // quad_perm [1,0,3,2]: lane ^ 1
    if constexpr (KS >= 4) v += dpp_quad<0x4E>(v);  // quad_perm [2,3,0,1]: lane ^ 2
    return v;
}

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations
// (lgkmcnt) but not for its outstanding global stores (vmcnt) — __syncthreads() would
// wait for every z / d store of the level to reach L2. No kernel here reads back,
// within the launch, global data another lane wrote.
__device__ __forceinline__ void lds_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}

template <class P>
struct RowsT {
    P base;
    int off;
    int stride;
    __device__ __forceinline__ P operator()(int j) const { return base + (size_t)(j - off) * stride; }
};
typedef RowsT<ldsd*> LRows;
typedef RowsT<glbd*> GRows;

template <class IP>
struct InfoT {
    IP nl;  // nonleaf records {ch_start, nch, class, stage}
    int n0;
    IP ch;  // child records {kind, pair, anc, 0}
    int c0;
    __device__ __forceinline__ Rec nonleaf(int i) const { return nl[i - n0]; }
    __device__ __forceinline__ Rec child(int j) const { return ch[j - c0]; }
};

// matrix tables as seen by a kernel: W, RG, KM in one address space, F in another;
// classes / pairs are rebased by c0 / p0 when a kernel stages only its stages' range
template <class PW, class PF>
struct TabsT {
    PW W;
    PW RG;
    PW KM;
    PF F;
    int c0, p0;
};
typedef TabsT<const glbd*, const glbd*> GTabs;
__device__ __forceinline__ GTabs dyn_tabs(const Dev& p) {
    return GTabs{(const glbd*)p.dW, (const glbd*)p.dRG, (const glbd*)p.dKM, (const glbd*)p.dF, 0, 0};
}

// ---- backward phase A: child products p_j = sign [B' ; A'] q_j for children [cb, ce) --
// qin(j): padded row (KP) of q_j (or x_j for leaf children, sign = -1); P(j): PS-row.
// KS lanes per output row (split-k); the caller picks KS from the level's width.
template <int KS, int NXc, int NUc, class TB, class INF, class QI, class PO>
__device__ __forceinline__ void back_phase_a_ks(const Dev& p, const TB& tb, const INF& inf, int cb, int ce, QI qin,
                                                double sign, PO pout, int tid, int nthr) {
    const Geo<NXc, NUc> g(p);
    constexpr int cKC = Geo<NXc, NUc>::cKP / KS;
    const int KC = g.KP / KS;
    const int per = g.R * KS;
    const int slots = nthr / per;
    const int slot = tid / per, rem = tid - slot * per, rho = rem / KS, sl = rem - rho * KS;
    for (int first = cb; first < ce; first += slots) {
        const int j = first + slot;
        if (slot < slots && j < ce) {
            const Rec cj = inf.child(j);
            const auto w = tb.W + ((size_t)cj.x * g.R + rho) * g.SKP + sl * KC;
            double acc = dot_slice<cKC>(w, qin(j) + sl * KC, KC);
            acc = ks_reduce<KS>(acc) * sign;
            if (sl == 0) pout(j)[rho < g.nu ? rho : g.PH + rho - g.nu] = acc;
        }
    }
}

template <int NXc, int NUc, class TB, class INF, class QI, class PO>
__device__ __forceinline__ void back_phase_a(const Dev& p, const TB& tb, const INF& inf, int cb, int ce, QI qin,
                                             double sign, PO pout, int tid, int nthr) {
    const int items = (ce - cb) * (NXc ? NXc + NUc : p.nx + p.nu);
    if (items * 4 <= nthr) back_phase_a_ks<4, NXc, NUc>(p, tb, inf, cb, ce, qin, sign, pout, tid, nthr);
    else if (items * 2 <= nthr) back_phase_a_ks<2, NXc, NUc>(p, tb, inf, cb, ce, qin, sign, pout, tid, nthr);
    else back_phase_a_ks<1, NXc, NUc>(p, tb, inf, cb, ce, qin, sign, pout, tid, nthr);
}

// ---- backward phase B: per node d = RG[0:nu] v, q = (-x + a) + RG[nu:] v ------------
template <int NXc, int NUc, class TB, class INF, class PI, class XI, class UI, class QO, class DO>
__device__ __forceinline__ void back_phase_b(const Dev& p, const TB& tb, const INF& inf, int b, int e, PI pin,
                                             XI xin, UI uin, QO qout, DO dout, int tid, int nthr) {
    const Geo<NXc, NUc> g(p);
    constexpr int cNUP = Geo<NXc, NUc>::cNUP;
    const int slots = nthr / g.R;
    const int slot = tid / g.R, t = tid - slot * g.R;
    for (int first = b; first < e; first += slots) {
        const int i = first + slot;
        if (slot < slots && i < e) {
            const Rec ni = inf.nonleaf(i);
            const auto u = uin(i);
            const auto rg = tb.RG + ((size_t)(ni.z - tb.c0) * g.R + t) * g.SNU;
            double out;
            if constexpr (cNUP > 0) {
                d2v v[cNUP / 2], m[cNUP / 2];
                _Pragma("unroll") for (int k = 0; k < cNUP / 2; ++k) {
                    m[k] = ld2(rg + 2 * k);
                    v[k] = ld2(u + 2 * k);
                }
                for (int q = 0; q < ni.y; ++q) {
                    const auto pr = pin(ni.x + q);
                    _Pragma("unroll") for (int k = 0; k < cNUP / 2; ++k) v[k] -= ld2(pr + 2 * k);
                }
                double s0 = 0.0, s1 = 0.0;
                _Pragma("unroll") for (int k = 0; k < cNUP / 2; ++k) {
                    s0 = fma(m[k].x, v[k].x, s0);
                    s1 = fma(m[k].y, v[k].y, s1);
                }
                out = s0 + s1;
            } else {
                double s0 = 0.0, s1 = 0.0;
                for (int k = 0; k < g.NUP; k += 2) {
                    d2v v = ld2(u + k);
                    for (int q = 0; q < ni.y; ++q) v -= ld2(pin(ni.x + q) + k);
                    const d2v m = ld2(rg + k);
                    s0 = fma(m.x, v.x, s0);
                    s1 = fma(m.y, v.y, s1);
                }
                out = s0 + s1;
            }
            if (t < g.nu) {
                dout(i)[t] = out;
            } else {
                const int r = t - g.nu;
                double a = 0.0;
                for (int q = 0; q < ni.y; ++q) a += pin(ni.x + q)[g.PH + r];
                qout(i)[r] = (-xin(i)[r] + a) + out;
            }
        }
    }
}

// ---- backward level in ONE phase (phases A and B folded) ------------------------------
// With the per-pair table WT_j = [-Rinv B_j' ; A_j' - G B_j'] (host) the level is
//     out = RG u_i + sign * sum_j WT_j q_j ;  d_i = out[0:nu] ,  q_i = -x_i + out[nu:]
// (the same algebra as phases A + B, re-associated): every output row is one split-k dot
// over the node's children and its own u, so a level costs one barrier instead of two and
// no P rows go through LDS. tb.W = WT (pairs rebased by tb.p0), tb.RG = RG (classes by c0).
template <int KS, int NXc, int NUc, class TB, class INF, class QI, class XI, class UI, class QO, class DO>
__device__ __forceinline__ void back_fold_ks(const Dev& p, const TB& tb, const INF& inf, int b, int e, QI qin,
                                             double sign, XI xin, UI uin, QO qout, DO dout, int tid, int nthr) {
    const Geo<NXc, NUc> g(p);
    constexpr int cKC = Geo<NXc, NUc>::cKP / KS;
    const int KC = g.KP / KS;
    const int per = g.R * KS;
    const int slots = nthr / per;
    const int slot = tid / per, rem = tid - slot * per, t = rem / KS, sl = rem - t * KS;
    for (int first = b; first < e; first += slots) {
        const int i = first + slot;
        if (slot < slots && i < e) {
            const Rec ni = inf.nonleaf(i);
            double acc = 0.0;
            for (int q = 0; q < ni.y; ++q) {
                const int j = ni.x + q;
                const Rec cj = inf.child(j);
                const auto w = tb.W + ((size_t)(cj.y - tb.p0) * g.R + t) * g.SKP + sl * KC;
                acc += dot_slice<cKC>(w, qin(j) + sl * KC, KC);
            }
            acc *= sign;
            const auto rg = tb.RG + ((size_t)(ni.z - tb.c0) * g.R + t) * g.SNU;
            const auto u = uin(i);
            for (int k = 2 * sl; k < g.NUP; k += 2 * KS) {
                const d2v m = ld2(rg + k), v = ld2(u + k);
                acc = fma(m.x, v.x, acc);
                acc = fma(m.y, v.y, acc);
            }
            acc = ks_reduce<KS>(acc);
            if (sl == 0) {
                if (t < g.nu) dout(i)[t] = acc;
                else qout(i)[t - g.nu] = -xin(i)[t - g.nu] + acc;
            }
        }
    }
}

template <int NXc, int NUc, class TB, class INF, class QI, class XI, class UI, class QO, class DO>
__device__ __forceinline__ void back_fold(const Dev& p, const TB& tb, const INF& inf, int b, int e, QI qin,
                                          double sign, XI xin, UI uin, QO qout, DO dout, int tid, int nthr) {
    const int items = (e - b) * (NXc ? NXc + NUc : p.nx + p.nu);
    if (items * 4 <= nthr) back_fold_ks<4, NXc, NUc>(p, tb, inf, b, e, qin, sign, xin, uin, qout, dout, tid, nthr);
    else if (items * 2 <= nthr) back_fold_ks<2, NXc, NUc>(p, tb, inf, b, e, qin, sign, xin, uin, qout, dout, tid, nthr);
    else back_fold_ks<1, NXc, NUc>(p, tb, inf, b, e, qin, sign, xin, uin, qout, dout, tid, nthr);
}

// ---- forward: u_i = K x_i + d_i (nodes [b, e)), x_j = F [x_i; d_i] (their children) ---
// xd(i): padded row [x_i | d_i | 0] (KF); child rows also go to xdo(j) when XOUT.
// SCX: the children's x rows are stored write-through (st_sc1): another workgroup of the
// same launch reads them (the split sweep, raocp_dynf.hip)
template <int KS, int NXc, int NUc, bool XOUT, bool SCX, class TB, class INF, class XDI, class XDO>
__device__ __forceinline__ void fwd_phase_ks(const Dev& p, const TB& tb, const INF& inf, int b, int e, int cb, int ce,
                                             XDI xd, glbd* z, XDO xdo, int tid, int nthr) {
    const Geo<NXc, NUc> g(p);
    constexpr int cKCP = Geo<NXc, NUc>::cKP / KS, cKCF = Geo<NXc, NUc>::cKF / KS;
    const int KCP = g.KP / KS, KCF = g.KF / KS;
    const int nU = (e - b) * g.nu * KS;    // u items (lanes)
    const int nX = (ce - cb) * g.nx * KS;  // x items (lanes)
    for (int base = 0; base < nU + nX; base += nthr) {
        const int vi = base + tid;
        if (vi < nU) {
            const int grp = vi / KS, sl = vi - grp * KS;
            const int i = b + grp / g.nu, r = grp - (grp / g.nu) * g.nu;
            const Rec ni = inf.nonleaf(i);
            const auto row = xd(i);
            const auto km = tb.KM + ((size_t)(ni.z - tb.c0) * g.nu + r) * g.SKP + sl * KCP;
            double acc = dot_slice<cKCP>(km, row + sl * KCP, KCP);
            acc = ks_reduce<KS>(acc);
            if (sl == 0) z[p.U0 + (size_t)i * g.nu + r] = acc + row[g.nx + r];
        } else if (vi < nU + nX) {
            const int wi = vi - nU;
            const int grp = wi / KS, sl = wi - grp * KS;
            const int j = cb + grp / g.nx, r = grp - (grp / g.nx) * g.nx;
            const Rec cj = inf.child(j);
            const auto f = tb.F + ((size_t)(cj.y - tb.p0) * g.nx + r) * g.SKF + sl * KCF;
            double acc = dot_slice<cKCF>(f, xd(cj.z) + sl * KCF, KCF);
            acc = ks_reduce<KS>(acc);
            if (sl == 0) {
                if constexpr (SCX) st_sc1((double*)(z + p.X0 + (size_t)j * g.nx + r), acc);
                else z[p.X0 + (size_t)j * g.nx + r] = acc;
                if (XOUT) xdo(j)[r] = acc;
            }
        }
    }
}

template <int NXc, int NUc, bool XOUT, bool SCX = false, class TB, class INF, class XDI, class XDO>
__device__ __forceinline__ void fwd_phase(const Dev& p, const TB& tb, const INF& inf, int b, int e, XDI xd, glbd* z,
                                          XDO xdo, int tid, int nthr) {
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    const int cb = inf.nonleaf(b).x;
    const Rec last = inf.nonleaf(e - 1);
    const int ce = last.x + last.y;
    const int items = (e - b) * nu + (ce - cb) * nx;
    if (items * 4 <= nthr) fwd_phase_ks<4, NXc, NUc, XOUT, SCX>(p, tb, inf, b, e, cb, ce, xd, z, xdo, tid, nthr);
    else if (items * 2 <= nthr) fwd_phase_ks<2, NXc, NUc, XOUT, SCX>(p, tb, inf, b, e, cb, ce, xd, z, xdo, tid, nthr);
    else fwd_phase_ks<1, NXc, NUc, XOUT, SCX>(p, tb, inf, b, e, cb, ce, xd, z, xdo, tid, nthr);
}


// the iterate the sweep projects: buffers arrive rotated for the iteration, so no ctl read
__device__ __forceinline__ glbd* dyn_z(const Bufs& bf, int zsel, const Ctl*) { return pick3(bf, zsel); }

// copy `rows` rows of `cols` doubles (source stride sstride) into padded rows of stride
// dstride, zero tail; loads batched so several are in flight per thread
template <class PD, class PS>
__device__ __forceinline__ void copy_rows(PD dst, int dstride, PS src, int sstride, int rows, int cols, int tid,
                                          int nthr) {
    const int total = rows * dstride;
    constexpr int U = 8;
    for (int base = tid; base < total; base += U * nthr) {
        double v[U];
        _Pragma("unroll") for (int k = 0; k < U; ++k) {
            const int e = base + k * nthr;
            const int r = e / dstride, c = e - r * dstride;
            v[k] = (e < total && c < cols) ? (double)src[(size_t)r * sstride + c] : 0.0;
        }
        _Pragma("unroll") for (int k = 0; k < U; ++k) {
            const int e = base + k * nthr;
            if (e < total) dst[e] = v[k];
        }
    }
}

template <class PD>
__device__ __forceinline__ void zero_fill(PD dst, int count, int tid, int nthr) {
    for (int e = tid; e < count; e += nthr) dst[e] = 0.0;
}

// ---- per-stage path on padded global rows (any tree) ----------------------------------
// gather: XQ[j] = x_j (padded KP), U[i] = u_i (padded NUP), XD[i] = [0 | 0 | 0]
template <int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_dyn_gather(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                        double* xq_, double* u_, double* xd_) {
    if (ctl && ctl->done) return;
    const Geo<NXc, NUc> g(p);
    const glbd* z = dyn_z(bf, zsel, ctl);
    const int tid = blockIdx.x * blockDim.x + threadIdx.x, nthr = gridDim.x * blockDim.x;
    copy_rows((glbd*)xq_, g.KP, z + p.X0, g.nx, p.n, g.nx, tid, nthr);
    copy_rows((glbd*)u_, g.NUP, z + p.U0, g.nu, p.m, g.nu, tid, nthr);
    zero_fill((glbd*)xd_, p.m * g.KF, tid, nthr);
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(kDynBlock) k_dyn_stage_a(Dev p, const Ctl* ctl, const double* xq_,
                                                         double* pb_, int cb, int ce, double sign) {
    if (ctl && ctl->done) return;
    const Geo<NXc, NUc> g(p);
    const InfoT<glbrec*> inf{(glbrec*)p.ninfo, 0, (glbrec*)p.cinfo, 0};
    const int per = g.R * kKS, slots = blockDim.x / per;
    const int c0 = cb + blockIdx.x * slots;
    back_phase_a<NXc, NUc>(p, dyn_tabs(p), inf, c0, min(ce, c0 + slots), GRows{(glbd*)xq_, 0, g.KP}, sign,
                           GRows{(glbd*)pb_, 0, g.PS}, threadIdx.x, blockDim.x);
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(kDynBlock) k_dyn_stage_b(Dev p, const Ctl* ctl, double* xq_,
                                                         const double* u_, const double* pb_, double* xd_, double* d_,
                                                         int b, int e) {
    if (ctl && ctl->done) return;
    const Geo<NXc, NUc> g(p);
    const InfoT<glbrec*> inf{(glbrec*)p.ninfo, 0, (glbrec*)p.cinfo, 0};
    const int slots = blockDim.x / g.R;
    const int b0 = b + blockIdx.x * slots;
    const GRows xq{(glbd*)xq_, 0, g.KP};
    // d goes to the padded forward rows (XD cols nx..) and to the d buffer
    struct DOut {
        glbd* xd;
        glbd* d;
        int KF, nx, nu;
        struct Ref {
            glbd* a;
            glbd* b;
            __device__ __forceinline__ void operator=(double v) const { *a = v; *b = v; }
        };
        struct Row {
            glbd* a;
            glbd* b;
            __device__ __forceinline__ Ref operator[](int r) const { return Ref{a + r, b + r}; }
        };
        __device__ __forceinline__ Row operator()(int i) const {
            return Row{xd + (size_t)i * KF + nx, d + (size_t)i * nu};
        }
    } dout{(glbd*)xd_, (glbd*)d_, g.KF, g.nx, g.nu};
    back_phase_b<NXc, NUc>(p, dyn_tabs(p), inf, b0, min(e, b0 + slots), GRows{(glbd*)pb_, 0, g.PS}, xq,
                           RowsT<const glbd*>{(const glbd*)u_, 0, g.NUP}, xq, dout, threadIdx.x, blockDim.x);
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(kDynBlock) k_dyn_stage_f(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                         double* xd_, const double* x0_, int b, int e) {
    if (ctl && ctl->done) return;
    const Geo<NXc, NUc> g(p);
    glbd* z = dyn_z(bf, zsel, ctl);
    glbd* xd = (glbd*)xd_;
    const InfoT<glbrec*> inf{(glbrec*)p.ninfo, 0, (glbrec*)p.cinfo, 0};
    if (b == 0) {  // x_0 = x0bar (cache.py:282): one workgroup, one node
        if ((int)threadIdx.x < g.nx) {
            const double v = ((const glbd*)x0_)[threadIdx.x];
            xd[threadIdx.x] = v;
            z[p.X0 + threadIdx.x] = v;
        }
        __syncthreads();
    }
    // blocks over (parent) nodes: each block takes whole parents so its children follow
    const int per_node = g.nu * kKS + p.cmax * g.nx * kKS;
    const int slots = max(1, (int)blockDim.x / per_node);
    const int b0 = b + blockIdx.x * slots;
    const int e0 = min(e, b0 + slots);
    const bool xout = inf.nonleaf(b).w + 1 < p.N;
    if (xout)
        fwd_phase<NXc, NUc, true>(p, dyn_tabs(p), inf, b0, e0, GRows{xd, 0, g.KF}, z, GRows{xd, 0, g.KF}, threadIdx.x,
                                  blockDim.x);
    else
        fwd_phase<NXc, NUc, false>(p, dyn_tabs(p), inf, b0, e0, GRows{xd, 0, g.KF}, z, GRows{xd, 0, g.KF},
                                   threadIdx.x, blockDim.x);
}

// ---- subtree-blocked sweep ------------------------------------------------------------
constexpr int kMaxLevels = 31;    // tier depth limit (host plans within it)
constexpr int kMaxTopStages = 62; // cut stage limit of k_dyn_top

struct Prologue {
    int lo[kMaxLevels + 1], hi[kMaxLevels + 1], off[kMaxLevels + 1];
    int sp[kMaxTopStages + 2];  // stage_ptr[0 .. s+1] (top)
    unsigned long long ts[64];  // diagnostics (p.stamps != nullptr)
    int nts;                    // next stamp slot (the split sweep)
};

// diagnostics: thread 0 records the 100 MHz clock in LDS; flushed at the end of the kernel
__device__ __forceinline__ void tstamp(const Dev& p, Prologue& pl, int slot) {
    if (kDiag && p.stamps && threadIdx.x == 0 && slot < 64) pl.ts[slot] = __builtin_amdgcn_s_memrealtime();
}
__device__ __forceinline__ void tflush(const Dev& p, const Prologue& pl, int n) {
    if (kDiag && p.stamps && threadIdx.x == 0 && blockIdx.x == 0)
        for (int k = 0; k < n && k < 64; ++k) p.stamps[k] = pl.ts[k];
}

// Prologue copies are LDS-DMA (global_load_lds_dwordx4): every wave issues its share of
// 16-B chunks straight into LDS and nothing waits until the single vmcnt(0) at the end,
// so a prologue costs about one memory round trip. The destination of one wave
// instruction is linear (base + lane * 16 B), the source is per lane: padded rows are
// filled chunk by chunk, tail chunks reading a page of zeros (p.zpage).
// Group g (64 chunks) goes to wave (g + rot) mod nw: callers staging many small regions
// rotate the start so the issue cost (≈100+ cycles per instruction) is spread over the
// waves instead of queueing on wave 0. Returns the number of groups.
template <class SrcF>
__device__ __forceinline__ int dma_gen(ldsd* dst, int chunks, SrcF src, int rot = 0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
    const int g0 = ((wave - rot) % nw + nw) % nw;
    for (int c0 = g0 * 64; c0 < chunks; c0 += nw * 64) {
        const int ch = c0 + lane;
        if (ch < chunks) __builtin_amdgcn_global_load_lds((const glbd*)src(ch), dst + 2 * c0, 16, 0, 0);
    }
    return (chunks + 63) >> 6;
}
// contiguous range of n (even) doubles, 16-B aligned at both ends
__device__ __forceinline__ void dma(ldsd* dst, const double* src, int n) {
    dma_gen(dst, n >> 1, [=](int ch) { return src + 2 * ch; });
}
// rows x cols (even) doubles, source row stride sstride (even, rows 16-B aligned) ->
// LDS rows of w (even) doubles with a zero tail
__device__ __forceinline__ void dma_rows(ldsd* dst, int w, const double* src, int sstride, int cols, int rows,
                                         const double* zp) {
    const int cpr = w >> 1, cc = cols >> 1;
    dma_gen(dst, rows * cpr, [=](int ch) {
        const int r = ch / cpr, c = ch - r * cpr;
        return c < cc ? src + (size_t)r * sstride + 2 * c : zp;
    });
}
__device__ __forceinline__ void dma_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }
// The CP stop flag, read by a kernel AFTER it has issued its prologue loads: the flag was
// written by the previous launch (another XCD's L2), so the load costs a memory round trip,
// and a scalar load is waited for where its value is first needed — at the top of the
// kernel, that wait serialised the round trip ahead of the whole prologue.
__device__ __forceinline__ int ctl_done(const Ctl* ctl) { return ctl ? ctl->done : 0; }

// register path for odd sizes / unaligned rows (same result as dma_rows; used only when
// nx or nu is odd)
__device__ __forceinline__ void copy_rows_reg(ldsd* dst, int w, const double* src, int sstride, int cols, int rows,
                                              int tid, int nthr) {
    for (int e = tid; e < rows * w; e += nthr) {
        const int r = e / w, c = e - r * w;
        dst[e] = c < cols ? ((const glbd*)src)[(size_t)r * sstride + c] : 0.0;
    }
}
__device__ __forceinline__ void rows_in(bool dmaok, ldsd* dst, int w, const double* src, int sstride, int cols,
                                        int rows, const double* zp, int tid, int nthr) {
    if (dmaok) dma_rows(dst, w, src, sstride, cols, rows, zp);
    else copy_rows_reg(dst, w, src, sstride, cols, rows, tid, nthr);
}
// The same copies with a rotating first wave (Dev::dyn_rot): a prologue of many small
// ranges would otherwise put the first (often only) instruction of every range on wave 0,
// which then issues them one after another. rot < 0: rotation off (every range starts at
// wave 0); else the next range starts where the previous one ended.
__device__ __forceinline__ void dma_r(ldsd* dst, const double* src, int n, int& rot) {
    const int g = dma_gen(dst, n >> 1, [=](int ch) { return src + 2 * ch; }, rot < 0 ? 0 : rot);
    if (rot >= 0) rot += g;
}
__device__ __forceinline__ void rows_in_r(bool dmaok, ldsd* dst, int w, const double* src, int sstride, int cols,
                                          int rows, const double* zp, int tid, int nthr, int& rot) {
    if (!dmaok) {
        copy_rows_reg(dst, w, src, sstride, cols, rows, tid, nthr);
        return;
    }
    const int cpr = w >> 1, cc = cols >> 1;
    const int g = dma_gen(dst, rows * cpr, [=](int ch) {
        const int r = ch / cpr, c = ch - r * cpr;
        return c < cc ? src + (size_t)r * sstride + 2 * c : zp;
    }, rot < 0 ? 0 : rot);
    if (rot >= 0) rot += g;
}

// level ranges of a tier's subtree: from the kernel argument when the tier is regular
// (every subtree the same shape, ids consecutive), else from the host table
struct TierArg {
    int regular;
    int boff;  // first subtree of this launch (a shard launches only the subtrees it owns)
    int lo0[kMaxLevels + 1];
    int cnt[kMaxLevels + 1];
    int pl0[kMaxLevels + 1];  // first (kind, class) pair of the parents of level l (absolute)
};

// level l's node range {lo, hi, off} of this workgroup's subtree: computed from the kernel
// argument when the tier is regular (wave-uniform arithmetic, no LDS round trip and no
// barrier before the prologue's row copies are issued), else read from the staged table
// (after tier_levels and a barrier)
struct LvR {
    int lo, hi, off;
};
__device__ __forceinline__ LvR lv_of(const Prologue& pl, const TierArg& ta, int l, int off) {
    if (ta.regular) {
        const int lo = ta.lo0[l] + (blockIdx.x + ta.boff) * ta.cnt[l];
        return LvR{lo, lo + ta.cnt[l], off};
    }
    return LvR{pl.lo[l], pl.hi[l], pl.off[l]};
}

__device__ __forceinline__ void tier_levels(Prologue& pl, const TierArg& ta, const Rec* __restrict__ sub_lv, int L) {
    const int l = threadIdx.x;
    if (l > L) return;
    if (ta.regular) {
        int off = 0;
        for (int k = 0; k < l; ++k) off += ta.cnt[k];
        pl.lo[l] = ta.lo0[l] + (blockIdx.x + ta.boff) * ta.cnt[l];
        pl.hi[l] = pl.lo[l] + ta.cnt[l];
        pl.off[l] = off;
    } else {
        const Rec r = sub_lv[(size_t)(blockIdx.x + ta.boff) * (L + 1) + l];
        pl.lo[l] = r.x;
        pl.hi[l] = r.y;
        pl.off[l] = r.z;
    }
}

// table sizes in doubles (host mirrors these in raocp_capi.hip)
template <int NXc, int NUc>
struct TabSize {
    int W1, RG1, KM1, F1;  // per kind / class / class / pair
    __device__ __forceinline__ TabSize(const Geo<NXc, NUc>& g) {
        W1 = g.R * g.SKP;
        RG1 = g.R * g.SNU;
        KM1 = g.nu * g.SKP;
        F1 = g.nx * g.SKF;
    }
};

// LDS plan (doubles from the dynamic base), tier backward:
//   [W (all kinds) | RG (classes c0..c1) | XQ rows (all subtree nodes, KP) | U rows (nonleaf, NUP)
//    | P rows (maxch, PS) | NL records | CH records]
// FOLD (one-phase levels): W -> WT (pairs p0..p1), no P rows.
// The boundary level (s1) holds the leaves' x (q = -x) or q of the next tier's roots.
template <int NXc, int NUc, bool FOLD>
__global__ void __launch_bounds__(kDynBlock) k_dyn_bottom_back(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                                double* qbuf_, double* dbuf_, int s, int s1, int maxch,
                                                                int c0, int c1, int p0, int p1,
                                                                const Rec* __restrict__ sub_lv, TierArg ta, ChkArg ck) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Prologue pl;
    // block 0 of a launch with ck.on: the previous CP iteration's stopping test (the host
    // shifts ta.boff by one, so the subtrees stay blocks 1..)
    if (ck.on && blockIdx.x == 0) {
        if (threadIdx.x < 64) cp_check_wave(ck);
        return;
    }
    tstamp(p, pl, 0);
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const bool dmaok = (g.nx % 2 == 0) && (g.nu % 2 == 0);
    const int tid = threadIdx.x, nthr = blockDim.x;
    ldsd* smem = (ldsd*)smem_;
    const int L = s1 - s;
    const bool leaves = s1 == p.N;
    const int nW = FOLD ? (p1 - p0) * ts.W1 : p.nkind * ts.W1;
    const int oW = 0, oRG = oW + nW, oXQ = oRG + (c1 - c0) * ts.RG1;
    const double* srcW = FOLD ? p.dWT + (size_t)p0 * ts.W1 : p.dW;
    const double* srcRG = p.dRG + (size_t)c0 * ts.RG1;
    int rot = p.dyn_rot ? 0 : -1;
    dma_r(smem + oW, srcW, nW, rot);
    dma_r(smem + oRG, srcRG, (c1 - c0) * ts.RG1, rot);
    tier_levels(pl, ta, sub_lv, L);
    glbd* z = dyn_z(bf, zsel, ctl);
    if (!ta.regular) lds_sync();
    tstamp(p, pl, 1);
    int nnl = 0;
    for (int l = 0; l < L; ++l) nnl += ta.regular ? ta.cnt[l] : 0;
    if (!ta.regular) nnl = pl.off[L];
    const int nall = nnl + (ta.regular ? ta.cnt[L] : pl.hi[L] - pl.lo[L]);
    ldsd* XQ = smem + oXQ;
    ldsd* U = XQ + (size_t)nall * g.KP;
    ldsd* PB = U + (size_t)nnl * g.NUP;
    ldsd* NLd = PB + (FOLD ? 0 : rup(maxch * g.PS, 2));
    ldsd* CHd = NLd + 2 * nnl;
    for (int l = 0, off = 0; l <= L; ++l) {
        const LvR lv = lv_of(pl, ta, l, off);
        const int cnt = lv.hi - lv.lo;
        off += cnt;
        if (l < L || leaves)
            rows_in_r(dmaok, XQ + (size_t)lv.off * g.KP, g.KP, (const double*)z + p.X0 + (size_t)lv.lo * g.nx,
                      g.nx, g.nx, cnt, p.zpage, tid, nthr, rot);
        else  // q rows of the next tier's roots, already padded
            dma_r(XQ + (size_t)lv.off * g.KP, qbuf_ + (size_t)lv.lo * g.KP, cnt * g.KP, rot);
        if (l < L) {
            rows_in_r(dmaok, U + (size_t)lv.off * g.NUP, g.NUP, (const double*)z + p.U0 + (size_t)lv.lo * g.nu,
                      g.nu, g.nu, cnt, p.zpage, tid, nthr, rot);
            dma_r(NLd + 2 * lv.off, (const double*)(p.ninfo + lv.lo), 2 * cnt, rot);
        }
        if (l > 0) dma_r(CHd + 2 * (lv.off - 1), (const double*)(p.cinfo + lv.lo), 2 * cnt, rot);
    }
    if (!FOLD) zero_fill(PB, maxch * g.PS, tid, nthr);
    const int done = ctl_done(ctl);
    dma_wait();
    lds_sync();
    tstamp(p, pl, 2);
    if (done) return;
    tstamp(p, pl, 3);
    const ldsrec* NL = (const ldsrec*)NLd;
    const ldsrec* CH = (const ldsrec*)CHd;
    const TabsT<const ldsd*, const ldsd*> tb{smem + oW, smem + oRG, nullptr, nullptr, c0, FOLD ? p0 : 0};
    const GRows dg{(glbd*)dbuf_, 0, g.nu};
    for (int l = L - 1; l >= 0; --l) {
        const InfoT<const ldsrec*> inf{NL + pl.off[l], pl.lo[l], CH + pl.off[l + 1] - 1, pl.lo[l + 1]};
        const LRows xq_l{XQ + (size_t)pl.off[l] * g.KP, pl.lo[l], g.KP};
        const LRows xq_c{XQ + (size_t)pl.off[l + 1] * g.KP, pl.lo[l + 1], g.KP};
        const LRows ur{U + (size_t)pl.off[l] * g.NUP, pl.lo[l], g.NUP};
        if constexpr (FOLD) {
            const double sign = (l + 1 == L && leaves) ? -1.0 : 1.0;
            if (l > 0) {
                back_fold<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], xq_c, sign, xq_l, ur, xq_l, dg, tid, nthr);
            } else {
                const GRows qroot{(glbd*)qbuf_, 0, g.KP};
                back_fold<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], xq_c, sign, xq_l, ur, qroot, dg, tid, nthr);
            }
            lds_sync();
            tstamp(p, pl, 4 + 2 * (L - 1 - l));
            continue;
        }
        const LRows pr{PB, pl.lo[l + 1], g.PS};
        back_phase_a<NXc, NUc>(p, tb, inf, pl.lo[l + 1], pl.hi[l + 1], xq_c, (l + 1 == L && leaves) ? -1.0 : 1.0, pr,
                               tid, nthr);
        lds_sync();
        tstamp(p, pl, 4 + 2 * (L - 1 - l));
        if (l > 0) {
            back_phase_b<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], pr, xq_l, ur, xq_l, dg, tid, nthr);
        } else {
            const GRows qroot{(glbd*)qbuf_, 0, g.KP};  // q of the subtree root, padded row
            back_phase_b<NXc, NUc>(p, tb, inf, pl.lo[l], pl.hi[l], pr, xq_l, ur, qroot, dg, tid, nthr);
        }
        lds_sync();
        tstamp(p, pl, 5 + 2 * (L - 1 - l));
    }
    tflush(p, pl, 4 + 2 * L);
}

// tier forward: [KM (classes c0..c1) | F | XD rows (nonleaf, KF) | NL | CH]
// XD rows = [x (the root's; the others are written by the sweep) | d | 0]
// FM: where the [A_bar | B] rows F live. 0: global (L2); 1: every pair of the tier (p0..p1)
// staged in the prologue; 2: only the pairs of one level's parents (ta.pl0[l] ..
// ta.pl0[l + 1]), restaged before each level — a deep tier whose whole F does not fit LDS
// reads its rows from LDS anyway, for one LDS round trip per level.
template <int NXc, int NUc, int FM>
__global__ void __launch_bounds__(kDynBlock) k_dyn_bottom_fwd(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                               const double* dbuf_, int s, int s1, int c0, int c1,
                                                               int p0, int p1, const Rec* __restrict__ sub_lv,
                                                               TierArg ta) {
    constexpr bool FL = FM != 0;
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Prologue pl;
    tstamp(p, pl, 0);
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const bool dmaok = (g.nx % 2 == 0) && (g.nu % 2 == 0);
    const int tid = threadIdx.x, nthr = blockDim.x;
    ldsd* smem = (ldsd*)smem_;
    const int L = s1 - s;
    int npl = p1 - p0;  // pairs held in LDS
    if constexpr (FM == 2) {
        npl = 0;
        for (int l = 0; l < L; ++l) npl = max(npl, ta.pl0[l + 1] - ta.pl0[l]);
    }
    const int oKM = 0, oF = oKM + (c1 - c0) * ts.KM1, oXD = oF + (FL ? npl * ts.F1 : 0);
    int rot = p.dyn_rot ? 0 : -1;
    dma_r(smem + oKM, p.dKM + (size_t)c0 * ts.KM1, (c1 - c0) * ts.KM1, rot);
    if (FM == 1) dma_r(smem + oF, p.dF + (size_t)p0 * ts.F1, (p1 - p0) * ts.F1, rot);
    if (FM == 2) dma_r(smem + oF, p.dF + (size_t)ta.pl0[0] * ts.F1, (ta.pl0[1] - ta.pl0[0]) * ts.F1, rot);
    tier_levels(pl, ta, sub_lv, L);
    glbd* z = dyn_z(bf, zsel, ctl);
    if (!ta.regular) lds_sync();
    tstamp(p, pl, 1);
    int nnl = 0;
    for (int l = 0; l < L; ++l) nnl += ta.regular ? ta.cnt[l] : 0;
    if (!ta.regular) nnl = pl.off[L];
    const int root = lv_of(pl, ta, 0, 0).lo;
    ldsd* XD = smem + oXD;
    ldsd* NLd = XD + (size_t)nnl * g.KF;
    ldsd* CHd = NLd + 2 * nnl;
    const double* xroot = (const double*)z + p.X0 + (size_t)root * g.nx;
    const double* zp = p.zpage;
    for (int l = 0, off = 0; l < L; ++l) {
        const LvR lv = lv_of(pl, ta, l, off);
        const LvR lc = lv_of(pl, ta, l + 1, off + (lv.hi - lv.lo));
        const int cnt = lv.hi - lv.lo;
        off += cnt;
        ldsd* xd = XD + (size_t)lv.off * g.KF;
        const double* dl = dbuf_ + (size_t)lv.lo * g.nu;
        if (dmaok) {
            const int cpr = g.KF >> 1, cx = g.nx >> 1, cd = (g.nx + g.nu) >> 1;
            const bool first = l == 0;
            const int gx = dma_gen(xd, cnt * cpr, [=](int ch) {
                const int r = ch / cpr, c = ch - r * cpr;
                if (c < cx) return (first && r == 0) ? xroot + 2 * c : zp;
                if (c < cd) return dl + (size_t)r * g.nu + 2 * (c - cx);
                return zp;
            }, rot < 0 ? 0 : rot);
            if (rot >= 0) rot += gx;
        } else {
            for (int e = tid; e < cnt * g.KF; e += nthr) {
                const int r = e / g.KF, c = e - r * g.KF;
                double v = 0.0;
                if (c < g.nx) v = (l == 0 && r == 0) ? ((const glbd*)xroot)[c] : 0.0;
                else if (c < g.nx + g.nu) v = ((const glbd*)dl)[(size_t)r * g.nu + c - g.nx];
                xd[e] = v;
            }
        }
        dma_r(NLd + 2 * lv.off, (const double*)(p.ninfo + lv.lo), 2 * cnt, rot);
        const int cc = lc.hi - lc.lo;
        dma_r(CHd + 2 * (lc.off - 1), (const double*)(p.cinfo + lc.lo), 2 * cc, rot);
    }
    const int done = ctl_done(ctl);
    dma_wait();
    lds_sync();
    tstamp(p, pl, 2);
    if (done) return;
    tstamp(p, pl, 3);
    const ldsrec* NL = (const ldsrec*)NLd;
    const ldsrec* CH = (const ldsrec*)CHd;
    typedef typename std::conditional<FL, const ldsd*, const glbd*>::type PF;
    TabsT<const ldsd*, PF> tb{nullptr, nullptr, smem + oKM,
                              FL ? (PF)(smem + oF) : (PF)((const glbd*)p.dF), c0, FL ? p0 : 0};
    for (int l = 0; l < L; ++l) {
        if constexpr (FM == 2) {
            tb.p0 = ta.pl0[l];
            if (l > 0) {  // level l-1's products are done (the barrier that ended it)
                dma(smem + oF, p.dF + (size_t)ta.pl0[l] * ts.F1, (ta.pl0[l + 1] - ta.pl0[l]) * ts.F1);
                dma_wait();
                lds_sync();
            }
        }
        const InfoT<const ldsrec*> inf{NL + pl.off[l], pl.lo[l], CH + pl.off[l + 1] - 1, pl.lo[l + 1]};
        const LRows xd_l{XD + (size_t)pl.off[l] * g.KF, pl.lo[l], g.KF};
        if (l + 1 < L) {
            const LRows xd_c{XD + (size_t)pl.off[l + 1] * g.KF, pl.lo[l + 1], g.KF};
            fwd_phase<NXc, NUc, true>(p, tb, inf, pl.lo[l], pl.hi[l], xd_l, z, xd_c, tid, nthr);
        } else {
            fwd_phase<NXc, NUc, false>(p, tb, inf, pl.lo[l], pl.hi[l], xd_l, z, xd_l, tid, nthr);
        }
        lds_sync();
        tstamp(p, pl, 4 + l);
    }
    tflush(p, pl, 4 + L);
}

// the top of the tree (stages < s, nodes 0..T-1) in one workgroup, backward then forward:
//   [W | RG | KM | F (if FL) | XQ (T, KP) | QB (boundary, KP) | U (T, NUP) | XD (T, KF) |
//    P (maxch, PS) | NL (T) | CH (T + nb - 1)]
// FOLD (one-phase backward levels): W -> WT (pairs 0..p1), no P rows.
template <int NXc, int NUc, bool FL, bool FOLD>
__global__ void __launch_bounds__(kDynBlock) k_dyn_top(Dev p, Bufs bf, const Ctl* ctl, int zsel,
                                                        const double* qbuf_, const double* x0_, int s, int maxch,
                                                        int c1, int p1, int T, int nb) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ Prologue pl;
    tstamp(p, pl, 0);
    const Geo<NXc, NUc> g(p);
    const TabSize<NXc, NUc> ts(g);
    const bool dmaok = (g.nx % 2 == 0) && (g.nu % 2 == 0);
    const int tid = threadIdx.x, nthr = blockDim.x;
    ldsd* smem = (ldsd*)smem_;
    const bool leaves = s == p.N;
    const int nW = FOLD ? p1 * ts.W1 : p.nkind * ts.W1;
    const int oW = 0, oRG = oW + nW, oKM = oRG + c1 * ts.RG1, oF = oKM + c1 * ts.KM1;
    const int oXQ = oF + (FL ? p1 * ts.F1 : 0), oQB = oXQ + T * g.KP, oU = oQB + nb * g.KP, oXD = oU + T * g.NUP;
    const int oP = oXD + T * g.KF, oNL = oP + (FOLD ? 0 : rup(maxch * g.PS, 2)), oCH = oNL + 2 * T;
    int rot = p.dyn_rot ? 0 : -1;
    dma_r(smem + oW, FOLD ? p.dWT : p.dW, nW, rot);
    dma_r(smem + oRG, p.dRG, c1 * ts.RG1, rot);
    dma_r(smem + oKM, p.dKM, c1 * ts.KM1, rot);
    if (FL) dma_r(smem + oF, p.dF, p1 * ts.F1, rot);
    dma_r(smem + oNL, (const double*)p.ninfo, 2 * T, rot);
    dma_r(smem + oCH, (const double*)(p.cinfo + 1), 2 * (T + nb - 1), rot);
    if (tid <= s + 1) pl.sp[tid] = p.stage_ptr[tid];
    glbd* z = dyn_z(bf, zsel, ctl);
    rows_in_r(dmaok, smem + oXQ, g.KP, (const double*)z + p.X0, g.nx, g.nx, T, p.zpage, tid, nthr, rot);
    if (leaves)
        rows_in_r(dmaok, smem + oQB, g.KP, (const double*)z + p.X0 + (size_t)T * g.nx, g.nx, g.nx, nb, p.zpage, tid,
                  nthr, rot);
    else
        dma_r(smem + oQB, qbuf_ + (size_t)T * g.KP, nb * g.KP, rot);
    rows_in_r(dmaok, smem + oU, g.NUP, (const double*)z + p.U0, g.nu, g.nu, T, p.zpage, tid, nthr, rot);
    zero_fill(smem + oXD, T * g.KF, tid, nthr);
    if (!FOLD) zero_fill(smem + oP, maxch * g.PS, tid, nthr);
    const int done = ctl_done(ctl);
    dma_wait();
    lds_sync();
    if (done) return;
    tstamp(p, pl, 1);
    tstamp(p, pl, 2 + 3 * s);
    tstamp(p, pl, 3 + 3 * s);
    typedef typename std::conditional<FL, const ldsd*, const glbd*>::type PF;
    const TabsT<const ldsd*, PF> tb{smem + oW, smem + oRG, smem + oKM,
                                    FL ? (PF)(smem + oF) : (PF)((const glbd*)p.dF), 0, 0};
    const InfoT<const ldsrec*> inf{(const ldsrec*)(smem + oNL), 0, (const ldsrec*)(smem + oCH), 1};
    ldsd* XD = smem + oXD;
    const LRows xq{smem + oXQ, 0, g.KP}, qb{smem + oQB, T, g.KP}, ur{smem + oU, 0, g.NUP}, xd{XD, 0, g.KF};
    const LRows dlds{XD + g.nx, 0, g.KF};  // d_i into XD row i, cols nx..
    for (int t = s - 1; t >= 0; --t) {
        const int b = pl.sp[t], e = pl.sp[t + 1];
        const int cb = e, ce = pl.sp[t + 2];
        if constexpr (FOLD) {
            const double sign = (t + 1 == s && leaves) ? -1.0 : 1.0;
            if (t + 1 < s) back_fold<NXc, NUc>(p, tb, inf, b, e, xq, sign, xq, ur, xq, dlds, tid, nthr);
            else back_fold<NXc, NUc>(p, tb, inf, b, e, qb, sign, xq, ur, xq, dlds, tid, nthr);
            lds_sync();
            tstamp(p, pl, 2 + 2 * (s - 1 - t));
            continue;
        }
        const LRows pr{smem + oP, cb, g.PS};
        if (t + 1 < s) back_phase_a<NXc, NUc>(p, tb, inf, cb, ce, xq, 1.0, pr, tid, nthr);
        else back_phase_a<NXc, NUc>(p, tb, inf, cb, ce, qb, leaves ? -1.0 : 1.0, pr, tid, nthr);
        lds_sync();
        tstamp(p, pl, 2 + 2 * (s - 1 - t));
        back_phase_b<NXc, NUc>(p, tb, inf, b, e, pr, xq, ur, xq, dlds, tid, nthr);
        lds_sync();
        tstamp(p, pl, 3 + 2 * (s - 1 - t));
    }
    if (tid < g.nx) {
        const double v = ((const glbd*)x0_)[tid];
        XD[tid] = v;
        z[p.X0 + tid] = v;  // x_0 = x0bar (cache.py:282)
    }
    lds_sync();
    for (int t = 0; t < s; ++t) {
        const int b = pl.sp[t], e = pl.sp[t + 1];
        if (t + 1 < s) fwd_phase<NXc, NUc, true>(p, tb, inf, b, e, xd, z, xd, tid, nthr);
        else fwd_phase<NXc, NUc, false>(p, tb, inf, b, e, xd, z, xd, tid, nthr);
        lds_sync();
        tstamp(p, pl, 2 + 2 * s + t);
    }
    tflush(p, pl, 4 + 3 * s);
}
