// raocp_dyn.hip — projection of (x, u) onto the tree dynamics (cache.py:259-288).
// Included by raocp_kernels.hip (inside namespace raocp).
//
// Reference recursion (offline P, K, Abar = A + BK, R~ = I + sum B'PB per node):
//   backward, stage N-1 .. 0, nonleaf i (a leaf child j has q_j = -x_j):
//     d_i = R~^-1 (u_i - sum_j B_j' q_j)
//     q_i = (-x_i + K_i'(d_i - u_i)) + sum_j Abar_j' (P_j B_j d_i + q_j)
//   forward, stage 0 .. N-1:  x_0 = x0bar ; u_i = K_i x_i + d_i ; x_j = Abar_j x_i + B_j d_i.
// Device form (same values, re-associated so only per-MODE A, B and per-CLASS
// Rinv, K, M = K' + sum_j Abar_j' P_j B_j are stored, and each backward step needs
// two group exchanges):
//     h = sum_j B_j' q_j ,  a = sum_j A_j' q_j            (lanes r < nu / r < nx)
//     d = Rinv (u - h) ,    w = (-x + K'(h - u)) + a      (exchange h)
//     q = w + M d                                          (exchange d)
//   forward: u = K x + d ; x_j = A_j x + B_j u            (exchange u)
//
// Launch structure. The recursion is sequential in the stage, so the number of
// dependent steps, not bandwidth, sets the time. The tree is cut at a stage s:
//   k_dyn_bottom_back — one workgroup per subtree rooted at stage s, levels N-1..s;
//   k_dyn_top        — ONE workgroup: stages s-1..0 backward, then 0..s-1 forward;
//   k_dyn_bottom_fwd — one workgroup per subtree, levels s..N-1 forward.
// Matrices of the stages a kernel covers are staged into LDS in its prologue (plus,
// for the top, the node records and the x/u/q rows it reads), so the dependent
// steps only touch LDS. Trees that do not fit fall back to one launch per stage
// (k_dyn_back_stage / k_dyn_fwd_stage, everything from global memory).
//
// Every pointer carries its address space in its type (ldsd / glbd), so loads are
// ds_read / global_load, never flat.
//
// Lane mapping: a node is handled by a group of G lanes (lane r owns row r).
// Matrix layouts (padded leading dimension, conflict-free LDS reads):
//   A[mode]  nx x (nx+1)  A(k, r) at k*(nx+1) + r      B[mode] nx x (nu+1)  B(k, c) at k*(nu+1) + c
//   R[cls]   Rinv(r, c) at c*(nu+1) + r                 K[cls]  K(c, r) at c*(nx+1) + r
//   M[cls]   M(r, c) at c*(nx+1) + r

template <class P>
struct RowsT {
    P base;
    int off;
    int stride;
    __device__ __forceinline__ P operator()(int j) const { return base + (size_t)(j - off) * stride; }
};
typedef RowsT<ldsd*> LRows;

// element-wise difference view a[k] - b[k] (for the batched dot products)
template <class PA, class PB>
struct Diff {
    PA a;
    PB b;
    __device__ __forceinline__ double operator[](int k) const { return a[k] - b[k]; }
};
typedef RowsT<glbd*> GRows;

template <class P>
struct MatsT {
    P A, B, R, K, M;
    int cls0;  // class id of slot 0
};

template <class IP>
struct InfoT {
    IP nl;  // nonleaf records {ch_start, nch, class, stage}
    int n0;
    IP ch;  // child records {iA, iB, anc, 0}
    int c0;
    __device__ __forceinline__ Rec nonleaf(int i) const { return nl[i - n0]; }
    __device__ __forceinline__ Rec child(int j) const { return ch[j - c0]; }
};

template <int NXc, int NUc>
struct Dims {
    int nx, nu, SA, SB, SR, SK;
    __device__ __forceinline__ Dims(const Dev& p) {
        nx = NXc ? NXc : p.nx;
        nu = NUc ? NUc : p.nu;
        SA = nx * (nx + 1);
        SB = nx * (nu + 1);
        SR = nu * (nu + 1);
        SK = nu * (nx + 1);
    }
};

// ---- backward step for nonleaf nodes [b, e) of one stage --------------------------
// qin(j): rows of the children's q, or of their x when qsign = -1 (leaf children).
template <int NXc, int NUc, class MT, class INF, class QI, class XI, class UI, class QO, class DO>
__device__ __forceinline__ void back_step(const Dev& p, const MT& mt, const INF& inf, int b, int e, QI qin,
                                          double qsign, XI xin, UI uin, QO qout, DO dout, ldsd* s_h, ldsd* s_d,
                                          int pass0, int pstride) {
    const Dims<NXc, NUc> D(p);
    const int nx = D.nx, nu = D.nu;
    const int G = nx > nu ? nx : nu;
    const int per = blockDim.x / G, gl = threadIdx.x / G, r = threadIdx.x - gl * G, base = gl * G;
    for (int pass = pass0;; pass += pstride) {
        const int first = b + pass * per;
        if (first >= e) break;  // uniform over the workgroup
        const int i = first + gl;
        const bool live = gl < per && i < e;
        Rec ni = {0, 0, 0, 0};
        if (live) ni = inf.nonleaf(i);
        const int cs = ni.x, c = ni.y, cl = ni.z - mt.cls0;
        double h = 0.0, a = 0.0;
        if (live) {
            for (int q = 0; q < c; ++q) {
                const int j = cs + q;
                const Rec cj = inf.child(j);
                const auto row = qin(j);
                if (r < nu) {
                    const auto Bm = mt.B + (size_t)cj.y * D.SB;
                    h += dotb<NXc>(Bm + r, nu + 1, row, nx);
                }
                if (r < nx) {
                    const auto Am = mt.A + (size_t)cj.x * D.SA;
                    a += dotb<NXc>(Am + r, nx + 1, row, nx);
                }
            }
            h *= qsign;
            a *= qsign;
        }
        s_h[threadIdx.x] = h;
        __syncthreads();
        double dr = 0.0, w = 0.0;
        if (live) {
            const auto u = uin(i);
            if (r < nu) {
                const auto Rm = mt.R + (size_t)cl * D.SR;
                dr = dotb<NUc>(Rm + r, nu + 1, Diff<decltype(u), ldsd*>{u, s_h + base}, nu);
                dout(i)[r] = dr;
            }
            if (r < nx) {
                const auto Km = mt.K + (size_t)cl * D.SK;
                const double s = dotb<NUc>(Km + r, nx + 1, Diff<ldsd*, decltype(u)>{s_h + base, u}, nu);
                w = (-xin(i)[r] + s) + a;
            }
        }
        s_d[threadIdx.x] = dr;
        __syncthreads();
        if (live && r < nx) {
            const auto Mm = mt.M + (size_t)cl * D.SK;
            qout(i)[r] = w + dotb<NUc>(Mm + r, nx + 1, s_d + base, nu);
        }
        __syncthreads();
    }
}

// ---- forward step for nonleaf nodes [b, e): u_i, then x of all their children ------
// xin must cover every parent (node 0 included: callers store x0bar there first);
// uio(i): LDS rows receiving u (read back by the children's lanes after a barrier);
// child rows also go to xout when XOUT.
template <int NXc, int NUc, bool XOUT, class MT, class INF, class XI, class DI>
__device__ __forceinline__ void fwd_step(const Dev& p, const MT& mt, const INF& inf, int b, int e, XI xin, DI din,
                                         LRows uio, glbd* z, LRows xout) {
    const Dims<NXc, NUc> D(p);
    const int nx = D.nx, nu = D.nu;
    {
        const int per = blockDim.x / nu, gl = threadIdx.x / nu, r = threadIdx.x - gl * nu;
        for (int first = b; first < e; first += per) {
            const int i = first + gl;
            if (gl < per && i < e) {
                const int cl = inf.nonleaf(i).z - mt.cls0;
                const auto x = xin(i);
                const auto Km = mt.K + (size_t)cl * D.SK;
                const double u = dotb<NXc>(Km + r * (nx + 1), 1, x, nx) + din(i)[r];
                z[p.U0 + (size_t)i * nu + r] = u;
                uio(i)[r] = u;
            }
        }
    }
    __syncthreads();
    {
        const int cb = inf.nonleaf(b).x;
        const Rec last = inf.nonleaf(e - 1);
        const int ce = last.x + last.y;
        const int per = blockDim.x / nx, gl = threadIdx.x / nx, r = threadIdx.x - gl * nx;
        for (int first = cb; first < ce; first += per) {
            const int j = first + gl;
            if (gl < per && j < ce) {
                const Rec cj = inf.child(j);
                const int i = cj.z;
                const auto x = xin(i);
                const ldsd* u = uio(i);
                const auto Am = mt.A + (size_t)cj.x * D.SA;
                const auto Bm = mt.B + (size_t)cj.y * D.SB;
                const double v = dotb<NXc>(Am + r * (nx + 1), 1, x, nx) + dotb<NUc>(Bm + r * (nu + 1), 1, u, nu);
                z[p.X0 + (size_t)j * nx + r] = v;
                if (XOUT) xout(j)[r] = v;
            }
        }
    }
    __syncthreads();
}

__device__ __forceinline__ glbd* pick3(const Bufs& bf, int k) {
    const int w = k % 3;
    return (glbd*)(w == 0 ? bf.z0 : (w == 1 ? bf.z1 : bf.z2));
}

__device__ __forceinline__ glbd* dyn_z(const Bufs& bf, int zsel, const Ctl* ctl) {
    return pick3(bf, (ctl ? ctl->k : 0) + zsel);
}

typedef MatsT<const glbd*> GMats;
typedef MatsT<const ldsd*> LMats;

__device__ __forceinline__ GMats global_mats(const Dev& p) {
    return GMats{(const glbd*)p.Ap, (const glbd*)p.Bp, (const glbd*)p.Rp, (const glbd*)p.Kp, (const glbd*)p.Mp, 0};
}

// cooperative global -> LDS copy
__device__ __forceinline__ void lds_copy(ldsd* dst, const glbd* src, size_t count) {
    for (size_t t = threadIdx.x; t < count; t += blockDim.x) dst[t] = src[t];
}

// stage the A/B tables of every mode and the class tables [c0, c1) into LDS at `dst`
template <int NXc, int NUc>
__device__ __forceinline__ LMats stage_mats(const Dev& p, ldsd* dst, int c0, int c1, ldsd** end) {
    const Dims<NXc, NUc> D(p);
    const GMats g = global_mats(p);
    ldsd* A = dst;
    ldsd* B = A + (size_t)p.nA * D.SA;
    ldsd* R = B + (size_t)p.nB * D.SB;
    ldsd* K = R + (size_t)(c1 - c0) * D.SR;
    ldsd* M = K + (size_t)(c1 - c0) * D.SK;
    lds_copy(A, g.A, (size_t)p.nA * D.SA);
    lds_copy(B, g.B, (size_t)p.nB * D.SB);
    lds_copy(R, g.R + (size_t)c0 * D.SR, (size_t)(c1 - c0) * D.SR);
    lds_copy(K, g.K + (size_t)c0 * D.SK, (size_t)(c1 - c0) * D.SK);
    lds_copy(M, g.M + (size_t)c0 * D.SK, (size_t)(c1 - c0) * D.SK);
    *end = M + (size_t)(c1 - c0) * D.SK;
    return LMats{A, B, R, K, M, c0};
}

// ---- per-stage fallback (any tree) ------------------------------------------------
template <int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_dyn_back_stage(Dev p, Bufs bf, const Ctl* __restrict__ ctl, int zsel,
                                                            double* qbuf_, double* dbuf_, int b, int e) {
    __shared__ double s_h[kBlock];
    __shared__ double s_d[kBlock];
    if (ctl && ctl->done) return;
    glbd* z = dyn_z(bf, zsel, ctl);
    glbd* qbuf = (glbd*)qbuf_;
    glbd* dbuf = (glbd*)dbuf_;
    const Dims<NXc, NUc> D(p);
    const InfoT<glbrec*> inf{(glbrec*)p.ninfo, 0, (glbrec*)p.cinfo, 0};
    const bool leaves = p.ninfo[b].x >= p.m;
    const GRows qin = leaves ? GRows{z + p.X0, 0, D.nx} : GRows{qbuf, 0, D.nx};
    back_step<NXc, NUc>(p, global_mats(p), inf, b, e, qin, leaves ? -1.0 : 1.0, GRows{z + p.X0, 0, D.nx},
                        GRows{z + p.U0, 0, D.nu}, GRows{qbuf, 0, D.nx}, GRows{dbuf, 0, D.nu}, (ldsd*)s_h,
                        (ldsd*)s_d, blockIdx.x, gridDim.x);
}

// forward, one stage, across workgroups: a child lane recomputes its parent's u = K x + d
// (the same FMA chain as the parent's u lanes, so the values agree bit for bit)
template <int NXc, int NUc>
__global__ void __launch_bounds__(kBlock) k_dyn_fwd_stage(Dev p, Bufs bf, const Ctl* __restrict__ ctl, int zsel,
                                                           const double* dbuf_, const double* x0_, int b, int e) {
    if (ctl && ctl->done) return;
    glbd* z = dyn_z(bf, zsel, ctl);
    const glbd* dbuf = (const glbd*)dbuf_;
    const glbd* x0 = (const glbd*)x0_;
    const GMats g = global_mats(p);
    const Dims<NXc, NUc> D(p);
    const int nx = D.nx, nu = D.nu;
    if (b == 0 && blockIdx.x == 0 && (int)threadIdx.x < nx) z[p.X0 + threadIdx.x] = x0[threadIdx.x];  // x_0 = x0bar
    const int nuB = cdiv_dev(e - b, blockDim.x / nu);
    if ((int)blockIdx.x < nuB) {
        const int per = blockDim.x / nu, gl = threadIdx.x / nu, r = threadIdx.x - gl * nu;
        const int i = b + blockIdx.x * per + gl;
        if (gl < per && i < e) {
            const glbd* x = i == 0 ? x0 : z + p.X0 + (size_t)i * nx;
            const glbd* Km = g.K + (size_t)p.ninfo[i].z * D.SK;
            double s = 0.0;
            _Pragma("unroll") for (int k = 0; k < nx; ++k) s = fma(Km[r * (nx + 1) + k], x[k], s);
            z[p.U0 + (size_t)i * nu + r] = s + dbuf[(size_t)i * nu + r];
        }
        return;
    }
    const int cb = p.ninfo[b].x;
    const int ce = p.ninfo[e - 1].x + p.ninfo[e - 1].y;
    const int per = blockDim.x / nx, gl = threadIdx.x / nx, r = threadIdx.x - gl * nx;
    const int j = cb + (blockIdx.x - nuB) * per + gl;
    if (gl >= per || j >= ce) return;
    const Rec cj = p.cinfo[j];
    const int i = cj.z;
    const glbd* x = i == 0 ? x0 : z + p.X0 + (size_t)i * nx;
    const glbd* Km = g.K + (size_t)p.ninfo[i].z * D.SK;
    const glbd* d = dbuf + (size_t)i * nu;
    const glbd* Am = g.A + (size_t)cj.x * D.SA;
    const glbd* Bm = g.B + (size_t)cj.y * D.SB;
    double s = 0.0, s2 = 0.0;
    _Pragma("unroll") for (int k = 0; k < nx; ++k) s = fma(Am[r * (nx + 1) + k], x[k], s);
    for (int cc = 0; cc < nu; ++cc) {
        double uc = 0.0;
        _Pragma("unroll") for (int k = 0; k < nx; ++k) uc = fma(Km[cc * (nx + 1) + k], x[k], uc);
        s2 = fma(Bm[r * (nu + 1) + cc], uc + d[cc], s2);
    }
    z[p.X0 + (size_t)j * nx + r] = s + s2;
}

// ---- subtree-blocked sweep ------------------------------------------------------------
constexpr int kMaxLevels = 67;  // 3 int arrays of 68: keeps the dynamic-LDS base 16-B aligned

// descendant id ranges of `root` per level (level l <-> stage s + l), levels 0..L; off[l] =
// LDS row offset of level l among the subtree's nonleaf nodes
__device__ __forceinline__ void subtree_levels(const Dev& p, int root, int L, int* lo, int* hi, int* off) {
    if (threadIdx.x == 0) {
        lo[0] = root;
        hi[0] = root + 1;
        int acc = 0;
        for (int l = 0; l < L; ++l) {
            off[l] = acc;
            acc += hi[l] - lo[l];
            const Rec a = p.ninfo[lo[l]], zz = p.ninfo[hi[l] - 1];
            lo[l + 1] = a.x;
            hi[l + 1] = zz.x + zz.y;
        }
        off[L] = acc;
    }
    __syncthreads();
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(512) k_dyn_bottom_back(Dev p, Bufs bf, const Ctl* __restrict__ ctl, int zsel,
                                                          double* qbuf_, double* dbuf_, int s) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ int lo[kMaxLevels + 1], hi[kMaxLevels + 1], off[kMaxLevels + 1];
    if (ctl && ctl->done) return;
    ldsd* smem = (ldsd*)smem_;
    glbd* z = dyn_z(bf, zsel, ctl);
    glbd* qbuf = (glbd*)qbuf_;
    glbd* dbuf = (glbd*)dbuf_;
    const Dims<NXc, NUc> D(p);
    const int nx = D.nx, nu = D.nu;
    const int L = p.N - s;
    const int root = p.stage_ptr[s] + blockIdx.x;
    ldsd* s_h = smem;
    ldsd* s_d = smem + blockDim.x;
    ldsd* qL;
    const LMats mt = stage_mats<NXc, NUc>(p, s_d + blockDim.x, p.cls_ptr[s], p.cls_ptr[p.N], &qL);
    subtree_levels(p, root, L, lo, hi, off);  // ends with a barrier (also covers the staging)
    const InfoT<glbrec*> inf{(glbrec*)p.ninfo, 0, (glbrec*)p.cinfo, 0};
    const GRows xg{z + p.X0, 0, nx}, ug{z + p.U0, 0, nu}, dg{dbuf, 0, nu}, qroot{qbuf, 0, nx};
    for (int l = L - 1; l >= 0; --l) {
        const LRows qmine{qL + (size_t)off[l] * nx, lo[l], nx};
        if (l + 1 == L) {  // children are leaves: q_j = -x_j
            if (l == 0) back_step<NXc, NUc>(p, mt, inf, lo[l], hi[l], xg, -1.0, xg, ug, qroot, dg, s_h, s_d, 0, 1);
            else back_step<NXc, NUc>(p, mt, inf, lo[l], hi[l], xg, -1.0, xg, ug, qmine, dg, s_h, s_d, 0, 1);
        } else {
            const LRows qkids{qL + (size_t)off[l + 1] * nx, lo[l + 1], nx};
            if (l == 0) back_step<NXc, NUc>(p, mt, inf, lo[l], hi[l], qkids, 1.0, xg, ug, qroot, dg, s_h, s_d, 0, 1);
            else back_step<NXc, NUc>(p, mt, inf, lo[l], hi[l], qkids, 1.0, xg, ug, qmine, dg, s_h, s_d, 0, 1);
        }
    }
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(512) k_dyn_bottom_fwd(Dev p, Bufs bf, const Ctl* __restrict__ ctl, int zsel,
                                                         const double* dbuf_, int s) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    __shared__ int lo[kMaxLevels + 1], hi[kMaxLevels + 1], off[kMaxLevels + 1];
    if (ctl && ctl->done) return;
    ldsd* smem = (ldsd*)smem_;
    glbd* z = dyn_z(bf, zsel, ctl);
    const glbd* dbuf = (const glbd*)dbuf_;
    const Dims<NXc, NUc> D(p);
    const int nx = D.nx, nu = D.nu;
    const int L = p.N - s;
    const int root = p.stage_ptr[s] + blockIdx.x;
    ldsd* xL;
    const LMats mt = stage_mats<NXc, NUc>(p, smem, p.cls_ptr[s], p.cls_ptr[p.N], &xL);
    subtree_levels(p, root, L, lo, hi, off);
    ldsd* uL = xL + (size_t)off[L] * nx;
    const InfoT<glbrec*> inf{(glbrec*)p.ninfo, 0, (glbrec*)p.cinfo, 0};
    const RowsT<const glbd*> dg{dbuf, 0, nu};
    const LRows none{nullptr, 0, 0};
    for (int l = 0; l < L; ++l) {
        const LRows uio{uL + (size_t)off[l] * nu, lo[l], nu};
        const bool more = l + 1 < L;
        const LRows xo = more ? LRows{xL + (size_t)off[l + 1] * nx, lo[l + 1], nx} : none;
        if (l == 0) {
            const GRows xin{z + p.X0, 0, nx};
            if (more) fwd_step<NXc, NUc, true>(p, mt, inf, lo[l], hi[l], xin, dg, uio, z, xo);
            else fwd_step<NXc, NUc, false>(p, mt, inf, lo[l], hi[l], xin, dg, uio, z, xo);
        } else {
            const LRows xin{xL + (size_t)off[l] * nx, lo[l], nx};
            if (more) fwd_step<NXc, NUc, true>(p, mt, inf, lo[l], hi[l], xin, dg, uio, z, xo);
            else fwd_step<NXc, NUc, false>(p, mt, inf, lo[l], hi[l], xin, dg, uio, z, xo);
        }
    }
}

// the top of the tree (stages < s, nodes 0..T-1) in one workgroup, everything in LDS
template <int NXc, int NUc>
__global__ void __launch_bounds__(1024) k_dyn_top(Dev p, Bufs bf, const Ctl* __restrict__ ctl, int zsel,
                                                   const double* qbuf_, const double* x0_, int s) {
    extern __shared__ __attribute__((aligned(16))) double smem_[];
    if (ctl && ctl->done) return;
    stamp(p, 0);
    ldsd* smem = (ldsd*)smem_;
    glbd* z = dyn_z(bf, zsel, ctl);
    const glbd* qbuf = (const glbd*)qbuf_;
    const glbd* x0 = (const glbd*)x0_;
    const Dims<NXc, NUc> D(p);
    const int nx = D.nx, nu = D.nu;
    const int T = p.stage_ptr[s];
    const int nb = p.stage_ptr[s + 1] - T;  // boundary nodes (stage s)
    const bool leaves = s == p.N;
    ldsd* s_h = smem;
    ldsd* s_d = smem + blockDim.x;
    ldsd* xS;
    const LMats mt = stage_mats<NXc, NUc>(p, s_d + blockDim.x, 0, p.cls_ptr[s], &xS);  // x rows of the top
    ldsd* uS = xS + (size_t)T * nx;  // u rows (inputs, then outputs)
    ldsd* qT = uS + (size_t)T * nu;
    ldsd* dT = qT + (size_t)T * nx;
    ldsd* qB = dT + (size_t)T * nu;  // boundary rows: q of stage s (or x of the leaves)
    ldsrec* nlS = (ldsrec*)(qB + (((size_t)nb * nx + 1) & ~(size_t)1));  // nonleaf records 0..T-1
    ldsrec* chS = nlS + T;                                              // child records 1..T+nb-1
    lds_copy(xS, z + p.X0, (size_t)T * nx);
    lds_copy(uS, z + p.U0, (size_t)T * nu);
    lds_copy(qB, leaves ? z + p.X0 + (size_t)T * nx : qbuf + (size_t)T * nx, (size_t)nb * nx);
    for (int t = threadIdx.x; t < T; t += blockDim.x) nlS[t] = p.ninfo[t];
    for (int t = threadIdx.x; t < T + nb - 1; t += blockDim.x) chS[t] = p.cinfo[t + 1];
    __syncthreads();
    stamp(p, 1);
    const InfoT<const ldsrec*> inf{nlS, 0, chS, 1};
    const LRows xr{xS, 0, nx}, ur{uS, 0, nu}, qr{qT, 0, nx}, dr{dT, 0, nu}, qbr{qB, T, nx};
    for (int t = s - 1; t >= 0; --t) {
        const int b = p.stage_ptr[t], e = p.stage_ptr[t + 1];
        if (t + 1 < s) back_step<NXc, NUc>(p, mt, inf, b, e, qr, 1.0, xr, ur, qr, dr, s_h, s_d, 0, 1);
        else back_step<NXc, NUc>(p, mt, inf, b, e, qbr, leaves ? -1.0 : 1.0, xr, ur, qr, dr, s_h, s_d, 0, 1);
        stamp(p, 2 + (s - 1 - t));
    }
    if ((int)threadIdx.x < nx) {
        xS[threadIdx.x] = x0[threadIdx.x];
        z[p.X0 + threadIdx.x] = x0[threadIdx.x];  // x_0 = x0bar (cache.py:282)
    }
    __syncthreads();
    for (int t = 0; t < s; ++t) {
        const int b = p.stage_ptr[t], e = p.stage_ptr[t + 1];
        if (t + 1 < s) fwd_step<NXc, NUc, true>(p, mt, inf, b, e, xr, dr, ur, z, xr);
        else fwd_step<NXc, NUc, false>(p, mt, inf, b, e, xr, dr, ur, z, xr);
        stamp(p, 2 + s + t);
    }
}
