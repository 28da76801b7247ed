// L and L^T (operators.py:19-53, 55-94) as node-range block kernels.
//
// Block b owns a range of nonleaf nodes [i0, i1) together with their children [c0, c1)
// (contiguous in the BFS numbering) and a range of leaves [l0, l1) (host table
// Dev::ell_tab). One LDS-DMA gather stages every input range the block reads (iterate
// slices and index records, packed back to back: one 64-lane instruction may span
// several ranges, since the source address is per lane) while the lanes load their
// weight row into registers; a block costs two memory round trips (its table, then the
// gather) and then computes from LDS. The matrix-vector products of 16 nodes that share
// a weight table are one MFMA tile (v_mfma_f64_16x16x4f64: nodes x weight rows, k in
// steps of 4), so each lane loads one input and one weight value per 64 FMAs instead
// of one per FMA; a tile whose nodes use different tables takes a per-lane path with
// the same result slots (the packer merges equal per-mode weights, so the benchmark
// trees are all-MFMA).
//
// Measured on MI355X (tools/ubench5.hip): an LDS-DMA instruction costs its CU ~45 ns of
// issue/landing slot whether it moves 1 KiB or 128 B, so the gather packs small ranges
// into full instructions; loads issued next to it would wait behind it (vmcnt is in
// order), which is why even the plain copies go through LDS.
//
// Weights are column-major M[k*rows + r] = M_rk; both L and L^T apply M itself (the
// reference applies sqrt_Q, not its transpose, in ell_transpose: sqrt-weights are symmetric).
//
// Algorithmic bytes per launch: 8 (|P| + |D|) over active entries.

// LDS-DMA gather: ranges added one after the other get consecutive 16-B chunk slots in
// LDS (a range may start 8 B into its first chunk: the returned pointer is shifted);
// issue() sends all chunks, 64 per wave instruction, groups spread over the waves.
template <int MAXR>
struct Gather {
    ldsd* base;
    int nr = 0, total = 0;
    const char* src[MAXR];
    int cum[MAXR];
    __device__ __forceinline__ explicit Gather(ldsd* b) : base(b) {}
    __device__ __forceinline__ const ldsd* add(const void* p, int nbytes) {
        const uintptr_t a = (uintptr_t)p;
        const int sh = (int)(a & 15);
        src[nr] = (const char*)(a - sh);
        cum[nr] = total;
        ldsd* dst = base + 2 * total;
        total += nbytes > 0 ? (sh + nbytes + 15) >> 4 : 0;
        ++nr;
        return dst + (sh >> 3);
    }
    template <class PT>
    __device__ __forceinline__ const ldsd* dbl(PT p, int count) { return add((const void*)p, count * 8); }
    __device__ __forceinline__ const ldsrec* rec(const Rec* p, int count) { return (const ldsrec*)add(p, count * 16); }
    __device__ __forceinline__ void issue() const {
        const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, nw = blockDim.x >> 6;
        for (int c0 = wave * 64; c0 < total; c0 += nw * 64) {
            const int ch = c0 + lane;
            if (ch < total) {
                const char* s = src[0];
                int c = cum[0];
                _Pragma("unroll") for (int r = 1; r < MAXR; ++r)
                    if (r < nr && ch >= cum[r]) { s = src[r]; c = cum[r]; }
                __builtin_amdgcn_global_load_lds((const glbd*)(s + 16 * (ch - c)), base + 2 * c0, 16, 0, 0);
            }
        }
    }
};

// sequential LDS regions filled by LDS-DMA (CP kernels). Region r occupies F_r 16-B chunk
// slots from chunk offset o / 2 (F_r = its bytes rounded up plus one pad chunk, the
// footprint the host's LDS plan counts). The regions are only recorded (source, first
// slot, slots: a table in LDS, a few instructions per region); issue() then sends them, one
// DMA pass per region (packing short regions into shared instructions through a slot ->
// region map measured neutral to 6 % slower: two more barriers per block).
// Only a region's data chunks are loaded (its first chunk may start up to 8 B before the
// range, its last end up to 15 B after it: inside the allocation or its 64-B slack).
// (Recording instead of issuing per call keeps the kernels small: the inlined per-region
// DMA loops made k_cpp 89 KB of code, more than the instruction cache.)
constexpr int kStgMaxR = 64;
// the recorded regions of one block (LDS tables: each kernel declares them, StgLds)
struct StgTable {
    __attribute__((address_space(3))) unsigned long long* tsrc = nullptr;  // per region: 16-B aligned source
    __attribute__((address_space(3))) int* tc0 = nullptr;                 // per region: first slot
    __attribute__((address_space(3))) int* tF = nullptr;                  // per region: chunks to load
    int nr = 0;
    __device__ __forceinline__ void record(const char* s16, int bytes, int c0) {
        if (threadIdx.x == 0 && nr < kStgMaxR) {
            tsrc[nr] = (unsigned long long)(uintptr_t)s16;
            tc0[nr] = c0;
            tF[nr] = bytes > 0 ? (bytes + 15) >> 4 : 0;
        }
        ++nr;
    }
    // send every recorded region into slots from `base` (call once, after the last region,
    // by the whole block); total = slots of the footprint
    __device__ __forceinline__ void issue(ldsd* base, int total) const {
        __syncthreads();  // the region table is written
        const int R = min(nr, kStgMaxR);
        (void)total;
        int rot = 0;
        _Pragma("unroll 1") for (int r = 0; r < R; ++r) {
            const char* src = (const char*)(uintptr_t)tsrc[r];
            rot += dma_gen(base + 2 * tc0[r], tF[r], [=](int ch) { return (const double*)(src + 16 * ch); }, rot);
        }
    }
};
// the LDS tables of a StgTable, declared once per kernel (a __shared__ array in an inlined
// device function is one allocation per kernel that uses it)
__device__ __forceinline__ StgTable stg_table() {
    __shared__ unsigned long long s_tsrc[kStgMaxR];
    __shared__ int s_tc0[kStgMaxR], s_tF[kStgMaxR];
    StgTable t;
    t.tsrc = (__attribute__((address_space(3))) unsigned long long*)s_tsrc;
    t.tc0 = (__attribute__((address_space(3))) int*)s_tc0;
    t.tF = (__attribute__((address_space(3))) int*)s_tF;
    return t;
}
struct Stg {
    ldsd* base;
    int o;  // next free offset (doubles), kept even
    StgTable tab;
    // a region of F slots whose first `bytes` from s16 (16-B aligned) are data
    __device__ __forceinline__ ldsd* region(const char* s16, int bytes, int F) {
        ldsd* dst = base + o;
        tab.record(s16, bytes, o >> 1);
        o += 2 * F;
        return dst;
    }
    template <class PT>
    __device__ __forceinline__ const ldsd* dbl(PT src, int count) {  // count doubles
        const uintptr_t a = (uintptr_t)src;
        const int sh = (int)(a & 15);
        return region((const char*)(a - sh), count > 0 ? sh + 8 * count : 0, (rup(count, 2) + 2) >> 1) + (sh >> 3);
    }
    __device__ __forceinline__ const ldsrec* rec(const Rec* src, int count) {  // 16-B records
        return (const ldsrec*)region((const char*)src, 16 * count, count + 1);
    }
    __device__ __forceinline__ const __attribute__((address_space(3))) int* ints(const int* src, int count) {
        const uintptr_t a = (uintptr_t)src;
        const int shb = (int)(a & 15);
        ldsd* dst = region((const char*)(a - shb), count > 0 ? count * 4 + shb : 0,
                           (rup((count * 4 + shb + 7) / 8, 2) + 2) >> 1);
        return (const __attribute__((address_space(3))) int*)((__attribute__((address_space(3))) char*)dst + shb);
    }
    __device__ __forceinline__ void issue() const { tab.issue(base, o >> 1); }
};

typedef __attribute__((address_space(4))) const Rec crec4;  // scalar (constant) loads

// block table: 4 records per block
//   {i0, i1, c0, c1}, {l0, l1, y0, y1}, {e7a, e7b, e14a, e14b}, {iSQ[c0], iSR[c0], iSP[l0], 0}
// (e7a/e7b, e14a/e14b: the eta7 / eta14 ranges of the block's nodes, placeholders included)
constexpr int kEllRecs = 4;




typedef double d4 __attribute__((ext_vector_type(4)));

// out[node][r0 + r] = sum_k M_t(node)[r0 + r][k] v_node[k] for the 16 nodes [first, first +
// min(cnt, 16)) and 16 weight rows from r0; column-major table M[k n + r]. MFMA operands:
// lane l: A = v_{node l%16}[k0 + l/16], B = M[r0 + l%16][k0 + l/16]; result lane l, element
// e -> node l/16 + 4e, row r0 + l%16 (tools/ubench6.hip). Called by a whole wave.
template <int NC, class SlotF, class TabF>
__device__ __forceinline__ d4 mrows16(const double* T, int nr, const ldsd* src, int first, int cnt, int r0,
                                      SlotF slot, TabF tab) {
    const int n = NC ? NC : nr;
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
    const int na = lo < cnt ? lo : 0;
    const int ta = tab(first + na);
    const int t0 = __builtin_amdgcn_readfirstlane(ta);
    d4 acc = {0.0, 0.0, 0.0, 0.0};
    const int r = r0 + lo;
    if (__all(ta == t0)) {
        const glbd* M = (const glbd*)(T + (size_t)t0 * n * n);
        const ldsd* va = src + slot(first + na) * n;
        const bool live_a = lo < cnt, live_b = r < n;
        _Pragma("unroll") for (int k0 = 0; k0 < (NC ? NC : 1 << 20); k0 += 4) {
            if (!NC && k0 >= n) break;
            const int k = k0 + hi;
            const double a = (live_a && k < n) ? va[k] : 0.0;
            const double b = (live_b && k < n) ? M[k * n + r] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc, 0, 0, 0);
        }
    } else {
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e;
            double s0 = 0.0, s1 = 0.0;
            if (nd < cnt && r < n) {
                const glbd* M = (const glbd*)(T + (size_t)tab(first + nd) * n * n) + r;
                const ldsd* x = src + slot(first + nd) * n;
                int k = 0;
                for (; k + 1 < n; k += 2) {
                    s0 = fma(M[k * n], x[k], s0);
                    s1 = fma(M[(k + 1) * n], x[k + 1], s1);
                }
                if (k < n) s0 = fma(M[k * n], x[k], s0);
            }
            acc[e] = s0 + s1;
        }
    }
    return acc;
}

// the tiles of one product family: nodes [first, first + cnt) x rows [0, n), tiles
// numbered (node tile) * rt + (row tile); put(node, r, value) for every live result
template <int NC, class SlotF, class TabF, class PutF>
__device__ __forceinline__ void mrows_tile(int tile, const double* T, int nr, const ldsd* src, int first, int cnt,
                                           SlotF slot, TabF tab, PutF put) {
    const int n = NC ? NC : nr, rt = (n + 15) >> 4;
    const int nt = tile / rt, r0 = (tile - nt * rt) * 16;
    const int f = first + nt * 16, c = cnt - nt * 16;
    const d4 d = mrows16<NC>(T, n, src, f, c, r0, slot, tab);
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
    _Pragma("unroll") for (int e = 0; e < 4; ++e) {
        const int nd = hi + 4 * e, r = r0 + lo;
        if (nd < c && r < n) put(f + nd, r, d[e]);
    }
}
__device__ __forceinline__ int ntiles(int cnt, int n) { return ((cnt + 15) >> 4) * ((n + 15) >> 4); }

// Weight-stationary MFMA streams. A product family (nodes [first, first + cnt), n weight
// rows) whose nodes all use table t (block table, -1 when mixed) is cut into "streams"
// (one per 16-row tile); a wave owns one stream, loads its weight fragments once (before
// the block's gather has landed: they depend only on t) and runs the stream's node
// tiles w0, w0 + ws, ... A mixed family falls back to mrows_tile per tile.
template <int NC>
struct WFrag {
    static constexpr int KS = NC > 0 ? (NC + 3) / 4 : 16;
    static constexpr int KV = KS <= 2 ? KS : KS <= 4 ? 4 : KS <= 8 ? 8 : 16;  // vector width
    typedef double bvec __attribute__((ext_vector_type(KV)));
    bvec b;  // a vector type stays in registers (a plain array member went to scratch)
    __device__ __forceinline__ void load(const double* T, int t, int n, int r0) {
        const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4, r = r0 + lo;
        const glbd* M = (const glbd*)(T + (size_t)t * n * n);
        _Pragma("unroll") for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + hi;
            b[s] = (r < n && k < n) ? M[k * n + r] : 0.0;
        }
    }
    // one tile whose A-row of this lane is va (live) or zero
    __device__ __forceinline__ d4 tile_at(const ldsd* va, int n, bool live) const {
        const int hi = (threadIdx.x & 63) >> 4;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        _Pragma("unroll") for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + hi;
            const double a = (live && k < n) ? va[k] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[s], acc, 0, 0, 0);
        }
        return acc;
    }
    // one 16-node tile: A from LDS rows src + slot(node) n
    template <class SlotF>
    __device__ __forceinline__ d4 tile(const ldsd* src, int n, int first, int cnt, SlotF slot) const {
        const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
        const bool live = lo < cnt;
        const ldsd* va = src + slot(first + (live ? lo : 0)) * n;
        d4 acc = {0.0, 0.0, 0.0, 0.0};
        _Pragma("unroll") for (int s = 0; s < KS; ++s) {
            const int k = 4 * s + hi;
            const double a = (live && k < n) ? va[k] : 0.0;
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b[s], acc, 0, 0, 0);
        }
        return acc;
    }
};

// families: up to 3 (role f: table T[f], uniform index tu[f], rows n[f], nodes [first,
// first + cnt), LDS input src[f]); streams are (family, row tile); waves are spread over
// the streams, several waves per stream splitting its node tiles.
struct Fam {
    const double* T;
    int tu, n, first, cnt;
    const ldsd* src;
};
__device__ __forceinline__ int fam_rt(const Fam& f) { return f.cnt > 0 ? (f.n + 15) >> 4 : 0; }

template <int NC, class SlotF, class TabF, class PutF>
__device__ __forceinline__ void fam_tiles(const Fam& F, const WFrag<NC>& wf, int r0, int part, int P, SlotF slot,
                                          TabF tab, PutF put) {
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4;
    for (int ti = part; ti * 16 < F.cnt; ti += P) {
        const int first = F.first + ti * 16, cnt = F.cnt - ti * 16;
        const d4 d = F.tu >= 0 ? wf.tile(F.src, F.n, first, cnt, slot)
                               : mrows16<NC>(F.T, F.n, F.src, first, cnt, r0, slot, tab);
        _Pragma("unroll") for (int e = 0; e < 4; ++e) {
            const int nd = hi + 4 * e, r = r0 + lo;
            if (nd < cnt && r < F.n) put(first + nd, r, d[e]);
        }
    }
}

// Per-parent tiles (k_ell_t on a regular block: C children per parent, children of block
// parent p at rows p C + [0, C) of F.src). MFMA result element e of lane group h is A-row
// h + 4e, so A-row h + 4e is given child e % C of parent h + 4 (e / C): the C products of
// one parent land in one lane, which sums them in child order after base(p, r) and stores
// the parent row with put(p, r, sum). A tile covers 4 (4 / C) parents.
template <int C, int NC, class BaseF, class PutF>
__device__ __forceinline__ void par_tiles_c(const Fam& F, const WFrag<NC>& wf, int r0, int part, int P, int np,
                                            BaseF base, PutF put) {
    constexpr int Q = 4 / C, PT = 4 * Q;
    const int l = threadIdx.x & 63, lo = l & 15, hi = l >> 4, r = r0 + lo;
    const int hA = lo & 3, eA = lo >> 2, pA = hA + 4 * (eA / C), kA = eA % C;
    for (int ti = part; ti * PT < np; ti += P) {
        const int pb = ti * PT;
        const bool live = eA < Q * C && pb + pA < np;
        const d4 d = wf.tile_at(F.src + (live ? (pb + pA) * C + kA : 0) * F.n, F.n, live);
        _Pragma("unroll") for (int s = 0; s < Q; ++s) {
            const int pp = pb + hi + 4 * s;
            if (pp < np && r < F.n) {
                double acc = base(pp, r);
                _Pragma("unroll") for (int k = 0; k < C; ++k) acc += d[s * C + k];
                put(pp, r, acc);
            }
        }
    }
}
template <int NC, class BaseF, class PutF>
__device__ __forceinline__ void par_tiles(int c, const Fam& F, const WFrag<NC>& wf, int r0, int part, int P, int np,
                                          BaseF base, PutF put) {
    switch (c) {
        case 1: par_tiles_c<1, NC>(F, wf, r0, part, P, np, base, put); break;
        case 2: par_tiles_c<2, NC>(F, wf, r0, part, P, np, base, put); break;
        case 3: par_tiles_c<3, NC>(F, wf, r0, part, P, np, base, put); break;
        default: par_tiles_c<4, NC>(F, wf, r0, part, P, np, base, put); break;
    }
}

// the three product families of L / L^T: 0 = Q rows over the children, 1 = R rows over
// the children, 2 = Pf rows over the leaves. Waves split the (family, row tile) streams;
// prefetch() loads the first stream's weight fragments (call before the gather wait),
// run() computes every stream of the wave.
template <int NXc, int NUc>
struct FamRun {
    Fam F0, F1, F2;  // separate members (a runtime-indexed array would live in scratch)
    int S0, S1, S, W, w, P;
    WFrag<NXc> f0, f2;  // one fragment set per family, each used only under its own branch
    WFrag<NUc> f1;
    __device__ __forceinline__ FamRun(const Fam& a, const Fam& b, const Fam& c) : F0(a), F1(b), F2(c) {
        S0 = fam_rt(F0);
        S1 = S0 + fam_rt(F1);
        S = S1 + fam_rt(F2);
        W = blockDim.x >> 6;
        w = threadIdx.x >> 6;
        P = S > 0 ? (W / S > 1 ? W / S : 1) : 1;
    }
    __device__ __forceinline__ void frag(int st) {
        if (st < S0) {
            if (F0.tu >= 0) f0.load(F0.T, F0.tu, F0.n, 16 * st);
        } else if (st < S1) {
            if (F1.tu >= 0) f1.load(F1.T, F1.tu, F1.n, 16 * (st - S0));
        } else {
            if (F2.tu >= 0) f2.load(F2.T, F2.tu, F2.n, 16 * (st - S1));
        }
    }
    __device__ __forceinline__ void prefetch() {
        if (w < S * P) frag(w % S);
    }
    // k_ell_t on a regular block: families 0 / 1 as per-parent tiles (par_tiles), family 2
    // as node tiles
    template <class Base0, class PPut0, class Base1, class PPut1, class Slot2, class Tab2, class Put2>
    __device__ __forceinline__ void run_par(int c, int np, Base0 b0, PPut0 q0, Base1 b1, PPut1 q1, Slot2 s2, Tab2 t2,
                                            Put2 p2) {
        for (int item = w; item < S * P; item += W) {
            const int st = item % S, part = item / S;
            if (item != w) frag(st);
            if (st < S0) par_tiles<NXc>(c, F0, f0, 16 * st, part, P, np, b0, q0);
            else if (st < S1) par_tiles<NUc>(c, F1, f1, 16 * (st - S0), part, P, np, b1, q1);
            else fam_tiles<NXc>(F2, f2, 16 * (st - S1), part, P, s2, t2, p2);
        }
    }
    template <class Slot0, class Tab0, class Put0, class Tab1, class Put1, class Slot2, class Tab2, class Put2>
    __device__ __forceinline__ void run(Slot0 s0, Tab0 t0, Put0 p0, Tab1 t1, Put1 p1, Slot2 s2, Tab2 t2, Put2 p2) {
        for (int item = w; item < S * P; item += W) {
            const int st = item % S, part = item / S;
            if (item != w) frag(st);
            if (st < S0) fam_tiles<NXc>(F0, f0, 16 * st, part, P, s0, t0, p0);
            else if (st < S1) fam_tiles<NUc>(F1, f1, 16 * (st - S0), part, P, s0, t1, p1);
            else fam_tiles<NXc>(F2, f2, 16 * (st - S1), part, P, s2, t2, p2);
        }
    }
};

template <int NXc, int NUc>
__global__ void __launch_bounds__(512) k_ell(Dev p, const double* __restrict__ z, double* __restrict__ eta) {
    extern __shared__ __attribute__((aligned(16))) double ell_smem[];
    stamp(p, 0);
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    const crec4* tb = (const crec4*)p.ell_tab + (size_t)blockIdx.x * kEllRecs;
    const Rec t0 = tb[0], t1 = tb[1];
    const int i0 = t0.x, i1 = t0.y, c0 = t0.z, c1 = t0.w, l0 = t1.x, l1 = t1.y, y0 = t1.z, y1 = t1.w;
    const int np = i1 - i0, nc = c1 - c0, nl = l1 - l0, ny = y1 - y0, tid = threadIdx.x, nt = blockDim.x;
    const glbd* zg = (const glbd*)z;
    glbd* eg = (glbd*)eta;
    Gather<12> g((ldsd*)ell_smem);
    const ldsd* X = g.dbl(zg + p.X0 + (size_t)i0 * nx, np * nx);  // parents' x, u, y, s
    const ldsd* U = g.dbl(zg + p.U0 + (size_t)i0 * nu, np * nu);
    const ldsd* Y = g.dbl(zg + p.Y0 + y0, ny);
    const ldsd* S = g.dbl(zg + p.S0 + i0, np);
    const ldsd* T = g.dbl(zg + p.T0 + c0, nc);                     // children's tau
    const ldsd* CD = g.dbl(p.cond + c0, nc);
    const ldsrec* FR = g.rec(p.frec + i0, np);   // {yrel, nch, ch_start, e7off}
    const ldsrec* CR = g.rec(p.crec + c0, nc);   // {anc, iSQ, iSR, 0}
    const ldsd* XL = g.dbl(zg + p.X0 + (size_t)l0 * nx, nl * nx);  // leaves' x, s
    const ldsd* SL = g.dbl(zg + p.S0 + l0, nl);
    const ldsrec* LR = g.rec(p.lrec + (l0 - p.m), nl);  // {iSP, iBl, e14off, 0}
    g.issue();
    const Rec t3 = tb[3];
    FamRun<NXc, NUc> fr(Fam{p.SQ, t3.x, nx, c0, nc, X}, Fam{p.SR, t3.y, nu, c0, nc, U}, Fam{p.SP, t3.z, nx, l0, nl, XL});
    fr.prefetch();
    stamp(p, 1);
    dma_wait();
    lds_sync();
    stamp(p, 2);
    // eta3_j = sqrtQ_j x_anc(j) | eta4_j = sqrtR_j u_anc(j) | eta11_l = sqrtPf_l x_l
    fr.run([&](int j) { return CR[j - c0].x - i0; }, [&](int j) { return CR[j - c0].y; },
           [&](int j, int r, double v) { eg[e3(p, j) + r] = v; }, [&](int j) { return CR[j - c0].z; },
           [&](int j, int r, double v) { eg[e4(p, j) + r] = v; }, [&](int l) { return l - l0; },
           [&](int l) { return LR[l - l0].x; }, [&](int l, int r, double v) { eg[e11(p, l) + r] = v; });
    stamp(p, 3);
    // copies: eta7 | eta14 | eta1 | eta2 | eta5,6 | eta12,13 as one flat task list
    const int nD = np * (nx + nu), nE = nD + nl * nx, nF = nE + ny, nG = nF + np, nH = nG + nc, nI = nH + nl;
    for (int t = tid; t < nI; t += nt) {
        if (t < nD) {  // eta7 = [x; u] on boxed nonleaf nodes
            const int q = t / (nx + nu), rr = t - q * (nx + nu);
            const int o7 = FR[q].w;
            if (o7 >= 0) eg[o7 + rr] = rr < nx ? X[q * nx + rr] : U[q * nu + rr - nx];
        } else if (t < nE) {  // eta14_l = x_l on boxed leaves
            const int e = t - nD, q = e / nx, r = e - q * nx;
            const int o14 = LR[q].z;
            if (o14 >= 0) eg[o14 + r] = XL[e];
        } else if (t < nF) {  // eta1 = y
            const int e = t - nE;
            eg[p.E1 + y0 + e] = Y[e];
        } else if (t < nG) {  // eta2 = s - b'y, b = [p; 0; 1]
            const int q = t - nF;
            const Rec fr = FR[q];
            const int c = fr.y, yo = fr.x - y0, cl = fr.z - c0;
            double by = 0.0;
            for (int k = 0; k < c; ++k) by = fma(CD[cl + k], Y[yo + k], by);
            for (int k = c; k < 2 * c; ++k) by += 0.0 * Y[yo + k];
            by += Y[yo + 2 * c];
            eg[p.E2 + i0 + q] = S[q] - by;
        } else if (t < nH) {  // eta5 = eta6 = tau_j / 2
            const int jj = t - nG;
            const double h = 0.5 * T[jj];
            eg[p.E5 + c0 + jj] = h;
            eg[p.E6 + c0 + jj] = h;
        } else {  // eta12 = eta13 = s_l / 2
            const int ll = t - nH;
            const double h = 0.5 * SL[ll];
            eg[p.E12 + l0 + ll] = h;
            eg[p.E13 + l0 + ll] = h;
        }
    }
    stamp(p, 4);
}

template <int NXc, int NUc>
__global__ void __launch_bounds__(512) k_ell_t(Dev p, const double* __restrict__ eta, double* __restrict__ z) {
    extern __shared__ __attribute__((aligned(16))) double ell_smem[];
    const int nx = NXc ? NXc : p.nx, nu = NUc ? NUc : p.nu;
    const crec4* tb = (const crec4*)p.ell_tab + (size_t)blockIdx.x * kEllRecs;
    const Rec t0 = tb[0], t1 = tb[1], t2 = tb[2];
    const int i0 = t0.x, i1 = t0.y, c0 = t0.z, c1 = t0.w, l0 = t1.x, l1 = t1.y, y0 = t1.z, y1 = t1.w;
    const int e7a = t2.x, e14a = t2.z;
    const int np = i1 - i0, nc = c1 - c0, nl = l1 - l0, tid = threadIdx.x, nt = blockDim.x;
    const glbd* eg = (const glbd*)eta;
    glbd* zg = (glbd*)z;
    Gather<16> g((ldsd*)ell_smem);
    const ldsd* D3 = g.dbl(eg + e3(p, c0), nc * nx);
    const ldsd* D4 = g.dbl(eg + e4(p, c0), nc * nu);
    const ldsd* D7 = g.dbl(eg + e7a, t2.y - e7a);
    const ldsd* D1 = g.dbl(eg + p.E1 + y0, y1 - y0);
    const ldsd* D2 = g.dbl(eg + p.E2 + i0, np);
    const ldsd* D5 = g.dbl(eg + p.E5 + c0, nc);
    const ldsd* D6 = g.dbl(eg + p.E6 + c0, nc);
    const ldsd* CD = g.dbl(p.cond + c0, nc);
    const ldsrec* FR = g.rec(p.frec + i0, np);   // {yrel, nch, ch_start, e7off}
    const ldsrec* CR = g.rec(p.crec + c0, nc);   // {anc, iSQ, iSR, 0}
    const ldsd* D11 = g.dbl(eg + e11(p, l0), nl * nx);
    const ldsd* D14 = g.dbl(eg + e14a, t2.w - e14a);
    const ldsd* D12 = g.dbl(eg + p.E12 + l0, nl);
    const ldsd* D13 = g.dbl(eg + p.E13 + l0, nl);
    const ldsrec* LR = g.rec(p.lrec + (l0 - p.m), nl);  // {iSP, iBl, e14off, 0}
    g.issue();
    // products sqrtQ_j eta3_j, sqrtR_j eta4_j (children) in LDS, summed per parent below; the
    // leaves' sqrtPf_l eta11_l (+ eta14_l) go straight from the MFMA tile to x_l
    ldsd* PX = (ldsd*)ell_smem + 2 * g.total;
    ldsd* PU = PX + nc * nx;
    const Rec t3 = tb[3];
    FamRun<NXc, NUc> fr(Fam{p.SQ, t3.x, nx, c0, nc, D3}, Fam{p.SR, t3.y, nu, c0, nc, D4},
                        Fam{p.SP, t3.z, nx, l0, nl, D11});
    fr.prefetch();
    dma_wait();
    lds_sync();
    auto leaf_put = [&](int l, int r, double v) {
        const int o14 = LR[l - l0].z;
        zg[p.X0 + (size_t)l * nx + r] = o14 >= 0 ? v + D14[o14 - e14a + r] : v;
    };
    // regular block with uniform Q / R tables: the parents' x, u rows come straight out of
    // the per-parent MFMA tiles (no product staging, no second barrier)
    const bool par = t3.w > 0 && t3.x >= 0 && t3.y >= 0;
    if (par) {
        fr.run_par(
            t3.w, np,
            [&](int q, int r) {
                const int o7 = FR[q].w;
                return o7 >= 0 ? D7[o7 - e7a + r] : 0.0;
            },
            [&](int q, int r, double v) { zg[p.X0 + (size_t)(i0 + q) * nx + r] = v; },
            [&](int q, int r) {
                const int o7 = FR[q].w;
                return o7 >= 0 ? D7[o7 - e7a + nx + r] : 0.0;
            },
            [&](int q, int r, double v) { zg[p.U0 + (size_t)(i0 + q) * nu + r] = v; }, [&](int l) { return l - l0; },
            [&](int l) { return LR[l - l0].x; }, leaf_put);
    } else {
        fr.run([&](int j) { return j - c0; }, [&](int j) { return CR[j - c0].y; },
               [&](int j, int r, double v) { PX[(j - c0) * nx + r] = v; }, [&](int j) { return CR[j - c0].z; },
               [&](int j, int r, double v) { PU[(j - c0) * nu + r] = v; }, [&](int l) { return l - l0; },
               [&](int l) { return LR[l - l0].x; }, leaf_put);
        lds_sync();
    }
    // x_i = [eta7_i]_x + sum_children (sqrtQ_j eta3_j) | u_i likewise (unless done above) |
    // y = eta1 - b eta2 | s = eta2 | tau | leaf s, as one flat task list
    const int G = 2 * p.cmax + 1;
    const int nA = par ? 0 : np * nx, nB = par ? 0 : nA + np * nu, nC = nB, nD = nC + np * G, nE = nD + np,
              nF = nE + nc;
    const int nH = nF + nl;
    for (int t = tid; t < nH; t += nt) {
        if (t < nB) {
            const bool isx = t < nA;
            const int e = isx ? t : t - nA, n = isx ? nx : nu, q = e / n, r = e - q * n;
            const Rec fr = FR[q];
            double acc = fr.w >= 0 ? D7[fr.w - e7a + (isx ? 0 : nx) + r] : 0.0;
            const ldsd* P = isx ? PX : PU;
            for (int j = fr.z; j < fr.z + fr.y; ++j) acc += P[(j - c0) * n + r];
            if (isx) zg[p.X0 + (size_t)(i0 + q) * nx + r] = acc;
            else zg[p.U0 + (size_t)(i0 + q) * nu + r] = acc;
        } else if (t < nD) {  // y = eta1 - b eta2
            const int e = t - nC, q = e / G, k = e - q * G;
            const Rec fr = FR[q];
            const int c = fr.y;
            if (k < 2 * c + 1) {
                const double b = k < c ? CD[fr.z - c0 + k] : (k < 2 * c ? 0.0 : 1.0);
                zg[p.Y0 + fr.x + k] = D1[fr.x - y0 + k] - b * D2[q];
            }
        } else if (t < nE) {  // s = eta2
            const int q = t - nD;
            zg[p.S0 + i0 + q] = D2[q];
        } else if (t < nF) {  // tau_j = (eta5 + eta6) / 2
            const int jj = t - nE;
            zg[p.T0 + c0 + jj] = 0.5 * (D5[jj] + D6[jj]);
        } else {  // s_l = (eta12 + eta13) / 2
            const int ll = t - nF;
            zg[p.S0 + l0 + ll] = 0.5 * (D12[ll] + D13[ll]);
        }
    }
}
