// raocp_capi.hip — host side of libraocp_hip.so: the C-ABI declared in
// include/raocp_hip.h. Owns one HIP device context per raocp_ctx: uploads the
// packed problem, keeps the CP iterate resident in HBM, launches the kernels of
// raocp_kernels.hip and replays the CP iteration as a captured hipGraph.

#include "raocp_kernels.hip"
#include "raocp_dynr.h"
#include "raocp_cp4.h"
#include "raocp_cp5.h"
#include "../../include/raocp_hip.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <string>
#include <vector>

using raocp::Ctl;
using raocp::Dev;
using raocp::kBlock;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define HIPCHK(expr)                                                                             \
    do {                                                                                         \
        hipError_t _e = (expr);                                                                  \
        if (_e != hipSuccess)                                                                    \
            return fail(RAOCP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));       \
    } while (0)

int cdiv(int a, int b) { return b <= 0 ? 0 : (a + b - 1) / b; }

// CP iterations per captured graph: a multiple of 6 (buffer rotation period, see rotated())
constexpr int kGraphBatch = 24;

}  // namespace

struct raocp_ctx {
    int device = 0;
    bool f32 = false;            // RAOCP_F32: iterate, tables and products in fp32
    bool dyn32 = false;          // the per-stage T-templated dynamics (raocp_dyn2.hip) is planned
    bool ell3 = false;           // L by streaming wave tasks (raocp_ell3.hip)
    int ell3_grid = 0;
    int box_mode = 0;            // k_ell3 / k_ellt3: bits 0-1 nonleaf, 2-3 leaf boxes (1 all, 2 none, 0 mixed)
    int unif_C = 0;              // uniform branching factor <= 4 with uniform tables (0 = not)
    int unif_branch = 0;         // uniform branching factor <= 4 (children 1 + C i ..), any tables (dyn3)
    int ellt3_C = 0;             // L^T by streaming wave tasks: uniform branching factor (0 = off)
    int ellt3_grid = 0;
    bool cp3 = false;            // the CP iteration after the dynamics as one streaming kernel (raocp_cp3.hip)
    bool cp4 = false;            // ... with every operand of a tile loaded at its start (raocp_cp4.hip; RAOCP_CP4=0: off)
    int cp4_wpb = 2;             // k_cp4's waves per workgroup, one task per workgroup: 2 = helper mode (wave 1
                                 // takes a leaf-parent tile's leaf children), 1 = one wave (RAOCP_CP4_HELPER=0);
                                 // one task per workgroup spreads the load bursts over all CUs (round 4: one
                                 // task per wave at four waves per workgroup 18.5 vs 16.7 us at one)
    bool cp5 = false;            // ... as a leaf launch and a family launch (raocp_cp5.hip: configs 3, 4, 5;
                                 // RAOCP_CP5=0: off)
    bool cp6 = false;            // ... as one family tile per workgroup of 2 C waves (raocp_cp5.hip k_cp6: config
                                 // 2; RAOCP_CP6=0: k_cp4)
    int cp6_grid = 0;
    raocp::Cp3Tasks cp5_tk{};    // k_cp5_fam's / k_cp6's task list (every parent, leaf parents first)
    int cp5_gl = 0, cp5_gf = 0;  // grids of the two launches
    raocp::Cp3Tasks cp5_et{};    // k_cp5_leaf's eta2 tasks (nonleaf ranges, 64 nodes per task)
    raocp::Cp3Tasks cp5_tkb{};   // a shard's second k_cp5 launch: the cut's parents, after X1
    int cp5_gfb = 0;             // ... its grid
    bool cp5_lpf = false;        // k_cp5_leaf's form (RAOCP_CP5_LPF, raocp_cp5.h)
    int cp3_grid = 0;            // workgroups of the (first) k_cp3 launch
    int cp3_mL = 0;              // first parent whose children are leaves (stage N - 1)
    int cp3_split = 0;           // leaves as tasks of their own (small trees: more waves, shorter chains)
    raocp::Cp3Tasks cp3_ta{};    // the launch's task list (a shard: its own families + the top)
    raocp::Cp3Tasks cp3_tb{};    // a shard's second launch: the cut's parents, after X1
    int cp3_gridb = 0;
    double* cp3img = nullptr;    // k_cp3's weight fragments in LDS order (k_cp3_image)
    // per-stage MFMA dynamics (raocp_dyn2.hip): tables, node lists, tile lists per stage
    bool dyn2 = false;           // fp32 contexts always; fp64 opt-in RAOCP_DYN2=1
    const double *W2 = nullptr, *RG2 = nullptr, *KM2 = nullptr, *F2 = nullptr;
    const int* d2_idx = nullptr;
    const raocp::DynTile* d2_tiles = nullptr;
    std::vector<int> d2_off;     // per stage t: [prod, node, fwdU, fwdX] tile offsets, 5 entries
    double *Q2 = nullptr, *PA2 = nullptr, *Dd2 = nullptr;
    // per-stage streaming dynamics (raocp_dyn3.hip): uniform branching, per-slot kinds and one
    // class per stage; fp32 contexts by default, fp64 opt-in RAOCP_DYN3=1
    bool dyn3 = false;
    std::vector<raocp::Dy3Stage> d3st;
    double *d3img_b = nullptr, *d3img_f = nullptr;  // per-stage table images (k_dy3_image)
    std::vector<raocp::Dy3Stage> d3own;  // a shard's stages (owned parent ranges below its cut)
    int d3ts = 0;  // the top stages k_dy3_top_back / k_dy3_top_fwd run in one workgroup (0: none)
    size_t d3nb = 0, d3nf = 0;  // doubles per stage image (backward, forward)
    int wsz = 8;                 // bytes per scalar of the iterate
    hipStream_t stream = nullptr;
    Dev dev{};
    int n = 0, m = 0, nx = 0, nu = 0, cmax = 0, N = 0;
    std::vector<int> stage_ptr;  // start id of each stage, size N+2
    int64_t P = 0, D = 0;
    // iterate and work buffers
    double* Z[3] = {nullptr, nullptr, nullptr};
    double* E[2] = {nullptr, nullptr};
    double* XI2 = nullptr;
    double* q = nullptr;         // q rows of the cut stage, padded (n x KP)
    double* d = nullptr;         // d rows (m x nu)
    // per-stage dynamics path: padded global rows
    double* gXQ = nullptr;       // n x KP  (x, then q)
    double* gU = nullptr;        // m x NUP
    double* gXD = nullptr;       // m x KF  ([x | d | 0])
    double* gP = nullptr;        // n x PS  (child products)
    int KP = 0, KF = 0, NUP = 0, PS = 0;
    int maxch_top = 0;
    std::vector<int> cls_ptr;    // first class of each stage (size N+1)
    std::vector<int> pair_ptr;   // first (kind, class) pair of each class (size n_k+1)
    int nkind = 0;
    bool f_lds_top = false;      // F table staged in LDS by k_dyn_top
    bool fold_top = false;       // k_dyn_top's backward levels in one phase (WT tables)
    struct TierPlan {            // a tier [s0, s1) below the top: one workgroup per subtree
        int s0, s1, nsub, maxch;
        size_t lds_b, lds_f;
        int fm;                  // F in the forward kernel: 0 global, 1 LDS, 2 LDS per level
        bool fold;               // one-phase backward levels (WT tables)
        const raocp::Rec* lv;    // level ranges of its subtrees
        raocp::TierArg ta;       // the same, as a kernel argument, when the tier is regular
    };
    std::vector<TierPlan> tiers;
    raocp::FuseArg fuse{};       // the split sweep's plan (counters / flags in fuse_sync)
    bool dyn_split = false;      // the tiered sweep in TWO launches (k_dyn_up / k_dyn_down)
    size_t lds_up = 0, lds_down = 0;
    unsigned* fuse_sync = nullptr;  // [epoch | error word | per tier: counters, flags]
    size_t fuse_words = 0;
    // the regular-tree sweep (raocp_dynr.hip): two launches, one workgroup per subtree of
    // every tier; the default for fp64 regular trees of the compiled sizes (RAOCP_DR=0: off)
    bool reg_ok = false;            // uniform branching, one class per stage, one pair per slot
    int reg_C = 0;
    std::vector<raocp::Dy3Stage> reg_st;
    bool dr = false;
    raocp::DrPlan drp{};
    int dr_block = 512;
    size_t dr_lds = 0;
    // k_drc (raocp_dynr.hip): k_dr with each subtree's CP families fused behind its forward
    // sweep, one launch per CP iteration (config 2: binary, 20 / 8, fp64, tiers of 4 levels, the
    // k_cp6 box patterns); RAOCP_DRC=0 keeps k_dr + k_cp6. Its residual rows alternate between two
    // sets of cp_rows rows (the extra workgroup tests the previous iteration beside the next)
    bool drc = false;
    raocp::DrcArg drca{};
    raocp::DrcArg* d_drca = nullptr;  // drca per iteration parity in device memory (k_drc reads it there)
    size_t drc_lds = 0;
    size_t dr_gran = 0;  // granules of each hand-off buffer
    double* x0 = nullptr;
    raocp::Bufs bufs{};          // {Z0, Z1, Z2, E0, E1}
    Ctl* ctl = nullptr;
    Ctl* h_ctl = nullptr;        // pinned host mirror
    raocp::CtlPub* h_pub = nullptr;  // pinned host memory the batch tail's stopping test publishes to
    raocp::CtlPub* d_pub = nullptr;  // (its device address)
    double* hist = nullptr;
    size_t hist_rows = 0;
    double* cur_z = nullptr;     // the Cache's current primal / dual
    double* cur_e = nullptr;
    double* tmpP = nullptr;      // staging for host-pointer calls
    double* tmpD = nullptr;
    double* part = nullptr;      // dot-product partials
    double* scal = nullptr;      // device scalars
    int cut = 0;                 // dynamics cut stage (0: per-stage kernels)
    double* redpart = nullptr;   // per-block residual maxima [red_rows][6]
    int red_rows = 0;
    size_t lds_top = 0;
    int dyn_block = 1024;        // tier workgroups (RAOCP_DYN_BLOCK)
    int dyn_top_block = 1024;    // the top's single workgroup (RAOCP_DYN_TOP_BLOCK)
    // node-block CP kernels (raocp_cp.hip): family / leaf block sizes, grid, LDS bytes
    int cp_FB = 1, cp_LB = 1, cp_nbF = 0, cp_nbL = 0;
    int ell_nb = 0, ell_threads = 512;  // L / L^T blocks (raocp_ell.hip), threads, LDS bytes
    size_t ell_lds = 0, ellt_lds = 0;
    size_t lds_cpd = 0, lds_cpp = 0;
    int cp_rows = 0;             // residual partial rows the CP iteration writes
    // MFMA CP kernels (raocp_cp2.hip): block shape, grid, LDS bytes; v1 = the scalar kernels
    int cp2_W = 4, cp2_FB = 1, cp2_LB = 16, cp2_nbF = 0, cp2_nbL = 0;
    size_t lds_cpd2 = 0, lds_cpp2 = 0;
    bool cp_v1 = false;          // RAOCP_CP_V1=1: the scalar k_cpd / k_cpp (raocp_cp.hip)
    // host copies the CP tables are (re)built from (build_cp_blocks)
    std::vector<int> h_yrel, h_chs, h_nch, h_pos7, h_pos14;
    std::vector<int> h_isq, h_isr, h_isp;  // per-node weight table indices (uniform-table blocks)
    // subtree sharding (raocp_shard_setup): R shards own contiguous blocks of the
    // subtrees rooted at the top's boundary stage sh_S; the top is replicated
    int sh_R = 1, sh_r = 0, sh_S = 0;
    std::vector<int> own_lo, own_hi;                // per stage: owned id range
    std::vector<std::pair<int, int>> tier_own;      // per tier: {first subtree, count}
    int x_max = 0;                                  // largest slice of stage sh_S
    int own_first = 0, own_cnt = 0;                 // this shard's slice
    double *x2_send = nullptr, *x2_recv = nullptr;  // q rows of the roots
    double *x1_send = nullptr, *x1_recv = nullptr;  // (eta+, xi2) eta2 entries of the roots
    const int* d_slc = nullptr;                     // [2R] {first id, count} per shard
    double* red8 = nullptr;                         // this shard's maxima, then all-reduced
    void* comm = nullptr;                           // ncclComm_t when the transport is RCCL
    bool eager = false;                             // iterations launched without a graph
    int n_sq = 0, n_sr = 0, n_sp = 0, nbn = 1, nbl = 1;
    const int* ph = nullptr;     // dual placeholder offsets
    int n_ph = 0;
    bool has_x0 = false;
    std::vector<double> h_x0;
    bool no_defer_check = false; // RAOCP_DEFER_CHECK=0: k_cp_check after every iteration (defer_check)
                                 // (measured slower than its own launch: DESIGN.md)
    // captured CP iterations
    hipGraphExec_t graph = nullptr;      // kGraphBatch iterations (raocp_cp_run, raocp_cp_bench)
    int graph_iters = 0;
    hipGraphExec_t graph_rem = nullptr;  // the remainder batch of raocp_cp_bench (exactly K iterations)
    int prepared = 0;                    // raocp_cp_prepare(x0) set up a run of this many iterations
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    int graph_rem_iters = 0;
    std::vector<void*> allocs;

    template <class T>
    int alloc(T** p, size_t count) {
        void* v = nullptr;
        if (count == 0) count = 1;
        hipError_t e = hipMalloc(&v, count * sizeof(T) + 64);  // slack: LDS-DMA reads whole 16-B chunks
        if (e != hipSuccess) return fail(RAOCP_ERR_HIP, std::string("hipMalloc: ") + hipGetErrorString(e));
        allocs.push_back(v);
        *p = (T*)v;
        return RAOCP_OK;
    }
    template <class T>
    int upload(const T** dst, const T* src, size_t count) {
        T* p = nullptr;
        int rc = alloc(&p, count);
        if (rc) return rc;
        if (count) HIPCHK(hipMemcpy(p, src, count * sizeof(T), hipMemcpyHostToDevice));
        *dst = p;
        return RAOCP_OK;
    }
    template <class T>
    int upload_vec(const T** dst, const std::vector<T>& v) {
        return upload(dst, v.data(), v.size());
    }
};

namespace {

// row-major table [cnt][rows][cols] -> column-major per matrix: out[k*rows + r] = M[r][k]
std::vector<double> to_colmajor(const double* src, int cnt, int rows, int cols) {
    std::vector<double> out((size_t)cnt * rows * cols);
    for (int t = 0; t < cnt; ++t)
        for (int r = 0; r < rows; ++r)
            for (int k = 0; k < cols; ++k)
                out[(size_t)t * rows * cols + (size_t)k * rows + r] = src[(size_t)t * rows * cols + (size_t)r * cols + k];
    return out;
}

std::vector<double> copy_table(const double* src, size_t count) {
    return std::vector<double>(src, src + count);
}

struct Launch {
    int G, per, blocks;
};

Launch groups(int G, int count) {
    Launch l;
    l.G = G;
    l.per = kBlock / G;
    l.blocks = cdiv(count, l.per);
    return l;
}

int check_group(int G, const char* what) {
    if (G > kBlock)
        return fail(RAOCP_ERR_ARG, std::string("group size of ") + what + " (" + std::to_string(G) +
                                       ") exceeds the 256-lane workgroup; nx/nu/children too large for this build");
    return RAOCP_OK;
}

// host fp64 arrays <-> the context's device vectors (fp32 contexts convert on the host;
// a device pointer is taken in the context's own type)
int copy_in(raocp_ctx* c, double* dst, const double* src, size_t count, int flags) {
    if (c->f32 && !(flags & RAOCP_DEVICE_PTR)) {
        std::vector<float> tmp(src, src + count);
        HIPCHK(hipMemcpyAsync(dst, tmp.data(), count * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        return RAOCP_OK;
    }
    HIPCHK(hipMemcpyAsync(dst, src, count * c->wsz,
                          (flags & RAOCP_DEVICE_PTR) ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, c->stream));
    return RAOCP_OK;
}

int copy_out(raocp_ctx* c, double* dst, const double* src, size_t count, int flags) {
    if (c->f32 && !(flags & RAOCP_DEVICE_PTR)) {
        std::vector<float> tmp(count);
        HIPCHK(hipMemcpyAsync(tmp.data(), src, count * sizeof(float), hipMemcpyDeviceToHost, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));
        std::copy(tmp.begin(), tmp.end(), dst);
        return RAOCP_OK;
    }
    HIPCHK(hipMemcpyAsync(dst, src, count * c->wsz,
                          (flags & RAOCP_DEVICE_PTR) ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
    if (!(flags & RAOCP_DEVICE_PTR)) HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

// a table as the context's scalar type (fp32 contexts keep float arrays in the Dev's
// double* fields; only the T-templated kernels read them)
int upload_t(raocp_ctx* c, const double** dst, const std::vector<double>& v) {
    if (!c->f32) return c->upload_vec(dst, v);
    std::vector<float> f(v.begin(), v.end());
    const float* p = nullptr;
    int rc = c->upload_vec(&p, f);
    *dst = (const double*)p;
    return rc;
}

// ---- template dispatch on (nx, nu): exact sizes get fully unrolled kernels,
// everything else runs the runtime-size instantiation <0, 0>.
template <class F, class... A>
void dispatch(int nx, int nu, F f, A... a) {
    if (nx == 20 && nu == 8) f.template run<20, 8>(a...);
    else if (nx == 32 && nu == 12) f.template run<32, 12>(a...);
    else if (nx == 64 && nu == 16) f.template run<64, 16>(a...);
    else if (nx == 3 && nu == 2) f.template run<3, 2>(a...);
    else f.template run<0, 0>(a...);
}

// the MFMA CP kernels are instantiated per (row tiles of nx, row tiles of nu)
template <class F, class... A>
void dispatch_rt(int nx, int nu, F f, A... a) {
    const int rx = (nx + 15) / 16, ru = (nu + 15) / 16;
    if (ru == 1) {
        if (rx == 1) f.template run<1, 1>(a...);
        else if (rx == 2) f.template run<2, 1>(a...);
        else if (rx == 3) f.template run<3, 1>(a...);
        else f.template run<4, 1>(a...);
    } else {
        if (rx == 1) f.template run<1, 2>(a...);
        else if (rx == 2) f.template run<2, 2>(a...);
        else if (rx == 3) f.template run<3, 2>(a...);
        else f.template run<4, 2>(a...);
    }
}
template <class K>
void allow_lds(K kernel, size_t bytes) {
    if (bytes > 64 * 1024) (void)hipFuncSetAttribute((const void*)kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                                      (int)bytes);
}

// ---- launches (all on c->stream)
struct EllOp {
    template <int NX, int NU>
    void run(raocp_ctx* c, const double* z, double* eta) {
        auto k = raocp::k_ell<NX, NU>;
        allow_lds(k, c->ell_lds);
        if (c->ell_nb) k<<<c->ell_nb, c->ell_threads, c->ell_lds, c->stream>>>(c->dev, z, eta);
    }
};
template <class T>
struct Ell2Op {
    template <int RX, int RU>
    void run(raocp_ctx* c, const double* z, double* eta, bool t) {
        if (t) {
            auto k = raocp::k_ellt2<T, RX, RU>;
            allow_lds(k, c->lds_cpp2);
            k<<<c->cp2_nbF + c->cp2_nbL, 64 * c->cp2_W, c->lds_cpp2, c->stream>>>(c->dev, z, eta, c->cp2_nbF);
        } else {
            auto k = raocp::k_ell2<T, RX, RU>;
            allow_lds(k, c->lds_cpd2);
            k<<<c->cp2_nbF + c->cp2_nbL, 64 * c->cp2_W, c->lds_cpd2, c->stream>>>(c->dev, z, eta, c->cp2_nbF);
        }
    }
};
// L as streaming wave tasks (raocp_ell3.hip): compile-time sizes of the benchmark configs
template <class T>
bool launch_ell3(raocp_ctx* c, const double* z, double* eta) {
    const int g = c->ell3_grid;
    if (c->nx == 20 && c->nu == 8) raocp::k_ell3<T, 20, 8><<<g, 256, 0, c->stream>>>(c->dev, z, eta, c->unif_C, c->box_mode);
    else if (c->nx == 32 && c->nu == 12) raocp::k_ell3<T, 32, 12><<<g, 256, 0, c->stream>>>(c->dev, z, eta, c->unif_C, c->box_mode);
    else if (c->nx == 64 && c->nu == 16) raocp::k_ell3<T, 64, 16><<<g, 256, 0, c->stream>>>(c->dev, z, eta, c->unif_C, c->box_mode);
    else return false;
    return true;
}
void launch_ell(raocp_ctx* c, const double* z, double* eta) {
    if (c->ell3 && (c->f32 ? launch_ell3<float>(c, z, eta) : launch_ell3<double>(c, z, eta))) return;
    if (c->f32) dispatch_rt(c->nx, c->nu, Ell2Op<float>{}, c, z, eta, false);
    else dispatch(c->nx, c->nu, EllOp{}, c, z, eta);
}

struct EllTOp {
    template <int NX, int NU>
    void run(raocp_ctx* c, const double* eta, double* z) {
        auto k = raocp::k_ell_t<NX, NU>;
        allow_lds(k, c->ellt_lds);
        if (c->ell_nb) k<<<c->ell_nb, c->ell_threads, c->ellt_lds, c->stream>>>(c->dev, eta, z);
    }
};
// L^T as streaming wave tasks (raocp_ell3.hip): uniform tables and branching
template <class T, int QM>
bool launch_ellt3q(raocp_ctx* c, const double* eta, double* z) {
    const int g = c->ellt3_grid, C = c->ellt3_C;
    if (c->nx == 20 && c->nu == 8) raocp::k_ellt3<T, 20, 8, QM><<<g, 256, 0, c->stream>>>(c->dev, eta, z, C, c->box_mode);
    else if (c->nx == 32 && c->nu == 12) raocp::k_ellt3<T, 32, 12, QM><<<g, 256, 0, c->stream>>>(c->dev, eta, z, C, c->box_mode);
    else if (c->nx == 64 && c->nu == 16) raocp::k_ellt3<T, 64, 16, QM><<<g, 256, 0, c->stream>>>(c->dev, eta, z, C, c->box_mode);
    else return false;
    return true;
}
template <class T>
bool launch_ellt3(raocp_ctx* c, const double* eta, double* z) {
    const int C = c->ellt3_C;
    if (C == 1) return launch_ellt3q<T, 4>(c, eta, z);
    if (C == 2) return launch_ellt3q<T, 2>(c, eta, z);
    return launch_ellt3q<T, 1>(c, eta, z);
}
void launch_ell_t(raocp_ctx* c, const double* eta, double* z) {
    if (c->ellt3_C && (c->f32 ? launch_ellt3<float>(c, eta, z) : launch_ellt3<double>(c, eta, z))) return;
    if (c->f32) dispatch_rt(c->nx, c->nu, Ell2Op<float>{}, c, eta, z, true);
    else dispatch(c->nx, c->nu, EllTOp{}, c, eta, z);
}

// ---- per-stage MFMA dynamics (raocp_dyn2.hip) on z = the iterate to project
template <class T>
struct Dyn2Op {
    template <int RX, int RU>
    void run(raocp_ctx* c, double* z, const Ctl* ctl) {
        const int N = c->N, nthr = 256, W = nthr / 64;
        auto grid = [&](int nt) { return std::max(1, cdiv(nt, W)); };
        for (int t = N - 1; t >= 0; --t) {
            const int* o = &c->d2_off[(size_t)t * 5];
            const bool leaf = t + 1 == N;
            if (o[1] > o[0])
                raocp::k_d2_prod<T, RX + RU, 4 * RX><<<grid(o[1] - o[0]), nthr, 0, c->stream>>>(
                    c->dev, ctl, c->d2_tiles + o[0], o[1] - o[0], c->d2_idx, c->W2, leaf ? z : c->Q2,
                    leaf ? c->dev.X0 : 0, leaf ? T(-1) : T(1), c->PA2);
            if (o[2] > o[1])
                raocp::k_d2_node<T, RX + RU, 4 * RU><<<grid(o[2] - o[1]), nthr, 0, c->stream>>>(
                    c->dev, ctl, c->d2_tiles + o[1], o[2] - o[1], c->d2_idx, c->RG2, z, c->PA2, c->Q2, c->Dd2);
        }
        raocp::k_d2_x0<T><<<1, 64, 0, c->stream>>>(ctl, z, c->dev.X0, c->x0, c->nx);
        for (int t = 0; t < N; ++t) {
            const int* o = &c->d2_off[(size_t)t * 5];
            if (o[3] > o[2])
                raocp::k_d2_fwd<T, RU, 4 * RX, false><<<grid(o[3] - o[2]), nthr, 0, c->stream>>>(
                    c->dev, ctl, c->d2_tiles + o[2], o[3] - o[2], c->d2_idx, c->KM2, z, c->Dd2);
            if (o[4] > o[3])
                raocp::k_d2_fwd<T, RX, 4 * (RX + RU), true><<<grid(o[4] - o[3]), nthr, 0, c->stream>>>(
                    c->dev, ctl, c->d2_tiles + o[3], o[4] - o[3], c->d2_idx, c->F2, z, c->Dd2);
        }
    }
};

// the per-stage streaming sweep (raocp_dyn3.hip) on z; ck: the previous iteration's stopping
// test in an extra workgroup of the first launch (defer_check)
// part: 0 the whole projection; 1 (a shard) the backward stages below its cut, on its owned
// parents; 2 the replicated top backward, then every forward stage (owned below the cut)
// the stages k_dy3_top_back / k_dy3_top_fwd run in one workgroup: a shard merges only stages of
// its replicated top (t < sh_S, run after X2), at least two of them
int dyn3_top_stages(const raocp_ctx* c) {
    if (c->sh_S == 0) return c->d3ts;
    const int ts = std::min(c->d3ts, c->sh_S);
    return ts >= 2 ? ts : 0;
}
template <class T, int NX, int NU>
void launch_dyn3t(raocp_ctx* c, double* z, const Ctl* ctl, const raocp::ChkArg* ck, int part) {
    typedef raocp::Dy3Lds<T, NX, NU> L;
    const int C = c->unif_branch;
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    // LDS: the stage's tables; the backward kernel's slot sums of a cooperative tile after them
    const size_t lb = (size_t)(L::back_n(C) + C * (RU + RX) * 4 * 64) * sizeof(T), lf = (size_t)L::fwd_n(C) * sizeof(T);
    const size_t lmax = std::max(lb, lf);
    const int thr = lmax > 64 * 1024 ? 512 : 256, wpb = thr / 64;
    // (1,024-lane workgroups for the wide stages when the tables allow one workgroup per CU
    // measured slower at config 5: 215.3 vs 190.9 us per projection, profiles/r03_v3)
    // the wide stages (a wave per tile, looping) in 256-lane workgroups: at config 5 (one
    // workgroup per CU by LDS) 4 waves of 4 tiles each beat 8 waves of 2 (projection 197.1 ->
    // 191.9 us); at least 2 tiles per wave measured slower at configs 4 and 5 (fewer waves in
    // flight: 113.6 -> 123.1, 197.1 -> 217.9 us; profiles/r05/dy3_geometry.log)
    const int thr_w = 256, wpb_w = thr_w / 64;
    const int per_cu = std::max<int>(1, std::min<int>(2048 / thr_w, (int)(160 * 1024 / lmax)));
    const int cap = 256 * per_cu;  // one round of resident workgroups; waves loop over tiles
    auto kb = raocp::k_dy3_back<T, NX, NU>;
    auto kf = raocp::k_dy3_fwd<T, NX, NU>;
    allow_lds(kb, lb);
    allow_lds(kf, lf);
    // stages of few tiles run slot-parallel (a wave per child slot): the dependent MFMA chain
    // of a tile is what a small stage costs. Decided on the whole stage, so a shard sums a
    // parent's child slots in the same order as the unsharded sweep (bit-identical results).
    // (every stage slot-parallel, a workgroup looping over its tiles, measured slower: config 4
    // 112.3 vs 110.4 us, config 5 227.5 vs 197.3 us per projection, profiles/r04/cp3_time_dy3.log)
    auto coop = [&](int t) { return (c->d3st[t].i1 - c->d3st[t].i0 + 15) / 16 * C <= 256 * wpb; };
    auto grid = [&](const raocp::Dy3Stage& st, int t, bool back) {
        const int tiles = (st.i1 - st.i0 + 15) / 16;
        if (coop(t)) return std::max(1, std::min(cap, back ? tiles : (tiles * C + wpb - 1) / wpb));
        return std::max(1, std::min(cap, (tiles + wpb_w - 1) / wpb_w));
    };
    auto threads = [&](int t) { return coop(t) ? thr : thr_w; };
    const int N = c->N, S = c->sh_S;  // S > 0: a shard owns the stages >= S partly
    auto stage = [&](int t) -> const raocp::Dy3Stage& { return S > 0 && t >= S ? c->d3own[t] : c->d3st[t]; };
    // the top stages t < ts in one workgroup per direction (dyn3_top_stages)
    const int ts = dyn3_top_stages(c);
    raocp::Dy3Top tp{};
    tp.ts = ts;
    for (int t = 0; t < ts; ++t) tp.st[t] = c->d3st[t];
    tp.same_kinds = 1;
    for (int t = 1; t < ts; ++t)
        for (int k = 0; k < C; ++k) tp.same_kinds &= c->d3st[t].kind[k] == c->d3st[0].kind[k];
    const size_t ltop = (size_t)(L::back_n(C) + (8 / C) * C * (RU + RX) * 4 * 64) * sizeof(T);
    auto ktb = raocp::k_dy3_top_back<T, NX, NU>;
    auto ktf = raocp::k_dy3_top_fwd<T, NX, NU>;
    if (ts) {
        allow_lds(ktb, ltop);
        allow_lds(ktf, lf);
    }
    for (int t = N - 1; t >= ts; --t) {
        if (part == 1 && t < S) break;
        if (part == 2 && t >= S) continue;
        const raocp::Dy3Stage& st = stage(t);
        if (st.i1 <= st.i0) continue;
        raocp::ChkArg ca{};
        if (ck && t == N - 1) ca = *ck;
        const double* img = (const double*)((const char*)c->d3img_b + (size_t)t * L::back_n(C) * sizeof(T));
        kb<<<grid(st, t, true) + ca.on, threads(t), lb, c->stream>>>(c->dev, ctl, ca, z, c->Q2, c->Dd2, st, C, img,
                                                                    coop(t) ? 1 : 0);
    }
    if (part == 1) return;
    if (ts) {
        ktb<<<1, 512, ltop, c->stream>>>(c->dev, ctl, z, c->Q2, c->Dd2, tp, C, (const double*)c->d3img_b);
        ktf<<<1, 512, lf, c->stream>>>(c->dev, ctl, z, c->Dd2, c->x0, tp, C, (const double*)c->d3img_f);
    }
    for (int t = ts; t < N; ++t) {
        const raocp::Dy3Stage& st = stage(t);
        if (st.i1 <= st.i0) continue;
        const double* img = (const double*)((const char*)c->d3img_f + (size_t)t * L::fwd_n(C) * sizeof(T));
        kf<<<grid(st, t, false), threads(t), lf, c->stream>>>(c->dev, ctl, z, c->Dd2, c->x0, st, C, img,
                                                               coop(t) ? 1 : 0);
    }
}
// LDS bytes of the sweep's larger launch (tables + the slot-parallel sums; launch_dyn3t)
template <class T, int NX, int NU>
size_t dyn3_lds(int C) {
    typedef raocp::Dy3Lds<T, NX, NU> L;
    constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
    return std::max((size_t)(L::back_n(C) + C * (RU + RX) * 4 * 64) * sizeof(T), (size_t)L::fwd_n(C) * sizeof(T));
}
bool dyn3_lds_fits(bool f32, int nx, int nu, int C) {
    size_t b = ~(size_t)0;
    if (nx == 20 && nu == 8) b = f32 ? dyn3_lds<float, 20, 8>(C) : dyn3_lds<double, 20, 8>(C);
    else if (nx == 32 && nu == 12) b = f32 ? dyn3_lds<float, 32, 12>(C) : dyn3_lds<double, 32, 12>(C);
    else if (nx == 64 && nu == 16 && f32) b = dyn3_lds<float, 64, 16>(C);
    // (fp64 at nx = 64: the tables exceed the LDS, so k_dy3 has no such instantiation)
    return b <= 160 * 1024;
}
// the per-stage table images of the sweep, laid out once (k_dy3_image, one workgroup per stage)
template <class T, int NX, int NU>
int dyn3_imagest(raocp_ctx* c) {
    typedef raocp::Dy3Lds<T, NX, NU> L;
    const int C = c->unif_branch, N = (int)c->d3st.size();
    const size_t nb = (size_t)L::back_n(C) * sizeof(T) / 8, nf = (size_t)L::fwd_n(C) * sizeof(T) / 8;
    c->d3nb = nb;
    c->d3nf = nf;
    int rc;
    if ((rc = c->alloc(&c->d3img_b, std::max<size_t>(1, N * nb))) || (rc = c->alloc(&c->d3img_f, std::max<size_t>(1, N * nf))))
        return rc;
    // the top stages of at most two rounds of 512 / (64 C) tiles run in one workgroup per
    // direction (k_dy3_top_back / k_dy3_top_fwd); RAOCP_DY3_TOP=0 keeps a launch per stage
    {
        constexpr int RX = (NX + 15) / 16, RU = (NU + 15) / 16;
        const int tpr = 8 / C;
        const size_t ltop = (size_t)(L::back_n(C) + tpr * C * (RU + RX) * 4 * 64) * sizeof(T);
        // (stages of up to 4 / 16 rounds measured slower: config 4 117.8 / 145.4 vs 111.6 us,
        // profiles/r04/cp3_time_dy3_rounds.log)
        const int rounds = 2;
        int ts = 0;
        while (ts < N - 1 && ts < raocp::kDy3TopMax && (c->d3st[ts].i1 - c->d3st[ts].i0 + 15) / 16 <= rounds * tpr) ++ts;
        if (ts < 2 || ltop > 159 * 1024 || (size_t)L::fwd_n(C) * sizeof(T) > 159 * 1024) ts = 0;
        if (const char* e = getenv("RAOCP_DY3_TOP")) ts = atoi(e) ? ts : 0;
        c->d3ts = ts;
    }
    for (int t = 0; t < N; ++t)
        raocp::k_dy3_image<T, NX, NU><<<1, 512, 0, c->stream>>>(c->d3st[t], C, c->W2, c->RG2, c->KM2, c->F2,
                                                                c->d3img_b + t * nb, c->d3img_f + t * nf);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}
int dyn3_images(raocp_ctx* c) {
    if (c->f32) {
        if (c->nx == 20) return dyn3_imagest<float, 20, 8>(c);
        if (c->nx == 32) return dyn3_imagest<float, 32, 12>(c);
        return dyn3_imagest<float, 64, 16>(c);
    }
    if (c->nx == 20) return dyn3_imagest<double, 20, 8>(c);
    if (c->nx == 32) return dyn3_imagest<double, 32, 12>(c);
    return fail(RAOCP_ERR_ARG, "k_dy3 has no fp64 form at nx = 64 (dyn3_lds_fits)");
}
void launch_dyn3(raocp_ctx* c, double* z, const Ctl* ctl, const raocp::ChkArg* ck, int part) {
    if (c->f32) {
        if (c->nx == 20) launch_dyn3t<float, 20, 8>(c, z, ctl, ck, part);
        else if (c->nx == 32) launch_dyn3t<float, 32, 12>(c, z, ctl, ck, part);
        else launch_dyn3t<float, 64, 16>(c, z, ctl, ck, part);
    } else {
        // (no fp64 nx = 64 form: dyn3_lds_fits keeps such contexts off k_dy3)
        if (c->nx == 20) launch_dyn3t<double, 20, 8>(c, z, ctl, ck, part);
        else if (c->nx == 32) launch_dyn3t<double, 32, 12>(c, z, ctl, ck, part);
    }
}

// workgroups per CU of the split sweep's two kernels at their LDS sizes (co-residency)
struct SplitOcc {
    template <int NX, int NU>
    void run(raocp_ctx* c, int* pu, int* pd) {
        auto ku = raocp::k_dyn_up<NX, NU>;
        auto kd = c->f_lds_top ? raocp::k_dyn_down<NX, NU, true> : raocp::k_dyn_down<NX, NU, false>;
        allow_lds(ku, c->lds_up);
        allow_lds(kd, c->lds_down);
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(pu, (const void*)ku, raocp::kFuseBlock, c->lds_up) != hipSuccess)
            *pu = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(pd, (const void*)kd, raocp::kFuseBlock, c->lds_down) != hipSuccess)
            *pd = 0;
    }
};

struct DynOp {
    // part: 0 whole projection; 1 the tiers' backward sweeps only; 2 the top and the
    // tiers' forward sweeps (a shard exchanges the roots' q rows in between)
    template <int NX, int NU>
    void run(raocp_ctx* c, raocp::Bufs bf, int zsel, const Ctl* ctl, int part, const raocp::ChkArg* ck) {
        const int s = c->cut;
        const int B = c->dyn_block;
        // diagnostics: each launch stamps into its own 64-slot region
        Dev dv = c->dev;
        int slot = 0;
        auto dev_for = [&]() {
            if (c->dev.stamps) dv.stamps = c->dev.stamps + 64 * slot++;
            return dv;
        };
        const bool sharded = c->sh_S > 0;
        auto tier_arg = [&](int k) {  // a shard launches only the subtrees it owns
            raocp::TierArg ta = c->tiers[k].ta;
            ta.boff = sharded ? c->tier_own[k].first : 0;
            return ta;
        };
        auto tier_blocks = [&](int k) { return sharded ? c->tier_own[k].second : c->tiers[k].nsub; };
        if (s > 0 && c->dyn_split && !sharded && part == 0) {
            // the tiered sweep in two launches (raocp_dynf.hip): one workgroup per subtree of
            // every tier plus the top; k_dyn_up runs the deferred stopping test in block 0
            raocp::FuseArg fa = c->fuse;
            if (ck) fa.ck = *ck;
            int nsub = 0;
            for (const auto& tp : c->tiers) nsub += tp.nsub;
            auto ku = raocp::k_dyn_up<NX, NU>;
            auto kd = c->f_lds_top ? raocp::k_dyn_down<NX, NU, true> : raocp::k_dyn_down<NX, NU, false>;
            allow_lds(ku, c->lds_up);
            allow_lds(kd, c->lds_down);
            ku<<<nsub + 1 + (fa.ck.on ? 1 : 0), raocp::kFuseBlock, c->lds_up, c->stream>>>(dev_for(), bf, ctl, zsel, c->q,
                                                                                           c->d, fa);
            kd<<<nsub + 1, raocp::kFuseBlock, c->lds_down, c->stream>>>(dev_for(), bf, ctl, zsel, c->d, c->x0, fa);
            return;
        }
        if (s > 0) {
            // tiers below the top, deepest first (backward), the top, then the tiers (forward)
            if (part != 2)
                for (int k = (int)c->tiers.size() - 1; k >= 0; --k) {
                    const auto& tp = c->tiers[k];
                    const int c0 = c->cls_ptr[tp.s0], c1 = c->cls_ptr[tp.s1];
                    const int p0 = c->pair_ptr[c0], p1 = c->pair_ptr[c1];
                    auto kb = tp.fold ? raocp::k_dyn_bottom_back<NX, NU, true> : raocp::k_dyn_bottom_back<NX, NU, false>;
                    allow_lds(kb, tp.lds_b);
                    // the deepest tier (launched first) carries the deferred stopping test
                    raocp::ChkArg cka{};
                    raocp::TierArg ta = tier_arg(k);
                    if (ck && k == (int)c->tiers.size() - 1) {
                        cka = *ck;
                        ta.boff -= 1;
                    }
                    if (tier_blocks(k) > 0)
                        kb<<<tier_blocks(k) + cka.on, B, tp.lds_b, c->stream>>>(dev_for(), bf, ctl, zsel, c->q, c->d, tp.s0,
                                                                               tp.s1, tp.maxch, c0, c1, p0, p1, tp.lv, ta, cka);
                }
            if (part == 1) return;
            {
                const int c1 = c->cls_ptr[s], p1 = c->pair_ptr[c1];
                auto kt = c->f_lds_top ? (c->fold_top ? raocp::k_dyn_top<NX, NU, true, true> : raocp::k_dyn_top<NX, NU, true, false>)
                                       : (c->fold_top ? raocp::k_dyn_top<NX, NU, false, true> : raocp::k_dyn_top<NX, NU, false, false>);
                allow_lds(kt, c->lds_top);
                const int T = c->stage_ptr[s], nb = c->stage_ptr[s + 1] - T;
                kt<<<1, c->dyn_top_block, c->lds_top, c->stream>>>(dev_for(), bf, ctl, zsel, c->q, c->x0, s, c->maxch_top, c1,
                                                                   p1, T, nb);
            }
            for (int k = 0; k < (int)c->tiers.size(); ++k) {
                const auto& tp = c->tiers[k];
                const int c0 = c->cls_ptr[tp.s0], c1 = c->cls_ptr[tp.s1], p0 = c->pair_ptr[c0], p1 = c->pair_ptr[c1];
                auto kf = tp.fm == 1 ? raocp::k_dyn_bottom_fwd<NX, NU, 1>
                                     : (tp.fm == 2 ? raocp::k_dyn_bottom_fwd<NX, NU, 2> : raocp::k_dyn_bottom_fwd<NX, NU, 0>);
                allow_lds(kf, tp.lds_f);
                if (tier_blocks(k) > 0)
                    kf<<<tier_blocks(k), B, tp.lds_f, c->stream>>>(dev_for(), bf, ctl, zsel, c->d, tp.s0, tp.s1, c0, c1,
                                                                  p0, p1, tp.lv, tier_arg(k));
            }
            return;
        }
        if (part == 2) return;  // the per-stage path runs whole in part 1 / 0
        // per-stage path on padded global rows
        const int R = c->nu + c->nx;
        raocp::k_dyn_gather<NX, NU><<<std::max(1, std::min(1024, cdiv(c->n * c->KP, kBlock))), kBlock, 0, c->stream>>>(
            c->dev, bf, ctl, zsel, c->gXQ, c->gU, c->gXD);
        for (int t = c->N - 1; t >= 0; --t) {
            const int b = c->stage_ptr[t], e = c->stage_ptr[t + 1];
            const int cb = e, ce = c->stage_ptr[t + 2];
            const int slots_a = B / (R * raocp::kKS), slots_b = B / R;
            raocp::k_dyn_stage_a<NX, NU><<<cdiv(ce - cb, slots_a), B, 0, c->stream>>>(
                c->dev, ctl, c->gXQ, c->gP, cb, ce, t + 1 == c->N ? -1.0 : 1.0);
            raocp::k_dyn_stage_b<NX, NU><<<cdiv(e - b, slots_b), B, 0, c->stream>>>(c->dev, ctl, c->gXQ, c->gU,
                                                                                         c->gP, c->gXD, c->d, b, e);
        }
        const int per_node = c->nu * raocp::kKS + c->cmax * c->nx * raocp::kKS;
        const int slots_f = std::max(1, B / per_node);
        for (int t = 0; t < c->N; ++t) {
            const int b = c->stage_ptr[t], e = c->stage_ptr[t + 1];
            raocp::k_dyn_stage_f<NX, NU><<<cdiv(e - b, slots_f), B, 0, c->stream>>>(c->dev, bf, ctl, zsel, c->gXD,
                                                                                         c->x0, b, e);
        }
    }
};
// dynamics projection on z = Z[(k + zsel) % 3] (k from ctl when ctl != null, else 0)
// ck: the previous CP iteration's stopping test, run by an extra workgroup of the first
// launch (only where defer_check(c) holds)
void launch_dynamics(raocp_ctx* c, raocp::Bufs bf, int zsel, const Ctl* ctl, int part = 0,
                     const raocp::ChkArg* ck = nullptr) {
    if (c->dr && c->sh_S == 0 && part == 0) {  // the regular-tree sweep (raocp_dynr.hip)
        raocp::DrPlan p = c->drp;
        if (c->dev.stamps) p.stamps = c->dev.stamps;
        raocp::dr_launch(p, c->nx, c->nu, c->dr_lds, bf, zsel, ctl,
                         ck ? *ck : raocp::ChkArg{nullptr, nullptr, nullptr, 0, 0}, c->stream);
        return;
    }
    if (c->dyn3) {
        double* z = zsel % 3 == 0 ? bf.z0 : (zsel % 3 == 1 ? bf.z1 : bf.z2);
        launch_dyn3(c, z, ctl, ck, part);
        return;
    }
    if (c->dyn2) {
        double* z = zsel % 3 == 0 ? bf.z0 : (zsel % 3 == 1 ? bf.z1 : bf.z2);
        if (c->f32) dispatch_rt(c->nx, c->nu, Dyn2Op<float>{}, c, z, ctl);
        else dispatch_rt(c->nx, c->nu, Dyn2Op<double>{}, c, z, ctl);
        return;
    }
    dispatch(c->nx, c->nu, DynOp{}, c, bf, zsel, ctl, part, ck);
}

// the device word a hand-off sweep sets when a wait times out (nullptr: no such sweep)
const unsigned* err_word(const raocp_ctx* c) {
    if (c->dr && c->sh_S == 0) return c->drp.sync + 1;
    if (c->dyn_split && c->fuse_sync) return (const unsigned*)c->fuse_sync + 1;
    return nullptr;
}
// the fused sweep's error word (a hand-off wait timed out, raocp_dynf.hip): checked after
// every synchronised run that may have launched it; the context is unusable afterwards
int fuse_err(raocp_ctx* c) {
    if (c->dr && c->sh_S == 0) {
        unsigned e = 0;
        HIPCHK(hipMemcpy(&e, c->drp.sync + 1, sizeof(unsigned), hipMemcpyDeviceToHost));
        if (e) {
            // clear the epoch, the error word and every granule: the next projection starts
            // from a clean protocol state
            HIPCHK(hipMemset(c->drp.sync, 0, 2 * sizeof(unsigned)));
            HIPCHK(hipMemset(c->drp.gq, 0, c->dr_gran * sizeof(unsigned long long)));
            HIPCHK(hipMemset(c->drp.gx, 0, c->dr_gran * sizeof(unsigned long long)));
            return fail(RAOCP_ERR_STATE, "dynamics sweep: a workgroup hand-off timed out (k_dr); "
                                         "RAOCP_DR=0 selects the tiered sweep");
        }
        return RAOCP_OK;
    }
    if (!c->dyn_split || !c->fuse_sync) return RAOCP_OK;
    int e = 0;
    HIPCHK(hipMemcpy(&e, c->fuse_sync + 1, sizeof(int), hipMemcpyDeviceToHost));
    if (e) HIPCHK(hipMemset(c->fuse_sync, 0, c->fuse_words * sizeof(unsigned)));  // clean protocol state
    if (e) return fail(RAOCP_ERR_STATE, "dynamics sweep: a workgroup hand-off timed out (k_dyn_up / k_dyn_down); "
                                        "RAOCP_DYN_SPLIT=0 selects the tier launches");
    return RAOCP_OK;
}

// ---- the regular-tree sweep (raocp_dynr.hip) -----------------------------------------------
// Tables in the kernel's LDS order, per nonleaf stage t (its class and the pairs of its child
// slots, c->reg_st[t]), element-pair-major [p][lane][2] so lane s reads its row pair p as one
// 16-B word:
//   backward lane s = r KS + k (row r < nx + nu, slot k; LB = (nx + nu) KS lanes): WT = [-Rinv B' ; A' - G B'] row r of
//            slot k's pair (zero for k >= C), then entries [k UP, (k + 1) UP) of RG = [Rinv ; G]
//            row r of the class;
//   forward  lane s = k nx + r (slot k, row r < nx; LF = C nx + nu lanes): [Abar_k | B_k] row r; lane C nx + r
//            (r < nu): [K row r | unit vector e_r] (u_r = K x + d_r as one dot product).
// The tier plan minimises a cost model of the critical path (us, fitted to measured cut lists:
// per level of each sweep a fixed part and a part per node, per tier boundary its two
// hand-offs) over cut lists of at most kDrMaxTiers tiers whose grid (one workgroup per subtree
// of every tier, plus the stopping test) is resident at once (occupancy x CU count): no wait
// then depends on the dispatch order. RAOCP_DR_CUTS="s1:s2:.." forces the cuts.
int dr_setup(raocp_ctx* c, const std::vector<double>& WT, int SKP, const std::vector<double>& RG, int SNU,
             const std::vector<double>& KM, const std::vector<double>& F, int SKF, int n_cus) {
    const int nx = c->nx, nu = c->nu, C = c->reg_C, N = c->N, R = nx + nu;
    const int KS = raocp::dr_ks(C), UP = raocp::dr_up(nu, C), LB = raocp::dr_lb(nx, nu, C),
              LF = raocp::dr_lf(nx, nu, C);
    const int nb = raocp::dr_tb_n(nx, nu, C), nf = raocp::dr_tf_n(nx, nu, C);
    auto npow = [&](int e) {
        long v = 1;
        for (int i = 0; i < e; ++i) v *= C;
        return v;
    };
    if (N >= raocp::kDrMaxStages) return RAOCP_OK;  // the sweep stays off
    int block = 512;
    // cost (us) of a cut list s = {0, s1, .., N}; 1e300 where it does not fit
    auto eval = [&](const std::vector<int>& s) -> double {
        const int T = (int)s.size() - 1;
        if (T < 1 || T > raocp::kDrMaxTiers) return 1e300;
        long wgs = 1;  // the stopping test
        size_t lds = 0;
        int lmax = 0;
        for (int k = 0; k < T; ++k) {
            const int L = s[k + 1] - s[k];
            if (L < 1 || L > raocp::kDrMaxL) return 1e300;
            lmax = std::max(lmax, L);
            wgs += npow(s[k]);
            lds = std::max(lds, raocp::dr_lds(nx, nu, C, L));
            if (k + 1 < T && npow(L) * 2 * nx > (long)raocp::kDrMaxGran * block) return 1e300;
        }
        if (lds > 160 * 1024 - 512) return 1e300;
        const int occ = raocp::dr_occupancy(nx, nu, C, lmax, lds);
        if (occ < 1 || wgs > (long)occ * n_cus) return 1e300;
        // fitted to the config-2 cut lists measured on MI355X (profiles/r04_*/dr_cuts.log): a
        // level 0.6 us plus 0.045 us per node beyond the first, each way; a tier boundary
        // 2.5 us (its two hand-offs)
        double cost = 2.5 * (T - 1);
        for (int k = 0; k < T; ++k)
            for (int l = 0; l < s[k + 1] - s[k]; ++l) cost += 2 * (0.6 + 0.045 * (double)(npow(l) - 1));
        return cost;
    };
    std::vector<int> cuts;
    if (const char* e = getenv("RAOCP_DR_CUTS")) {
        cuts.push_back(0);
        for (const char* p = e; *p;) {
            char* q = nullptr;
            const long v = strtol(p, &q, 10);
            if (q == p) break;
            if (v > 0 && v < N) cuts.push_back((int)v);
            p = *q ? q + 1 : q;
        }
        cuts.push_back(N);
        if (!std::is_sorted(cuts.begin(), cuts.end()) || eval(cuts) >= 1e299)
            return fail(RAOCP_ERR_ARG, std::string("RAOCP_DR_CUTS=") + e + ": not a valid tier plan for this tree");
    } else {
        double best = 1e300;
        std::vector<int> s{0};
        // every increasing cut list of at most kDrMaxTiers tiers
        auto rec = [&](auto&& self, int from) -> void {
            s.push_back(N);
            const double v = eval(s);
            if (v < best) {
                best = v;
                cuts = s;
            }
            s.pop_back();
            if ((int)s.size() >= raocp::kDrMaxTiers) return;
            for (int a = from; a < N; ++a) {
                s.push_back(a);
                self(self, a + 1);
                s.pop_back();
            }
        };
        rec(rec, 1);
        if (best >= 1e299) return RAOCP_OK;  // no plan: the sweep stays off
    }
    std::vector<double> bimg((size_t)N * nb, 0.0), fimg((size_t)N * nf, 0.0);
    for (int t = 0; t < N; ++t) {
        const raocp::Dy3Stage& st = c->reg_st[t];
        double* b = &bimg[(size_t)t * nb];
        auto bset = [&](int e, int lane, double v) { b[((size_t)(e / 2) * LB + lane) * 2 + (e & 1)] = v; };
        for (int r = 0; r < R; ++r)
            for (int k = 0; k < KS; ++k) {
                const int lane = r * KS + k;
                if (k < C)
                    for (int e = 0; e < nx; ++e) bset(e, lane, WT[((size_t)st.pair[k] * R + r) * SKP + e]);
                for (int e = 0; e < UP && k * UP + e < nu; ++e)
                    bset(nx + e, lane, RG[((size_t)st.cls * R + r) * SNU + k * UP + e]);
            }
        double* f = &fimg[(size_t)t * nf];
        auto fset = [&](int e, int lane, double v) { f[((size_t)(e / 2) * LF + lane) * 2 + (e & 1)] = v; };
        for (int k = 0; k < C; ++k)
            for (int r = 0; r < nx; ++r)
                for (int e = 0; e < nx + nu; ++e) fset(e, k * nx + r, F[((size_t)st.pair[k] * nx + r) * SKF + e]);
        for (int r = 0; r < nu; ++r) {
            for (int e = 0; e < nx; ++e) fset(e, C * nx + r, KM[((size_t)st.cls * nu + r) * SKP + e]);
            fset(nx + r, C * nx + r, 1.0);
        }
    }
    raocp::DrPlan& p = c->drp;
    memset(&p, 0, sizeof(p));
    const int T = (int)cuts.size() - 1;
    p.T = T;
    p.C = C;
    p.N = N;
    int w = 0, b0 = 0;
    for (int k = T - 1; k >= 0; --k) {  // the deepest tier first, the top last
        p.t[k].b0 = b0;
        b0 += (int)npow(cuts[k]);
    }
    c->dr_lds = 0;
    for (int k = 0; k < T; ++k) {
        raocp::DrTier& tt = p.t[k];
        tt.s0 = cuts[k];
        tt.L = cuts[k + 1] - cuts[k];
        tt.nsub = (int)npow(cuts[k]);
        tt.w0 = w;
        w += tt.nsub;
        c->dr_lds = std::max(c->dr_lds, raocp::dr_lds(nx, nu, C, tt.L));
    }
    p.nblk = b0;
    for (int t = 0; t <= N; ++t) p.sbase[t] = (int)((npow(t) - 1) / (C - 1));
    p.X0 = c->dev.X0;
    p.U0 = c->dev.U0;
    c->dr_block = block;
    // error-path test (tests/test_gpu_dynr.py): RAOCP_DR_FAULT=1 makes the deepest tier's first
    // subtree skip its publish, so its parent's wait times out and the call fails; the
    // timing-only bits (no DMA / arithmetic / write-out) exist in diagnostic builds only
    // (the timing bits pass where the sweep's unit is a diagnostic build: VAR_UNIT=dynr variants)
    if (const char* e = getenv("RAOCP_DR_FAULT")) p.fault = atoi(e) & ((raocp::kDiag || raocp::dr_diag_build()) ? ~0 : 1);
    int rc;
    const double *bi = nullptr, *fi = nullptr;
    unsigned long long *gq = nullptr, *gx = nullptr;
    unsigned* sy = nullptr;
    c->dr_gran = (size_t)w * 2 * nx;
    if ((rc = c->upload_vec(&bi, bimg)) || (rc = c->upload_vec(&fi, fimg)) || (rc = c->alloc(&gq, c->dr_gran)) ||
        (rc = c->alloc(&gx, c->dr_gran)) || (rc = c->alloc(&sy, 2)))
        return rc;
    HIPCHK(hipMemset(sy, 0, 2 * sizeof(unsigned)));
    HIPCHK(hipMemset(gq, 0, c->dr_gran * sizeof(unsigned long long)));
    HIPCHK(hipMemset(gx, 0, c->dr_gran * sizeof(unsigned long long)));
    p.bimg = bi;
    p.fimg = fi;
    p.gq = gq;
    p.gx = gx;
    p.sync = sy;
    long long ms = 1000;  // a wait normally lasts microseconds
    if (const char* e = getenv("RAOCP_FUSE_TIMEOUT_MS")) ms = std::max(1, atoi(e));
    p.timeout = ms * 100000LL;  // 100 MHz ticks
    c->dr = true;
    return RAOCP_OK;
}

// k_drc (raocp_dynr.hip): where k_dr and k_cp6 both run and every tier of the plan has 4 levels
// (binary trees, 20 / 8, fp64, every node boxed or none), the fused launch replaces the pair;
// RAOCP_DRC=0 keeps them. Its weight image is k_cp3's [sqrtQ | sqrtR | sqrtPf] followed by the
// one box table of each kind [lo_nl | hi_nl | lo_l | hi_l] (zeros when unboxed); its residual rows
// are two sets of one row per sweep wave (8 per workgroup, drc_part).
double* drc_part(raocp_ctx* c, int q);
int drc_nanbit(int q);
int drc_setup(raocp_ctx* c) {
    c->drc = false;
    if (!c->dr || !c->cp6 || c->f32 || c->sh_S > 0 || !raocp::drc_supported(c->nx, c->nu, c->reg_C)) return RAOCP_OK;
    if (const char* e = getenv("RAOCP_DRC"))
        if (!atoi(e)) return RAOCP_OK;
    const raocp::DrPlan& p = c->drp;
    for (int k = 0; k < p.T; ++k)
        if (p.t[k].L != 4) return RAOCP_OK;
    const int bx = c->box_mode;
    if (bx != 5 && bx != 10) return RAOCP_OK;
    const size_t lds = raocp::drc_lds(c->nx, c->nu, 2);
    int n_cus = 0, dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n_cus <= 0)
        n_cus = 256;
    const int occ = raocp::drc_occupancy(lds);
    if (occ < 1 || (long)p.nblk + 1 > (long)occ * n_cus) return RAOCP_OK;  // the grid must be resident
    const int nx = c->nx, nu = c->nu, R = nx + nu;
    const size_t nimg = raocp::kDrcWa + raocp::kDrcWb;
    double* img = nullptr;
    int rc;
    if ((rc = c->alloc(&img, nimg))) return rc;
    HIPCHK(hipMemset(img, 0, nimg * sizeof(double)));
    HIPCHK(hipMemcpy(img, c->cp3img, (size_t)(raocp::kDrcWa + 640) * sizeof(double), hipMemcpyDeviceToDevice));
    if ((bx & 3) == 1) {
        double* bx0 = img + raocp::kDrcWa + 640;
        HIPCHK(hipMemcpy(bx0, c->dev.blo_nl, R * sizeof(double), hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(bx0 + R, c->dev.bhi_nl, R * sizeof(double), hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(bx0 + 2 * R, c->dev.blo_l, nx * sizeof(double), hipMemcpyDeviceToDevice));
        HIPCHK(hipMemcpy(bx0 + 2 * R + nx, c->dev.bhi_l, nx * sizeof(double), hipMemcpyDeviceToDevice));
    }
    const int rows = 8 * p.nblk;
    if (2 * rows > c->red_rows) {
        c->red_rows = 2 * rows;
        if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return rc;
        HIPCHK(hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)));
    }
    c->cp_rows = rows;
    raocp::DrcArg& a = c->drca;
    const raocp::Dev& D = c->dev;
    a = raocp::DrcArg{};
    a.m = c->m;
    a.Y0 = D.Y0;
    a.T0 = D.T0;
    a.S0 = D.S0;
    a.E1 = D.E1; a.E2 = D.E2; a.E3 = D.E3; a.E4 = D.E4; a.E5 = D.E5; a.E6 = D.E6; a.E7 = D.E7;
    a.E11 = D.E11; a.E12 = D.E12; a.E13 = D.E13; a.E14 = D.E14;
    a.cond = D.cond;
    a.alpha_r = D.alpha_r;
    a.blo_nl = D.blo_nl; a.bhi_nl = D.bhi_nl; a.blo_l = D.blo_l; a.bhi_l = D.bhi_l;
    a.img = img;
    a.ctl = c->ctl;
    a.box = (bx & 3) == 1 ? 1 : 2;
    // the launch's arguments in device memory, one copy per iteration parity (part / nanbit)
    {
        raocp::DrcArg two[2] = {a, a};
        for (int q = 0; q < 2; ++q) {
            two[q].part = drc_part(c, q);
            two[q].nanbit = drc_nanbit(q);
        }
        double* d = nullptr;
        const size_t words = (2 * sizeof(raocp::DrcArg) + 7) / 8;
        if ((rc = c->alloc(&d, words))) return rc;
        HIPCHK(hipMemcpy(d, two, sizeof(two), hipMemcpyHostToDevice));
        c->d_drca = (raocp::DrcArg*)d;
    }
    c->drc_lds = lds;
    c->drc = true;
    return RAOCP_OK;
}

// role: 0 all blocks; 1 nonleaf blocks only; 2 leaf blocks only (op_bench timing)
struct CpPrimalOp {
    template <int NX, int NU>
    void run(raocp_ctx* c, bool full, int role) {
        const Launch a = groups(c->nx + c->nu + c->cmax + 1, c->m);
        const Launch l = groups(c->nx, c->n - c->m);
        int grid = a.blocks + l.blocks, blk0 = 0;
        if (role == 1) grid = a.blocks;
        if (role == 2) { grid = l.blocks; blk0 = a.blocks; }
        if (full)
            raocp::k_cp_primal<true, NX, NU><<<grid, kBlock, 0, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2,
                                                                              c->redpart, a.blocks, blk0);
        else
            raocp::k_cp_primal<false, NX, NU><<<grid, kBlock, 0, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2,
                                                                               c->redpart, a.blocks, blk0);
    }
};
void launch_cp_primal(raocp_ctx* c, bool full, int role = 0) { dispatch(c->nx, c->nu, CpPrimalOp{}, c, full, role); }

// role: 0 all blocks; 1 child; 2 nonleaf; 3 leaf blocks only (op_bench timing)
struct CpDualOp {
    template <int NX, int NU>
    void run(raocp_ctx* c, bool with_l, double* dsolo, int mode, int role) {
        const Launch a = groups(c->nx + c->nu + 2, c->n - 1);
        const Launch b = groups(2 * c->cmax + 2 + c->nx + c->nu, c->m);
        const Launch l = groups(2 * c->nx + 2, c->n - c->m);
        int grid = a.blocks + b.blocks + l.blocks, blk0 = 0;
        if (role == 1) grid = a.blocks;
        if (role == 2) { grid = b.blocks; blk0 = a.blocks; }
        if (role == 3) { grid = l.blocks; blk0 = a.blocks + b.blocks; }
        if (with_l)
            raocp::k_cp_dual<true, NX, NU><<<grid, kBlock, 0, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2,
                                                                            nullptr, c->redpart, a.blocks, b.blocks,
                                                                            raocp::kDualAll, blk0);
        else
            raocp::k_cp_dual<false, NX, NU><<<grid, kBlock, 0, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2,
                                                                             dsolo, c->redpart, a.blocks, b.blocks, mode,
                                                                             blk0);
    }
};
void launch_cp_dual(raocp_ctx* c, bool with_l, double* dsolo, int mode = raocp::kDualAll, int role = 0) {
    dispatch(c->nx, c->nu, CpDualOp{}, c, with_l, dsolo, mode, role);
}

// One CP iteration for iteration index `it` within a graph batch. Graph batches are a
// multiple of 6 iterations and always start at k = 0 mod 6, so the buffer rotation
// Z[k % 3], E[k % 2] is static per captured node: the kernels get the buffers already
// rotated and never read the iteration counter to choose them.
raocp::Bufs rotated(raocp_ctx* c, int it) {
    return raocp::Bufs{c->Z[it % 3], c->Z[(it + 1) % 3], c->Z[(it + 2) % 3], c->E[it % 2], c->E[(it + 1) % 2]};
}

template <class T>
struct Cpd2Op {
    template <int RX, int RU>
    void run(raocp_ctx* c) {
        auto k = raocp::k_cpd2<T, RX, RU>;
        allow_lds(k, c->lds_cpd2);
        k<<<c->cp2_nbF + c->cp2_nbL, 64 * c->cp2_W, c->lds_cpd2, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2,
                                                                                c->redpart, c->cp2_nbF);
    }
};
template <class T>
struct Cpp2Op {
    template <int RX, int RU>
    void run(raocp_ctx* c) {
        auto k = raocp::k_cpp2<T, RX, RU>;
        allow_lds(k, c->lds_cpp2);
        k<<<c->cp2_nbF + c->cp2_nbL, 64 * c->cp2_W, c->lds_cpp2, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2,
                                                                                c->redpart, c->cp2_nbF);
    }
};
// the node-block kernels (raocp_cp.hip): fp64 at every size; fp32 contexts whose CP blocks
// mix weight tables (per-mode costs) at runtime sizes
template <class T>
struct CpdOp {
    template <int NX, int NU>
    void run(raocp_ctx* c) {
        auto k = raocp::k_cpd<T, NX, NU>;
        allow_lds(k, c->lds_cpd);
        k<<<c->cp_nbF + c->cp_nbL, kBlock, c->lds_cpd, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2, c->redpart,
                                                                     c->cp_nbF);
    }
};
template <class T>
struct CppOp {
    template <int NX, int NU>
    void run(raocp_ctx* c) {
        auto k = raocp::k_cpp<T, NX, NU>;
        allow_lds(k, c->lds_cpp);
        k<<<c->cp_nbF + c->cp_nbL, kBlock, c->lds_cpp, c->stream>>>(c->dev, c->ctl, c->bufs, c->XI2, c->redpart,
                                                                     c->cp_nbF);
    }
};
void launch_cpd(raocp_ctx* c) {
    if (c->f32 && c->cp_v1) CpdOp<float>{}.run<0, 0>(c);
    else if (c->f32) dispatch_rt(c->nx, c->nu, Cpd2Op<float>{}, c);
    else if (c->cp_v1) dispatch(c->nx, c->nu, CpdOp<double>{}, c);
    else dispatch_rt(c->nx, c->nu, Cpd2Op<double>{}, c);
}
void launch_cpp(raocp_ctx* c) {
    if (c->f32 && c->cp_v1) CppOp<float>{}.run<0, 0>(c);
    else if (c->f32) dispatch_rt(c->nx, c->nu, Cpp2Op<float>{}, c);
    else if (c->cp_v1) dispatch(c->nx, c->nu, CppOp<double>{}, c);
    else dispatch_rt(c->nx, c->nu, Cpp2Op<double>{}, c);
}
// the fused CP iteration (raocp_cp3.hip): compile-time sizes of the benchmark configs
// instantiated for the fp64 sizes of configs 2 and 4 and the fp32 sizes of configs 2, 4, 5
bool cp3_sizes(bool f32, int nx, int nu) {
    return (nx == 20 && nu == 8) || (nx == 32 && nu == 12) || (f32 && nx == 64 && nu == 16);
}
// a k_cp3 task list: split leaf tiles [l0, l1), then the parent ranges in order; returns
// the tiles, or -1 when the nonempty ranges exceed the kernel argument's kCp3MaxR slots (the
// caller must not launch it: a dropped range would leave its parents uncomputed)
long cp3_tasks(raocp::Cp3Tasks& tk, const std::vector<std::pair<int, int>>& ranges, int l0, int l1, int split,
               int mL, int gran = 16) {
    tk = raocp::Cp3Tasks{};
    tk.l0 = l0;
    tk.l1 = std::max(l0, l1);
    tk.split = split;
    tk.mL = mL;
    long tiles = (tk.l1 - tk.l0 + 15) / 16;
    for (const auto& r : ranges) {
        if (r.second <= r.first) continue;
        if (tk.nr >= raocp::kCp3MaxR) return -1;
        tk.lo[tk.nr] = r.first;
        tk.hi[tk.nr] = r.second;
        tk.t0[tk.nr + 1] = tk.t0[tk.nr] + (r.second - r.first + gran - 1) / gran;
        ++tk.nr;
    }
    if (tk.nr == 0) {  // an empty launch still needs one range (no tiles)
        tk.nr = 1;
        tk.t0[1] = 0;
    }
    return tiles + tk.t0[tk.nr];
}
int cp3_grid_of(long tiles) { return (int)std::max(1L, std::min((tiles + 3) / 4, 2048L)); }
// part 0: the unsharded launch, or a shard's first; 1: a shard's second (after X1), whose
// residual partials follow the first launch's rows
template <bool SH>
void launch_cp3t(raocp_ctx* c, int g, double* rp, const raocp::Cp3Tasks& tk) {
    const int C = c->unif_C, bx = c->box_mode;
    const double* im = c->cp3img;
    if (c->f32) {
        if (c->nx == 20) raocp::k_cp3<float, 20, 8, SH><<<g, 256, 0, c->stream>>>(c->dev, c->ctl, c->bufs, rp, c->XI2, C, bx, tk, im);
        else if (c->nx == 32) raocp::k_cp3<float, 32, 12, SH><<<g, 256, 0, c->stream>>>(c->dev, c->ctl, c->bufs, rp, c->XI2, C, bx, tk, im);
        else raocp::k_cp3<float, 64, 16, SH><<<g, 256, 0, c->stream>>>(c->dev, c->ctl, c->bufs, rp, c->XI2, C, bx, tk, im);
    } else {
        if (c->nx == 20) raocp::k_cp3<double, 20, 8, SH><<<g, 256, 0, c->stream>>>(c->dev, c->ctl, c->bufs, rp, c->XI2, C, bx, tk, im);
        else raocp::k_cp3<double, 32, 12, SH><<<g, 256, 0, c->stream>>>(c->dev, c->ctl, c->bufs, rp, c->XI2, C, bx, tk, im);
    }
}
// k_cp3's weight image (one workgroup, at context creation)
template <class T, int NX, int NU>
int cp3_imaget(raocp_ctx* c) {
    typedef raocp::WL<T, NX, NX> WQ;
    typedef raocp::WL<T, NU, NU> WR;
    int rc;
    if ((rc = c->alloc(&c->cp3img, (size_t)(2 * WQ::N + WR::N) * sizeof(T) / 8))) return rc;
    raocp::k_cp3_image<T, NX, NU><<<1, 256, 0, c->stream>>>(c->dev, c->cp3img);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}
int cp3_image(raocp_ctx* c) {
    if (c->f32) {
        if (c->nx == 20) return cp3_imaget<float, 20, 8>(c);
        if (c->nx == 32) return cp3_imaget<float, 32, 12>(c);
        return cp3_imaget<float, 64, 16>(c);
    }
    if (c->nx == 20) return cp3_imaget<double, 20, 8>(c);
    return cp3_imaget<double, 32, 12>(c);
}
void launch_cp3(raocp_ctx* c, int part = 0) {
    if (c->cp6 && c->sh_S == 0) {
        raocp::cp6_launch(c->dev, c->ctl, c->bufs, c->redpart, c->box_mode, c->cp5_tk, c->cp6_grid, c->cp3img, c->stream);
        return;
    }
    if (c->cp5) {
        // a shard: its eta2 tasks, leaves and families, then (part 1, after X1) the cut's parents
        const bool sh = c->sh_S > 0;
        if (part == 0)
            raocp::cp5_launch(c->dev, c->ctl, c->bufs, c->redpart, c->unif_C, c->box_mode, c->cp5_et,
                              sh ? c->own_lo[c->N] : c->m, sh ? c->own_hi[c->N] : c->n, c->cp5_gl, c->cp5_tk, c->cp5_gf,
                              c->cp3img, c->cp5_lpf, c->stream);
        else
            raocp::cp5_launch(c->dev, c->ctl, c->bufs, c->redpart + (size_t)raocp::cp5_rows(c->cp5_gl, c->cp5_gf) * 6,
                              c->unif_C, c->box_mode, c->cp5_et, 0, 0, 0, c->cp5_tkb, c->cp5_gfb, c->cp3img, c->cp5_lpf,
                              c->stream);
        return;
    }
    if (c->cp4 && c->sh_S == 0) {
        raocp::cp4_launch(c->dev, c->ctl, c->bufs, c->redpart, c->unif_C, c->box_mode, c->cp3_ta, c->cp3img, c->cp3_grid,
                          c->cp4_wpb, c->stream);
        return;
    }
    if (c->sh_S > 0)
        launch_cp3t<true>(c, part ? c->cp3_gridb : c->cp3_grid, c->redpart + (part ? (size_t)c->cp3_grid * 6 : 0),
                          part ? c->cp3_tb : c->cp3_ta);
    else
        launch_cp3t<false>(c, c->cp3_grid, c->redpart, c->cp3_ta);
}
// the solve's first half step Z[1] = prox-part(Z[0] - alpha L^T E[0]) (s_0 relaxation,
// kernel projection): k_cp_primal; an fp32 context runs k_cpp2 on {p = z+ = Z[0], d = eta+ =
// E[0]} (its residual partials are overwritten by iteration 0 before they are read)
void launch_first_half(raocp_ctx* c) {
    if (!c->f32) {
        launch_cp_primal(c, false);
        return;
    }
    const raocp::Bufs keep = c->bufs;
    c->bufs = raocp::Bufs{c->Z[0], c->Z[0], c->Z[1], c->E[0], c->E[0]};
    launch_cpp(c);
    c->bufs = keep;
}
// Deferred stopping test (default for the tiered dynamics; RAOCP_DEFER_CHECK=0 disables):
// iteration k's test runs in an extra workgroup of iteration k + 1's first dynamics launch
// instead of its own k_cp_check launch after k_cpp, and a batch ends with one k_cp_check
// for its last iteration. Iteration k + 1's kernels that start before the test fires only
// write the next iterate's buffers (Z[(k + 1) % 3] projected in place, nothing of
// z+_k = Z[k % 3] or eta+_k = E[k % 2]), and every later kernel exits on ctl->done, so the
// result and the history are those of the eager test.
bool defer_check(const raocp_ctx* c) {
    if (c->dr && c->sh_S == 0) return !(c->comm || c->sh_R != 1 || c->no_defer_check);
    if (c->dyn3 && c->sh_S == 0) return !(c->comm || c->sh_R != 1 || c->no_defer_check || c->N < 1);
    if (c->comm || c->sh_R != 1 || c->dyn2 || c->cut <= 0 || c->tiers.empty() || c->no_defer_check)
        return false;
    return c->tiers.back().nsub > 0;
}

// ---- RCCL, loaded on demand (dlopen) so single-GPU users never load it
struct Rccl {
    void* h = nullptr;
    ncclResult_t (*get_id)(ncclUniqueId*) = nullptr;
    ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*destroy)(ncclComm_t) = nullptr;
    const char* (*err)(ncclResult_t) = nullptr;
};
Rccl g_rccl;
int rccl_load() {
    if (g_rccl.h) return RAOCP_OK;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) return fail(RAOCP_ERR_HIP, std::string("cannot load librccl: ") + dlerror());
    g_rccl.get_id = (decltype(g_rccl.get_id))dlsym(h, "ncclGetUniqueId");
    g_rccl.init_rank = (decltype(g_rccl.init_rank))dlsym(h, "ncclCommInitRank");
    g_rccl.all_gather = (decltype(g_rccl.all_gather))dlsym(h, "ncclAllGather");
    g_rccl.all_reduce = (decltype(g_rccl.all_reduce))dlsym(h, "ncclAllReduce");
    g_rccl.destroy = (decltype(g_rccl.destroy))dlsym(h, "ncclCommDestroy");
    g_rccl.err = (decltype(g_rccl.err))dlsym(h, "ncclGetErrorString");
    if (!g_rccl.get_id || !g_rccl.init_rank || !g_rccl.all_gather || !g_rccl.all_reduce || !g_rccl.destroy)
        return fail(RAOCP_ERR_HIP, "librccl lacks the collectives used here");
    g_rccl.h = h;
    return RAOCP_OK;
}

// The two exchanges of a sharded iteration:
//   X2  after the tiers' backward sweeps: q rows of the boundary roots (all-gather);
//   X1  after k_cpd: eta+ and xi2 of the roots' eta2 (all-gather), read by the
//       replicated top families of k_cpp, carrying the previous iteration's 16-double
//       residual record too (k_cp_reduce after k_cpp packs it; the stopping test runs one
//       iteration late, k_cp_check_gather), so SURVEY.md's X3 all-reduce is not needed.
// pack/unpack run on every shard; the collective itself is RCCL, or, for shards that
// share a process (raocp_group_cp_run), host-driven copies between the phases.
// X2 rows: the tiered sweep's q rows (KP doubles each), or the per-stage sweep's (nx scalars
// of the context's type, raocp_dyn3.hip)
int x2_row(const raocp_ctx* c) { return c->dyn3 ? c->nx : c->KP; }
int x2_elt(const raocp_ctx* c) { return c->dyn3 ? c->wsz : 8; }
double* x2_q(const raocp_ctx* c) { return c->dyn3 ? c->Q2 : c->q; }
size_t x2_bytes(const raocp_ctx* c) { return (size_t)c->x_max * x2_row(c) * x2_elt(c); }
void shard_pack_x2(raocp_ctx* c) {
    const size_t row = (size_t)x2_row(c) * x2_elt(c);
    if (c->own_cnt)
        (void)hipMemcpyAsync(c->x2_send, (char*)x2_q(c) + (size_t)c->own_first * row, (size_t)c->own_cnt * row,
                             hipMemcpyDeviceToDevice, c->stream);
}
void shard_unpack_x2(raocp_ctx* c) {
    const int tot = c->sh_R * c->x_max * x2_row(c);
    const int g = std::max(1, std::min(256, cdiv(tot, kBlock)));
    if (x2_elt(c) == 4)
        raocp::k_scatter_rows<float><<<g, kBlock, 0, c->stream>>>((const float*)c->x2_recv, (float*)x2_q(c), c->d_slc,
                                                                   c->sh_R, c->x_max, x2_row(c));
    else
        raocp::k_scatter_rows<double><<<g, kBlock, 0, c->stream>>>(c->x2_recv, x2_q(c), c->d_slc, c->sh_R, c->x_max,
                                                                    x2_row(c));
}
// X1 carries two entries per root and the previous iteration's residual record: under k_cp3
// the roots' (eta+, xi2) eta2 entries, under k_cp5 the roots' s of the half step before their
// parents' kernel projection (k_cp5_leaf's eta2 tasks write it, the cut's parents' family tiles
// read it) and eta+ of their eta2
int x1_len(const raocp_ctx* c) { return 2 * c->x_max + 16; }
struct X1Src {
    double *a, *b;  // buffers (of the context's type) and element offsets of root 0's entries
    int oa, ob;
};
X1Src x1_src(const raocp_ctx* c) {
    if (c->cp5) return X1Src{c->bufs.z2, c->bufs.e1, c->dev.S0, c->dev.E2};
    return X1Src{c->bufs.e1, c->XI2, c->dev.E2, c->dev.E2};
}
void shard_pack_x1(raocp_ctx* c) {
    const int g = std::max(1, cdiv(c->own_cnt, kBlock)), o = c->own_first;
    const X1Src x = x1_src(c);
    if (c->f32)
        raocp::k_pack_x1<float><<<g, kBlock, 0, c->stream>>>(c->x1_send, (const float*)x.a + x.oa + o,
                                                             (const float*)x.b + x.ob + o, c->own_cnt, c->x_max, c->red8);
    else
        raocp::k_pack_x1<double><<<g, kBlock, 0, c->stream>>>(c->x1_send, x.a + x.oa + o, x.b + x.ob + o, c->own_cnt,
                                                              c->x_max, c->red8);
}
void shard_unpack_x1(raocp_ctx* c) {
    const int g = std::max(1, cdiv(c->sh_R * c->x_max, kBlock));
    const X1Src x = x1_src(c);
    if (c->f32)
        raocp::k_unpack_x1<float><<<g, kBlock, 0, c->stream>>>(c->x1_recv, (float*)x.a + x.oa, (float*)x.b + x.ob, c->d_slc,
                                                               c->sh_R, c->x_max);
    else
        raocp::k_unpack_x1<double><<<g, kBlock, 0, c->stream>>>(c->x1_recv, x.a + x.oa, x.b + x.ob, c->d_slc, c->sh_R,
                                                                c->x_max);
    raocp::k_cp_check_gather<<<1, 64, 0, c->stream>>>(c->ctl, c->hist, c->x1_recv, c->sh_R, c->x_max);
}
int rccl_check(ncclResult_t r, const char* what) {
    if (r != ncclSuccess)
        return fail(RAOCP_ERR_HIP, std::string(what) + ": " + (g_rccl.err ? g_rccl.err(r) : "rccl error"));
    return RAOCP_OK;
}

// one CP iteration of a shard whose transport is RCCL (graph-capturable)
int enqueue_shard_iteration(raocp_ctx* c) {
    ncclComm_t comm = (ncclComm_t)c->comm;
    int rc;
    launch_dynamics(c, c->bufs, 1, c->ctl, 1);
    shard_pack_x2(c);
    if ((rc = rccl_check(g_rccl.all_gather(c->x2_send, c->x2_recv, (size_t)c->x_max * x2_row(c),
                                           x2_elt(c) == 4 ? ncclFloat32 : ncclFloat64, comm, c->stream),
                         "ncclAllGather(q)")))
        return rc;
    shard_unpack_x2(c);
    launch_dynamics(c, c->bufs, 1, c->ctl, 2);
    if (c->cp3) launch_cp3(c, 0);
    else launch_cpd(c);
    shard_pack_x1(c);
    if ((rc = rccl_check(g_rccl.all_gather(c->x1_send, c->x1_recv, (size_t)x1_len(c), ncclFloat64, comm, c->stream),
                         "ncclAllGather(eta2, residuals)")))
        return rc;
    shard_unpack_x1(c);  // + the previous iteration's stopping test
    if (c->cp3) launch_cp3(c, 1);
    else launch_cpp(c);
    raocp::k_cp_reduce<<<1, kBlock, 0, c->stream>>>(c->ctl, c->redpart, c->cp_rows, c->red8);
    return RAOCP_OK;
}

// the last iteration's stopping test (its record has no next iteration to ride on): the
// X1 all-gather with only the residual record meaningful
int enqueue_shard_tail(raocp_ctx* c) {
    shard_pack_x1(c);
    int rc;
    if ((rc = rccl_check(g_rccl.all_gather(c->x1_send, c->x1_recv, (size_t)x1_len(c), ncclFloat64, (ncclComm_t)c->comm,
                                           c->stream),
                         "ncclAllGather(residuals)")))
        return rc;
    raocp::k_cp_check_gather<<<1, 64, 0, c->stream>>>(c->ctl, c->hist, c->x1_recv, c->sh_R, c->x_max);
    return RAOCP_OK;
}

// returns the first failure of an RCCL call (launch errors surface at the next sync)
// k_drc's residual rows of iteration parity q, and the ctl->flags bit of its NaN-in-box flag
double* drc_part(raocp_ctx* c, int q) { return c->redpart + (size_t)(q & 1) * c->cp_rows * 6; }
int drc_nanbit(int q) { return 2 << (q & 1); }
// the fused launch of iteration `it` (k = it mod 2 within a batch that starts at k = 0 mod 6)
void launch_drc(raocp_ctx* c, int it, bool with_check) {
    raocp::DrPlan p = c->drp;
    if (c->dev.stamps) p.stamps = c->dev.stamps;
    const raocp::ChkArg ck{c->ctl, c->hist, drc_part(c, it - 1), c->cp_rows, with_check ? 1 : 0, drc_nanbit(it - 1)};
    raocp::drc_launch(p, c->d_drca + (it & 1), c->drca.box, c->drc_lds, c->bufs, ck, c->stream);
}
int enqueue_cp_iteration(raocp_ctx* c, int it) {
    const raocp::Bufs keep = c->bufs;
    c->bufs = rotated(c, it);
    if (c->comm) {
        const int rc = enqueue_shard_iteration(c);
        c->bufs = keep;
        return rc;
    }
    const bool defer = defer_check(c);
    if (c->drc && c->sh_S == 0) {
        launch_drc(c, it, defer && it > 0);
        c->bufs = keep;
        if (!defer)
            raocp::k_cp_check<<<1, kBlock, 0, c->stream>>>(c->ctl, c->hist, drc_part(c, it), c->cp_rows, drc_nanbit(it), nullptr, nullptr);
        return RAOCP_OK;
    }
    const raocp::ChkArg ck{c->ctl, c->hist, c->redpart, c->cp_rows, 1};
    launch_dynamics(c, c->bufs, 1, c->ctl, 0, defer && it > 0 ? &ck : nullptr);
    if (c->cp3) {
        launch_cp3(c);
    } else {
        launch_cpd(c);
        launch_cpp(c);
    }
    c->bufs = keep;
    if (!defer) raocp::k_cp_check<<<1, kBlock, 0, c->stream>>>(c->ctl, c->hist, c->redpart, c->cp_rows, 0, nullptr, nullptr);
    return RAOCP_OK;
}
// the kernel the default selection launches for op (raocp_op_bench numbering: 0 L, 1 L^T,
// 2 dual CP kernel, 6 primal CP kernel, 9 the dynamics projection), as rocprofv3 names it
std::string kernel_name(const raocp_ctx* c, int op) {
    const std::string T = c->f32 ? "float" : "double";
    const bool exact = (c->nx == 20 && c->nu == 8) || (c->nx == 32 && c->nu == 12) || (c->nx == 64 && c->nu == 16) ||
                       (c->nx == 3 && c->nu == 2);
    const std::string nn = exact ? std::to_string(c->nx) + ", " + std::to_string(c->nu) : "0, 0";
    const int rx = std::min(4, (c->nx + 15) / 16), ru = c->nu <= 16 ? 1 : 2;
    const std::string rr = std::to_string(rx) + ", " + std::to_string(ru);
    const bool big = (c->nx == 20 && c->nu == 8) || (c->nx == 32 && c->nu == 12) || (c->nx == 64 && c->nu == 16);
    switch (op) {
        case 0:
            if (c->ell3 && big) return "k_ell3<" + T + ", " + nn + ">";
            return c->f32 ? "k_ell2<float, " + rr + ">" : "k_ell<" + nn + ">";
        case 1:
            if (c->ellt3_C && big) return "k_ellt3<" + T + ", " + nn + ", " + std::to_string(4 / c->ellt3_C) + ">";
            return c->f32 ? "k_ellt2<float, " + rr + ">" : "k_ell_t<" + nn + ">";
        case 2:
            if (c->cp_v1) return "k_cpd<" + T + ", " + (c->f32 ? std::string("0, 0") : nn) + ">";
            return "k_cpd2<" + T + ", " + rr + ">";
        case 6:
            if (c->cp_v1) return "k_cpp<" + T + ", " + (c->f32 ? std::string("0, 0") : nn) + ">";
            return "k_cpp2<" + T + ", " + rr + ">";
        case 9: {
            // the launches of one projection as "name xcount" terms (bench.py sums the PMC
            // traffic of these terms)
            std::vector<std::pair<std::string, int>> terms;
            auto add = [&](const std::string& k) {
                for (auto& t : terms)
                    if (t.first == k) {
                        ++t.second;
                        return;
                    }
                terms.push_back({k, 1});
            };
            auto b = [](bool v) { return std::string(v ? "true" : "false"); };
            if (c->dr && c->sh_S == 0) {
                return std::string(raocp::dr_name(c->nx, c->nu)) + " x1";
            } else if (c->dyn3) {  // a backward and a forward launch per nonleaf stage below the top
                const int ts = dyn3_top_stages(c);
                for (int t = ts; t < c->N; ++t) add("k_dy3_back<" + T + ", " + nn + ">");
                if (ts) add("k_dy3_top_back<" + T + ", " + nn + ">");
                if (ts) add("k_dy3_top_fwd<" + T + ", " + nn + ">");
                for (int t = ts; t < c->N; ++t) add("k_dy3_fwd<" + T + ", " + nn + ">");
            } else if (c->dyn2) {
                return "k_d2_prod + k_d2_node + k_d2_x0 + k_d2_fwd (per stage, " + T + ")";
            } else if (c->cut > 0 && c->dyn_split && c->sh_S == 0) {
                return "k_dyn_up<" + nn + "> x1 + k_dyn_down<" + nn + ", " + b(c->f_lds_top) + "> x1";
            } else if (c->cut > 0) {
                for (int k = (int)c->tiers.size() - 1; k >= 0; --k)
                    add("k_dyn_bottom_back<" + nn + ", " + b(c->tiers[k].fold) + ">");
                add("k_dyn_top<" + nn + ", " + b(c->f_lds_top) + ", " + b(c->fold_top) + ">");
                for (const auto& tp : c->tiers) add("k_dyn_bottom_fwd<" + nn + ", " + std::to_string(tp.fm) + ">");
            } else {
                return "k_dyn_gather + k_dyn_stage_a / _b / _f (per stage)";
            }
            std::string s;
            for (const auto& t : terms) s += (s.empty() ? "" : " + ") + t.first + " x" + std::to_string(t.second);
            return s;
        }
        case 11:  // the CP loop's fused launch (dynamics projection + CP iteration), if any
            return c->drc && c->sh_S == 0 ? raocp::drc_name() : "";
        case 12:  // the forms of the k_cp5 launches, when they run ("" otherwise)
            if (!c->cp5) return "";
            return std::string("leaf_pf=") + (c->cp5_lpf ? "1" : "0");
        case 10:
            if (c->cp6 && c->sh_S == 0) return raocp::cp6_name();
            if (c->cp5) return std::string(raocp::cp5_name(c->f32, c->nx)) + (c->sh_S > 0 ? " (+ fams x1 after X1)" : "");
            if (c->cp4 && c->sh_S == 0) return raocp::cp4_name(c->f32, c->nx, c->nu);
            if (c->cp3) return "k_cp3<" + T + ", " + nn + (c->sh_S > 0 ? ", true> x2" : ", false>");
            return kernel_name(c, 2) + " + " + kernel_name(c, 6);
        default: return "";
    }
}

// the end of a batch of `iters` iterations: the deferred test of its last iteration
void enqueue_batch_tail(raocp_ctx* c, int iters) {
    if (!defer_check(c)) return;
    if (c->drc && c->sh_S == 0)
        raocp::k_cp_check<<<1, kBlock, 0, c->stream>>>(c->ctl, c->hist, drc_part(c, iters - 1), c->cp_rows,
                                                       drc_nanbit(iters - 1), c->d_pub, err_word(c));
    else
        raocp::k_cp_check<<<1, kBlock, 0, c->stream>>>(c->ctl, c->hist, c->redpart, c->cp_rows, 0, c->d_pub, err_word(c));
}


int set_ctl_alpha(raocp_ctx* c, double alpha) {
    HIPCHK(hipMemcpyAsync(&c->ctl->alpha, &alpha, sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

void drop_graphs(raocp_ctx* c) {
    if (c->graph) (void)hipGraphExecDestroy(c->graph);
    if (c->graph_rem) (void)hipGraphExecDestroy(c->graph_rem);
    c->graph = c->graph_rem = nullptr;
    c->graph_iters = c->graph_rem_iters = 0;
}

int ensure_hist(raocp_ctx* c, size_t rows) {
    if (rows <= c->hist_rows) return RAOCP_OK;
    if (c->hist) {
        (void)hipFree(c->hist);
        c->allocs.erase(std::remove(c->allocs.begin(), c->allocs.end(), (void*)c->hist), c->allocs.end());
        c->hist = nullptr;
    }
    int rc = c->alloc(&c->hist, rows * 6);
    if (rc) return rc;
    c->hist_rows = rows;
    drop_graphs(c);  // the graphs reference the history buffer
    return RAOCP_OK;
}

// Prepare a CP run: the starting primal / dual go to Z[0] / E[0] and ctl is reset.
// warm: start from the context's current primal / dual (the reference's chock continues
// from the cached old primal / dual, solver.py:27-61 with cache.py:58-66, 186-196), with
// x0 written into node 0's state (cache_initial_state, cache.py:79-82); otherwise from
// (x0 at node 0, zeros) / 0.
int cp_init(raocp_ctx* c, const double* x0, int max_iters, double tol, double alpha, bool warm = false) {
    if (warm) {
        if (c->cur_z != c->Z[0])
            HIPCHK(hipMemcpyAsync(c->Z[0], c->cur_z, c->P * c->wsz, hipMemcpyDeviceToDevice, c->stream));
        if (c->cur_e != c->E[0])
            HIPCHK(hipMemcpyAsync(c->E[0], c->cur_e, c->D * c->wsz, hipMemcpyDeviceToDevice, c->stream));
    } else {
        HIPCHK(hipMemsetAsync(c->Z[0], 0, c->P * sizeof(double), c->stream));
        HIPCHK(hipMemsetAsync(c->E[0], 0, c->D * sizeof(double), c->stream));
    }
    if (c->red8) HIPCHK(hipMemsetAsync(c->red8, 0, 16 * sizeof(double), c->stream));  // no previous record
    for (int b = 1; b < 3; ++b) HIPCHK(hipMemsetAsync(c->Z[b], 0, c->P * sizeof(double), c->stream));
    HIPCHK(hipMemsetAsync(c->E[1], 0, c->D * sizeof(double), c->stream));
    HIPCHK(hipMemsetAsync(c->XI2, 0, c->D * sizeof(double), c->stream));
    if (c->f32) {
        const std::vector<float> f(x0, x0 + c->nx);
        HIPCHK(hipMemcpyAsync((float*)c->Z[0] + c->dev.X0, f.data(), c->nx * sizeof(float), hipMemcpyHostToDevice,
                              c->stream));
        HIPCHK(hipMemcpyAsync(c->x0, f.data(), c->nx * sizeof(float), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipStreamSynchronize(c->stream));  // f leaves scope
    } else {
        HIPCHK(hipMemcpyAsync(c->Z[0] + c->dev.X0, x0, c->nx * sizeof(double), hipMemcpyHostToDevice, c->stream));
        HIPCHK(hipMemcpyAsync(c->x0, x0, c->nx * sizeof(double), hipMemcpyHostToDevice, c->stream));
    }
    Ctl h{};
    h.alpha = alpha;
    h.k = 0;
    h.done = 0;
    h.final_k = -1;
    h.flags = 0;
    h.max_iters = max_iters;
    h.tol = tol;
    *c->h_ctl = h;
    HIPCHK(hipMemcpyAsync(c->ctl, c->h_ctl, sizeof(Ctl), hipMemcpyHostToDevice, c->stream));
    launch_first_half(c);
    return RAOCP_OK;
}

// the captured batch of `iters` CP iterations: kGraphBatch in the main slot, any other
// count (a benchmark's remainder, always launched after whole batches, so it also starts
// at k = 0 mod 6) in the remainder slot
int ensure_graph(raocp_ctx* c, int iters) {
    if (c->eager) return RAOCP_OK;
    const bool rem = iters != kGraphBatch;
    hipGraphExec_t& slot = rem ? c->graph_rem : c->graph;
    int& slot_iters = rem ? c->graph_rem_iters : c->graph_iters;
    if (slot && slot_iters == iters) return RAOCP_OK;
    if (slot) {
        (void)hipGraphExecDestroy(slot);
        slot = nullptr;
    }
    hipGraph_t g = nullptr;
    HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
    int rc_enq = RAOCP_OK;
    for (int it = 0; it < iters && rc_enq == RAOCP_OK; ++it) rc_enq = enqueue_cp_iteration(c, it);
    if (rc_enq == RAOCP_OK) enqueue_batch_tail(c, iters);
    hipError_t e = hipStreamEndCapture(c->stream, &g);
    if (rc_enq != RAOCP_OK) {
        if (g) (void)hipGraphDestroy(g);
        (void)hipGetLastError();
        if (!c->comm) return rc_enq;
        // an RCCL shard whose collectives cannot be captured: launch iterations eagerly
        c->eager = true;
        return RAOCP_OK;
    }
    if (e == hipSuccess) {
        e = hipGraphInstantiate(&slot, g, nullptr, nullptr, 0);
        (void)hipGraphDestroy(g);
        // the executable graph's device-side setup now, not inside its first (timed) launch
        if (e == hipSuccess) e = hipGraphUpload(slot, c->stream);
    }
    if (e != hipSuccess) {
        if (!c->comm) return fail(RAOCP_ERR_HIP, std::string("graph capture: ") + hipGetErrorString(e));
        // an RCCL shard whose collectives cannot be captured: launch iterations eagerly
        (void)hipGetLastError();
        slot = nullptr;
        c->eager = true;
        return RAOCP_OK;
    }
    slot_iters = iters;
    return RAOCP_OK;
}

// launch one batch of `iters` CP iterations (the captured graph, or eagerly)
int launch_batch(raocp_ctx* c, int iters) {
    if (c->eager) {
        for (int it = 0; it < iters; ++it) {
            const int rc = enqueue_cp_iteration(c, it);
            if (rc) return rc;
        }
        enqueue_batch_tail(c, iters);
        HIPCHK(hipGetLastError());
        return RAOCP_OK;
    }
    HIPCHK(hipGraphLaunch(iters == kGraphBatch ? c->graph : c->graph_rem, c->stream));
    return RAOCP_OK;
}


// ---- node-block CP tables (raocp_cp.hip) for given owned parent / leaf id ranges ----
struct CpFam { int cb, ce, y0, y1, e7a, e7b; };
CpFam cp_fam(const raocp_ctx* c, int i0, int i1) {
    CpFam f;
    f.cb = c->h_chs[i0];
    f.ce = c->h_chs[i1 - 1] + c->h_nch[i1 - 1];
    f.y0 = c->h_yrel[i0];
    f.y1 = c->h_yrel[i1 - 1] + 2 * c->h_nch[i1 - 1] + 1;
    f.e7a = c->h_pos7[i0];
    f.e7b = c->h_pos7[i1];
    return f;
}

// LDS doubles of one block (k_cpd, k_cpp), mirroring the Stg regions of raocp_cp.hip
std::pair<long, long> cp_block_need(const raocp_ctx* c, bool family, int a0, int a1) {
    const long nx = c->nx, nu = c->nu;
    auto dbl = [](long cnt) { return (cnt + 1) / 2 * 2 + 2; };
    auto recs = [](long cnt) { return 2 * cnt + 2; };
    auto ints = [](long cnt) { return (cnt * 4 + 22) / 8 / 2 * 2 + 4; };
    const long nQ = (long)c->n_sq * nx * nx, nR = (long)c->n_sr * nu * nu, nP = (long)c->n_sp * nx * nx;
    const long nBx = (long)c->nbn * (nx + nu), nBlx = (long)c->nbl * nx;
    if (family) {
        const long P = a1 - a0;
        const CpFam f = cp_fam(c, a0, a1);
        const long C = f.ce - f.cb, Y = f.y1 - f.y0, E7n = f.e7b - f.e7a;
        const long nd = 2 * dbl(P * nx) + 2 * dbl(P * nu) + 2 * dbl(Y) + 2 * dbl(P) + 2 * dbl(C) + dbl(C) + dbl(Y) +
                        dbl(P) + dbl(E7n) + dbl(C * nx) + dbl(C * nu) + 2 * dbl(C) + recs(P) + recs(C) + ints(P) +
                        dbl(nQ) + dbl(nR) + 2 * dbl(nBx);
        const long npp = 3 * (dbl(Y) + dbl(P) + dbl(C * nx) + dbl(C * nu) + 2 * dbl(C) + dbl(E7n) + 3 * dbl(C)) +
                         2 * dbl(P * nx) + 2 * dbl(P * nu) + 2 * dbl(Y) + 2 * dbl(C) + 2 * dbl(C) + dbl(C) + dbl(P) +
                         recs(P) + recs(C) + dbl(nQ) + dbl(nR);
        return {nd, npp};
    }
    const long Lc = a1 - a0;
    const long E14n = c->h_pos14[a1 - c->m] - c->h_pos14[a0 - c->m];
    const long nd = 2 * dbl(Lc * nx) + 2 * dbl(Lc) + dbl(Lc * nx) + 2 * dbl(Lc) + dbl(E14n) + recs(Lc) + dbl(nP) +
                    2 * dbl(nBlx);
    const long npp = 3 * (dbl(Lc * nx) + dbl(E14n)) + 2 * dbl(Lc * nx) + recs(Lc) + dbl(nP);
    return {nd, npp};
}

long cp_need(const raocp_ctx* c, const std::vector<std::pair<int, int>>& pr_, const std::vector<std::pair<int, int>>& lr_,
             int FB, int LB) {
    long w = 0;
    for (const auto& r : pr_)
        for (int i0 = r.first; i0 < r.second; i0 += FB) {
            const auto nd = cp_block_need(c, true, i0, std::min(r.second, i0 + FB));
            w = std::max(w, std::max(nd.first, nd.second));
        }
    for (const auto& r : lr_)
        for (int l0 = r.first; l0 < r.second; l0 += LB) {
            const auto nd = cp_block_need(c, false, l0, std::min(r.second, l0 + LB));
            w = std::max(w, std::max(nd.first, nd.second));
        }
    return w;
}

// ---- MFMA CP blocks (raocp_cp2.hip): LDS bytes of one block, mirroring StgB (worst-case
// misalignment of each region: 15 B)
long cp2_region(long nbytes) { return nbytes > 0 ? 16 * ((nbytes + 30) >> 4) + 16 : 16; }
std::pair<long, long> cp2_block_need(const raocp_ctx* c, bool family, int a0, int a1, bool regular) {
    const long nx = c->nx, nu = c->nu, w = c->wsz;
    auto R = [&](long cnt) { return cp2_region(cnt * w); };
    auto Rr = [&](long cnt) { return cp2_region(cnt * 16); };
    auto Ri = [&](long cnt) { return cp2_region(cnt * 4); };
    const long nBx = (long)c->nbn * (nx + nu), nBlx = (long)c->nbl * nx;
    if (family) {
        const long P = a1 - a0;
        const CpFam f = cp_fam(c, a0, a1);
        const long C = f.ce - f.cb, Y = f.y1 - f.y0, E7n = f.e7b - f.e7a;
        const long nd = 2 * R(P * nx) + 2 * R(P * nu) + 2 * R(Y) + 2 * R(P) + 3 * R(C) + R(Y) + R(P) + R(E7n) +
                        R(C * nx) + R(C * nu) + 2 * R(C) + Rr(P) + Rr(C) + Ri(P) + 2 * R(nBx);
        long npp = 3 * (R(Y) + R(P) + R(C * nx) + R(C * nu) + 2 * R(C) + R(E7n) + 3 * R(C)) + 2 * R(P * nx) +
                   2 * R(P * nu) + 2 * R(Y) + 5 * R(C) + R(P) + Rr(P) + Rr(C);
        if (!regular) npp += 3 * C * (nx + nu) * w;
        return {nd, npp};
    }
    const long Lc = a1 - a0;
    const long E14n = c->h_pos14[a1 - c->m] - c->h_pos14[a0 - c->m];
    const long nd = 2 * R(Lc * nx) + 2 * R(Lc) + R(Lc * nx) + 2 * R(Lc) + R(E14n) + Rr(Lc) + 2 * R(nBlx);
    const long npp = 3 * (R(Lc * nx) + R(E14n)) + 2 * R(Lc * nx) + Rr(Lc);
    return {nd, npp};
}

// largest LDS bytes of a MFMA CP block over a range of parents (families of FB) or leaves (LB)
long cp2_need(const raocp_ctx* c, int a, int b, int per, bool family);

// the uniform table index of nodes [a, b) (-1 when they differ or the range is empty)
int uniform_idx(const std::vector<int>& idx, int a, int b) {
    if (b <= a) return -1;
    for (int q = a + 1; q < b; ++q)
        if (idx[q] != idx[a]) return -1;
    return idx[a];
}

bool cp2_regular(const raocp_ctx* c, int i0, int i1) {
    const CpFam f = cp_fam(c, i0, i1);
    int creg = c->h_nch[i0] <= 4 ? c->h_nch[i0] : 0;
    for (int q = i0; q < i1 && creg; ++q)
        if (c->h_nch[q] != creg || c->h_chs[q] != f.cb + (q - i0) * creg) creg = 0;
    return creg > 0 && uniform_idx(c->h_isq, f.cb, f.ce) >= 0 && uniform_idx(c->h_isr, f.cb, f.ce) >= 0;
}
long cp2_need(const raocp_ctx* c, int a, int b, int per, bool family) {
    long w = 0;
    for (int x0 = a; x0 < b; x0 += per) {
        const int x1 = std::min(b, x0 + per);
        const auto nd = cp2_block_need(c, family, x0, x1, family ? cp2_regular(c, x0, x1) : true);
        w = std::max(w, std::max(nd.first, nd.second));
    }
    return w;
}

// (re)build the CP block table for the owned parent ranges and leaf ranges
int build_cp_blocks(raocp_ctx* c, const std::vector<std::pair<int, int>>& pranges,
                    const std::vector<std::pair<int, int>>& lranges) {
    std::vector<raocp::Rec> fam, leaf;
    long need_d = 0, need_p = 0;
    for (const auto& r : pranges)
        for (int i0 = r.first; i0 < r.second; i0 += c->cp_FB) {
            const int i1 = std::min(r.second, i0 + c->cp_FB);
            const CpFam f = cp_fam(c, i0, i1);
            fam.push_back(raocp::Rec{f.cb, f.ce, f.y0, f.y1});
            fam.push_back(raocp::Rec{f.e7a, f.e7b, i0, i1});
            const auto nd = cp_block_need(c, true, i0, i1);
            need_d = std::max(need_d, nd.first);
            need_p = std::max(need_p, nd.second);
        }
    for (const auto& r : lranges)
        for (int l0 = r.first; l0 < r.second; l0 += c->cp_LB) {
            const int l1 = std::min(r.second, l0 + c->cp_LB);
            leaf.push_back(raocp::Rec{c->h_pos14[l0 - c->m], c->h_pos14[l1 - c->m], l0, l1});
            const auto nd = cp_block_need(c, false, l0, l1);
            need_d = std::max(need_d, nd.first);
            need_p = std::max(need_p, nd.second);
        }
    if (std::max(need_d, need_p) * 8 > 150 * 1024)
        return fail(RAOCP_ERR_ARG, "CP node block does not fit LDS (nx, nu or branching too large)");
    std::vector<raocp::Rec> tab = fam;
    tab.insert(tab.end(), leaf.begin(), leaf.end());
    if (tab.empty()) tab.push_back(raocp::Rec{0, 0, 0, 0});
    const raocp::Rec* dtab = nullptr;
    int rc = c->upload_vec(&dtab, tab);
    if (rc) return rc;
    c->dev.cpd_tab = dtab;
    c->cp_nbF = (int)fam.size() / 2;
    c->cp_nbL = (int)leaf.size();
    c->lds_cpd = (size_t)need_d * 8;
    c->lds_cpp = (size_t)need_p * 8;
    c->cp_rows = c->cp_nbF + c->cp_nbL;
    // MFMA CP blocks (raocp_cp2.hip) over the same ranges
    {
        std::vector<raocp::Rec> fam2, leaf2;
        long nd2 = 0, np2 = 0;
        for (const auto& r : pranges)
            for (int i0 = r.first; i0 < r.second; i0 += c->cp2_FB) {
                const int i1 = std::min(r.second, i0 + c->cp2_FB);
                const CpFam f = cp_fam(c, i0, i1);
                // regular: every parent has the same child count creg <= 4, children in parent order
                int creg = c->h_nch[i0] <= 4 ? c->h_nch[i0] : 0;
                for (int q = i0; q < i1 && creg; ++q)
                    if (c->h_nch[q] != creg || c->h_chs[q] != f.cb + (q - i0) * creg) creg = 0;
                fam2.push_back(raocp::Rec{f.cb, f.ce, f.y0, f.y1});
                fam2.push_back(raocp::Rec{f.e7a, f.e7b, i0, i1});
                const int tq = uniform_idx(c->h_isq, f.cb, f.ce), tr = uniform_idx(c->h_isr, f.cb, f.ce);
                fam2.push_back(raocp::Rec{tq, tr, creg, 0});
                const auto nd = cp2_block_need(c, true, i0, i1, creg > 0 && tq >= 0 && tr >= 0);
                nd2 = std::max(nd2, nd.first);
                np2 = std::max(np2, nd.second);
            }
        for (const auto& r : lranges)
            for (int l0 = r.first; l0 < r.second; l0 += c->cp2_LB) {
                const int l1 = std::min(r.second, l0 + c->cp2_LB);
                leaf2.push_back(raocp::Rec{c->h_pos14[l0 - c->m], c->h_pos14[l1 - c->m], l0, l1});
                leaf2.push_back(raocp::Rec{uniform_idx(c->h_isp, l0, l1), 0, 0, 0});
                const auto nd = cp2_block_need(c, false, l0, l1, true);
                nd2 = std::max(nd2, nd.first);
                np2 = std::max(np2, nd.second);
            }
        if (std::max(nd2, np2) > 150 * 1024)
            return fail(RAOCP_ERR_ARG, "MFMA CP block does not fit LDS (nx, nu or branching too large)");
        std::vector<raocp::Rec> tab2 = fam2;
        tab2.insert(tab2.end(), leaf2.begin(), leaf2.end());
        if (tab2.empty()) tab2.push_back(raocp::Rec{0, 0, 0, 0});
        const raocp::Rec* dtab2 = nullptr;
        if ((rc = c->upload_vec(&dtab2, tab2))) return rc;
        c->dev.cp2_tab = dtab2;
        c->cp2_nbF = (int)fam2.size() / raocp::kCpFamRecs;
        c->cp2_nbL = (int)leaf2.size() / raocp::kCpLeafRecs;
        // the MFMA kernels need every block's nodes on one weight table (per-mode tables the
        // packer could not merge): otherwise the scalar kernels (raocp_cp.hip) run
        for (int b = 0; b < c->cp2_nbF; ++b)
            if (fam2[raocp::kCpFamRecs * b].y > fam2[raocp::kCpFamRecs * b].x &&
                (fam2[raocp::kCpFamRecs * b + 2].x < 0 || fam2[raocp::kCpFamRecs * b + 2].y < 0))
                c->cp_v1 = true;
        for (int b = 0; b < c->cp2_nbL; ++b)
            if (leaf2[raocp::kCpLeafRecs * b + 1].x < 0) c->cp_v1 = true;
        c->lds_cpd2 = (size_t)nd2;
        c->lds_cpp2 = (size_t)np2;
        c->cp_rows = c->cp_v1 ? c->cp_nbF + c->cp_nbL : c->cp2_nbF + c->cp2_nbL;
    }
    return RAOCP_OK;
}


// Every entry point that takes a context runs on that context's device: the current
// device is switched for the call and restored afterwards (a process may hold contexts
// on several devices; allocations and graph captures must land on c->device).
// The co-resident sweeps (k_dr, k_drc and the split tier sweep k_dyn_up / k_dyn_down) spin on
// hand-off flags and need every workgroup of their launch resident at once. Two of them from
// different contexts on one device could each hold part of the CUs and wait for the other
// (until the hand-off timeout returns RAOCP_ERR_STATE). One active context per device: the entry
// points that launch them hold a per-device lock for the call (each synchronises its stream
// before it returns), so threads of one process run such contexts one at a time. Processes
// sharing a device are not serialised (docs: INTEGRATION.md "one active context per device").
std::recursive_mutex g_sweep_mu[64];
struct SweepLock {
    std::unique_lock<std::recursive_mutex> l;
    explicit SweepLock(const raocp_ctx* c) {
        if (c && (c->dr || c->dyn_split)) l = std::unique_lock<std::recursive_mutex>(g_sweep_mu[c->device & 63]);
    }
};

struct DevGuard {
    int prev = -1;
    explicit DevGuard(const raocp_ctx* c) {
        if (!c) return;
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != c->device) (void)hipSetDevice(c->device);
        else prev = -1;
    }
    ~DevGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

}  // namespace

extern "C" {

const char* raocp_last_error(void) { return g_err.c_str(); }

int raocp_device_synchronize(int device) {
    HIPCHK(hipSetDevice(device));
    HIPCHK(hipDeviceSynchronize());
    return RAOCP_OK;
}

int raocp_ctx_create(const raocp_tree_desc* t, const raocp_problem_desc* pr, int device, raocp_ctx** out) {
    if (!t || !pr || !out) return fail(RAOCP_ERR_ARG, "null argument");
    *out = nullptr;
    const int n = t->n, m = t->m, nx = t->nx, nu = t->nu;
    if (n < 2 || m < 1 || m >= n || nx < 1 || nu < 1) return fail(RAOCP_ERR_ARG, "bad tree sizes");
    // ---- validate the layout invariants the kernels rely on
    if (t->anc[0] != -1 || t->stage[0] != 0) return fail(RAOCP_ERR_TREE, "node 0 must be the root");
    for (int i = 1; i < n; ++i) {
        if (t->stage[i] < t->stage[i - 1]) return fail(RAOCP_ERR_TREE, "stage must be non-decreasing in node id");
        if (t->anc[i] < 0 || t->anc[i] >= i) return fail(RAOCP_ERR_TREE, "ancestor must precede its child");
    }
    const int N = t->stage[n - 1];
    int expect = 1, cmax = 0;
    for (int i = 0; i < m; ++i) {
        if (t->stage[i] >= N) return fail(RAOCP_ERR_TREE, "nonleaf nodes must be ids 0..m-1");
        if (t->nch[i] < 1 || t->ch_start[i] != expect)
            return fail(RAOCP_ERR_TREE, "children must be contiguous id ranges in parent order");
        for (int k = 0; k < t->nch[i]; ++k)
            if (t->anc[expect + k] != i || t->stage[expect + k] != t->stage[i] + 1)
                return fail(RAOCP_ERR_TREE, "child range inconsistent with ancestors/stages");
        expect += t->nch[i];
        cmax = std::max(cmax, (int)t->nch[i]);
    }
    if (expect != n) return fail(RAOCP_ERR_TREE, "children ranges do not cover nodes 1..n-1");
    for (int i = m; i < n; ++i)
        if (t->stage[i] != N) return fail(RAOCP_ERR_TREE, "leaves must all be at the last stage");
    // group sizes of every kernel must fit one workgroup
    int rc;
    if ((rc = check_group(nx + nu + 2, "child block")) || (rc = check_group(2 * cmax + 2 + nx + nu, "nonleaf block")) ||
        (rc = check_group(2 * nx + 2, "leaf block")) || (rc = check_group(nx + nu + 2 * cmax + 2 + cmax, "L^T nonleaf")) ||
        (rc = check_group(nx + nu + cmax + 1, "CP primal nonleaf")))
        return rc;

    int prev_dev = -1;
    (void)hipGetDevice(&prev_dev);
    HIPCHK(hipSetDevice(device));
    struct Restore {
        int d;
        ~Restore() { if (d >= 0) (void)hipSetDevice(d); }
    } restore_{prev_dev != device ? prev_dev : -1};
    if (pr->dtype != RAOCP_F64 && pr->dtype != RAOCP_F32) return fail(RAOCP_ERR_ARG, "dtype must be RAOCP_F64 or RAOCP_F32");
    raocp_ctx* c = new raocp_ctx();
    c->device = device;
    c->n = n; c->m = m; c->nx = nx; c->nu = nu; c->cmax = cmax; c->N = N;
    c->f32 = pr->dtype == RAOCP_F32;
    c->wsz = c->f32 ? 4 : 8;
    auto bail = [&](int code) { raocp_ctx_destroy(c); return code; };
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess)
        return bail(fail(RAOCP_ERR_HIP, "hipStreamCreate failed"));

    c->stage_ptr.assign(N + 2, n);
    for (int i = n - 1; i >= 0; --i) c->stage_ptr[t->stage[i]] = i;
    c->stage_ptr[N + 1] = n;

    // ---- flat layout (cache.py:126-170)
    Dev& D = c->dev;
    D.n = n; D.m = m; D.nx = nx; D.nu = nu; D.cmax = cmax;
    std::vector<int> yrel(m), e7off(m, -1), e14off(n - m, -1), rank(n, 0);
    int ysum = 0;
    for (int i = 0; i < m; ++i) {
        yrel[i] = ysum;
        ysum += 2 * t->nch[i] + 1;
        for (int k = 0; k < t->nch[i]; ++k) rank[t->ch_start[i] + k] = k;
    }
    int64_t off = 0;
    D.X0 = (int)off; off += (int64_t)n * nx;
    D.U0 = (int)off; off += (int64_t)m * nu;
    D.Y0 = (int)off; off += ysum;
    D.T0 = (int)off; off += n;
    D.S0 = (int)off; off += n;
    c->P = off; D.P = (int)off;
    off = 0;
    D.E1 = (int)off; off += ysum + (n - m);
    D.E2 = (int)off; off += n;
    D.E3 = (int)off; off += 1 + (int64_t)(n - 1) * nx;
    D.E4 = (int)off; off += 1 + (int64_t)(n - 1) * nu;
    D.E5 = (int)off; off += n;
    D.E6 = (int)off; off += n;
    D.E7 = (int)off;
    for (int i = 0; i < n; ++i) {
        if (i < m && pr->i_box_nl[i] >= 0) { e7off[i] = (int)off; off += nx + nu; }
        else off += 1;
    }
    D.E11 = (int)off; off += m + (int64_t)(n - m) * nx;
    D.E12 = (int)off; off += n;
    D.E13 = (int)off; off += n;
    D.E14 = (int)off;
    for (int i = 0; i < n; ++i) {
        if (i >= m && pr->i_box_l[i] >= 0) { e14off[i - m] = (int)off; off += nx; }
        else off += 1;
    }
    c->D = off; D.D = (int)off;
    // dual placeholders: (1,1) blocks no projection touches; prox_g* maps them to exactly 0
    std::vector<int> ph;
    for (int l = m; l < n; ++l) ph.push_back(D.E1 + ysum + (l - m));
    for (int l = m; l < n; ++l) ph.push_back(D.E2 + l);
    ph.push_back(D.E3); ph.push_back(D.E4); ph.push_back(D.E5); ph.push_back(D.E6);
    {
        int o = D.E7;
        for (int i = 0; i < n; ++i) {
            if (i < m && e7off[i] >= 0) o += nx + nu;
            else ph.push_back(o++);
        }
        o = D.E14;
        for (int i = 0; i < n; ++i) {
            if (i >= m && e14off[i - m] >= 0) o += nx;
            else ph.push_back(o++);
        }
    }
    for (int i = 0; i < m; ++i) { ph.push_back(D.E11 + i); ph.push_back(D.E12 + i); ph.push_back(D.E13 + i); }
    if (c->P >= (int64_t)1 << 31 || c->D >= (int64_t)1 << 31)
        return bail(fail(RAOCP_ERR_ARG, "flat vectors exceed 2^31 entries (int32 offsets)"));

    // ---- tables
    std::vector<int> ch_start(t->ch_start, t->ch_start + m), nch(t->nch, t->nch + m), anc(t->anc, t->anc + n);
    c->n_ph = (int)ph.size();
    if ((rc = c->upload_vec(&c->ph, ph))) return bail(rc);
    if ((rc = c->upload_vec(&D.anc, anc)) || (rc = c->upload_vec(&D.ch_start, ch_start)) ||
        (rc = c->upload_vec(&D.nch, nch)) || (rc = c->upload_vec(&D.rank, rank)) || (rc = c->upload_vec(&D.yrel, yrel)) ||
        (rc = c->upload_vec(&D.e7off, e7off)) || (rc = c->upload_vec(&D.e14off, e14off)))
        return bail(rc);
    if ((rc = upload_t(c, &D.SQ, to_colmajor(pr->sqrt_q, pr->n_sq, nx, nx))) ||
        (rc = upload_t(c, &D.SR, to_colmajor(pr->sqrt_r, pr->n_sr, nu, nu))) ||
        (rc = upload_t(c, &D.SP, to_colmajor(pr->sqrt_pf, pr->n_sp, nx, nx))) ||
        (rc = c->upload(&D.SQr, pr->sqrt_q, (size_t)pr->n_sq * nx * nx)) ||
        (rc = c->upload(&D.SRr, pr->sqrt_r, (size_t)pr->n_sr * nu * nu)) ||
        (rc = c->upload(&D.SPr, pr->sqrt_pf, (size_t)pr->n_sp * nx * nx)) ||
        (rc = c->upload(&D.iSQ, pr->i_sq, n)) || (rc = c->upload(&D.iSR, pr->i_sr, n)) ||
        (rc = c->upload(&D.iSP, pr->i_sp, n)) || (rc = upload_t(c, &D.alpha_r, copy_table(pr->alpha_r, m))) ||
        ((D.nSQ = pr->n_sq), (D.nSR = pr->n_sr), (D.nSP = pr->n_sp), false) ||
        (rc = upload_t(c, &D.cond, copy_table(pr->cond, n))))
        return bail(rc);
    const int nbn = std::max(1, pr->n_box_nl), nbl = std::max(1, pr->n_box_l);
    std::vector<double> lo_nl(nbn * (nx + nu), 0.0), hi_nl(nbn * (nx + nu), 0.0), lo_l(nbl * nx, 0.0), hi_l(nbl * nx, 0.0);
    if (pr->n_box_nl) {
        std::copy(pr->box_nl_lo, pr->box_nl_lo + lo_nl.size(), lo_nl.begin());
        std::copy(pr->box_nl_hi, pr->box_nl_hi + hi_nl.size(), hi_nl.begin());
    }
    if (pr->n_box_l) {
        std::copy(pr->box_l_lo, pr->box_l_lo + lo_l.size(), lo_l.begin());
        std::copy(pr->box_l_hi, pr->box_l_hi + hi_l.size(), hi_l.begin());
    }
    if ((rc = upload_t(c, &D.blo_nl, lo_nl)) || (rc = upload_t(c, &D.bhi_nl, hi_nl)) ||
        (rc = upload_t(c, &D.blo_l, lo_l)) || (rc = upload_t(c, &D.bhi_l, hi_l)) ||
        (rc = c->upload(&D.iBnl, pr->i_box_nl, m)) || (rc = c->upload(&D.iBl, pr->i_box_l, n)))
        return bail(rc);
    // dynamics tables (raocp_dyn.hip header): per child kind W = [B'; A'], per class
    // RG = [R~^-1; G = M R~^-1 - K'] and K, per (kind, parent class) pair F = [A + B K | B]
    const int R = nx + nu;
    const int KP = raocp::rup(nx, 2 * raocp::kKS), KF = raocp::rup(nx + nu, 2 * raocp::kKS), NUP = raocp::rup(nu, 2);
    c->KP = KP; c->KF = KF; c->NUP = NUP; c->PS = NUP + raocp::rup(nx, 2);
    const int SKP = raocp::tstride(KP), SKF = raocp::tstride(KF), SNU = raocp::tstride(NUP);  // table row strides
    if (R * raocp::kKS > raocp::kDynBlock)
        return bail(fail(RAOCP_ERR_ARG, "nx + nu > 256 is not supported by the dynamics sweep"));
    {
        const int nk = pr->n_k;
        for (int j = 1; j < n; ++j)
            if (pr->i_a[j] < 0 || pr->i_a[j] >= pr->n_a || pr->i_b[j] < 0 || pr->i_b[j] >= pr->n_b)
                return bail(fail(RAOCP_ERR_ARG, "dynamics index out of range"));
        for (int i = 0; i < m; ++i)
            if (pr->i_k[i] < 0 || pr->i_k[i] >= nk) return bail(fail(RAOCP_ERR_ARG, "class index out of range"));
        auto A = [&](int t, int r, int k) { return pr->A[((size_t)t * nx + r) * nx + k]; };
        auto Bm = [&](int t, int r, int k) { return pr->B[((size_t)t * nx + r) * nu + k]; };
        auto K = [&](int c_, int r, int k) { return pr->K[((size_t)c_ * nu + r) * nx + k]; };
        auto Ri = [&](int c_, int r, int k) { return pr->Rinv[((size_t)c_ * nu + r) * nu + k]; };
        auto M = [&](int c_, int r, int k) { return pr->M[((size_t)c_ * nx + r) * nu + k]; };
        // child kinds (A, B index pairs) and (kind, parent class) pairs
        std::vector<int> kind(n, 0), pair(n, 0);
        std::vector<std::pair<int, int>> kinds, pairs;
        {
            std::vector<std::pair<std::pair<int, int>, int>> seen_k;
            std::vector<std::pair<std::pair<int, int>, int>> seen_p;
            auto find = [](std::vector<std::pair<std::pair<int, int>, int>>& v, std::pair<int, int> key, int next) {
                for (auto& e : v)
                    if (e.first == key) return e.second;
                v.push_back({key, next});
                return next;
            };
            for (int j = 1; j < n; ++j) {
                const std::pair<int, int> kk{pr->i_a[j], pr->i_b[j]};
                const int kid = find(seen_k, kk, (int)kinds.size());
                if (kid == (int)kinds.size()) kinds.push_back(kk);
                kind[j] = kid;
                const std::pair<int, int> pk{kid, pr->i_k[t->anc[j]]};
                const int pid = find(seen_p, pk, (int)pairs.size());
                if (pid == (int)pairs.size()) pairs.push_back(pk);
                pair[j] = pid;
            }
        }
        // number pairs by parent class (so the pairs of a stage range are contiguous)
        {
            std::vector<int> order(pairs.size());
            for (size_t q = 0; q < order.size(); ++q) order[q] = (int)q;
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return pairs[a].second < pairs[b].second; });
            std::vector<int> newid(pairs.size());
            std::vector<std::pair<int, int>> sorted(pairs.size());
            for (size_t q = 0; q < order.size(); ++q) {
                newid[order[q]] = (int)q;
                sorted[q] = pairs[order[q]];
            }
            pairs = sorted;
            for (int j = 1; j < n; ++j) pair[j] = newid[pair[j]];
        }
        // classes must be numbered by stage: stage t owns classes [cls_ptr[t], cls_ptr[t+1])
        c->cls_ptr.assign(N + 1, nk);
        for (int i = m - 1; i >= 0; --i) c->cls_ptr[t->stage[i]] = std::min(c->cls_ptr[t->stage[i]], pr->i_k[i]);
        for (int st = N - 1; st >= 0; --st) c->cls_ptr[st] = std::min(c->cls_ptr[st], c->cls_ptr[st + 1]);
        for (int i = 0; i < m; ++i)
            if (pr->i_k[i] < c->cls_ptr[t->stage[i]] || pr->i_k[i] >= c->cls_ptr[t->stage[i] + 1])
                return bail(fail(RAOCP_ERR_ARG, "classes must be numbered by stage"));
        c->pair_ptr.assign(nk + 1, (int)pairs.size());
        for (int q = (int)pairs.size() - 1; q >= 0; --q) c->pair_ptr[pairs[q].second] = q;
        for (int c_ = nk - 1; c_ >= 0; --c_) c->pair_ptr[c_] = std::min(c->pair_ptr[c_], c->pair_ptr[c_ + 1]);
        c->nkind = (int)kinds.size();
        D.nkind = c->nkind;
        std::vector<double> W(std::max<size_t>(1, kinds.size()) * R * SKP, 0.0);
        for (size_t q = 0; q < kinds.size(); ++q)
            for (int rho = 0; rho < R; ++rho)
                for (int k = 0; k < nx; ++k)
                    W[(q * R + rho) * SKP + k] =
                        rho < nu ? Bm(kinds[q].second, k, rho) : A(kinds[q].first, k, rho - nu);  // B', A'
        std::vector<double> RG((size_t)nk * R * SNU, 0.0), KM((size_t)nk * nu * SKP, 0.0);
        for (int c_ = 0; c_ < nk; ++c_) {
            for (int r = 0; r < nu; ++r) {
                for (int k = 0; k < nu; ++k) RG[((size_t)c_ * R + r) * SNU + k] = Ri(c_, r, k);
                for (int k = 0; k < nx; ++k) KM[((size_t)c_ * nu + r) * SKP + k] = K(c_, r, k);
            }
            for (int r = 0; r < nx; ++r)
                for (int k = 0; k < nu; ++k) {
                    double g = 0.0;
                    for (int t2 = 0; t2 < nu; ++t2) g += M(c_, r, t2) * Ri(c_, t2, k);
                    RG[((size_t)c_ * R + nu + r) * SNU + k] = g - K(c_, k, r);
                }
        }
        std::vector<double> F(std::max<size_t>(1, pairs.size()) * nx * SKF, 0.0);
        for (size_t q = 0; q < pairs.size(); ++q) {
            const int ia = kinds[pairs[q].first].first, ib = kinds[pairs[q].first].second, c_ = pairs[q].second;
            for (int r = 0; r < nx; ++r) {
                for (int k = 0; k < nx; ++k) {
                    double bk = 0.0;
                    for (int t2 = 0; t2 < nu; ++t2) bk += Bm(ib, r, t2) * K(c_, t2, k);
                    F[(q * nx + r) * SKF + k] = A(ia, r, k) + bk;  // Abar = A + B K (cache.py:226)
                }
                for (int k = 0; k < nu; ++k) F[(q * nx + r) * SKF + nx + k] = Bm(ib, r, k);
            }
        }
        // one-phase backward levels: WT[pair] = [-Rinv B' ; A' - G B'] of (child kind, parent class)
        std::vector<double> WT(std::max<size_t>(1, pairs.size()) * R * SKP, 0.0);
        for (size_t q = 0; q < pairs.size(); ++q) {
            const int ia = kinds[pairs[q].first].first, ib = kinds[pairs[q].first].second, c_ = pairs[q].second;
            for (int tr = 0; tr < R; ++tr)
                for (int k = 0; k < nx; ++k) {
                    double v = 0.0;
                    if (tr < nu) {
                        for (int t2 = 0; t2 < nu; ++t2) v -= Ri(c_, tr, t2) * Bm(ib, k, t2);
                    } else {
                        const double* grow = &RG[((size_t)c_ * R + tr) * SNU];
                        for (int t2 = 0; t2 < nu; ++t2) v -= grow[t2] * Bm(ib, k, t2);
                        v += A(ia, k, tr - nu);
                    }
                    WT[(q * R + tr) * SKP + k] = v;
                }
        }
        if ((rc = c->upload_vec(&D.dW, W)) || (rc = c->upload_vec(&D.dRG, RG)) || (rc = c->upload_vec(&D.dKM, KM)) ||
            (rc = c->upload_vec(&D.dF, F)) || (rc = c->upload_vec(&D.dWT, WT)))
            return bail(rc);
        // per-stage MFMA dynamics (raocp_dyn2.hip): column-major tables M[k R + r] and, per
        // stage, tiles of <= 16 nodes sharing a table (fp32 contexts; fp64 opt-in RAOCP_DYN2=1)
        c->dyn2 = c->f32;
        if (const char* e = getenv("RAOCP_DYN2")) c->dyn2 = c->dyn2 || atoi(e) != 0;
        {
            // the per-stage streaming sweep (raocp_dyn3.hip): one branching factor C <= 4, the
            // children's slot k of one kind at every parent of a stage, one class per stage, and
            // the compile-time sizes
            const int C = t->nch[0];
            // (fp64 at nx = 64: the stage's tables exceed the 160 KB of LDS)
            bool ok = C >= 1 && C <= 4 && ((nx == 20 && nu == 8) || (nx == 32 && nu == 12) || (nx == 64 && nu == 16)) &&
                      dyn3_lds_fits(c->f32, nx, nu, C);
            for (int i = 0; i < m && ok; ++i)
                if (t->nch[i] != C || t->ch_start[i] != 1 + C * i) ok = false;
            std::vector<raocp::Dy3Stage> sts;
            for (int st = 0; st < N && ok; ++st) {
                raocp::Dy3Stage d{};
                d.i0 = c->stage_ptr[st];
                d.i1 = c->stage_ptr[st + 1];
                d.leaf = st + 1 == N;
                d.cls = pr->i_k[d.i0];
                for (int k = 0; k < 4; ++k) {
                    d.kind[k] = k < C ? kind[1 + C * d.i0 + k] : 0;
                    d.pair[k] = k < C ? pair[1 + C * d.i0 + k] : 0;
                }
                for (int i = d.i0; i < d.i1 && ok; ++i) {
                    if (pr->i_k[i] != d.cls) ok = false;
                    for (int k = 0; k < C && ok; ++k)
                        if (kind[1 + C * i + k] != d.kind[k] || pair[1 + C * i + k] != d.pair[k]) ok = false;
                }
                sts.push_back(d);
            }
            c->reg_ok = ok && C >= 2;
            c->reg_C = C;
            c->reg_st = sts;
            // default: fp32, and fp64 trees of >= 64k nodes (config 4: 118 vs 143 us for the
            // tiers; config 2 keeps the tiers, whose few launches win on small trees)
            c->dyn3 = ok && (c->f32 || n >= 65536);
            if (const char* e = getenv("RAOCP_DYN3")) c->dyn3 = ok && atoi(e) != 0;
            if (c->dyn3) {
                c->d3st = sts;
                c->dyn2 = false;
                c->unif_branch = C;
            }
        }
        if (c->dyn2 || c->dyn3) {
            const size_t nkd = std::max<size_t>(1, kinds.size()), npr = std::max<size_t>(1, pairs.size());
            std::vector<double> W2(nkd * R * nx, 0.0), RG2((size_t)std::max(1, nk) * R * nu, 0.0),
                KM2((size_t)std::max(1, nk) * nu * nx, 0.0), F2(npr * nx * (nx + nu), 0.0);
            for (size_t q = 0; q < kinds.size(); ++q)
                for (int r = 0; r < R; ++r)
                    for (int k = 0; k < nx; ++k) W2[(q * nx + k) * R + r] = W[(q * R + r) * SKP + k];
            for (int c_ = 0; c_ < nk; ++c_) {
                for (int r = 0; r < R; ++r)
                    for (int k = 0; k < nu; ++k) RG2[((size_t)c_ * nu + k) * R + r] = RG[((size_t)c_ * R + r) * SNU + k];
                for (int r = 0; r < nu; ++r)
                    for (int k = 0; k < nx; ++k) KM2[((size_t)c_ * nx + k) * nu + r] = KM[((size_t)c_ * nu + r) * SKP + k];
            }
            for (size_t q = 0; q < pairs.size(); ++q)
                for (int r = 0; r < nx; ++r)
                    for (int k = 0; k < nx + nu; ++k) F2[(q * (nx + nu) + k) * nx + r] = F[(q * nx + r) * SKF + k];
            if ((rc = upload_t(c, &c->W2, W2)) || (rc = upload_t(c, &c->RG2, RG2)) || (rc = upload_t(c, &c->KM2, KM2)) ||
                (rc = upload_t(c, &c->F2, F2)))
                return bail(rc);
        }
        if (c->dyn3) {
            if ((rc = c->alloc(&c->Q2, (size_t)n * nx)) || (rc = c->alloc(&c->Dd2, (size_t)m * nu)) ||
                (rc = dyn3_images(c)))
                return bail(rc);
            c->dyn32 = c->f32;
        }
        if (c->dyn2) {
            std::vector<int> idx;
            std::vector<raocp::DynTile> tl;
            // nodes [a, b) grouped by table (stable), cut into tiles of <= 16
            auto add = [&](int a, int b, auto table_of) {
                std::vector<std::pair<int, int>> it;
                for (int v = a; v < b; ++v) it.push_back({table_of(v), v});
                std::stable_sort(it.begin(), it.end(), [](const auto& x, const auto& y) { return x.first < y.first; });
                for (size_t q = 0; q < it.size();) {
                    size_t e = q;
                    while (e < it.size() && e - q < 16 && it[e].first == it[q].first) ++e;
                    tl.push_back(raocp::DynTile{(int)idx.size(), (int)(e - q), it[q].first, 0});
                    for (size_t k = q; k < e; ++k) idx.push_back(it[k].second);
                    q = e;
                }
            };
            c->d2_off.assign((size_t)N * 5, 0);
            for (int st = 0; st < N; ++st) {
                int* o = &c->d2_off[(size_t)st * 5];
                const int pb = c->stage_ptr[st], pe = c->stage_ptr[st + 1], cb_ = pe, ce_ = c->stage_ptr[st + 2];
                o[0] = (int)tl.size();
                add(cb_, ce_, [&](int j) { return kind[j]; });
                o[1] = (int)tl.size();
                add(pb, pe, [&](int i) { return pr->i_k[i]; });
                o[2] = (int)tl.size();
                add(pb, pe, [&](int i) { return pr->i_k[i]; });
                o[3] = (int)tl.size();
                add(cb_, ce_, [&](int j) { return pair[j]; });
                o[4] = (int)tl.size();
            }
            if ((rc = c->upload_vec(&c->d2_idx, idx)) || (rc = c->upload_vec(&c->d2_tiles, tl)) ||
                (rc = c->alloc(&c->Q2, (size_t)n * nx)) || (rc = c->alloc(&c->PA2, (size_t)n * R)) ||
                (rc = c->alloc(&c->Dd2, (size_t)m * nu)))
                return bail(rc);
            c->dyn32 = c->f32;
        }
        // the regular-tree sweep (raocp_dynr.hip): fp64 regular trees of the compiled sizes
        c->dr = false;
        // (RAOCP_DYN3=1 / RAOCP_DYN2=1 keep the per-stage sweeps they ask for)
        if (c->reg_ok && !c->f32 && !c->dyn3 && !c->dyn2 && raocp::dr_supported(nx, nu, c->reg_C) && N >= 2) {
            bool want = true;
            if (const char* e = getenv("RAOCP_DR")) want = atoi(e) != 0;
            int n_cus = 0;
            if (hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cus <= 0)
                n_cus = 256;
            if (want && (rc = dr_setup(c, WT, SKP, RG, SNU, KM, F, SKF, n_cus))) return bail(rc);
        }
        std::vector<raocp::Rec> ninfo(m), cinfo(n);
        for (int i = 0; i < m; ++i) ninfo[i] = raocp::Rec{t->ch_start[i], t->nch[i], pr->i_k[i], t->stage[i]};
        cinfo[0] = raocp::Rec{0, 0, -1, 0};
        for (int j = 1; j < n; ++j) cinfo[j] = raocp::Rec{kind[j], pair[j], t->anc[j], 0};
        // CP child blocks (k_cp_dual): child records and each block's parent range
        {
            std::vector<raocp::Rec> crec(n, raocp::Rec{0, 0, 0, 0});
            for (int j = 1; j < n; ++j) crec[j] = raocp::Rec{t->anc[j], pr->i_sq[j], pr->i_sr[j], 0};
            const int per = kBlock / (nx + nu + 2);
            std::vector<raocp::Rec> dblk;
            for (int j0 = 1; j0 < n; j0 += per) {
                const int j1 = std::min(n, j0 + per), J = j1 - j0;
                const int a0 = t->anc[j0], a1 = t->anc[j1 - 1], na = a1 - a0 + 1;
                auto reg = [](int cnt) { return (cnt + 1) / 2 * 2 + 2; };
                const int need = 2 * reg(na * nx) + 2 * reg(na * nu) + 2 * reg(J) + reg(J * nx) + reg(J * nu) +
                                 2 * reg(J) + reg(2 * J);
                if (need > raocp::kStageDual)
                    return bail(fail(RAOCP_ERR_ARG, "dual child block staging exceeds the LDS buffer"));
                dblk.push_back(raocp::Rec{a0, a1, 0, 0});
            }
            if ((rc = c->upload_vec(&D.crec, crec)) || (rc = c->upload_vec(&D.dblk, dblk))) return bail(rc);
        }
        if ((rc = c->upload_vec(&D.ninfo, ninfo)) || (rc = c->upload_vec(&D.cinfo, cinfo)) ||
            (rc = c->upload_vec(&D.stage_ptr, c->stage_ptr)))
            return bail(rc);
    }
    D.N = N;

    // ---- dynamics plan. The stages are split into tiers 0 = s_0 < s_1 < ... < s_T = N:
    // tier 0 (stages < s_1) runs backward + forward in ONE workgroup (k_dyn_top); every
    // deeper tier [s_k, s_k+1) runs one workgroup per subtree rooted at stage s_k
    // (k_dyn_bottom_back / _fwd), its boundary being the leaves or the next tier's roots.
    // Vectors and matrix tables live in LDS (F when it fits). The cut list minimises a
    // cost model: a level costs one unit per phase plus its lane work over 384, a tier
    // kernel five units of launch + prologue. Per-stage launches when nothing fits.
    {
        const size_t kLds = 160 * 1024 - 2 * 1024;  // minus the static LDS (Prologue, ~1.2 KB)
        const size_t W1 = (size_t)R * SKP, RG1 = (size_t)R * SNU, KM1 = (size_t)nu * SKP, F1 = (size_t)nx * SKF;
        const std::vector<int>& cp = c->cls_ptr;
        const std::vector<int>& pp = c->pair_ptr;
        const int PS = c->PS;
        auto stage_n = [&](int st) { return c->stage_ptr[st + 1] - c->stage_ptr[st]; };
        int n_cus = 0;
        if (hipDeviceGetAttribute(&n_cus, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cus <= 0)
            n_cus = 256;
        // workgroup sizes (multiples of 64, at most 1024). The plan below is costed for
        // 1024-lane workgroups; launching its tiers with 512 lanes measured 98.0 vs 106.5 us
        // per CP iteration at config 2 and 577 vs 589 us at config 4 (more co-resident
        // workgroups per CU, cheaper barriers), while re-costing the plan for 512 or 256
        // lanes picked worse plans (config 4: 906 / 815 us). RAOCP_DYN_BLOCK /
        // RAOCP_DYN_TOP_BLOCK override.
        auto wg_env = [](const char* name, int def) {
            const char* e = getenv(name);
            const int v = e ? atoi(e) : def;
            return v >= 64 && v <= 1024 && v % 64 == 0 ? v : def;
        };
        c->dyn_block = wg_env("RAOCP_DYN_BLOCK", 512);
        // the top on 512 lanes like the split sweep's top workgroups (kFuseBlock): the level
        // routines pick their split-k width from the lane count, so a sharded solve (tier
        // launches) reproduces the unsharded one (split sweep) bit for bit
        c->dyn_top_block = wg_env("RAOCP_DYN_TOP_BLOCK", raocp::kFuseBlock);
        if (R * raocp::kKS > c->dyn_block) c->dyn_block = 1024;  // a child's split-k rows in one workgroup
        const long wg_per_cu = 2;
        auto level_cost = [&](double P, double C) { return 3.0 + (C * R + P * R + P * nu + C * nx) / 384.0; };
        auto recs = [](size_t cnt) { return 2 * cnt; };  // 16-B records in doubles
        // fold: one-phase backward levels (per-pair WT tables instead of per-kind W, no P rows)
        // the default: config 2's split sweep 47.1 vs 49.5 us, the tier launches 51.4 vs 51.5 us
        // (profiles/r03_v5/dyn_time.log); RAOCP_DYN_FOLD=0 keeps the two-phase levels
        bool fold_ok = true;
        if (const char* env = getenv("RAOCP_DYN_FOLD")) fold_ok = atoi(env) != 0;
        auto top_bytes = [&](int s_, int& maxch, bool fl, bool fold) {
            const size_t T = c->stage_ptr[s_], nb = stage_n(s_);
            maxch = 0;
            for (int st = 1; st <= s_; ++st) maxch = std::max(maxch, stage_n(st));
            const size_t mats = (fold ? pp[cp[s_]] * W1 : c->nkind * W1) + cp[s_] * (RG1 + KM1) + (fl ? pp[cp[s_]] * F1 : 0);
            const size_t dbl = mats + T * KP + nb * KP + T * NUP + T * KF + (fold ? 0 : raocp::rup(maxch * PS, 2)) +
                               recs(T + T + nb - 1);
            return 8 * dbl;
        };
        struct Tier {
            size_t nall = 0, nnl = 0;
            int maxch = 0;
            double cost = 0;
            size_t bb = 0, bf = 0;
            int fm = 1;
            bool ok = false, fold = false;
        };
        auto tier = [&](int a, int b) {  // subtrees rooted at stage a, levels a..b-1, boundary b (worst case)
            Tier w;
            if (b - a > raocp::kMaxLevels) return w;
            std::vector<double> lvl(b - a, 0.0);
            for (int r = c->stage_ptr[a]; r < c->stage_ptr[a + 1]; ++r) {
                int lo = r, hi = r + 1, mc = 0;
                size_t nall = 0;
                for (int st = a; st < b; ++st) {
                    nall += hi - lo;
                    const int nlo = t->ch_start[lo], nhi = t->ch_start[hi - 1] + t->nch[hi - 1];
                    lvl[st - a] = std::max(lvl[st - a], level_cost(hi - lo, nhi - nlo));
                    mc = std::max(mc, nhi - nlo);
                    lo = nlo;
                    hi = nhi;
                }
                w.nnl = std::max(w.nnl, nall);
                w.nall = std::max(w.nall, nall + (hi - lo));
                w.maxch = std::max(w.maxch, mc);
            }
            for (double v : lvl) w.cost += v;
            const size_t ncl = cp[b] - cp[a], npr = pp[cp[b]] - pp[cp[a]];
            const size_t st_b = 0, st_f = 0;
            w.bb = 8 * (c->nkind * W1 + ncl * RG1 + w.nall * KP + w.nnl * NUP + raocp::rup(w.maxch * PS, 2) +
                        recs(w.nnl + w.nall - 1) + st_b);
            const size_t bb_fold = 8 * (npr * W1 + ncl * RG1 + w.nall * KP + w.nnl * NUP + recs(w.nnl + w.nall - 1) + st_b);
            if (fold_ok && bb_fold <= kLds) {
                w.fold = true;
                w.bb = bb_fold;
                w.cost -= (b - a);  // one barrier phase per backward level instead of two
            }
            w.bf = 8 * (ncl * KM1 + npr * F1 + w.nnl * KF + recs(w.nnl + w.nall - 1) + st_f);
            if (w.bf > kLds) {
                // the pairs of one level at a time (restaged per level: one LDS round trip each),
                // else F from L2: measured 86.7 us for the config-4 tier [6,10) forward, whose
                // leaf level alone took 18.7 us per round (profiles/r03_v2/stamps_c4.log)
                size_t npl = 0;
                for (int t = a; t < b; ++t) npl = std::max<size_t>(npl, pp[cp[t + 1]] - pp[cp[t]]);
                const size_t bf2 = w.bf - 8 * (npr - npl) * F1;
                if (bf2 <= kLds) {
                    w.fm = 2;
                    w.bf = bf2;
                    w.cost += (b - a - 1);
                } else {
                    w.fm = 0;
                    w.bf -= 8 * npr * F1;
                    w.cost += 8 * (b - a);
                }
            }
            // the tier's subtrees run as rounds of co-resident workgroups (2048 lanes per CU
            // at most, fewer workgroups when their LDS does not fit): every round
            // pays the levels again (measured at configs 3 / 4: deep tiers of thousands of
            // subtrees lost to one-level tiers)
            {
                const size_t lds = std::max(w.bb, w.bf);
                const long per_cu = std::max<long>(1, std::min<long>(wg_per_cu, lds ? (long)(160 * 1024 / lds) : wg_per_cu));
                const long nsub = c->stage_ptr[a + 1] - c->stage_ptr[a];
                const long rounds = (nsub + (long)n_cus * per_cu - 1) / ((long)n_cus * per_cu);
                w.cost *= (double)std::max<long>(1, rounds);
            }
            w.cost += 10.0;  // two launches and their prologues
            w.ok = w.bb <= kLds && w.bf <= kLds;
            return w;
        };
        // f[a]: best cost of tiers covering [a, N); nxt[a]: the end of the first of them
        std::vector<double> f(N + 1, 1e300);
        std::vector<int> nxt(N + 1, N);
        f[N] = 0.0;
        for (int a = N - 1; a >= 1; --a)
            for (int b = a + 1; b <= N; ++b) {
                if (f[b] >= 1e299) continue;
                const Tier w = tier(a, b);
                if (!w.ok) continue;
                if (w.cost + f[b] < f[a]) {
                    f[a] = w.cost + f[b];
                    nxt[a] = b;
                }
            }
        double best = 1e300;
        int best_s = 0;
        double top_cost = 5.0;
        for (int s_ = 1; s_ <= N && s_ <= raocp::kMaxTopStages; ++s_) {
            top_cost += level_cost(stage_n(s_ - 1), stage_n(s_));
            bool any = false;
            for (int v = 0; v < 4; ++v) {  // (F in LDS, fold) = (1,1), (1,0), (0,1), (0,0)
                const bool fl = v < 2, fold = (v % 2 == 0);
                if (fold && !fold_ok) continue;
                int mt = 0;
                const size_t tb = top_bytes(s_, mt, fl, fold);
                if (tb > kLds) continue;
                any = true;
                const double cost = top_cost + (fl ? 0.0 : 2.0 * s_) - (fold ? s_ : 0) + f[s_];
                if (cost < best) {
                    best = cost;
                    best_s = s_;
                    c->lds_top = tb;
                    c->maxch_top = mt;
                    c->f_lds_top = fl;
                    c->fold_top = fold;
                }
            }
            if (!any) break;
        }
        c->cut = best_s;
        if (const char* env = getenv("RAOCP_DYN_PER_STAGE"))
            if (env[0] == '1') c->cut = 0;
        if (c->cut > 0 && f[c->cut] >= 1e299) c->cut = 0;
        for (int a = c->cut; c->cut > 0 && a < N; a = nxt[a]) {
            const int b = nxt[a], L = b - a;
            const Tier w = tier(a, b);
            raocp_ctx::TierPlan tp;
            tp.s0 = a;
            tp.s1 = b;
            tp.nsub = stage_n(a);
            tp.maxch = w.maxch;
            tp.lds_b = w.bb;
            tp.lds_f = w.bf;
            tp.fm = w.fm;
            tp.fold = w.fold;
            std::vector<raocp::Rec> lv;  // level ranges {lo, hi, off} of every subtree of the tier
            for (int r = c->stage_ptr[a]; r < c->stage_ptr[a + 1]; ++r) {
                int lo = r, hi = r + 1, acc = 0;
                for (int l = 0; l <= L; ++l) {
                    lv.push_back(raocp::Rec{lo, hi, acc, 0});
                    acc += hi - lo;
                    if (l < L) {
                        const int nlo = t->ch_start[lo], nhi = t->ch_start[hi - 1] + t->nch[hi - 1];
                        lo = nlo;
                        hi = nhi;
                    }
                }
            }
            if ((rc = c->upload_vec(&tp.lv, lv))) return bail(rc);
            // regular tier: every subtree has the same level sizes and consecutive ids
            memset(&tp.ta, 0, sizeof(tp.ta));
            for (int l = 0; l <= L; ++l) tp.ta.pl0[l] = c->pair_ptr[c->cls_ptr[a + l]];
            tp.ta.regular = 1;
            for (int l = 0; l <= L; ++l) {
                tp.ta.lo0[l] = lv[l].x;
                tp.ta.cnt[l] = lv[l].y - lv[l].x;
            }
            for (int r = 0; r < tp.nsub && tp.ta.regular; ++r)
                for (int l = 0; l <= L; ++l) {
                    const raocp::Rec& e = lv[(size_t)r * (L + 1) + l];
                    if (e.x != tp.ta.lo0[l] + r * tp.ta.cnt[l] || e.y - e.x != tp.ta.cnt[l]) {
                        tp.ta.regular = 0;
                        break;
                    }
                }
            c->tiers.push_back(tp);
        }
        // ---- the split sweep (raocp_dynf.hip): the same tiers in TWO launches, one workgroup
        // per subtree of every tier plus the top, for regular tiers of >= 2 subtrees per parent
        // subtree with the top's F in LDS (RAOCP_DYN_SPLIT=0 keeps the tier launches). Its
        // waits are for workgroups of the same launch, so it runs only where the whole grid is
        // co-resident (the occupancy query): no wait then depends on the dispatch order.
        {
            c->dyn_split = false;
            bool fz = c->cut > 0 && !c->tiers.empty() && c->tiers.size() <= (size_t)raocp::kFuseTiers && c->f_lds_top;
            bool split = true;
            if (const char* e = getenv("RAOCP_DYN_SPLIT")) split = atoi(e) != 0;
            size_t up = 0, down = 0;  // doubles
            raocp::FuseArg& fa = c->fuse;
            memset(&fa, 0, sizeof(fa));
            for (size_t k = 0; fz && k < c->tiers.size(); ++k) {
                const auto& tp = c->tiers[k];
                const int L = tp.s1 - tp.s0;
                const int above = k == 0 ? 1 : c->tiers[k - 1].nsub;
                const int r = tp.nsub / above;
                const int per_parent = k == 0 ? stage_n(c->cut) : c->tiers[k - 1].ta.cnt[c->tiers[k - 1].s1 - c->tiers[k - 1].s0];
                fz = fz && tp.ta.regular && tp.fm != 0 && r >= 2 && r * above == tp.nsub && r == per_parent;
                if (!fz) break;
                raocp::FuseTier& ft = fa.t[k];
                size_t nnl = 0;
                for (int l = 0; l < L; ++l) nnl += tp.ta.cnt[l];
                const size_t nall = nnl + tp.ta.cnt[L];
                const int c0 = cp[tp.s0], c1 = cp[tp.s1], p0 = pp[c0], p1 = pp[c1];
                size_t npl = p1 - p0;
                if (tp.fm == 2) {
                    npl = 0;
                    for (int l = 0; l < L; ++l) npl = std::max<size_t>(npl, tp.ta.pl0[l + 1] - tp.ta.pl0[l]);
                }
                ft.s0 = tp.s0;
                ft.s1 = tp.s1;
                ft.r = r;
                ft.c0 = c0;
                ft.c1 = c1;
                ft.p0 = p0;
                ft.p1 = p1;
                ft.maxch = tp.maxch;
                ft.fm = tp.fm;
                ft.fold = tp.fold;
                ft.nnl = (int)nnl;
                ft.ngroups = above;
                ft.ta = tp.ta;
                ft.ta.boff = 0;
                const size_t back = (tp.fold ? (size_t)(p1 - p0) * W1 : c->nkind * W1) + (c1 - c0) * RG1 + nall * KP +
                                    nnl * NUP + (tp.fold ? 0 : raocp::rup(tp.maxch * PS, 2)) + recs(nnl + nall - 1);
                const size_t fwd = (c1 - c0) * KM1 + npl * F1 + recs(nnl + nall - 1);
                up = std::max(up, back);
                down = std::max(down, (size_t)raocp::rup((int)(nnl * KF), 2) + fwd);
            }
            if (fz) {  // the top's backward (k_dyn_up) and forward (k_dyn_down) layouts
                const size_t T = c->stage_ptr[c->cut], nb = stage_n(c->cut);
                const int c1 = cp[c->cut], p1 = pp[c1];
                up = std::max(up, (c->fold_top ? (size_t)p1 * W1 : c->nkind * W1) + c1 * RG1 + T * KP + nb * KP + T * NUP +
                                      T * KF + (c->fold_top ? 0 : raocp::rup(c->maxch_top * PS, 2)) + recs(T + T + nb - 1));
                down = std::max(down, c1 * KM1 + (c->f_lds_top ? (size_t)p1 * F1 : 0) + T * KF + recs(T + T + nb - 1));
                c->lds_up = 8 * up;
                c->lds_down = 8 * down;
                split = split && c->lds_up <= kLds && c->lds_down <= kLds;
            }
            if (fz && split) {
                fa.K = (int)c->tiers.size();
                long grid = 2;  // the top and the deferred stopping test's workgroup
                for (const auto& tp : c->tiers) grid += tp.nsub;
                int pu = 0, pd = 0;
                dispatch(nx, nu, SplitOcc{}, c, &pu, &pd);
                c->dyn_split = pu > 0 && pd > 0 && grid <= (long)n_cus * std::min(pu, pd);
            }
            if (c->dyn_split) {
                size_t words = 2;
                for (int k = 0; k < fa.K; ++k) words += 2 * (size_t)fa.t[k].ngroups;
                if ((rc = c->alloc(&c->fuse_sync, words))) return bail(rc);
                if (hipMemset(c->fuse_sync, 0, words * sizeof(unsigned)) != hipSuccess)
                    return bail(fail(RAOCP_ERR_HIP, "hipMemset failed"));
                c->fuse_words = words;
                fa.epoch = c->fuse_sync;
                fa.err = (int*)(c->fuse_sync + 1);
                unsigned* w = c->fuse_sync + 2;
                for (int k = 0; k < fa.K; ++k) {
                    fa.t[k].cnt = w;
                    fa.t[k].flag = w + fa.t[k].ngroups;
                    w += 2 * (size_t)fa.t[k].ngroups;
                }
                fa.s = c->cut;
                fa.T = c->stage_ptr[c->cut];
                fa.nb = stage_n(c->cut);
                fa.c1 = cp[c->cut];
                fa.p1 = pp[fa.c1];
                fa.maxch_top = c->maxch_top;
                fa.fold_top = c->fold_top;
                long long ms = 1000;  // a wait normally lasts tens of microseconds
                if (const char* e = getenv("RAOCP_FUSE_TIMEOUT_MS")) ms = std::max(1, atoi(e));
                fa.timeout = ms * 100000LL;  // 100 MHz ticks
            }
        }
    }

    // ---- node-block CP kernels (raocp_cp.hip): records, block tables, block sizes
    {
        std::vector<int>& pos7 = c->h_pos7;
        std::vector<int>& pos14 = c->h_pos14;
        pos7.assign(m + 1, 0);
        pos14.assign(n - m + 1, 0);
        {
            int o = D.E7;
            for (int i = 0; i < m; ++i) { pos7[i] = o; o += e7off[i] >= 0 ? nx + nu : 1; }
            pos7[m] = o;
            o = D.E14 + m;  // the E14 segment has one placeholder per nonleaf node first
            for (int l = m; l < n; ++l) { pos14[l - m] = o; o += e14off[l - m] >= 0 ? nx : 1; }
            pos14[n - m] = o;
        }
        c->h_yrel = yrel;
        c->h_chs.assign(t->ch_start, t->ch_start + m);
        c->h_nch.assign(t->nch, t->nch + m);
        c->h_isq.assign(pr->i_sq, pr->i_sq + n);
        c->h_isr.assign(pr->i_sr, pr->i_sr + n);
        c->h_isp.assign(pr->i_sp, pr->i_sp + n);
        c->n_sq = pr->n_sq;
        c->n_sr = pr->n_sr;
        c->n_sp = pr->n_sp;
        c->nbn = nbn;
        c->nbl = nbl;
        std::vector<raocp::Rec> frec(m), lrec(n - m);
        for (int i = 0; i < m; ++i) frec[i] = raocp::Rec{yrel[i], t->nch[i], t->ch_start[i], e7off[i]};
        for (int l = m; l < n; ++l) lrec[l - m] = raocp::Rec{pr->i_sp[l], pr->i_box_l[l] >= 0 ? pr->i_box_l[l] : 0, e14off[l - m], 0};
        D.nBnl = nbn;
        D.nBl = nbl;
        if ((rc = c->upload_vec(&D.frec, frec)) || (rc = c->upload_vec(&D.lrec, lrec))) return bail(rc);
        // block sizes: about 256 family and 256 leaf blocks, within the LDS budget
        const long kCpLds = 64 * 1024 / 8;  // doubles: keeps >= 2 blocks per CU
        // family blocks of one k_cpp lane chunk (kBlock / (nx + nu + cmax + 1) parents: the
        // chunks of a block run one after the other; measured +3.7 % it/s at config 2 over
        // 256 blocks of 16 parents), leaf blocks of ~1/256 of the leaves
        int FB = std::max(1, std::min((m + 255) / 256, kBlock / (nx + nu + cmax + 1))),
            LB = std::max(1, (n - m + 255) / 256);
        const std::vector<std::pair<int, int>> allp{{0, m}}, alll{{m, n}};
        while (FB > 1 && cp_need(c, allp, {}, FB, LB) > kCpLds) FB = FB * 3 / 4;
        while (LB > 1 && cp_need(c, {}, alll, FB, LB) > kCpLds) LB = LB * 3 / 4;
        c->cp_FB = FB;
        c->cp_LB = LB;
        // MFMA CP kernels: W waves per block, one 16-node tile per wave and pass; W from the
        // tile count (about two blocks per CU), at least the lanes of a parent-row group
        if (nx > 64 || nu > 32)
            return bail(fail(RAOCP_ERR_ARG, "the CP kernels support nx <= 64 and nu <= 32"));
        {
            // four waves per block measured faster than one or two at configs 2 and 4 (the
            // per-block gather and barriers amortise over more tiles)
            int W = 4;
            const int lanes = std::max(2 * cmax + 2 + nx + nu, cmax + 1);
            W = std::max(W, (lanes + 63) / 64);
            if (W > 4) return bail(fail(RAOCP_ERR_ARG, "parent rows exceed a 256-lane CP block (branching too large)"));
            const double cavg = (double)(n - 1) / m;
            c->cp2_W = W;
            c->cp2_FB = std::max(1, (int)(16.0 * W / cavg + 1e-9));
            c->cp2_LB = 16 * W;
            // within 64 KB of LDS per block (two blocks per CU)
            const long kLds2 = 64 * 1024;
            while (c->cp2_FB > 1 && cp2_need(c, 0, m, c->cp2_FB, true) > kLds2)
                c->cp2_FB = std::min(c->cp2_FB - 1, c->cp2_FB * 3 / 4);
            while (c->cp2_LB > 1 && cp2_need(c, m, n, c->cp2_LB, false) > kLds2)
                c->cp2_LB = std::min(c->cp2_LB - 1, c->cp2_LB * 3 / 4);
            // small trees (config 2: 8,191 nodes, ~770 tiles) run the scalar kernels, which
            // spread a latency-bound launch over more lanes (measured 17.0 / 21.1 us vs 21.3 /
            // 23.6 us for k_cpd / k_cpp); from ~4k tiles the MFMA kernels win (config 4:
            // 200 / 196 us vs 210 / 318 us; config 3 464 vs 505 us per iteration)
            c->cp_v1 = (long)(n - 1 + 15) / 16 + (long)(n - m + 15) / 16 < 4096;
            if (c->f32) c->cp_v1 = false;  // fp32: the MFMA kernels unless blocks mix weight tables
            if (const char* e = getenv("RAOCP_CP_V1")) c->cp_v1 = atoi(e) != 0;
        }
        if ((rc = build_cp_blocks(c, allp, alll))) return bail(rc);
    }

    // ---- L / L^T node-range blocks (raocp_ell.hip): nonleaf and leaf ranges split evenly
    // over B blocks; B from the node count (64 nodes per block), raised until every block's LDS stage fits 64 KB
    {
        // measured (round-2 A/B of the block size): 512-thread blocks while the grid is one block per CU,
        // 256-thread blocks of 64 nodes once there are several per CU
        int per = 64;
        int thr = (n + per - 1) / per > 512 ? 256 : 512;
        c->ell_threads = thr;
        const int Bmax = std::max(1, std::max(m, n - m));
        int B = std::max(1, std::min(std::max(256, (n + per - 1) / per), Bmax));
        std::vector<raocp::Rec> tab;
        long need_l = 0, need_t = 0;
        // LDS doubles of one gathered range (raocp_ell.hip Gather): 16-B chunks, +1 for a
        // range that starts 8 B into its first chunk
        auto dbl = [](long cnt) { return 2 * ((cnt * 8 + 15) / 16 + 1); };
        auto rec = [](long cnt) { return 2 * cnt + 2; };
        for (;;) {
            tab.assign((size_t)B * raocp::kEllRecs, raocp::Rec{0, 0, 0, 0});
            need_l = need_t = 0;
            for (int b = 0; b < B; ++b) {
                raocp::Rec* T = tab.data() + (size_t)b * raocp::kEllRecs;
                const int i0 = (int)((int64_t)b * m / B), i1 = (int)((int64_t)(b + 1) * m / B);
                const int l0 = m + (int)((int64_t)b * (n - m) / B), l1 = m + (int)((int64_t)(b + 1) * (n - m) / B);
                int c0 = 0, c1 = 0, y0 = 0, y1 = 0;
                if (i1 > i0) {
                    c0 = t->ch_start[i0];
                    c1 = t->ch_start[i1 - 1] + t->nch[i1 - 1];
                    y0 = yrel[i0];
                    y1 = yrel[i1 - 1] + 2 * t->nch[i1 - 1] + 1;
                }
                const int e7a = c->h_pos7[i0], e7b = c->h_pos7[i1];
                const int e14a = c->h_pos14[l0 - m], e14b = c->h_pos14[l1 - m];
                T[0] = raocp::Rec{i0, i1, c0, c1};
                T[1] = raocp::Rec{l0, l1, y0, y1};
                T[2] = raocp::Rec{e7a, e7b, e14a, e14b};
                // the block's table index of each product family, -1 when its nodes differ
                auto uni = [](const int* idx, int a, int b) {
                    if (b <= a) return -1;
                    for (int q = a + 1; q < b; ++q)
                        if (idx[q] != idx[a]) return -1;
                    return idx[a];
                };
                // regular block (k_ell_t's per-parent MFMA tiles): every parent has the same
                // child count c <= 4 and its children are c0 + (i - i0) c + [0, c)
                int creg = 0;
                if (i1 > i0 && t->nch[i0] >= 1 && t->nch[i0] <= 4) {
                    creg = t->nch[i0];
                    for (int q = i0; q < i1 && creg; ++q)
                        if (t->nch[q] != creg || t->ch_start[q] != c0 + (q - i0) * creg) creg = 0;
                }
                T[3] = raocp::Rec{uni(pr->i_sq, c0, c1), uni(pr->i_sr, c0, c1), uni(pr->i_sp, l0, l1), creg};
                const long np = i1 - i0, nc = c1 - c0, nl = l1 - l0, Y = y1 - y0;
                need_l = std::max(need_l, dbl(np * nx) + dbl(np * nu) + dbl(Y) + dbl(np) + 2 * dbl(nc) + rec(np) +
                                              rec(nc) + dbl(nl * nx) + dbl(nl) + rec(nl));
                need_t = std::max(need_t, dbl(nc * nx) + dbl(nc * nu) + dbl(e7b - e7a) + dbl(Y) + dbl(np) +
                                              3 * dbl(nc) + rec(np) + rec(nc) + dbl(nl * nx) + dbl(e14b - e14a) +
                                              2 * dbl(nl) + rec(nl) + nc * (nx + nu));
            }
            if (std::max(need_l, need_t) * 8 <= 64 * 1024 || B >= Bmax) break;
            B = std::min(Bmax, B * 2);
        }
        if (std::max(need_l, need_t) * 8 > 64 * 1024)
            return bail(fail(RAOCP_ERR_ARG, "L block does not fit LDS (node dimension too large)"));
        if ((rc = c->upload_vec(&D.ell_tab, tab))) return bail(rc);
        c->ell_nb = B;
        c->ell_lds = need_l * 8;
        c->ellt_lds = need_t * 8;
    }

    // ---- iterate and work buffers
    for (int b = 0; b < 3; ++b)
        if ((rc = c->alloc(&c->Z[b], c->P))) return bail(rc);
    for (int b = 0; b < 2; ++b)
        if ((rc = c->alloc(&c->E[b], c->D))) return bail(rc);
    if ((rc = c->alloc(&c->XI2, c->D)) || (rc = c->alloc(&c->q, (size_t)n * c->KP)) || (rc = c->alloc(&c->d, (size_t)m * nu + 2)) ||
        (rc = c->alloc(&c->gXQ, (size_t)n * c->KP)) || (rc = c->alloc(&c->gU, (size_t)m * c->NUP)) ||
        (rc = c->alloc(&c->gXD, (size_t)m * c->KF)) || (rc = c->alloc(&c->gP, (size_t)n * c->PS)) ||
        (rc = c->alloc(&c->x0, nx)) || (rc = c->alloc(&c->ctl, 1)) || (rc = c->alloc(&c->tmpP, c->P)) ||
        (rc = c->alloc(&c->tmpD, c->D)) || (rc = c->alloc(&c->part, 1024)) || (rc = c->alloc(&c->scal, 8)))
        return bail(rc);
    if (hipHostMalloc((void**)&c->h_ctl, sizeof(Ctl), 0) != hipSuccess) return bail(fail(RAOCP_ERR_HIP, "hipHostMalloc"));
    if (hipHostMalloc((void**)&c->h_pub, sizeof(raocp::CtlPub), hipHostMallocCoherent) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->d_pub, c->h_pub, 0) != hipSuccess)
        return bail(fail(RAOCP_ERR_HIP, "hipHostMalloc"));
    memset(c->h_pub, 0, sizeof(raocp::CtlPub));
    {
        double* zp = nullptr;
        if ((rc = c->alloc(&zp, 16))) return bail(rc);
        if (hipMemset(zp, 0, 16 * sizeof(double)) != hipSuccess) return bail(fail(RAOCP_ERR_HIP, "memset"));
        c->dev.zpage = zp;
    }
    {
        const int g_dual = groups(nx + nu + 2, n - 1).blocks + groups(2 * cmax + 2 + nx + nu, m).blocks +
                           groups(2 * nx + 2, n - m).blocks;
        const int g_primal = groups(nx + nu + cmax + 1, m).blocks + groups(nx, n - m).blocks;
        c->red_rows = std::max(std::max(g_dual, g_primal), std::max(c->cp_nbF + c->cp_nbL, c->cp2_nbF + c->cp2_nbL));
        if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return bail(rc);
        if (hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)) != hipSuccess)
            return bail(fail(RAOCP_ERR_HIP, "memset"));
    }
    for (int b = 0; b < 3; ++b)
        if (hipMemset(c->Z[b], 0, c->P * sizeof(double)) != hipSuccess) return bail(fail(RAOCP_ERR_HIP, "memset"));
    for (int b = 0; b < 2; ++b)
        if (hipMemset(c->E[b], 0, c->D * sizeof(double)) != hipSuccess) return bail(fail(RAOCP_ERR_HIP, "memset"));
    if (hipMemset(c->XI2, 0, c->D * sizeof(double)) != hipSuccess || hipMemset(c->ctl, 0, sizeof(Ctl)) != hipSuccess ||
        hipMemset(c->q, 0, (size_t)n * c->KP * sizeof(double)) != hipSuccess ||
        hipMemset(c->gP, 0, (size_t)n * c->PS * sizeof(double)) != hipSuccess ||
        hipMemset(c->d, 0, (size_t)m * nu * sizeof(double)) != hipSuccess)
        return bail(fail(RAOCP_ERR_HIP, "memset"));
    c->bufs = raocp::Bufs{c->Z[0], c->Z[1], c->Z[2], c->E[0], c->E[1]};
    // RAOCP_EAGER=1: CP iterations launched one kernel at a time instead of the captured
    // graph (for rocprofv3 --kernel-trace --stats, which crashes replaying this graph)
    if (const char* e = getenv("RAOCP_EAGER")) c->eager = atoi(e) != 0;
    c->cur_z = c->Z[0];
    c->cur_e = c->E[0];
    c->dev.dyn_rot = 1;  // the tier kernels rotate the first wave of each staged range
    if ((rc = ensure_hist(c, 1024))) return bail(rc);

    {
        // L by streaming wave tasks (raocp_ell3.hip): compile-time sizes, and one sqrtQ / sqrtR
        // table over all children and one sqrtPf over all leaves (the waves keep them in registers)
        bool uni = (nx == 20 && nu == 8) || (nx == 32 && nu == 12) || (nx == 64 && nu == 16);
        for (int j = 2; j < n && uni; ++j)
            if (pr->i_sq[j] != pr->i_sq[1] || pr->i_sr[j] != pr->i_sr[1]) uni = false;
        for (int l = m + 1; l < n && uni; ++l)
            if (pr->i_sp[l] != pr->i_sp[m]) uni = false;
        // measured (tools/ell3_check.py): config 2 fp64 4.9 vs 5.5 us, config 5 fp32 210 vs
        // 265 us, config 4 fp64 equal; RAOCP_ELL3=0 keeps the block kernels
        c->ell3 = uni;
        if (const char* e = getenv("RAOCP_ELL3")) c->ell3 = uni && atoi(e) != 0;
        const long tasks = (long)(n - 1 + 15) / 16 + (n - m + 15) / 16 + ((long)m * (nx + nu) + (c->dev.T0 - c->dev.Y0) + m + 63) / 64;
        // grid sweep (profiles/r02_v2/ab_order.log): config 4 fp64 best at 2,048 blocks (25.3 us
        // vs 26.7 at 4,096), config 5 fp32 at 1,024 (116 vs 137 us at 4,096)
        c->ell3_grid = (int)std::max(1L, std::min((tasks + 3) / 4, c->f32 ? 1024L : 2048L));
        // L^T by streaming wave tasks: additionally one branching factor C <= 4 over all
        // nonleaf nodes (children 1 + C i .., y_i at (2C + 1) i); RAOCP_ELLT3=0 keeps k_ell_t
        int C = m > 0 ? t->nch[0] : 0;
        bool reg = uni && C >= 1 && C <= 4;
        for (int i = 0; i < m && reg; ++i)
            if (t->nch[i] != C || t->ch_start[i] != 1 + C * i) reg = false;
        c->unif_C = reg ? C : 0;
        {
            int nb = 0, lb = 0;
            for (int i = 0; i < m; ++i) nb += pr->i_box_nl[i] >= 0;
            for (int l = m; l < n; ++l) lb += pr->i_box_l[l] >= 0;
            c->box_mode = (nb == m ? 1 : nb == 0 ? 2 : 0) | ((lb == n - m ? 1 : lb == 0 ? 2 : 0) << 2);
            // RAOCP_BOX_MODE=0 forces the offset tables (always valid); any other value must
            // agree with the computed pattern (a forced "all boxed" on a tree with unboxed nodes
            // would compute eta7 / eta14 offsets for slots that do not exist)
            if (const char* e = getenv("RAOCP_BOX_MODE")) {
                const int v = atoi(e);
                if (v != 0 && v != c->box_mode)
                    return bail(fail(RAOCP_ERR_ARG, "RAOCP_BOX_MODE=" + std::to_string(v) + " disagrees with the tree's box "
                                                    "pattern (" + std::to_string(c->box_mode) + "); only 0 may override"));
                c->box_mode = v;
            }
        }
        if (const char* e = getenv("RAOCP_ELLT3")) reg = reg && atoi(e) != 0;
        c->ellt3_C = reg ? C : 0;
        const long tasks_t = (long)(m + 4 * (4 / std::max(C, 1)) - 1) / (4 * (4 / std::max(C, 1))) + (n - m + 15) / 16 +
                             ((long)(c->dev.T0 - c->dev.Y0) + 2L * n - 1 + 63) / 64;
        // grid sweep (profiles/r02_v4/ab_grid.log): 1,536 blocks best at config 4 fp64 (24.0 us
        // vs 24.9 at 4,096, 28.0 at 1,024) and config 5 fp32 (109.4 vs 111.1 at 2,048)
        c->ellt3_grid = (int)std::max(1L, std::min((tasks_t + 3) / 4, 1536L));
        // the fused CP iteration (raocp_cp3.hip): uniform branching and tables (unif_C), the
        // compile-time sizes; RAOCP_CP3=0 keeps k_cpd* + k_cpp*
        c->cp3 = c->unif_C > 0 && c->ell3 && cp3_sizes(c->f32, nx, nu);
        if (const char* e = getenv("RAOCP_CP3")) c->cp3 = c->cp3 && atoi(e) != 0;
        if (c->cp3) {
            c->cp3_mL = c->stage_ptr[N - 1];
            const long ptiles = (long)(m - c->cp3_mL + 15) / 16 + (c->cp3_mL + 15) / 16;
            // small trees (latency-bound: config 2 has 256 family tiles, one wave each) split
            // the leaves into tasks of their own: twice the waves, half the longest chain
            c->cp3_split = ptiles < 1024;
            if (const char* e = getenv("RAOCP_CP3_SPLIT")) c->cp3_split = atoi(e) != 0;
            // leaf-parent tiles first (heavier), then the rest
            const long tiles = cp3_tasks(c->cp3_ta, {{c->cp3_mL, m}, {0, c->cp3_mL}}, m, c->cp3_split ? n : m,
                                         c->cp3_split, c->cp3_mL);
            if (tiles < 0) return bail(fail(RAOCP_ERR_ARG, "k_cp3 task list exceeds its parent-range slots"));
            c->cp3_grid = cp3_grid_of(tiles);
            if (c->cp3_grid > c->red_rows) {
                c->red_rows = c->cp3_grid;
                if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return bail(rc);
                if (hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)) != hipSuccess)
                    return bail(fail(RAOCP_ERR_HIP, "memset"));
            }
            c->cp_rows = c->cp3_grid;
            if ((rc = cp3_image(c))) return bail(rc);
            c->cp6 = raocp::cp6_supported(c->f32, nx, nu, c->unif_C, c->box_mode, c->dev.nBnl, c->dev.nBl);
            if (const char* e = getenv("RAOCP_CP6")) c->cp6 = c->cp6 && atoi(e) != 0;
            c->cp4 = !c->cp6 && raocp::cp4_supported(c->f32, nx, nu, c->unif_C, c->box_mode);
            if (const char* e = getenv("RAOCP_CP4")) c->cp4 = c->cp4 && atoi(e) != 0;
            if (c->cp4) {  // k_cp4: cp4_wpb waves per workgroup, the same waves over more CUs
                if (const char* e = getenv("RAOCP_CP4_HELPER")) c->cp4_wpb = atoi(e) ? 2 : 1;
                c->cp3_grid = (int)std::max(1L, std::min(tiles, 8192L));  // one task per workgroup
                if (c->cp3_grid > c->red_rows) {
                    c->red_rows = c->cp3_grid;
                    if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return bail(rc);
                    if (hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)) != hipSuccess)
                        return bail(fail(RAOCP_ERR_HIP, "memset"));
                }
                c->cp_rows = c->cp3_grid;
            }
            // k_cp5: the leaf tiles and the family tiles as two launches with small register
            // files (configs 3, 4, 5; k_cp4 keeps config 2)
            c->cp5 = !c->cp4 && !c->cp6 && raocp::cp5_supported(c->f32, nx, nu, c->unif_C, c->box_mode, c->dev.nBnl, c->dev.nBl);
            if (const char* e = getenv("RAOCP_CP5")) c->cp5 = c->cp5 && atoi(e) != 0;
            if (c->cp6) {
                if (cp3_tasks(c->cp5_tk, {{c->cp3_mL, m}, {0, c->cp3_mL}}, 0, 0, 1, c->cp3_mL) < 0)
                    return bail(fail(RAOCP_ERR_ARG, "k_cp6 task list exceeds its parent-range slots"));
                c->cp6_grid = raocp::cp6_grid(c->cp5_tk);
                if (const char* e = getenv("RAOCP_CP6_GRID")) c->cp6_grid = std::max(1, atoi(e));
                c->cp_rows = raocp::cp6_rows(c->cp6_grid);
                if (c->cp_rows > c->red_rows) {
                    c->red_rows = c->cp_rows;
                    if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return bail(rc);
                    if (hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)) != hipSuccess)
                        return bail(fail(RAOCP_ERR_HIP, "memset"));
                }
            }
            if (c->cp5) {
                if (cp3_tasks(c->cp5_tk, {{c->cp3_mL, m}, {0, c->cp3_mL}}, 0, 0, 1, c->cp3_mL) < 0)
                    return bail(fail(RAOCP_ERR_ARG, "k_cp5 task list exceeds its parent-range slots"));
                // the leaf launch's form is read here, per context (a later context with another
                // RAOCP_CP5_LPF gets its own)
                c->cp5_lpf = raocp::cp5_leaf_pf_default(c->f32);
                if (const char* e = getenv("RAOCP_CP5_LPF")) c->cp5_lpf = atoi(e) != 0;
                cp3_tasks(c->cp5_et, {{0, m}}, 0, 0, 1, 0, 64);
                c->cp5_gl = raocp::cp5_leaf_grid(c->cp5_et, m, n, c->cp5_lpf);
                // k_cp5_fams (profiles/r05/cp_time_fams*.log: config 4 100.7 -> 90.9 us, config 5
                // 335.3 -> 334.8 us, config 3 60.9 -> 57.4 us with the compacted slot sums)
                c->cp5_gf = raocp::cp5_fam_grid(c->cp5_tk);
                if (const char* e = getenv("RAOCP_CP5_LGRID")) c->cp5_gl = std::max(1, atoi(e));
                if (const char* e = getenv("RAOCP_CP5_FGRID")) c->cp5_gf = std::max(1, atoi(e));
                c->cp_rows = raocp::cp5_rows(c->cp5_gl, c->cp5_gf);
                if (c->cp_rows > c->red_rows) {
                    c->red_rows = c->cp_rows;
                    if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return bail(rc);
                    if (hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)) != hipSuccess)
                        return bail(fail(RAOCP_ERR_HIP, "memset"));
                }
            }
        }
    }
    if ((rc = drc_setup(c))) return bail(rc);
    if (const char* e = getenv("RAOCP_DEFER_CHECK")) c->no_defer_check = atoi(e) == 0;
    c->drp.zpage = c->dev.zpage;
    c->drp.x0 = c->x0;
    *out = c;
    return RAOCP_OK;
}

void raocp_ctx_destroy(raocp_ctx* c) {
    if (!c) return;
    DevGuard dg_(c);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    if (c->comm && g_rccl.destroy) (void)g_rccl.destroy((ncclComm_t)c->comm);
    drop_graphs(c);
    if (c->ev0) (void)hipEventDestroy(c->ev0);
    if (c->ev1) (void)hipEventDestroy(c->ev1);
    for (void* p : c->allocs) (void)hipFree(p);
    if (c->h_ctl) (void)hipHostFree(c->h_ctl);
    if (c->h_pub) (void)hipHostFree(c->h_pub);
    if (c->stream) (void)hipStreamDestroy(c->stream);
    delete c;
}

int raocp_sizes(raocp_ctx* c, int64_t* P, int64_t* D) {
    DevGuard dg_(c);
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    if (P) *P = c->P;
    if (D) *D = c->D;
    return RAOCP_OK;
}

int raocp_ell(raocp_ctx* c, const double* z, double* eta, int flags) {
    DevGuard dg_(c);
    if (!c || !z || !eta) return fail(RAOCP_ERR_ARG, "null argument");
    int rc;
    if (flags & RAOCP_DEVICE_PTR) {
        launch_ell(c, z, eta);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->stream));
        return RAOCP_OK;
    }
    if ((rc = copy_in(c, c->tmpP, z, c->P, 0)) || (rc = copy_in(c, c->tmpD, eta, c->D, 0))) return rc;
    launch_ell(c, c->tmpP, c->tmpD);
    HIPCHK(hipGetLastError());
    return copy_out(c, eta, c->tmpD, c->D, 0);
}

int raocp_ell_t(raocp_ctx* c, const double* eta, double* z, int flags) {
    DevGuard dg_(c);
    if (!c || !z || !eta) return fail(RAOCP_ERR_ARG, "null argument");
    int rc;
    if (flags & RAOCP_DEVICE_PTR) {
        launch_ell_t(c, eta, z);
        HIPCHK(hipGetLastError());
        HIPCHK(hipStreamSynchronize(c->stream));
        return RAOCP_OK;
    }
    if ((rc = copy_in(c, c->tmpD, eta, c->D, 0)) || (rc = copy_in(c, c->tmpP, z, c->P, 0))) return rc;
    launch_ell_t(c, c->tmpD, c->tmpP);
    HIPCHK(hipGetLastError());
    return copy_out(c, z, c->tmpP, c->P, 0);
}

int raocp_set_primal(raocp_ctx* c, const double* z, int flags) {
    DevGuard dg_(c);
    if (!c || !z) return fail(RAOCP_ERR_ARG, "null argument");
    int rc = copy_in(c, c->cur_z, z, c->P, flags);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}
int raocp_get_primal(raocp_ctx* c, double* z, int flags) {
    DevGuard dg_(c);
    if (!c || !z) return fail(RAOCP_ERR_ARG, "null argument");
    return copy_out(c, z, c->cur_z, c->P, flags);
}
int raocp_set_dual(raocp_ctx* c, const double* e, int flags) {
    DevGuard dg_(c);
    if (!c || !e) return fail(RAOCP_ERR_ARG, "null argument");
    int rc = copy_in(c, c->cur_e, e, c->D, flags);
    if (rc) return rc;
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}
int raocp_get_dual(raocp_ctx* c, double* e, int flags) {
    DevGuard dg_(c);
    if (!c || !e) return fail(RAOCP_ERR_ARG, "null argument");
    return copy_out(c, e, c->cur_e, c->D, flags);
}

// the cold start of Solver.chock on a fresh Cache: primal and dual zero on the device
int raocp_reset_iterate(raocp_ctx* c) {
    DevGuard dg_(c);
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    HIPCHK(hipMemsetAsync(c->cur_z, 0, c->P * c->wsz, c->stream));
    HIPCHK(hipMemsetAsync(c->cur_e, 0, c->D * c->wsz, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

int raocp_kernel_info(raocp_ctx* c, int op, char* buf, int cap) {
    DevGuard dg_(c);
    if (!c || !buf || cap < 1) return fail(RAOCP_ERR_ARG, "bad argument");
    const std::string s = kernel_name(c, op);
    if (s.empty() && op != 11 && op != 12) return fail(RAOCP_ERR_ARG, "unknown op " + std::to_string(op));
    snprintf(buf, (size_t)cap, "%s", s.c_str());
    return RAOCP_OK;
}

int raocp_set_initial_state(raocp_ctx* c, const double* x0) {
    DevGuard dg_(c);
    if (!c || !x0) return fail(RAOCP_ERR_ARG, "null argument");
    c->h_x0.assign(x0, x0 + c->nx);
    if (c->f32) {
        const std::vector<float> f(x0, x0 + c->nx);
        HIPCHK(hipMemcpy(c->x0, f.data(), c->nx * sizeof(float), hipMemcpyHostToDevice));
    } else {
        HIPCHK(hipMemcpy(c->x0, x0, c->nx * sizeof(double), hipMemcpyHostToDevice));
    }
    c->has_x0 = true;
    return RAOCP_OK;
}

int raocp_relax_s0(raocp_ctx* c, double alpha) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    raocp::k_relax_s0<<<1, 1, 0, c->stream>>>(c->dev, c->cur_z, alpha);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

int raocp_project_on_dynamics(raocp_ctx* c) {
    DevGuard dg_(c);
    SweepLock sl_(c);
    if (c && c->f32 && !c->dyn32) return fail(RAOCP_ERR_ARG, "fp32 context without a dynamics plan");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    if (!c->has_x0) return fail(RAOCP_ERR_STATE, "initial state not cached (call cache_initial_state first)");
    const raocp::Bufs solo{c->cur_z, c->cur_z, c->cur_z, c->cur_e, c->cur_e};
    launch_dynamics(c, solo, 0, nullptr);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return fuse_err(c);
}

int raocp_project_on_kernel(raocp_ctx* c) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    const Launch L = groups(c->cmax + 1, c->m);
    raocp::k_kernel_proj<<<L.blocks, kBlock, 0, c->stream>>>(c->dev, c->cur_z);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

int raocp_prox_f(raocp_ctx* c, double alpha) {
    DevGuard dg_(c);
    int rc;
    if ((rc = raocp_relax_s0(c, alpha)) || (rc = raocp_project_on_dynamics(c)) || (rc = raocp_project_on_kernel(c)))
        return rc;
    return RAOCP_OK;
}

int raocp_prox_gconj(raocp_ctx* c, double alpha) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    int rc = set_ctl_alpha(c, alpha);
    if (rc) return rc;
    HIPCHK(hipMemsetAsync(&c->ctl->flags, 0, sizeof(int), c->stream));
    launch_cp_dual(c, false, c->cur_e);
    if (c->n_ph) raocp::k_zero_idx<<<cdiv(c->n_ph, kBlock), kBlock, 0, c->stream>>>(c->cur_e, c->ph, c->n_ph);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->h_ctl, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int fe = fuse_err(c)) return fe;
    if (c->h_ctl->flags & 1) return fail(RAOCP_ERR_NAN_IN_BOX, "Rectangle constraint - 'nan' value cannot be constrained");
    return RAOCP_OK;
}

int raocp_dual_scale(raocp_ctx* c, double alpha) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    raocp::k_div<<<std::min(2048, cdiv((int)c->D, kBlock)), kBlock, 0, c->stream>>>(c->cur_e, alpha, (int)c->D);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

int raocp_dual_add_halves(raocp_ctx* c) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    const Dev& D = c->dev;
    const int nb = cdiv(c->n, kBlock);
    raocp::k_add_const<<<nb, kBlock, 0, c->stream>>>(c->cur_e, -0.5, D.E5, D.E6);
    raocp::k_add_const<<<nb, kBlock, 0, c->stream>>>(c->cur_e, 0.5, D.E6, D.E7);
    raocp::k_add_const<<<nb, kBlock, 0, c->stream>>>(c->cur_e, -0.5, D.E12, D.E13);
    raocp::k_add_const<<<nb, kBlock, 0, c->stream>>>(c->cur_e, 0.5, D.E13, D.E14);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

int raocp_dual_project(raocp_ctx* c, int which) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c) return fail(RAOCP_ERR_ARG, "null context");
    HIPCHK(hipMemsetAsync(&c->ctl->flags, 0, sizeof(int), c->stream));
    const int mode = (which & 1 ? raocp::kDualNonleaf : 0) | (which & 2 ? raocp::kDualLeaf : 0);
    launch_cp_dual(c, false, c->cur_e, mode);
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(c->h_ctl, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    if (int fe = fuse_err(c)) return fe;
    if (c->h_ctl->flags & 1) return fail(RAOCP_ERR_NAN_IN_BOX, "Rectangle constraint - 'nan' value cannot be constrained");
    return RAOCP_OK;
}

int raocp_dual_moreau(raocp_ctx* c, double alpha, const double* modified) {
    DevGuard dg_(c);
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c || !modified) return fail(RAOCP_ERR_ARG, "null argument");
    int rc = copy_in(c, c->tmpD, modified, c->D, 0);
    if (rc) return rc;
    raocp::k_moreau<<<std::min(2048, cdiv((int)c->D, kBlock)), kBlock, 0, c->stream>>>(c->cur_e, c->tmpD, alpha,
                                                                                        (int)c->D);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

// ---- step size: Lanczos on L'L with device mat-vecs (replaces ARPACK, solver.py:109-118)
static double tridiag_max_eig(const std::vector<double>& a, const std::vector<double>& b) {
    // largest eigenvalue of the symmetric tridiagonal (a diag, b off-diag) by Sturm bisection
    const int k = (int)a.size();
    double lo = a[0], hi = a[0];
    for (int i = 0; i < k; ++i) {
        const double r = (i > 0 ? std::fabs(b[i - 1]) : 0.0) + (i + 1 < k ? std::fabs(b[i]) : 0.0);
        lo = std::min(lo, a[i] - r);
        hi = std::max(hi, a[i] + r);
    }
    auto count_greater = [&](double x) {
        int cnt = 0;
        double dd = 1.0;
        for (int i = 0; i < k; ++i) {
            const double bb = i > 0 ? b[i - 1] * b[i - 1] : 0.0;
            dd = (a[i] - x) - (i > 0 ? bb / dd : 0.0);
            if (dd == 0.0) dd = -1e-300;
            if (dd > 0) ++cnt;
        }
        return cnt;  // number of eigenvalues > x
    };
    for (int it = 0; it < 200 && hi - lo > 1e-16 * std::max(1.0, std::fabs(hi)); ++it) {
        const double mid = 0.5 * (lo + hi);
        if (count_greater(mid) >= 1) lo = mid;
        else hi = mid;
    }
    return 0.5 * (lo + hi);
}

static int dev_dot(raocp_ctx* c, const double* a, const double* b, int n, double* out) {
    const int nb = std::min(1024, cdiv(n, kBlock));
    if (c->f32) raocp::k_dot_partial<float><<<nb, kBlock, 0, c->stream>>>((const float*)a, (const float*)b, n, c->part);
    else raocp::k_dot_partial<double><<<nb, kBlock, 0, c->stream>>>(a, b, n, c->part);
    raocp::k_dot_final<<<1, kBlock, 0, c->stream>>>(c->part, nb, c->scal);
    HIPCHK(hipMemcpyAsync(out, c->scal, sizeof(double), hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
    return RAOCP_OK;
}

static void dev_scale_copy(raocp_ctx* c, int nb, double sc, const double* x, double* y, int n) {
    if (c->f32) raocp::k_scale_copy<float><<<nb, kBlock, 0, c->stream>>>(sc, (const float*)x, (float*)y, n);
    else raocp::k_scale_copy<double><<<nb, kBlock, 0, c->stream>>>(sc, x, y, n);
}
static void dev_axpby(raocp_ctx* c, int nb, double a, const double* x, double b, double* y, int n) {
    if (c->f32) raocp::k_axpby<float><<<nb, kBlock, 0, c->stream>>>(a, (const float*)x, b, (float*)y, n);
    else raocp::k_axpby<double><<<nb, kBlock, 0, c->stream>>>(a, x, b, y, n);
}

int raocp_step_size(raocp_ctx* c, double* lambda_max, int max_it, double rtol) {
    DevGuard dg_(c);
    if (!c || !lambda_max) return fail(RAOCP_ERR_ARG, "null argument");
    if (max_it <= 0) max_it = 300;
    if (rtol <= 0) rtol = 1e-14;
    const int P = (int)c->P;
    max_it = std::min<int64_t>(max_it, c->P);
    double *v = nullptr, *vprev = nullptr, *w = nullptr, *eta = nullptr;
    int rc;
    if ((rc = c->alloc(&v, P)) || (rc = c->alloc(&vprev, P)) || (rc = c->alloc(&w, P)) || (rc = c->alloc(&eta, c->D)))
        return rc;
    std::vector<double> h(P);
    std::mt19937_64 gen(12345);
    std::normal_distribution<double> nd(0.0, 1.0);
    for (int i = 0; i < P; ++i) h[i] = nd(gen);
    h[c->dev.T0] = 0.0;  // tau_0 is outside the range of L'L (the reference's template keeps it 0)
    if ((rc = copy_in(c, v, h.data(), P, 0))) return rc;
    HIPCHK(hipMemsetAsync(vprev, 0, P * sizeof(double), c->stream));
    HIPCHK(hipMemsetAsync(w, 0, P * sizeof(double), c->stream));
    HIPCHK(hipMemsetAsync(eta, 0, c->D * sizeof(double), c->stream));
    const int nbv = std::min(2048, cdiv(P, kBlock));
    double nrm2;
    if ((rc = dev_dot(c, v, v, P, &nrm2))) return rc;
    dev_scale_copy(c, nbv, 1.0 / std::sqrt(nrm2), v, v, P);
    std::vector<double> al, be;
    double beta = 0.0, lam = 0.0, lam_prev = -1.0;
    int stable = 0;
    for (int j = 0; j < max_it; ++j) {
        launch_ell(c, v, eta);
        HIPCHK(hipMemsetAsync(w, 0, P * sizeof(double), c->stream));
        launch_ell_t(c, eta, w);          // w = L'L v (tau_0 = 0)
        dev_axpby(c, nbv, -beta, vprev, 1.0, w, P);
        double a;
        if ((rc = dev_dot(c, w, v, P, &a))) return rc;
        dev_axpby(c, nbv, -a, v, 1.0, w, P);
        double bb;
        if ((rc = dev_dot(c, w, w, P, &bb))) return rc;
        al.push_back(a);
        lam = tridiag_max_eig(al, be);
        beta = std::sqrt(bb);
        if (std::fabs(lam - lam_prev) <= rtol * std::fabs(lam)) {
            if (++stable >= 3) break;
        } else {
            stable = 0;
        }
        lam_prev = lam;
        if (beta <= 1e-300) break;
        be.push_back(beta);
        // vprev <- v ; v <- w / beta
        HIPCHK(hipMemcpyAsync(vprev, v, P * c->wsz, hipMemcpyDeviceToDevice, c->stream));
        dev_scale_copy(c, nbv, 1.0 / beta, w, v, P);
    }
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(c->stream));
    for (double* p : {v, vprev, w, eta}) {
        (void)hipFree(p);
        c->allocs.erase(std::remove(c->allocs.begin(), c->allocs.end(), (void*)p), c->allocs.end());
    }
    *lambda_max = lam;
    return RAOCP_OK;
}

int raocp_cp_run(raocp_ctx* c, const double* x0, int max_iters, double tol, double alpha, int* status, int* iters,
                 double* err_hist, double* delta_hist) {
    DevGuard dg_(c);
    SweepLock sl_(c);
    if (c && c->f32 && !c->dyn32) return fail(RAOCP_ERR_ARG, "fp32 CP loop unavailable: no fp32 dynamics plan");
    if (!c || !x0) return fail(RAOCP_ERR_ARG, "null argument");
    if (max_iters < 0) return fail(RAOCP_ERR_ARG, "max_iters must be >= 0");
    int rc;
    if ((rc = ensure_hist(c, (size_t)max_iters + 1))) return rc;
    if ((rc = raocp_set_initial_state(c, x0))) return rc;
    if ((rc = cp_init(c, x0, max_iters, tol, alpha, true))) return rc;
    {
        const int batch = kGraphBatch;
        if ((rc = ensure_graph(c, batch))) return rc;
        const bool pub = defer_check(c);
        for (;;) {
            if (pub) c->h_pub->ctl.final_k = -2;
            if ((rc = launch_batch(c, batch))) return rc;
            if (!pub) HIPCHK(hipMemcpyAsync(c->h_ctl, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
            HIPCHK(hipStreamSynchronize(c->stream));
            if (pub) *c->h_ctl = c->h_pub->ctl;  // published by the batch's last stopping test
            if (c->h_ctl->done) break;
        }
    }
    const int fk = c->h_ctl->final_k;
    std::vector<double> h((size_t)(fk + 1) * 6);
    HIPCHK(hipMemcpy(h.data(), c->hist, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int k = 0; k <= fk; ++k)
        for (int q = 0; q < 3; ++q) {
            if (err_hist) err_hist[k * 3 + q] = h[(size_t)k * 6 + q];
            if (delta_hist) delta_hist[k * 3 + q] = h[(size_t)k * 6 + 3 + q];
        }
    c->cur_z = c->Z[(fk + 1) % 3];
    c->cur_e = c->E[(fk + 1) % 2];
    if (iters) *iters = fk + 1;
    if (status) *status = fk < max_iters ? 0 : 1;
    if (int fe = fuse_err(c)) return fe;
    if (c->h_ctl->flags & 1) return fail(RAOCP_ERR_NAN_IN_BOX, "Rectangle constraint - 'nan' value cannot be constrained");
    return RAOCP_OK;
}

int raocp_cp_prepare(raocp_ctx* c, const double* x0, int iters, double alpha) {
    DevGuard dg_(c);
    if (c && c->f32 && !c->dyn32) return fail(RAOCP_ERR_ARG, "fp32 CP loop unavailable: no fp32 dynamics plan");
    if (!c || iters < 1) return fail(RAOCP_ERR_ARG, "bad argument");
    int rc;
    if ((rc = ensure_hist(c, (size_t)iters + 1))) return rc;
    if (iters / kGraphBatch && (rc = ensure_graph(c, kGraphBatch))) return rc;
    if (iters % kGraphBatch && (rc = ensure_graph(c, iters % kGraphBatch))) return rc;
    if (x0) {
        // one dry replay of each graph the run launches, with ctl->done set (every kernel leaves
        // without arithmetic): the graphs' first-launch cost (measured ~20 us at K = 20 beyond
        // hipGraphUpload, tools/k_sweep.py) falls here instead of in the timed call
        if (!c->eager) {
            HIPCHK(hipStreamSynchronize(c->stream));
            Ctl h{};
            h.done = 1;
            h.final_k = -1;
            *c->h_ctl = h;
            HIPCHK(hipMemcpyAsync(c->ctl, c->h_ctl, sizeof(Ctl), hipMemcpyHostToDevice, c->stream));
            if (iters / kGraphBatch && (rc = launch_batch(c, kGraphBatch))) return rc;
            if (iters % kGraphBatch && (rc = launch_batch(c, iters % kGraphBatch))) return rc;
            HIPCHK(hipStreamSynchronize(c->stream));
            if (int fe = fuse_err(c)) return fe;
        }
        // the run's initial state: the following raocp_cp_bench(ctx, NULL, iters, ...) starts here
        if ((rc = cp_init(c, x0, iters - 1, 0.0, alpha))) return rc;
        HIPCHK(hipStreamSynchronize(c->stream));
        c->prepared = iters;
    }
    return RAOCP_OK;
}

int raocp_cp_bench(raocp_ctx* c, const double* x0, int iters, double alpha, float* ms) {
    DevGuard dg_(c);
    SweepLock sl_(c);
    if (c && c->f32 && !c->dyn32) return fail(RAOCP_ERR_ARG, "fp32 CP loop unavailable: no fp32 dynamics plan");
    if (!c || iters < 1) return fail(RAOCP_ERR_ARG, "bad argument");
    int rc;
    if ((rc = ensure_hist(c, (size_t)iters + 1))) return rc;
    const int batch = kGraphBatch, full = iters / batch, rem = iters % batch;
    if (full && (rc = ensure_graph(c, batch))) return rc;
    if (rem && (rc = ensure_graph(c, rem))) return rc;
    if (x0) {
        if ((rc = cp_init(c, x0, iters - 1, 0.0, alpha))) return rc;
    } else if (c->prepared != iters) {
        return fail(RAOCP_ERR_STATE, "raocp_cp_bench without x0 needs raocp_cp_prepare(ctx, x0, iters, alpha) first");
    }
    c->prepared = 0;
    if (!c->ev0) {
        HIPCHK(hipEventCreate(&c->ev0));
        HIPCHK(hipEventCreate(&c->ev1));
    }
    hipEvent_t e0 = c->ev0, e1 = c->ev1;
    if (x0) HIPCHK(hipStreamSynchronize(c->stream));
    // the batch tail's stopping test publishes the control block and the error word to pinned
    // host memory (k_cp_check pub): no device-to-host copy behind the timed kernels
    const bool pub = defer_check(c);
    raocp::CtlPub* hp = c->h_pub;
    if (pub) hp->ctl.final_k = -2;
    HIPCHK(hipEventRecord(e0, c->stream));
    // exactly `iters` iterations' kernels: whole batches, then the remainder batch (an RCCL
    // shard then runs the last iteration's deferred stopping test)
    for (int b = 0; b < full; ++b)
        if ((rc = launch_batch(c, batch))) return rc;
    if (rem && (rc = launch_batch(c, rem))) return rc;
    if (c->comm && (rc = enqueue_shard_tail(c))) return rc;
    HIPCHK(hipEventRecord(e1, c->stream));
    const unsigned* ew = err_word(c);
    if (!pub) {
        HIPCHK(hipMemcpyAsync(&hp->ctl, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
        hp->err = 0;
        if (ew) HIPCHK(hipMemcpyAsync(&hp->err, ew, sizeof(unsigned), hipMemcpyDeviceToHost, c->stream));
    }
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipEventElapsedTime(ms, e0, e1));
    *c->h_ctl = hp->ctl;
    if (ew && hp->err)
        if (int fe = fuse_err(c)) return fe;  // a timed-out hand-off skipped its arithmetic
    if (c->h_ctl->final_k != iters - 1) return fail(RAOCP_ERR_STATE, "bench did not run the requested iterations");
    c->cur_z = c->Z[iters % 3];
    c->cur_e = c->E[iters % 2];
    return RAOCP_OK;
}

// diagnostics: run the dynamics projection once on the current primal with in-kernel
// stamps enabled (k_dyn_top: prologue, each backward / forward stage); returns up to
// `cap` raw 100 MHz timestamps.
int raocp_debug_dyn_stamps(raocp_ctx* c, unsigned long long* out, int cap) {
    DevGuard dg_(c);
    SweepLock sl_(c);
    // the regular-tree sweeps' stamps need only their own unit built with them (VAR_UNIT=dynr)
    if (!raocp::kDiag && !(c && c->dr && raocp::dr_diag_build()))
        return fail(RAOCP_ERR_ARG, "in-kernel stamps need a diagnostic build (make DIAG=1)");
    if (c && c->f32) return fail(RAOCP_ERR_ARG, "not available on an fp32 context (the CP loop and L / L^T are)");
    if (!c || !out || cap <= 0) return fail(RAOCP_ERR_ARG, "bad argument");
    // k_dr / k_drc stamp 4 slots per workgroup from slot 1024 (raocp_dynr.hip wg_stamp) and
    // k_drc's CP waves 128 slots from 3072
    if (c->dr && (size_t)cap < std::max(c->drc ? (size_t)3072 + 128 : (size_t)0, 1024 + 4 * ((size_t)c->drp.nblk + 1)))
        return fail(RAOCP_ERR_ARG, "stamp buffer too small for the regular-tree sweep's workgroup stamps");
    // the tiered sweep stamps 64 slots per launch (2 per tier + the top)
    if (c->cut > 0 && (size_t)cap < 64 * (2 * c->tiers.size() + 1))
        return fail(RAOCP_ERR_ARG, "stamp buffer too small: 64 slots per dynamics launch");
    unsigned long long* st = nullptr;
    int rc = c->alloc(&st, (size_t)cap);
    if (rc) return rc;
    HIPCHK(hipMemset(st, 0, cap * sizeof(unsigned long long)));
    Dev saved = c->dev;
    c->dev.stamps = st;
    const raocp::Bufs solo{c->cur_z, c->cur_z, c->cur_z, c->cur_e, c->cur_e};
    // RAOCP_STAMP_KERNEL: the launch to stamp (its first letter) and, for the CP kernels, the
    // workgroup / task that records (the number after it, e.g. "c200")
    const char* which = getenv("RAOCP_STAMP_KERNEL");
    if (which && which[0]) c->dev.cp_dbg = atoi(which + 1);
    if (which && which[0] == 'p') {  // k_cpp on a valid control block (diagnostics)
        std::vector<double> x0(c->nx, 0.0);
        int rc2 = cp_init(c, x0.data(), 1 << 30, 0.0, 0.5);
        if (rc2) return rc2;
        launch_cpp(c);
    } else if (which && which[0] == 'c') {  // the fused CP kernel (k_cp4 / k_cp3) on a valid control block
        if (!c->cp3) return fail(RAOCP_ERR_ARG, "no fused CP kernel on this context");
        std::vector<double> x0(c->nx, 0.0);
        int rc2 = cp_init(c, x0.data(), 1 << 30, 0.0, 0.5);
        if (rc2) return rc2;
        launch_cp3(c);
    } else if (which && which[0] == 'f') {  // the fused dynamics + CP launch (k_drc) on a valid control block
        if (!c->drc) return fail(RAOCP_ERR_ARG, "no fused dynamics + CP launch on this context");
        std::vector<double> x0(c->nx, 0.0);
        int rc2 = cp_init(c, x0.data(), 1 << 30, 0.0, 0.5);
        if (rc2) return rc2;
        const raocp::Bufs keep = c->bufs;
        c->bufs = rotated(c, 0);
        launch_drc(c, 0, false);
        c->bufs = keep;
    } else if (which && which[0] == 'l') {  // k_ell on the staging buffers
        launch_ell(c, c->tmpP, c->tmpD);
    } else if (which && which[0] == 't') {  // k_ell_t
        launch_ell_t(c, c->tmpD, c->tmpP);
    } else {
        launch_dynamics(c, solo, 0, nullptr);
    }
    c->dev = saved;
    HIPCHK(hipStreamSynchronize(c->stream));
    HIPCHK(hipMemcpy(out, st, cap * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    return RAOCP_OK;
}


// ---- subtree sharding ---------------------------------------------------------------
int raocp_shard_setup(raocp_ctx* c, int nranks, int rank) {
    DevGuard dg_(c);
    if (c && c->f32 && !c->dyn3)
        return fail(RAOCP_ERR_ARG, "fp32 sharding needs the per-stage streaming dynamics (uniform branching and slots)");
    if (!c || nranks < 1 || rank < 0 || rank >= nranks) return fail(RAOCP_ERR_ARG, "bad shard arguments");
    // one shard is the unsharded solve, unless forced (tests run the exchange path with R = 1)
    if (nranks == 1 && !getenv("RAOCP_SHARD_FORCE")) return RAOCP_OK;
    const int N = c->N;
    int S = c->cut;
    if (c->dyn3) {
        // the per-stage sweep: cut at the first stage with at least 8 subtrees per shard (the
        // replicated top above it is a few hundred nodes at most)
        S = 0;
        for (int t = 1; t < N && !S; ++t)
            if (c->stage_ptr[t + 1] - c->stage_ptr[t] >= 8 * nranks) S = t;
        if (!S) return fail(RAOCP_ERR_ARG, "tree too small to shard (no stage with 8 subtrees per shard)");
    } else if (S <= 0 || S >= N || c->tiers.empty()) {
        return fail(RAOCP_ERR_ARG, "tree too small to shard (the dynamics plan has no tier below the top)");
    }
    const int nb = c->stage_ptr[S + 1] - c->stage_ptr[S];
    if (nb < nranks) return fail(RAOCP_ERR_ARG, "fewer subtrees at the cut stage than shards");
    c->sh_R = nranks;
    c->sh_r = rank;
    c->sh_S = S;
    std::vector<int> slc(2 * nranks);
    int xmax = 0;
    for (int r = 0; r < nranks; ++r) {
        const int lo = c->stage_ptr[S] + (int)((long)r * nb / nranks), hi = c->stage_ptr[S] + (int)((long)(r + 1) * nb / nranks);
        slc[2 * r] = lo;
        slc[2 * r + 1] = hi - lo;
        xmax = std::max(xmax, hi - lo);
    }
    c->x_max = xmax;
    c->own_first = slc[2 * rank];
    c->own_cnt = slc[2 * rank + 1];
    // owned id range per stage: the whole stage above the cut, descendants below
    c->own_lo.assign(N + 1, 0);
    c->own_hi.assign(N + 1, 0);
    for (int t = 0; t < S; ++t) {
        c->own_lo[t] = c->stage_ptr[t];
        c->own_hi[t] = c->stage_ptr[t + 1];
    }
    int lo = c->own_first, hi = c->own_first + c->own_cnt;
    for (int t = S; t <= N; ++t) {
        c->own_lo[t] = lo;
        c->own_hi[t] = hi;
        if (t < N && hi > lo) {
            const int nlo = c->h_chs[lo], nhi = c->h_chs[hi - 1] + c->h_nch[hi - 1];
            lo = nlo;
            hi = nhi;
        }
    }
    c->tier_own.clear();
    if (!c->dyn3)
        for (const auto& tp : c->tiers)
            c->tier_own.push_back({c->own_lo[tp.s0] - c->stage_ptr[tp.s0], c->own_hi[tp.s0] - c->own_lo[tp.s0]});
    c->d3own = c->d3st;
    for (int t = S; t < N && c->dyn3; ++t) {
        c->d3own[t].i0 = c->own_lo[t];
        c->d3own[t].i1 = c->own_hi[t];
    }
    // CP blocks: the replicated top families plus the owned ones, the owned leaves
    std::vector<std::pair<int, int>> pr_;
    pr_.push_back({0, c->stage_ptr[S]});
    for (int t = S; t < N; ++t)
        if (c->own_hi[t] > c->own_lo[t]) pr_.push_back({c->own_lo[t], c->own_hi[t]});
    std::vector<std::pair<int, int>> lr_{{c->own_lo[N], c->own_hi[N]}};
    int rc;
    if ((rc = build_cp_blocks(c, pr_, lr_))) return rc;
    if (c->cp3) {
        // k_cp3 in two launches: the owned families and leaves plus the replicated top above
        // the cut's parents (storing its roots' xi2 for X1), then the cut's parents with the
        // roots' eta2 entries from X1
        std::vector<std::pair<int, int>> ra;
        if (N - 1 >= S) ra.push_back({c->own_lo[N - 1], c->own_hi[N - 1]});
        for (int t = S; t < N - 1; ++t) ra.push_back({c->own_lo[t], c->own_hi[t]});
        if (S >= 2) ra.push_back({0, c->stage_ptr[S - 1]});
        const long ta = cp3_tasks(c->cp3_ta, ra, c->own_lo[N], c->cp3_split ? c->own_hi[N] : c->own_lo[N], c->cp3_split,
                                  c->cp3_mL);
        c->cp3_ta.xlo = c->own_first;
        c->cp3_ta.xhi = c->own_first + c->own_cnt;
        const long tb = cp3_tasks(c->cp3_tb, {{c->stage_ptr[S - 1], c->stage_ptr[S]}}, 0, 0, c->cp3_split, c->cp3_mL);
        if (ta < 0 || tb < 0)
            return fail(RAOCP_ERR_ARG, "shard's k_cp3 task list exceeds its " + std::to_string(raocp::kCp3MaxR) +
                                           " parent-range slots (too many stages below the cut)");
        c->cp3_tb.ext2 = 1;
        c->cp3_grid = cp3_grid_of(ta);
        c->cp3_gridb = cp3_grid_of(tb);
        c->cp_rows = c->cp3_grid + c->cp3_gridb;
        if (c->cp_rows > c->red_rows) {
            c->red_rows = c->cp_rows;
            if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return rc;
        }
        HIPCHK(hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)));
    }
    if (c->cp5) {
        // k_cp5 in two launch pairs: the eta2 tasks of the replicated top and the owned stages,
        // the owned leaves, and the owned families plus the top above the cut's parents; after
        // X1 (the roots' s of the half step) the cut's parents' family tiles alone
        std::vector<std::pair<int, int>> er{{0, c->stage_ptr[S]}};
        for (int t = S; t < N; ++t) er.push_back({c->own_lo[t], c->own_hi[t]});
        std::vector<std::pair<int, int>> ra;
        if (N - 1 >= S) ra.push_back({c->own_lo[N - 1], c->own_hi[N - 1]});
        for (int t = S; t < N - 1; ++t) ra.push_back({c->own_lo[t], c->own_hi[t]});
        if (S >= 2) ra.push_back({0, c->stage_ptr[S - 1]});
        if (cp3_tasks(c->cp5_et, er, 0, 0, 1, 0, 64) < 0 || cp3_tasks(c->cp5_tk, ra, 0, 0, 1, c->cp3_mL) < 0 ||
            cp3_tasks(c->cp5_tkb, {{c->stage_ptr[S - 1], c->stage_ptr[S]}}, 0, 0, 1, c->cp3_mL) < 0)
            return fail(RAOCP_ERR_ARG, "shard's k_cp5 task lists exceed their " + std::to_string(raocp::kCp3MaxR) +
                                           " range slots (too many stages below the cut)");
        c->cp5_gl = raocp::cp5_leaf_grid(c->cp5_et, c->own_lo[N], c->own_hi[N], c->cp5_lpf);
        c->cp5_gf = raocp::cp5_fam_grid(c->cp5_tk);
        c->cp5_gfb = raocp::cp5_fam_grid(c->cp5_tkb);
        c->cp_rows = raocp::cp5_rows(c->cp5_gl, c->cp5_gf) + c->cp5_gfb;
        if (c->cp_rows > c->red_rows) {
            c->red_rows = c->cp_rows;
            if ((rc = c->alloc(&c->redpart, (size_t)c->red_rows * 6))) return rc;
        }
        HIPCHK(hipMemset(c->redpart, 0, (size_t)c->red_rows * 6 * sizeof(double)));
    }
    if ((rc = c->alloc(&c->x2_send, (size_t)xmax * std::max(c->KP, c->nx))) ||
        (rc = c->alloc(&c->x2_recv, (size_t)nranks * xmax * std::max(c->KP, c->nx))) ||
        (rc = c->alloc(&c->x1_send, (size_t)2 * xmax + 16)) || (rc = c->alloc(&c->x1_recv, (size_t)nranks * (2 * xmax + 16))) ||
        (rc = c->alloc(&c->red8, 16)) || (rc = c->upload_vec(&c->d_slc, slc)))
        return rc;
    drop_graphs(c);
    return RAOCP_OK;
}

int raocp_shard_owned(raocp_ctx* c, int32_t* lo, int32_t* hi, int cap) {
    DevGuard dg_(c);
    if (!c || !lo || !hi) return fail(RAOCP_ERR_ARG, "null argument");
    for (int t = 0; t <= c->N && t < cap; ++t) {
        lo[t] = c->sh_S > 0 ? c->own_lo[t] : c->stage_ptr[t];
        hi[t] = c->sh_S > 0 ? c->own_hi[t] : c->stage_ptr[t + 1];
    }
    return RAOCP_OK;
}

int raocp_comm_unique_id(unsigned char* out128) {
    if (!out128) return fail(RAOCP_ERR_ARG, "null argument");
    int rc;
    if ((rc = rccl_load())) return rc;
    ncclUniqueId id;
    if ((rc = rccl_check(g_rccl.get_id(&id), "ncclGetUniqueId"))) return rc;
    memcpy(out128, id.internal, NCCL_UNIQUE_ID_BYTES);
    return RAOCP_OK;
}

int raocp_comm_init(raocp_ctx* c, const unsigned char* id128, int nranks, int rank) {
    DevGuard dg_(c);
    if (!c || !id128) return fail(RAOCP_ERR_ARG, "null argument");
    if (c->sh_R != nranks || c->sh_r != rank) return fail(RAOCP_ERR_STATE, "call raocp_shard_setup with the same ranks first");
    int rc;
    if ((rc = rccl_load())) return rc;
    HIPCHK(hipSetDevice(c->device));
    ncclUniqueId id;
    memcpy(id.internal, id128, NCCL_UNIQUE_ID_BYTES);
    ncclComm_t comm = nullptr;
    if ((rc = rccl_check(g_rccl.init_rank(&comm, nranks, id, rank), "ncclCommInitRank"))) return rc;
    c->comm = comm;
    drop_graphs(c);
    return RAOCP_OK;
}

// Shards that share one process and one device (tests, and a host-driven transport):
// the CP loop runs eagerly, the exchanges are device copies between the shards' buffers.
int raocp_group_cp_run(raocp_ctx** cs, int R, const double* x0, int max_iters, double tol, double alpha, int* status,
                       int* iters, double* err_hist, double* delta_hist) {
    if (!cs || R < 1 || !x0) return fail(RAOCP_ERR_ARG, "null argument");
    DevGuard dg_(cs[0]);
    for (int r = 0; r < R; ++r)
        if (!cs[r] || cs[r]->sh_R != R || cs[r]->sh_r != r) return fail(RAOCP_ERR_STATE, "shards not set up for this group");
    int rc;
    for (int r = 0; r < R; ++r) {
        raocp_ctx* c = cs[r];
        HIPCHK(hipSetDevice(c->device));
        if ((rc = ensure_hist(c, (size_t)max_iters + 1))) return rc;
        if ((rc = raocp_set_initial_state(c, x0))) return rc;
        if ((rc = cp_init(c, x0, max_iters, tol, alpha))) return rc;
    }
    auto sync_all = [&]() -> int {
        for (int r = 0; r < R; ++r) HIPCHK(hipStreamSynchronize(cs[r]->stream));
        return RAOCP_OK;
    };
    // the RCCL iteration's protocol with device copies as the transport: X2 after the tiers'
    // backward sweeps, X1 (roots' eta2 entries + the previous iteration's residual record,
    // whose stopping test runs on arrival) after k_cpd; the loop ends once the (deferred)
    // test has fired
    for (int k = 0;; ++k) {
        for (int r = 0; r < R; ++r) {
            raocp_ctx* c = cs[r];
            c->bufs = rotated(c, k % 6);
            launch_dynamics(c, c->bufs, 1, c->ctl, 1);
            shard_pack_x2(c);
        }
        if ((rc = sync_all())) return rc;
        for (int r = 0; r < R; ++r) {
            raocp_ctx* c = cs[r];
            for (int q = 0; q < R; ++q)
                HIPCHK(hipMemcpyAsync((char*)c->x2_recv + (size_t)q * x2_bytes(c), cs[q]->x2_send, x2_bytes(c),
                                      hipMemcpyDeviceToDevice, c->stream));
            shard_unpack_x2(c);
            launch_dynamics(c, c->bufs, 1, c->ctl, 2);
            if (c->cp3) launch_cp3(c, 0);
            else launch_cpd(c);
            shard_pack_x1(c);
        }
        if ((rc = sync_all())) return rc;
        for (int r = 0; r < R; ++r) {
            raocp_ctx* c = cs[r];
            for (int q = 0; q < R; ++q)
                HIPCHK(hipMemcpyAsync(c->x1_recv + (size_t)q * x1_len(c), cs[q]->x1_send, (size_t)x1_len(c) * sizeof(double),
                                      hipMemcpyDeviceToDevice, c->stream));
            shard_unpack_x1(c);
            if (c->cp3) launch_cp3(c, 1);
            else launch_cpp(c);
            raocp::k_cp_reduce<<<1, kBlock, 0, c->stream>>>(c->ctl, c->redpart, c->cp_rows, c->red8);
            HIPCHK(hipMemcpyAsync(c->h_ctl, c->ctl, sizeof(Ctl), hipMemcpyDeviceToHost, c->stream));
        }
        if ((rc = sync_all())) return rc;
        HIPCHK(hipGetLastError());
        if (cs[0]->h_ctl->done) break;
    }
    for (int r = 0; r < R; ++r) cs[r]->bufs = raocp::Bufs{cs[r]->Z[0], cs[r]->Z[1], cs[r]->Z[2], cs[r]->E[0], cs[r]->E[1]};
    raocp_ctx* c = cs[0];
    const int fk = c->h_ctl->final_k;
    std::vector<double> h((size_t)(fk + 1) * 6);
    HIPCHK(hipMemcpy(h.data(), c->hist, h.size() * sizeof(double), hipMemcpyDeviceToHost));
    for (int k = 0; k <= fk; ++k)
        for (int q = 0; q < 3; ++q) {
            if (err_hist) err_hist[k * 3 + q] = h[(size_t)k * 6 + q];
            if (delta_hist) delta_hist[k * 3 + q] = h[(size_t)k * 6 + 3 + q];
        }
    for (int r = 0; r < R; ++r) {
        cs[r]->cur_z = cs[r]->Z[(fk + 1) % 3];
        cs[r]->cur_e = cs[r]->E[(fk + 1) % 2];
    }
    if (iters) *iters = fk + 1;
    if (status) *status = fk < max_iters ? 0 : 1;
    if (int fe = fuse_err(c)) return fe;
    if (c->h_ctl->flags & 1) return fail(RAOCP_ERR_NAN_IN_BOX, "Rectangle constraint - 'nan' value cannot be constrained");
    return RAOCP_OK;
}

int raocp_op_bench(raocp_ctx* c, int op, int reps, float* ms_per_launch) {
    DevGuard dg_(c);
    SweepLock sl_(c);
    if (!c || reps < 1 || !ms_per_launch) return fail(RAOCP_ERR_ARG, "bad argument");
    // random inputs (seed 1), resident in HBM
    std::vector<double> hz(c->P), he(c->D);
    std::mt19937_64 gen(1);
    std::normal_distribution<double> nd(0.0, 1.0);
    for (auto& v : hz) v = nd(gen);
    for (auto& v : he) v = nd(gen);
    int rci;
    if ((rci = copy_in(c, c->tmpP, hz.data(), c->P, 0)) || (rci = copy_in(c, c->tmpD, he.data(), c->D, 0))) return rci;
    HIPCHK(hipStreamSynchronize(c->stream));
    double* outP = c->Z[2];
    double* outD = c->E[1];
    // ops >= 2 time the CP kernels (or one role of them) on a valid control block
    if (op >= 2) {
        if (c->f32 && (!c->dyn32 || (op != 2 && op != 6 && op != 9 && op != 10)))
            return fail(RAOCP_ERR_ARG, "fp32 context: ops 0, 1, 2, 6, 9 and 10 can be timed");
        if (int rh = ensure_hist(c, (size_t)reps + 16)) return rh;
        std::vector<double> x0(c->nx, 0.0);
        int rc = cp_init(c, x0.data(), 1 << 30, 0.0, 0.5);
        if (rc) return rc;
        for (int b = 0; b < 3; ++b) HIPCHK(hipMemcpyAsync(c->Z[b], c->tmpP, c->P * c->wsz, hipMemcpyDeviceToDevice, c->stream));
        for (int b = 0; b < 2; ++b) HIPCHK(hipMemcpyAsync(c->E[b], c->tmpD, c->D * c->wsz, hipMemcpyDeviceToDevice, c->stream));
    }
    auto run = [&]() {
        switch (op) {
            case 0: launch_ell(c, c->tmpP, outD); break;
            case 1: launch_ell_t(c, c->tmpD, outP); break;
            case 2: launch_cpd(c); break;
            case 3: case 4: case 5: launch_cp_dual(c, true, nullptr, raocp::kDualAll, op - 2); break;
            case 6: launch_cpp(c); break;
            case 7: case 8: launch_cp_primal(c, true, op - 6); break;
            case 9: launch_dynamics(c, c->bufs, 1, c->ctl); break;
            case 10:  // the CP iteration's kernels after the dynamics
                if (c->cp3) {
                    launch_cp3(c);
                } else {
                    launch_cpd(c);
                    launch_cpp(c);
                }
                break;
            case 11: launch_drc(c, 0, false); break;  // the fused dynamics + CP launch (k_drc)
            default: raocp::k_cp_check<<<1, kBlock, 0, c->stream>>>(c->ctl, c->hist, c->redpart, c->cp_rows, 0, nullptr, nullptr);
        }
    };
    for (int i = 0; i < 3; ++i) run();  // warm-up
    // the reps launches replay as one graph (as in the CP loop), so the time is the
    // kernels' back to back, not the host's launch rate; RAOCP_EAGER=1 launches them
    // one by one (rocprofv3 kernel tracing)
    hipGraphExec_t gx = nullptr;
    if (!c->eager) {
        hipGraph_t g = nullptr;
        HIPCHK(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
        for (int i = 0; i < reps; ++i) run();
        HIPCHK(hipStreamEndCapture(c->stream, &g));
        HIPCHK(hipGraphInstantiate(&gx, g, nullptr, nullptr, 0));
        (void)hipGraphDestroy(g);
        HIPCHK(hipGraphLaunch(gx, c->stream));  // warm-up replay
    }
    hipEvent_t e0, e1;
    HIPCHK(hipEventCreate(&e0));
    HIPCHK(hipEventCreate(&e1));
    HIPCHK(hipEventRecord(e0, c->stream));
    if (gx) HIPCHK(hipGraphLaunch(gx, c->stream));
    else for (int i = 0; i < reps; ++i) run();
    HIPCHK(hipEventRecord(e1, c->stream));
    HIPCHK(hipEventSynchronize(e1));
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (gx) (void)hipGraphExecDestroy(gx);
    HIPCHK(hipGetLastError());
    *ms_per_launch = ms / reps;
    return fuse_err(c);
}

// L (op 0) or L^T (op 1) with the launches cycling over `nsets` input / output buffer pairs:
// with nsets (|P| + |D|) scalars beyond the 256 MiB Infinity Cache, every launch reads its
// input from HBM (the repeated-buffer op_bench is L3-assisted once a working set fits)
int raocp_op_bench_rot(raocp_ctx* c, int op, int reps, int nsets, float* ms_per_launch) {
    DevGuard dg_(c);
    SweepLock sl_(c);
    if (!c || reps < 1 || nsets < 1 || nsets > 16 || !ms_per_launch || (op != 0 && op != 1))
        return fail(RAOCP_ERR_ARG, "bad argument");
    std::vector<double> hz(c->P), he(c->D);
    std::mt19937_64 gen(1);
    std::normal_distribution<double> nd(0.0, 1.0);
    for (auto& v : hz) v = nd(gen);
    for (auto& v : he) v = nd(gen);
    int rci;
    if ((rci = copy_in(c, c->tmpP, hz.data(), c->P, 0)) || (rci = copy_in(c, c->tmpD, he.data(), c->D, 0))) return rci;
    std::vector<void*> mem;
    auto release = [&]() {
        for (void* q : mem) (void)hipFree(q);
    };
    std::vector<double*> P(nsets), D(nsets);
    for (int k = 0; k < nsets; ++k) {
        void* a = nullptr;
        void* b = nullptr;
        if (hipMalloc(&a, c->P * c->wsz + 64) != hipSuccess || (mem.push_back(a), hipMalloc(&b, c->D * c->wsz + 64)) != hipSuccess) {
            release();
            return fail(RAOCP_ERR_HIP, "hipMalloc (rotating buffer sets)");
        }
        mem.push_back(b);
        P[k] = (double*)a;
        D[k] = (double*)b;
        (void)hipMemcpyAsync(P[k], c->tmpP, c->P * c->wsz, hipMemcpyDeviceToDevice, c->stream);
        (void)hipMemcpyAsync(D[k], c->tmpD, c->D * c->wsz, hipMemcpyDeviceToDevice, c->stream);
    }
    auto run = [&](int i) {
        const int k = i % nsets;
        if (op == 0) launch_ell(c, P[k], D[k]);
        else launch_ell_t(c, D[k], P[k]);
    };
    for (int i = 0; i < nsets; ++i) run(i);  // warm-up
    hipGraphExec_t gx = nullptr;
    hipGraph_t g = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    float ms = 0;
    bool ok = hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal) == hipSuccess;
    if (ok) {
        for (int i = 0; i < reps; ++i) run(i);
        ok = hipStreamEndCapture(c->stream, &g) == hipSuccess && hipGraphInstantiate(&gx, g, nullptr, nullptr, 0) == hipSuccess;
    }
    if (g) (void)hipGraphDestroy(g);
    ok = ok && hipGraphLaunch(gx, c->stream) == hipSuccess;  // warm-up replay
    ok = ok && hipEventCreate(&e0) == hipSuccess && hipEventCreate(&e1) == hipSuccess;
    ok = ok && hipEventRecord(e0, c->stream) == hipSuccess && hipGraphLaunch(gx, c->stream) == hipSuccess &&
         hipEventRecord(e1, c->stream) == hipSuccess && hipEventSynchronize(e1) == hipSuccess &&
         hipEventElapsedTime(&ms, e0, e1) == hipSuccess;
    if (e0) (void)hipEventDestroy(e0);
    if (e1) (void)hipEventDestroy(e1);
    if (gx) (void)hipGraphExecDestroy(gx);
    (void)hipStreamSynchronize(c->stream);
    release();
    if (!ok) return fail(RAOCP_ERR_HIP, std::string("op_bench_rot: ") + hipGetErrorString(hipGetLastError()));
    *ms_per_launch = ms / reps;
    return RAOCP_OK;
}

}  // extern "C"
