/*
 * raocp_hip.h — C-ABI of libraocp_hip.so, the MI355X (gfx950) implementation of
 * raocp's Chambolle–Pock inner loop.
 *
 * The reference (smokinmirror/raocp-toolbox) is pure Python and has no FFI; its
 * "operator API" is a set of Python methods. Each entry point below replaces one
 * of them and is what the drop-in Python layer (raocp-toolbox_amd/raocp/core,
 * via ctypes) binds. Citations are /root/reference paths.
 *
 * Conventions
 *  - All functions return 0 on success or a negative RAOCP_ERR_* code;
 *    raocp_last_error() returns the message of the last failure on this thread.
 *  - Vectors crossing the boundary are FLAT fp64 arrays in the reference's block
 *    order (np.vstack of the block lists built in cache.py:126-170), placeholders
 *    included: primal length raocp_sizes(..)[0], dual length [1].
 *  - Pointers are host pointers unless RAOCP_DEVICE_PTR is passed in `flags`,
 *    in which case they are device (HBM) pointers on the context's device.
 *  - A context is bound to one device and one HIP stream; it is not thread-safe
 *    (neither is the reference: shared cone instances, cache.py:180-182).
 *  - Matrix tables are row-major, one matrix after another; per-node int32
 *    index arrays select a table entry (the packer dedupes shared matrices).
 */
#ifndef RAOCP_HIP_H
#define RAOCP_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RAOCP_OK 0
#define RAOCP_ERR_ARG -1          /* bad argument / shape (cache.py:84-122 shape errors) */
#define RAOCP_ERR_HIP -2          /* HIP runtime failure (no device, OOM, launch) */
#define RAOCP_ERR_TREE -3         /* tree violates a layout invariant (see raocp_tree_desc) */
#define RAOCP_ERR_NAN_IN_BOX -4   /* NaN reached a box projection (rectangle.py:50-59) */
#define RAOCP_ERR_STATE -5        /* call out of order (e.g. prox_f before an initial state) */

#define RAOCP_DEVICE_PTR 1

typedef struct raocp_ctx raocp_ctx;

/* Scenario tree (scenario_tree.py:21-154). Invariants checked at create:
 * nodes numbered so stage[] is non-decreasing, nonleaf nodes are 0..m-1, and the
 * children of node i are the contiguous ids ch_start[i] .. ch_start[i]+nch[i]-1
 * (true for every tree MarkovChainScenarioTreeFactory builds, scenario_tree.py:273-315). */
typedef struct {
    int32_t n;              /* num_nodes */
    int32_t m;              /* num_nonleaf_nodes */
    int32_t nx, nu;         /* state / control sizes */
    const int32_t* anc;     /* [n] ancestor, anc[0] = -1 */
    const int32_t* stage;   /* [n] stage of each node */
    const int32_t* ch_start;/* [m] first child */
    const int32_t* nch;     /* [m] number of children (>= 1) */
} raocp_tree_desc;

/* Problem data (raocp_spec.py, costs.py, risks.py, rectangle.py) and the offline
 * products of the dynamics projection (cache.py:207-233), computed by the host
 * packer (raocp/core/_pack.py). Index arrays are per node; -1 = not applicable. */
typedef struct {
    /* L / L^T weights (operators.py:19-94): sqrtm of Q, R (node j >= 1) and Pf (leaves) */
    int32_t n_sq, n_sr, n_sp;
    const double* sqrt_q;   /* [n_sq][nx][nx] */
    const double* sqrt_r;   /* [n_sr][nu][nu] */
    const double* sqrt_pf;  /* [n_sp][nx][nx] */
    const int32_t* i_sq;    /* [n] */
    const int32_t* i_sr;    /* [n] */
    const int32_t* i_sp;    /* [n] */
    /* AVaR (risks.py:28-35): b_i = [p; 0; 1]; p_k stored at child ch_start[i]+k */
    const double* alpha_r;  /* [m] risk parameter alpha of node i */
    const double* cond;     /* [n] conditional probability of node j given its parent */
    /* boxes (rectangle.py): nonleaf rows nx+nu, leaf rows nx */
    int32_t n_box_nl, n_box_l;
    const double* box_nl_lo; const double* box_nl_hi;   /* [n_box_nl][nx+nu] */
    const double* box_l_lo;  const double* box_l_hi;    /* [n_box_l][nx] */
    const int32_t* i_box_nl;/* [m] -1 = No constraint */
    const int32_t* i_box_l; /* [n] (leaves used) -1 = No constraint */
    /* dynamics projection: per-mode A, B (state / control dynamics of node j) and,
     * per subtree class (classes numbered by stage), the offline products
     * K, Rinv = (I + sum_j B_j'P_j B_j)^-1 and M = K' + sum_j Abar_j' P_j B_j */
    int32_t n_a, n_b, n_k;
    const double* A;        /* [n_a][nx][nx] */
    const double* B;        /* [n_b][nx][nu] */
    const double* K;        /* [n_k][nu][nx] */
    const double* Rinv;     /* [n_k][nu][nu] */
    const double* M;        /* [n_k][nx][nu] */
    const int32_t* i_a;     /* [n] */
    const int32_t* i_b;     /* [n] */
    const int32_t* i_k;     /* [m] class of nonleaf node i */
    /* arithmetic of the context: RAOCP_F64 (the reference's) or RAOCP_F32 (BASELINE
     * configs[4]: iterate, tables and products in fp32; vectors still cross the host
     * boundary as fp64 arrays, device pointers (RAOCP_DEVICE_PTR) are then float*) */
    int32_t dtype;
} raocp_problem_desc;

#define RAOCP_F64 0
#define RAOCP_F32 1

/* Create a context on HIP device `device`: validates the tree, uploads all tables
 * to HBM, allocates the iterate and work buffers. Replaces Cache.__init__
 * (cache.py:13-52) + Operator.__init__ (operators.py:10-17). */
int raocp_ctx_create(const raocp_tree_desc* tree, const raocp_problem_desc* prob, int device,
                     raocp_ctx** out);
void raocp_ctx_destroy(raocp_ctx* ctx);
const char* raocp_last_error(void);
/* hipDeviceSynchronize on `device` through this library's HIP runtime (bench.py
 * brackets its timed region with it; see bench.py for why not torch.cuda). */
int raocp_device_synchronize(int device);

/* Flat primal / dual lengths (placeholders included), cache.py:126-170. */
int raocp_sizes(raocp_ctx* ctx, int64_t* primal_size, int64_t* dual_size);

/* eta <- L z (Operator.ell, operators.py:19-53 / linop_ell 96-107). Only slots L
 * writes are stored; every other slot of `eta` keeps its input value, exactly like
 * the reference's output template. */
int raocp_ell(raocp_ctx* ctx, const double* z, double* eta, int flags);
/* z <- L^T eta (Operator.ell_transpose, operators.py:55-94 / linop_ell_transpose
 * 109-120). tau_0 keeps its input value. */
int raocp_ell_t(raocp_ctx* ctx, const double* eta, double* z, int flags);

/* The context's current iterate (Cache.__primal / __dual, cache.py:84-122). */
int raocp_set_primal(raocp_ctx* ctx, const double* z, int flags);
int raocp_get_primal(raocp_ctx* ctx, double* z, int flags);
int raocp_set_dual(raocp_ctx* ctx, const double* eta, int flags);
int raocp_get_dual(raocp_ctx* ctx, double* eta, int flags);
/* Cache.cache_initial_state (cache.py:79-82): x0 has nx entries. */
int raocp_set_initial_state(raocp_ctx* ctx, const double* x0);
/* Zero the current primal and dual on the device: the iterate of a fresh Cache
 * (cache.py:126-170 zero templates), without a host upload (cold-started chock). */
int raocp_reset_iterate(raocp_ctx* ctx);
/* Name of the kernel the context's default selection launches for `op` (raocp_op_bench
 * numbering: 0 L, 1 L^T, 2 dual CP kernel, 6 primal CP kernel, 9 dynamics projection,
 * 10 fused CP iteration, 11 the CP loop's one launch of dynamics projection + CP iteration
 * (k_drc; "" when the loop runs 9 and 10 as separate launches)), as rocprofv3 reports it;
 * op 12: the forms of the k_cp5 launches ("leaf_pf=. fams=. fam_pf=.", "" when k_cp5 does not
 * run); written NUL-terminated to buf. */
int raocp_kernel_info(raocp_ctx* ctx, int op, char* buf, int cap);

/* prox of f on the current primal (Cache.proximal_of_f, cache.py:248-257) and its steps */
int raocp_prox_f(raocp_ctx* ctx, double alpha);
int raocp_relax_s0(raocp_ctx* ctx, double alpha);        /* cache.py:253-257 */
int raocp_project_on_dynamics(raocp_ctx* ctx);           /* cache.py:259-288 */
int raocp_project_on_kernel(raocp_ctx* ctx);             /* cache.py:290-317 */
/* prox of alpha g* on the current dual (Cache.proximal_of_g_conjugate, cache.py:321-393) */
int raocp_prox_gconj(raocp_ctx* ctx, double alpha);

/* Sub-steps of prox_g* on the current dual, for the Cache API (cache.py:329-393):
 * modify_dual (eta /= alpha over every slot), add_halves (-1/2 on eta5, eta12 and
 * +1/2 on eta6, eta13, all blocks incl. placeholders), the cone/box projections
 * (which: 1 = project_on_constraints_nonleaf, 2 = _leaf, 3 = both) and
 * modify_projection (eta <- alpha (modified - eta), `modified` a host flat dual). */
int raocp_dual_scale(raocp_ctx* ctx, double alpha);
int raocp_dual_add_halves(raocp_ctx* ctx);
int raocp_dual_project(raocp_ctx* ctx, int which);
int raocp_dual_moreau(raocp_ctx* ctx, double alpha, const double* modified);

/* lambda_max(L'L) by device Lanczos (replaces ARPACK eigs, solver.py:104-118).
 * alpha = 0.999 / lambda_max. */
int raocp_step_size(raocp_ctx* ctx, double* lambda_max, int max_it, double rtol);

/* The whole Chambolle–Pock loop (Solver.chock, solver.py:97-171) on the device.
 * Starts from the context's current primal / dual (raocp_set_primal / raocp_set_dual;
 * both zero after raocp_ctx_create) with x0 written into node 0's state, as the
 * reference's chock continues from the cache's old primal / dual (solver.py:27-61,
 * cache.py:79-82, 186-196); runs until
 * k >= max_iters or max(error) <= tol, like the reference. Outputs:
 *   status    0 converged (k < max_iters) / 1 not converged (solver.py:166-169)
 *   iters     number of iterations run (rows of the error caches)
 *   err_hist, delta_hist: [max_iters+1][3] host arrays (row k = iteration k)
 * The final iterate is left as the context's current primal/dual. */
int raocp_cp_run(raocp_ctx* ctx, const double* x0, int max_iters, double tol, double alpha,
                 int* status, int* iters, double* err_hist, double* delta_hist);

/* Benchmark helpers (bench.py): raocp_cp_bench runs exactly `iters` CP iterations
 * (tol = 0) from (x0 at node 0, zeros) / 0 on the device, graph-replayed (whole
 * batches of 24 iterations, then one remainder batch), without host syncs inside;
 * returns device ms. raocp_cp_prepare captures the graphs a run of `iters` iterations
 * uses and, given x0, also resets the iterate for it, so that a following
 * raocp_cp_bench(ctx, NULL, iters, alpha, &ms) only launches the iterations. */
int raocp_cp_prepare(raocp_ctx* ctx, const double* x0, int iters, double alpha);
int raocp_cp_bench(raocp_ctx* ctx, const double* x0, int iters, double alpha, float* ms);
/* Time `reps` back-to-back launches of L (op=0) or L^T (op=1) on device-resident
 * vectors with HIP events on the context's stream; returns average ms per launch. */
int raocp_op_bench(raocp_ctx* ctx, int op, int reps, float* ms_per_launch);
/* The same for L (op 0) / L^T (op 1) with the launches cycling over `nsets` (<= 16) freshly
 * allocated input / output buffer pairs, so that a working set beyond the 256 MiB Infinity
 * Cache is read from HBM on every launch. */
int raocp_op_bench_rot(raocp_ctx* ctx, int op, int reps, int nsets, float* ms_per_launch);
/* Diagnostics: one dynamics projection with in-kernel s_memrealtime stamps (100 MHz). */
int raocp_debug_dyn_stamps(raocp_ctx* ctx, unsigned long long* stamps, int cap);

/* Subtree sharding across GPUs (north_star "scenarios shard naturally
 * by subtree"). Shard `rank` of `nranks` owns a contiguous block of the subtrees rooted
 * at the boundary stage of the replicated top of the tree; the CP iteration then runs on
 * the owned nodes only, with two all-gathers per iteration: the q rows of the roots
 * (dynamics backward sweep), and the roots' eta2 / xi2 entries together with the previous
 * iteration's residual record (the stopping test runs one iteration late, so the residual
 * reduction needs no collective of its own).
 * raocp_shard_setup restricts this context to its shard; raocp_comm_init binds an RCCL
 * communicator (one process per GPU; the 128-byte id comes from raocp_comm_unique_id on
 * one rank); raocp_cp_run / raocp_cp_bench then run the sharded iteration.
 * raocp_group_cp_run runs the shards of one process (tests: shards sharing a device),
 * exchanging through device copies. raocp_shard_owned: owned id range per stage. */
int raocp_shard_setup(raocp_ctx* ctx, int nranks, int rank);
int raocp_shard_owned(raocp_ctx* ctx, int32_t* stage_lo, int32_t* stage_hi, int cap);
int raocp_comm_unique_id(unsigned char* id128);
int raocp_comm_init(raocp_ctx* ctx, const unsigned char* id128, int nranks, int rank);
int raocp_group_cp_run(raocp_ctx** ctxs, int nranks, const double* x0, int max_iters, double tol, double alpha,
                       int* status, int* iters, double* err_hist, double* delta_hist);

#ifdef __cplusplus
}
#endif
#endif /* RAOCP_HIP_H */
