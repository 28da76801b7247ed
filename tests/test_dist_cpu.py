"""CPU, world_size 2-3: the host side of the multi-GPU paths.

* the gloo max / all-gather pattern of a timed region (the slowest rank sets the job time;
  every rank solves its own instance in bench.py's replica headline);
* the SocketGroup rendezvous (uid broadcast, max, barrier) bench.py uses (torch must not
  share a process with the RCCL the library binds);
* bench.py --gpus N without WORLD_SIZE starting its own rank processes;
* subtree sharding on the host: the dynamics projection by two processes that see only
  their own subtrees below the replicated top, exchanging the roots' q rows (X2); the dual
  step, next half step and residual record with the roots' eta2 entries + record (X1).
The device side of sharding is covered by tests/test_gpu_shard.py.
"""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    wall = 1.0 + rank  # the slowest rank sets the job time
    t = torch.tensor([wall], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    x0 = np.random.default_rng(1000 + rank).standard_normal(4)  # bench.py: per-rank instance
    g = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(g, torch.tensor(x0))
    out.put((rank, float(t[0]), [list(v.numpy()) for v in g]))
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_replicas_reduction():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gloo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, wall, xs in res:
        assert wall == 2.0
        assert not np.allclose(xs[0], xs[1])


def _socket_worker(rank, world, port, out):
    sys.path.insert(0, ROOT)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from bench import SocketGroup
    g = SocketGroup(rank, world)
    uid = g.bcast(bytes(range(128)) if rank == 0 else b"")
    m = g.max(float(10 * rank + 3))
    g.barrier()
    out.put((rank, uid, m))


@pytest.mark.parametrize("world", [2, 3])
def test_socket_group_rendezvous(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_socket_worker, args=(r, world, port - 1, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, uid, m in res:
        assert uid == bytes(range(128))
        assert m == float(10 * (world - 1) + 3)


# ---------------------------------------------------------------------------------------
# subtree sharding on the host: two gloo processes each own a contiguous
# block of the subtrees rooted at stage S (raocp_shard_setup's rule), see NaN everywhere
# else below the replicated top, and run the dynamics projection (cache.py:259-288) with
# the X2 exchange (all-gather of the roots' q rows) as their only communication. Their
# owned and top entries must equal the unsharded projection, NaN-free.
# ---------------------------------------------------------------------------------------
def shard_slices(stage_start, nb, R):
    """[first id, count] of each shard's roots (raocp_capi.hip raocp_shard_setup)."""
    return [(stage_start + r * nb // R, (r + 1) * nb // R - r * nb // R) for r in range(R)]


def owned_nodes(orc, S, first, cnt):
    """ids of the subtrees of roots [first, first + cnt) (stage S and below)."""
    out, lo, hi = [], first, first + cnt
    for t in range(S, orc.N + 1):
        out.extend(range(lo, hi))
        if t < orc.N and hi > lo:
            lo, hi = int(orc.chs[lo]), int(orc.chs[hi - 1] + orc.nch[hi - 1])
    return np.array(out, dtype=np.int64)


def _shard_worker(rank, world, port, S, out):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    from oracle.raocp_oracle import OracleProblem
    from raocp.problems import build_problem, recipe_bin6
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = recipe_bin6()
    orc = OracleProblem(build_problem(r)[1])
    st0 = int(np.flatnonzero(orc.stage == S)[0])
    nb = int(np.sum(orc.stage == S))
    sl = shard_slices(st0, nb, world)
    first, cnt = sl[rank]
    mine = owned_nodes(orc, S, first, cnt)
    top = np.flatnonzero(orc.stage < S)
    z = np.random.default_rng(3).standard_normal(orc.P)
    ref = orc.project_on_dynamics(z, r["x0"])
    # NaN outside the top and this shard's subtrees
    local = np.full(orc.P, np.nan)
    keep = np.zeros(orc.n, dtype=bool)
    keep[top] = True
    keep[mine] = True
    X = slice(orc.X0, orc.U0)
    local[orc.Y0:] = z[orc.Y0:]
    lx = local[X].reshape(orc.n, orc.nx)
    lx[keep] = z[X].reshape(orc.n, orc.nx)[keep]
    lu = local[orc.U0:orc.Y0].reshape(orc.m, orc.nu)
    km = keep[:orc.m]
    lu[km] = z[orc.U0:orc.Y0].reshape(orc.m, orc.nu)[km]

    def x2(q_stage):  # every shard's roots' q rows, the X2 all-gather
        maxc = max(c for _, c in sl)
        send = torch.zeros(maxc, orc.nx, dtype=torch.float64)
        send[:cnt] = torch.from_numpy(q_stage[first - st0:first - st0 + cnt])
        recv = [torch.zeros_like(send) for _ in range(world)]
        dist.all_gather(recv, send)
        full = q_stage.copy()
        for (f, c), buf in zip(sl, recv):
            full[f - st0:f - st0 + c] = buf[:c].numpy()
        return full

    got = orc.project_on_dynamics(local, r["x0"], exchange=(S, x2))
    gx = got[X].reshape(orc.n, orc.nx)[keep]
    rx = ref[X].reshape(orc.n, orc.nx)[keep]
    gu = got[orc.U0:orc.Y0].reshape(orc.m, orc.nu)[km]
    ru = ref[orc.U0:orc.Y0].reshape(orc.m, orc.nu)[km]
    ok = bool(np.all(np.isfinite(gx)) and np.all(np.isfinite(gu)))
    err = float(max(np.max(np.abs(gx - rx)), np.max(np.abs(gu - ru))))
    # without the exchange the other shard's NaN reaches the top: the X2 rows are needed
    bare = orc.project_on_dynamics(local, r["x0"])
    needed = not np.all(np.isfinite(bare[X].reshape(orc.n, orc.nx)[top]))
    out.put((rank, ok and needed, err, int(keep.sum())))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("S", [2, 3])
def test_sharded_dynamics_projection_two_processes(S):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok, err, nkeep in res:
        assert ok, f"rank {rank}: NaN reached an owned / top entry, or the X2 rows were not needed"
        assert err <= 1e-12, (rank, err)
    # the shards' subtrees partition the nodes below the top
    assert sum(nk for *_, nk in res) > 0


# ---------------------------------------------------------------------------------------
# X1 on the host: the dual step, the next half step with the AVaR kernel projection and the
# residual record (solver.py:63-95, 124-143) by shards that hold only the replicated top,
# their own subtrees and the roots' tau / s (written by the top families). Entries outside
# are garbage, not NaN (the rectangle projection raises on NaN, rectangle.py:50-59). The
# only message is raocp_capi.hip's X1: the owned roots' (eta+, xi2) eta2 entries plus the
# 16-double residual record, all-gathered. Local outputs must equal the unsharded step and
# the max over the gathered records must equal the unsharded error / delta-error.
# ---------------------------------------------------------------------------------------
def _x1_masks(orc, top, mine, roots):
    """local primal / dual entry masks of a shard (node blocks, placeholders included)."""
    n, m = orc.n, orc.m
    node = np.zeros(n, dtype=bool)
    node[top] = True
    node[mine] = True
    with_roots = node.copy()
    with_roots[roots] = True
    pm = np.zeros(orc.P, dtype=bool)
    pm[orc.x_idx[node].reshape(-1)] = True
    pm[orc.u_idx[node[:m]].reshape(-1)] = True
    pm[_blocks(orc.y_off[node[:m]], (2 * orc.nch + 1)[node[:m]])] = True
    pm[orc.T0 + np.flatnonzero(with_roots)] = True
    pm[orc.S0 + np.flatnonzero(with_roots)] = True
    dm = np.zeros(orc.D, dtype=bool)
    for k, off in enumerate(orc.d_off):
        sel = with_roots if k in (2, 3, 4, 5) else node  # eta3..eta6 of the roots: top families
        dm[_blocks(off[sel], orc.d_sizes[k][sel])] = True
    return pm, dm


def _blocks(starts, sizes):
    starts, sizes = np.asarray(starts, np.int64), np.asarray(sizes, np.int64)
    if starts.size == 0:
        return np.zeros(0, np.int64)
    return np.repeat(starts - np.concatenate([[0], np.cumsum(sizes)[:-1]]), sizes) + np.arange(sizes.sum())


def _x1_worker(rank, world, port, S, out):
    import torch
    import torch.distributed as dist
    sys.path[:0] = [os.path.join(ROOT, "raocp-toolbox_amd"), ROOT]
    from oracle.raocp_oracle import OracleProblem
    from raocp.problems import build_problem, recipe_bin6
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = recipe_bin6()
    orc = OracleProblem(build_problem(r)[1])
    x0 = r["x0"]
    st0 = int(np.flatnonzero(orc.stage == S)[0])
    nb = int(np.sum(orc.stage == S))
    sl = shard_slices(st0, nb, world)
    first, cnt = sl[rank]
    mine = owned_nodes(orc, S, first, cnt)
    top = np.flatnonzero(orc.stage < S)
    roots = np.arange(st0, st0 + nb)
    _, alpha = orc.step_size()
    # a mid-solve state: old primal / dual after a few iterations, then z+ (prox_f is shard-
    # local given X2, tested above)
    p, d = orc.initial_primal(x0), np.zeros(orc.D)
    for _ in range(4):
        p, d, _, _ = orc.cp_iteration(p, d, alpha, x0)
    zp = orc.prox_f(p - alpha * orc.ell_t(d, template=p), alpha, x0)
    # unsharded: dual step, residuals, next half step + kernel projection
    ep_r = orc.prox_gconj(d + alpha * orc.ell(2 * zp - p, template=d), alpha)
    nxt_r = _next_half_step(orc, zp, ep_r, alpha)
    _, _, err_r, derr_r = orc.cp_iteration(p, d, alpha, x0)

    pm, dm = _x1_masks(orc, top, mine, roots)
    dm_d = dm.copy()
    dm_d[orc.E2[roots]] = True  # the old dual's roots' eta2: the previous iteration's X1
    junk = np.random.default_rng(50 + rank)
    loc = lambda v, msk: np.where(msk, v, 1e6 + junk.standard_normal(v.size))
    p_l, zp_l, d_l = loc(p, pm), loc(zp, pm), loc(d, dm_d)
    ep = orc.prox_gconj(d_l + alpha * orc.ell(2 * zp_l - p_l, template=d_l), alpha)
    xi2 = (d_l - ep) / alpha + orc.ell(zp_l - p_l, template=d_l)
    e2_own = orc.E2[first:first + cnt]

    def residual_record(ep, xi2):
        xi1 = (p_l - zp_l) / alpha - orc.ell_t(d_l - ep, template=p_l)
        xi0 = xi1 + orc.ell_t(xi2, template=p_l)
        dl1 = zp_l - p_l
        dl2 = ep - d_l
        dl0 = dl1 - orc.ell_t(dl2, template=p_l)
        rec = np.zeros(16)
        for k, (v, msk) in enumerate(((xi0, pm), (xi1, pm), (xi2, dm), (dl0, pm), (dl1, pm), (dl2, dm))):
            rec[k] = np.max(np.abs(v[msk]), initial=0.0)
        return rec

    # X1 message: [eta+ of the owned roots' eta2 | xi2 of the same | residual record]
    maxc = max(c for _, c in sl)
    # the record's xi0 / xi1 / delta0 on the roots' s entries need the gathered eta2 entries,
    # so a record rides the NEXT iteration's X1 (k_cp_check_gather, one iteration late):
    # here a second gather of the same message layout
    msg = np.zeros(2 * maxc + 16)
    msg[:cnt] = ep[e2_own]
    msg[maxc:maxc + cnt] = xi2[e2_own]
    recv = [torch.zeros(msg.size, dtype=torch.float64) for _ in range(world)]
    dist.all_gather(recv, torch.from_numpy(msg))
    bare_ep = ep.copy()
    for (f, c), buf in zip(sl, recv):
        b = buf.numpy()
        ep[orc.E2[f:f + c]] = b[:c]
        xi2[orc.E2[f:f + c]] = b[maxc:maxc + c]
    nxt = _next_half_step(orc, zp_l, ep, alpha)
    err_next = float(np.max(np.abs(nxt[pm] - nxt_r[pm])))
    err_dual = float(np.max(np.abs(ep[dm] - ep_r[dm])))
    msg[2 * maxc:] = residual_record(ep, xi2)
    dist.all_gather(recv, torch.from_numpy(msg))
    rec = np.max(np.stack([b.numpy()[2 * maxc:] for b in recv]), axis=0)
    err_rec = float(max(np.max(np.abs(rec[:3] - err_r)), np.max(np.abs(rec[3:6] - derr_r))))
    # without X1 the other shards' garbage reaches the top families' kernel projection
    bare = _next_half_step(orc, zp_l, bare_ep, alpha)
    tmask = np.zeros(orc.P, dtype=bool)
    tmask[orc.y_off[orc.stage[:orc.m] == S - 1]] = True
    needed = (world == 1) or not np.allclose(bare[tmask], nxt_r[tmask], atol=1e-3)
    out.put((rank, err_next, err_dual, err_rec, needed))
    dist.barrier()
    dist.destroy_process_group()


def _next_half_step(orc, zp, ep, alpha):
    """the primal half step of the next iteration up to its dynamics projection
    (solver.py:124-131, cache.py:248-257): the kernel projection acts on (y, tau, s) only,
    so it commutes with the dynamics projection on (x, u)."""
    zh = zp - alpha * orc.ell_t(ep, template=zp)
    zh[orc.S0] -= alpha
    return orc.project_on_kernel(zh)


@pytest.mark.parametrize("S,world", [(2, 2), (3, 2), (3, 3)])
def test_x1_exchange_two_processes(S, world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_x1_worker, args=(r, world, port, S, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, err_next, err_dual, err_rec, needed in res:
        assert err_dual <= 1e-12, (rank, err_dual)
        assert err_next <= 1e-12, (rank, err_next)
        assert err_rec <= 1e-12, (rank, err_rec)
        assert needed, f"rank {rank}: the top families did not need the X1 entries"


def test_shard_slices_partition_the_roots():
    for nb in (3, 8, 27, 64, 243):
        for R in (1, 2, 3, 4, 8):
            if nb < R:
                continue
            sl = shard_slices(100, nb, R)
            assert sl[0][0] == 100 and sum(c for _, c in sl) == nb
            assert all(sl[i][0] + sl[i][1] == sl[i + 1][0] for i in range(R - 1))
            assert max(c for _, c in sl) - min(c for _, c in sl) <= 1
