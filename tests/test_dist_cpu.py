"""CPU, world_size 2-3: the host side of the multi-GPU paths.

* the gloo max / all-gather pattern of a timed region (the slowest rank sets the job time;
  every rank solves its own instance in bench.py's replica headline);
* the SocketGroup rendezvous (uid broadcast, max, barrier) bench.py uses (torch must not
  share a process with the RCCL the library binds);
* bench.py --gpus N without WORLD_SIZE starting its own rank processes;
* subtree sharding on the host: the dynamics projection by two processes that see only
  their own subtrees below the replicated top, exchanging the roots' q rows (X2).
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


def test_shard_slices_partition_the_roots():
    for nb in (3, 8, 27, 64, 243):
        for R in (1, 2, 3, 4, 8):
            if nb < R:
                continue
            sl = shard_slices(100, nb, R)
            assert sl[0][0] == 100 and sum(c for _, c in sl) == nb
            assert all(sl[i][0] + sl[i][1] == sl[i + 1][0] for i in range(R - 1))
            assert max(c for _, c in sl) - min(c for _, c in sl) <= 1
