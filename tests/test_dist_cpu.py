"""CPU, world_size 2: the host side of bench.py's multi-GPU modes.

* --mode replicas: gloo process group; the timed region's wall time is the MAX over
  ranks and every rank solves its own instance (distinct initial states);
* --mode shard: the SocketGroup rendezvous (uid broadcast, max, barrier) that replaces
  torch.distributed there (torch must not share a process with the RCCL the library binds).
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
