#!/usr/bin/env python3
"""Benchmark: Chambolle–Pock iterations/s + L-sweep HBM GB/s (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2] [--no-cpu]

One step = one CP iteration (solver.py:124-161: L^T half step, prox_f with the
dynamics sweeps and AVaR kernel projection, L half step, prox_g*, residuals and
the stopping test) on the BASELINE configs[1] tree (i.i.d. binary, N = 12:
8,191 nodes, nx = 20, nu = 8), with the iterate already
resident in HBM. The loop runs entirely on the device (graph-replayed, on-device
stopping test); tol = 0 so exactly K iterations run.

Multi-GPU (N > 1, one process per GPU launched by torch.distributed.run):
  --mode replicas (default): every rank solves its own tree instance (an MPC-style
      batch of independent problems: same tree, its own x0), no collective on the data
      path; value = total CP iterations/s of the job (weak scaling).
  --mode shard: ONE tree, its subtrees below the replicated top sharded across the
      ranks; per iteration an RCCL all-gather of the roots' q rows, one
      of the roots' eta2/xi2 entries and an all-reduce of the residual maxima; value =
      CP iterations/s of that one tree (strong scaling).

The JSON line also carries
  roofline: the L-sweep kernel (k_ell, operators.py:19-53) timed with HIP events
            on its own stream over a graph of back-to-back launches, algorithmic bytes =
            8 (|P| + |D|) per launch, against the 8 TB/s HBM3E peak
            (cache-resident at this size);
  l_sweep_hbm: the same kernels at config 4 (104.6 MB per launch, the HBM regime);
  cpu_baseline: the oracle (vectorised NumPy restatement, oracle/raocp_oracle.py)
            timed on this host on a bounded sample of the same workload.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raocp-toolbox_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0


def algorithmic_bytes(cache):
    """w (|P| + |D|) over ACTIVE entries: placeholders excluded."""
    pk = cache.packed
    n, m, nx, nu = pk.n, pk.m, pk.nx, pk.nu
    nl = n - m
    P = n * nx + m * nu + (2 * (n - 1) + m) + (n - 1) + n
    nl_box = int((pk.i_box_nl >= 0).sum())
    l_box = int((pk.i_box_l[m:] >= 0).sum())
    D = (2 * (n - 1) + m) + m + (n - 1) * (nx + nu + 2) + nl_box * (nx + nu) + nl * (nx + 2) + l_box * nx
    return 8 * P, 8 * D


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/<round>/traffic.json, written by tools/traffic.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this bench), or None."""
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json")), reverse=True):
        try:
            k = json.load(open(f))["kernels"].get(kernel)
        except Exception:
            continue
        if k:
            return k["traffic_bytes"], os.path.relpath(f, ROOT)
    return None, None


def cpu_baseline(recipe, budget_s=12.0):
    """Oracle CP iterations on the host (bounded sample of the same workload)."""
    from oracle.raocp_oracle import OracleProblem
    from raocp.problems import build_problem
    try:
        from threadpoolctl import threadpool_info
        blas_threads = max([t.get("num_threads", 1) for t in threadpool_info()] or [1])
    except Exception:
        blas_threads = 1
    tree, prob = build_problem(recipe)
    orc = OracleProblem(prob)
    orc.offline()
    lam, alpha = orc.step_size()
    p = orc.initial_primal(recipe["x0"])
    d = np.zeros(orc.D)
    orc.cp_iteration(p, d, alpha, recipe["x0"])  # warm-up
    k = 0
    t0 = time.perf_counter()
    while True:
        p, d, _, _ = orc.cp_iteration(p, d, alpha, recipe["x0"])
        k += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return {"value": k / dt, "unit": "it/s", "cores": int(blas_threads), "kind": "port",
            "sample": f"{k} CP iterations of the oracle (NumPy fp64) on the same {orc.n}-node tree in {dt:.1f} s; "
                      f"elementwise work single-threaded, BLAS up to {blas_threads} threads"}


class SocketGroup:
    """Minimal host rendezvous for --mode shard (rank 0 serves; MASTER_ADDR, MASTER_PORT+1).
    torch is not imported in shard mode: its wheel bundles a second ROCm runtime, and the
    RCCL that libraocp_hip.so binds cannot initialise in a process that imported it."""

    def __init__(self, rank, world):
        import socket
        import struct
        self.rank, self.world, self._struct = rank, world, struct
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + 1
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            self.peers = [None] * world
            for _ in range(world - 1):
                conn, _ = srv.accept()
                r = struct.unpack("!i", self._recv(conn, 4))[0]
                self.peers[r] = conn
            srv.close()
        else:
            t0 = time.time()
            while True:
                try:
                    self.conn = socket.create_connection((addr, port), timeout=60)
                    break
                except OSError:
                    if time.time() - t0 > 120:
                        raise
                    time.sleep(0.2)
            self.conn.sendall(struct.pack("!i", rank))

    @staticmethod
    def _recv(conn, n):
        buf = b""
        while len(buf) < n:
            chunk = conn.recv(n - len(buf))
            if not chunk:
                raise ConnectionError("peer closed")
            buf += chunk
        return buf

    def bcast(self, data):
        if self.rank == 0:
            for c in self.peers[1:]:
                c.sendall(self._struct.pack("!i", len(data)) + data)
            return data
        n = self._struct.unpack("!i", self._recv(self.conn, 4))[0]
        return self._recv(self.conn, n)

    def max(self, v):
        st = self._struct
        if self.rank == 0:
            m = v
            for c in self.peers[1:]:
                m = max(m, st.unpack("!d", self._recv(c, 8))[0])
            for c in self.peers[1:]:
                c.sendall(st.pack("!d", m))
            return m
        self.conn.sendall(st.pack("!d", v))
        return st.unpack("!d", self._recv(self.conn, 8))[0]

    def barrier(self):
        self.max(0.0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--op-reps", type=int, default=2000)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-hbm", action="store_true", help="skip the config-4 L / L^T measurement")
    ap.add_argument("--mode", choices=["replicas", "shard"], default="replicas",
                    help="N > 1: independent tree per GPU (replicas, weak scaling) or ONE tree sharded by "
                         "subtree across the GPUs with RCCL exchanges (shard, strong scaling)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    import raocp.core as core
    from raocp.core._native import load_library
    load_library()  # bind /opt/rocm's HIP runtime before torch (gloo only, no torch.cuda) is imported
    group = None
    if world > 1 and args.mode == "replicas":
        import torch.distributed as dist
        dist.init_process_group("gloo")
    elif world > 1:
        group = SocketGroup(rank, world)

    from raocp.problems import build_problem, recipe_config

    recipe = recipe_config(args.config, seed=0)
    shard = world > 1 and args.mode == "shard"
    if world > 1 and not shard:  # replicas: each rank its own instance (same tree/dynamics, own initial state)
        recipe["x0"] = np.random.default_rng(1000 + rank).standard_normal(recipe["x0"].size)
    tree, prob = build_problem(recipe)
    cache = core.Cache(prob)
    nat = cache.native
    lam = nat.step_size()
    alpha = 0.999 / lam
    if shard:
        # one tree, subtrees sharded across the ranks; RCCL communicator from a uid broadcast
        from raocp.core._native import comm_unique_id
        nat.shard(rank, world)
        uid = group.bcast(comm_unique_id() if rank == 0 else b"")
        nat.comm_init(uid, rank, world)

    # warm-up (W untimed iterations; also captures the CP graph)
    if args.warmup > 0:
        nat.cp_bench(recipe["x0"], args.warmup, alpha)

    def barrier():
        if dist is not None:
            dist.barrier()
        if group is not None:
            group.barrier()

    # The timed region is bracketed by barrier + device synchronize. The synchronize is
    # hipDeviceSynchronize through libraocp_hip.so: torch's wheel bundles its own
    # libamdhip64 (ROCm 7.0) with the same soname as /opt/rocm's (7.2) the library is
    # built against, so torch.cuda must not be initialised in this process.
    from raocp.core._native import device_synchronize
    barrier()
    device_synchronize(nat.device)
    t0 = time.perf_counter()
    dev_ms = nat.cp_bench(recipe["x0"], args.steps, alpha)
    device_synchronize(nat.device)
    barrier()
    wall = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([wall], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall = float(t[0])
    if group is not None:
        wall = group.max(wall)
    its = (1 if shard else world) * args.steps / wall

    # L-sweep roofline: k_ell timed with HIP events on the context's stream
    bP, bD = algorithmic_bytes(cache)
    ms_l = nat.op_bench(0, args.op_reps)
    ms_lt = nat.op_bench(1, args.op_reps)
    gbs_l = (bP + bD) / (ms_l * 1e-3) / 1e9
    gbs_lt = (bP + bD) / (ms_lt * 1e-3) / 1e9

    if rank != 0:
        barrier()
        return
    traffic, traffic_src = pmc_traffic(f"k_ell<{cache.packed.nx}, {cache.packed.nu}>")
    # HBM regime: the same L / L^T kernels at config 4 (88,573 nodes,
    # nx = 32, nu = 12: 104.6 MB per application, past L2)
    hbm = None
    if not args.no_hbm:
        r4 = recipe_config(4, seed=0)
        c4 = core.Cache(build_problem(r4)[1])
        b4P, b4D = algorithmic_bytes(c4)
        m4l, m4t = c4.native.op_bench(0, 200), c4.native.op_bench(1, 200)
        hbm = {"config": "SURVEY.md 8(d) config 4: 88,573 nodes, nx=32, nu=12", "bytes_per_launch": b4P + b4D,
               "L": {"us_per_launch": m4l * 1e3, "achieved": (b4P + b4D) / (m4l * 1e-3) / 1e9,
                     "frac": (b4P + b4D) / (m4l * 1e-3) / 1e9 / HBM_PEAK_GBS},
               "L_transpose": {"us_per_launch": m4t * 1e3, "achieved": (b4P + b4D) / (m4t * 1e-3) / 1e9,
                               "frac": (b4P + b4D) / (m4t * 1e-3) / 1e9 / HBM_PEAK_GBS},
               "unit": "GB/s", "peak": HBM_PEAK_GBS}
    out = {
        "metric": "Chambolle–Pock iterations/sec + L-sweep HBM GB/s, 10k-node tree nₓ=20",
        "value": its, "unit": "it/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * wall / args.steps, "higher_is_better": True,
        "scaling": "strong" if shard else "weak", "vs_baseline": None, "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"BASELINE configs[1]: i.i.d. binary scenario tree, N=12, {cache.packed.n} nodes, "
                               f"nx={cache.packed.nx}, nu={cache.packed.nu}, AVaR 0.9, boxes +-1 "
                               f"(SURVEY.md 8(d) config {args.config})",
                   "nodes": cache.packed.n, "nx": cache.packed.nx, "nu": cache.packed.nu,
                   "alpha": alpha, "tol": 0.0,
                   "parallelism": (f"shard{world}: one tree, subtrees sharded across GPUs, RCCL exchanges" if shard else
                                   f"replicas{world}: one independent tree instance per GPU") if world > 1 else "1 GPU"},
        "device_ms_per_step": dev_ms / args.steps,
        "roofline": {"bound": "hbm", "kernel": "k_ell (L sweep)", "achieved": gbs_l, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": gbs_l / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "bytes_per_launch": bP + bD, "us_per_launch": ms_l * 1e3,
                     "note": "working set L2/MALL-resident at this size (SURVEY.md 8(d))"},
        "l_transpose": {"kernel": "k_ell_t", "achieved": gbs_lt, "unit": "GB/s", "us_per_launch": ms_lt * 1e3},
        "l_sweep_hbm": hbm,
    }
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(recipe, args.cpu_seconds)
    print(json.dumps(out))
    barrier()


if __name__ == "__main__":
    main()
