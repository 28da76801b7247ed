#!/usr/bin/env python3
"""Benchmark: Chambolle–Pock iterations/s + L-sweep HBM GB/s (BASELINE.json `metric`).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2] [--no-cpu] [--no-shard]

One step = one CP iteration (solver.py:124-161: L^T half step, prox_f with the
dynamics sweeps and AVaR kernel projection, L half step, prox_g*, residuals and
the stopping test) on the BASELINE configs[1] tree (i.i.d. binary, N = 12:
8,191 nodes, nx = 20, nu = 8), with the iterate already
resident in HBM. The loop runs entirely on the device (graph-replayed, on-device
stopping test); tol = 0 so exactly K iterations run, and exactly K iterations'
kernels are launched (whole 24-iteration graphs plus one remainder graph, all
captured before the timed region).

Multi-GPU (one process per GPU): launched by torch.distributed.run (RANK / WORLD_SIZE /
LOCAL_RANK / MASTER_* in the environment), or, with --gpus N and no WORLD_SIZE, this
script starts the N rank processes itself before anything touches a GPU.
  value: every rank solves its own config-2 tree instance (an MPC-style batch of
      independent problems: same tree, its own x0), no collective on the data path;
      value = total CP iterations/s of the job (weak scaling).
  sharded: ONE config-4 tree (BASELINE configs[3]: branching 3, N = 10, 88,573 nodes,
      nx = 32, nu = 12) whose subtrees below the replicated top are sharded across the N
      GPUs, with RCCL exchanges each iteration; CP iterations/s of that
      one tree (strong scaling; N = 1 is the unsharded solve). Run by N fresh child
      processes under a time limit so that a failure there cannot take the line down.

torch is never imported: its wheel bundles a second ROCm runtime with the same soname
as the /opt/rocm one libraocp_hip.so links, and RCCL (dlopen'ed by the library) cannot
initialise next to it. Barriers and the max-over-ranks go through a socket group.

The JSON line also carries
  roofline: the dominant kernel of the timed CP iteration (largest device time per
            iteration), timed with HIP events on the context's stream over a graph of
            back-to-back launches on a valid control block; algorithmic bytes per launch
            over active entries; peak 8 TB/s HBM3E (cache-resident at this
            size);
  kernels:  the same figure for every kernel of the iteration;
  l_sweep:  L and L^T at config 2, at config 4 (104.6 MB per launch, the HBM regime) and in
            fp32 at config 5 (383.4 MB per launch);
  fp32_config5: BASELINE configs[4] (fp32, 349,525 nodes, nx = 64): L / L^T and CP it/s;
  cpu_baseline: the oracle (vectorised NumPy restatement, oracle/raocp_oracle.py)
            timed on this host on a bounded sample of the same workload, next to the
            reference's own CPU figure measured in the build container.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "raocp-toolbox_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0
METRIC = "Chambolle–Pock iterations/sec + L-sweep HBM GB/s, 10k-node tree nₓ=20"
# the reference's Solver.chock at config 2 on one core of the
# survey container (interpreter-bound), 3.85 s per iteration
REFERENCE_CPU = {"value": 0.26, "unit": "it/s", "cores": 1, "kind": "reference",
                 "sample": "reference Solver.chock (pure Python/NumPy), config 2, 20 iterations, 3.85 s/it, "
                           "measured in the build container (Intel Xeon, 8 cores; BASELINE.md 2)"}


def active_sizes(cache):
    """|P|, |D| over ACTIVE entries: placeholders excluded."""
    pk = cache.packed
    n, m, nx, nu = pk.n, pk.m, pk.nx, pk.nu
    nl = n - m
    P = n * nx + m * nu + (2 * (n - 1) + m) + (n - 1) + n
    nl_box = int((pk.i_box_nl >= 0).sum())
    l_box = int((pk.i_box_l[m:] >= 0).sum())
    D = (2 * (n - 1) + m) + m + (n - 1) * (nx + nu + 2) + nl_box * (nx + nu) + nl * (nx + 2) + l_box * nx
    return P, D


def algorithmic_bytes(cache):
    P, D = active_sizes(cache)
    return 8 * P, 8 * D


def kernel_bytes(cache):
    """Algorithmic bytes per launch of each kernel of the CP iteration:
    every input vector read once, every output written once, tables excluded."""
    P, D = active_sizes(cache)
    pk = cache.packed
    dyn = 2 * (pk.n * pk.nx + pk.m * pk.nu)
    return {
        "k_ell": 8 * (P + D),                # z -> L z
        "k_ell_t": 8 * (P + D),              # eta -> L^T eta
        "k_cpd": 8 * (2 * P + 3 * D),        # p, z+, d -> eta+, xi2
        "k_cpp": 8 * (3 * P + 3 * D),        # p, z+, d, eta+, xi2 -> next half step
        "dynamics": 8 * dyn,                 # x, u in and out (all tier launches of one projection)
    }


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


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


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
            "nproc": os.cpu_count(), "cpu_model": cpu_model(), "blas_threads": int(blas_threads),
            "sample": f"{k} CP iterations of the oracle (NumPy fp64) on the same {orc.n}-node tree in {dt:.1f} s; "
                      f"elementwise work single-threaded, BLAS up to {blas_threads} threads",
            "reference_cpu": REFERENCE_CPU}


class SocketGroup:
    """Minimal host rendezvous (rank 0 serves on MASTER_ADDR, MASTER_PORT + offset): byte
    broadcast, max of a double, barrier."""

    def __init__(self, rank, world, offset=1):
        import struct
        self.rank, self.world, self._struct = rank, world, struct
        addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
        port = int(os.environ.get("MASTER_PORT", "29500")) + offset
        if rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
            srv.bind((addr, port))
            srv.listen(world)
            srv.settimeout(300)
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
                    self.conn = socket.create_connection((addr, port), timeout=600)
                    break
                except OSError:
                    if time.time() - t0 > 300:
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


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_env(rank, world, port):
    env = dict(os.environ)
    env.update({"RANK": str(rank), "LOCAL_RANK": str(rank), "WORLD_SIZE": str(world),
                "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host (RCCL)
    return env


def spawn(world, argv, timeout=None):
    """Start `world` rank processes of this script (fresh, before any GPU call here).
    Returns (rank-0 stdout, return codes); kills the group on timeout."""
    port = free_port()
    procs = []
    for r in range(world):
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=rank_env(r, world, port),
                                      stdout=subprocess.PIPE if r == 0 else None, start_new_session=True))
    out, rcs = b"", []
    t_end = None if timeout is None else time.time() + timeout
    try:
        out = procs[0].communicate(timeout=timeout)[0] or b""
        for p in procs:
            left = None if t_end is None else max(1.0, t_end - time.time())
            p.wait(timeout=left)
    except subprocess.TimeoutExpired:
        pass
    for p in procs:
        if p.poll() is None:
            try:
                os.killpg(p.pid, 9)
            except OSError:
                pass
            p.wait()
        rcs.append(p.returncode)
    return out.decode(errors="replace"), rcs


def timed_cp(nat, x0, alpha, steps, warmup, group):
    """W untimed iterations, then exactly `steps` iterations bracketed by barrier + device
    synchronize; returns (max wall over ranks, device ms of this rank)."""
    from raocp.core._native import device_synchronize
    if warmup > 0:
        nat.cp_bench(x0, warmup, alpha)
    # graphs for exactly `steps` iterations and the run's initial iterate, set up outside the
    # timing: the timed call launches the K iterations' kernels only
    nat.cp_prepare(steps, x0, alpha)
    if group:
        group.barrier()
    device_synchronize(nat.device)
    t0 = time.perf_counter()
    dev_ms = nat.cp_bench(None, steps, alpha)
    device_synchronize(nat.device)
    if group:
        group.barrier()
    wall = time.perf_counter() - t0
    if group:
        wall = group.max(wall)
    return wall, dev_ms


def shard_leg(args):
    """One process of the sharded config-4 solve (a child of rank 0, see spawn)."""
    import raocp.core as core
    from raocp.core._native import comm_unique_id, load_library
    from raocp.problems import build_problem, recipe_config
    load_library()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    group = SocketGroup(rank, world) if world > 1 else None
    recipe = recipe_config(args.shard_config, seed=0)
    cache = core.Cache(build_problem(recipe)[1])
    nat = cache.native
    alpha = 0.999 / nat.step_size()
    if world > 1:
        nat.shard(rank, world)
        uid = group.bcast(comm_unique_id() if rank == 0 else b"")
        nat.comm_init(uid, rank, world)
    wall, dev_ms = timed_cp(nat, recipe["x0"], alpha, args.shard_steps, args.shard_warmup, group)
    if rank == 0:
        lo, hi = nat.shard_owned() if world > 1 else (None, None)
        print(json.dumps({"its": args.shard_steps / wall, "wall_s": wall, "device_ms": dev_ms, "steps": args.shard_steps,
                          "nodes": cache.packed.n, "owned_leaves_rank0": None if lo is None else int(hi[-1] - lo[-1])}),
              flush=True)
    if group:
        group.barrier()


def sharded_entry(args, world):
    """The config-4 strong-scaling leg: N = 1 in this process (no shards, no RCCL); N > 1 by
    N fresh child processes (one per GPU) under a time limit."""
    desc = {"config": f"SURVEY.md 8(d) config {args.shard_config} (BASELINE configs[{args.shard_config - 1}]): "
                      "ONE tree, subtrees below the replicated top sharded across the GPUs",
            "n_gpus": world, "steps": args.shard_steps, "unit": "it/s", "scaling": "strong"}
    argv = ["--shard-leg", "--shard-config", str(args.shard_config), "--shard-steps", str(args.shard_steps),
            "--shard-warmup", str(args.shard_warmup)]
    out, rcs = spawn(world, argv, timeout=args.shard_timeout)
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    if any(rc != 0 for rc in rcs) or not line:
        desc.update({"value": None, "error": f"shard leg failed: return codes {rcs}"})
        return desc
    r = json.loads(line[-1])
    desc.update({"value": r["its"], "ms_per_step": 1e3 * r["wall_s"] / r["steps"], "nodes": r["nodes"],
                 "device_ms_per_step": r["device_ms"] / r["steps"],
                 "exchanges": "per iteration: all-gather of the boundary roots' q rows (dynamics), all-gather of "
                              "their eta2 entries, all-reduce (max) of the residual maxima" if world > 1 else None})
    return desc


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
    ap.add_argument("--no-shard", action="store_true", help="skip the sharded config-4 leg")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 config-5 leg")
    ap.add_argument("--fp32-steps", type=int, default=48)
    ap.add_argument("--shard-config", type=int, default=4)
    ap.add_argument("--shard-steps", type=int, default=200)
    ap.add_argument("--shard-warmup", type=int, default=20)
    ap.add_argument("--shard-timeout", type=float, default=240.0)
    ap.add_argument("--shard-leg", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.shard_leg:
        return shard_leg(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start the N rank processes (no GPU has been touched in this one)
        out, rcs = spawn(args.gpus, sys.argv[1:])
        sys.stdout.write(out)
        sys.stdout.flush()
        return rcs[0] if rcs[0] else max(abs(rc) for rc in rcs)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch one process per GPU)")

    import raocp.core as core
    from raocp.core._native import load_library
    from raocp.problems import build_problem, recipe_config
    load_library()
    group = SocketGroup(rank, world) if world > 1 else None

    recipe = recipe_config(args.config, seed=0)
    if world > 1:  # each rank its own instance (same tree / dynamics, its own initial state)
        recipe["x0"] = np.random.default_rng(1000 + rank).standard_normal(recipe["x0"].size)
    tree, prob = build_problem(recipe)
    cache = core.Cache(prob)
    nat = cache.native
    alpha = 0.999 / nat.step_size()

    wall, dev_ms = timed_cp(nat, recipe["x0"], alpha, args.steps, args.warmup, group)
    its = world * args.steps / wall

    if rank != 0:
        group.barrier()  # rank 0 measures the rest; the sharded leg uses every GPU
        return 0

    # per-kernel HIP-event timings of the CP iteration's kernels (graph of back-to-back
    # launches on a valid control block, the context's stream), algorithmic bytes / time
    kb = kernel_bytes(cache)
    reps = args.op_reps
    ms = {"k_cpd": nat.op_bench(2, reps), "k_cpp": nat.op_bench(6, reps), "dynamics": nat.op_bench(9, max(1, reps // 4)),
          "k_ell": nat.op_bench(0, reps), "k_ell_t": nat.op_bench(1, reps)}
    kernels = {}
    for k, t in ms.items():
        gbs = kb[k] / (t * 1e-3) / 1e9
        kernels[k] = {"us_per_launch": t * 1e3, "bytes_per_launch": kb[k], "achieved": gbs, "frac": gbs / HBM_PEAK_GBS,
                      "in_cp_iteration": k in ("k_cpd", "k_cpp", "dynamics")}
    # the dominant single kernel of the timed iteration (the dynamics projection is a chain of
    # launches, one per tier, reported under kernels["dynamics"] as a whole)
    dom = max(("k_cpd", "k_cpp"), key=lambda k: ms[k])
    tname = {"k_cpd": f"k_cpd<{cache.packed.nx}, {cache.packed.nu}>", "k_cpp": f"k_cpp<{cache.packed.nx}, {cache.packed.nu}>"}
    traffic, traffic_src = pmc_traffic(tname.get(dom, dom))
    roofline = {"bound": "hbm", "kernel": dom, "achieved": kernels[dom]["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": kernels[dom]["frac"], "traffic": traffic, "traffic_source": traffic_src,
                "bytes_per_launch": kb[dom], "us_per_launch": kernels[dom]["us_per_launch"],
                "note": "dominant kernel of the timed CP iteration; working set L2/MALL-resident at this size "
                        "(SURVEY.md 8(d)), so the HBM fraction is an effective cache-resident bandwidth"}

    # HBM regime: the L / L^T kernels at config 4 (88,573 nodes, nx = 32,
    # nu = 12: 104.6 MB per application, past L2)
    # the kernels the default selection launches on these uniform trees (the
    # rocprofv3 names in profiles/<latest>/prof_kernel_stats.csv)
    l_sweep = {"config2": {"L": dict(kernels["k_ell"], kernel="k_ell3<double, 20, 8>"),
                           "L_transpose": dict(kernels["k_ell_t"], kernel="k_ellt3<double, 20, 8, 2>")}}
    if not args.no_hbm:
        r4 = recipe_config(4, seed=0)
        c4 = core.Cache(build_problem(r4)[1])
        b4P, b4D = algorithmic_bytes(c4)
        m4l, m4t = c4.native.op_bench(0, 200), c4.native.op_bench(1, 200)
        bb = b4P + b4D
        l_sweep["config4"] = {"config": "SURVEY.md 8(d) config 4: 88,573 nodes, nx=32, nu=12", "bytes_per_launch": bb,
                              "L": {"kernel": "k_ell3<double, 32, 12>", "us_per_launch": m4l * 1e3,
                                    "achieved": bb / (m4l * 1e-3) / 1e9,
                                    "frac": bb / (m4l * 1e-3) / 1e9 / HBM_PEAK_GBS},
                              "L_transpose": {"kernel": "k_ellt3<double, 32, 12, 1>", "us_per_launch": m4t * 1e3,
                                              "achieved": bb / (m4t * 1e-3) / 1e9,
                                              "frac": bb / (m4t * 1e-3) / 1e9 / HBM_PEAK_GBS},
                              "unit": "GB/s", "peak": HBM_PEAK_GBS}
        del c4
    # BASELINE configs[4]: fp32, 349,525 nodes, nx = 64, nu = 16 (383.4 MB per L): L / L^T and
    # the CP loop of an fp32 context
    fp32 = None
    if not args.no_fp32:
        r5 = recipe_config(5, seed=0)
        c5 = core.Cache(build_problem(r5)[1], dtype="float32")
        P5, D5 = active_sizes(c5)
        b5 = 4 * (P5 + D5)
        m5l, m5t = c5.native.op_bench(0, 100), c5.native.op_bench(1, 100)
        a5 = 0.999 / c5.native.step_size(rtol=1e-7)
        w5, d5 = timed_cp(c5.native, r5["x0"], a5, args.fp32_steps, 2, None)
        fp32 = {"config": "SURVEY.md 8(d) config 5 (BASELINE configs[4]): branching 4, N=9, 349,525 nodes, nx=64, "
                          "nu=16, fp32 iterate / tables / products (MFMA f32 tiles)", "dtype": "f32",
                "bytes_per_launch": b5,
                "L": {"kernel": "k_ell3<float, 64, 16>", "us_per_launch": m5l * 1e3, "achieved": b5 / (m5l * 1e-3) / 1e9,
                      "frac": b5 / (m5l * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "L_transpose": {"kernel": "k_ellt3<float, 64, 16, 1>", "us_per_launch": m5t * 1e3,
                                "achieved": b5 / (m5t * 1e-3) / 1e9,
                                "frac": b5 / (m5t * 1e-3) / 1e9 / HBM_PEAK_GBS},
                "cp": {"value": args.fp32_steps / w5, "unit": "it/s", "steps": args.fp32_steps,
                       "ms_per_step": 1e3 * w5 / args.fp32_steps},
                "unit": "GB/s", "peak": HBM_PEAK_GBS}
        l_sweep["config5_fp32"] = {k: fp32[k] for k in ("config", "bytes_per_launch", "L", "L_transpose", "unit", "peak")}
        del c5

    out = {
        "metric": METRIC, "value": its, "unit": "it/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": 1e3 * wall / args.steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f64", "data": "synthetic",
        "config": {"workload": f"BASELINE configs[1]: i.i.d. binary scenario tree, N=12, {cache.packed.n} nodes, "
                               f"nx={cache.packed.nx}, nu={cache.packed.nu}, AVaR 0.9, boxes +-1 "
                               f"(SURVEY.md 8(d) config {args.config})",
                   "nodes": cache.packed.n, "nx": cache.packed.nx, "nu": cache.packed.nu, "alpha": alpha, "tol": 0.0,
                   "parallelism": f"replicas{world}: one independent tree instance per GPU" if world > 1 else "1 GPU"},
        "device_ms_per_step": dev_ms / args.steps,
        "roofline": roofline,
        "kernels": kernels,
        "l_sweep": l_sweep,
        "fp32_config5": fp32,
    }
    if not args.no_shard:
        out["sharded"] = sharded_entry(args, world) if world > 1 else None
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(recipe, args.cpu_seconds)
    if world == 1 and not args.no_shard:
        # N = 1 point of the strong-scaling leg: the same config-4 tree unsharded in this process
        r4 = recipe_config(args.shard_config, seed=0)
        c4 = core.Cache(build_problem(r4)[1])
        a4 = 0.999 / c4.native.step_size()
        w4, d4 = timed_cp(c4.native, r4["x0"], a4, args.shard_steps, args.shard_warmup, None)
        out["sharded"] = {"config": f"SURVEY.md 8(d) config {args.shard_config} (BASELINE configs[{args.shard_config - 1}]): "
                                    "ONE tree, unsharded on 1 GPU (the N = 1 point of the strong-scaling leg)",
                          "n_gpus": 1, "steps": args.shard_steps, "unit": "it/s", "scaling": "strong",
                          "value": args.shard_steps / w4, "ms_per_step": 1e3 * w4 / args.shard_steps,
                          "device_ms_per_step": d4 / args.shard_steps, "nodes": c4.packed.n}
    print(json.dumps(out), flush=True)
    if group:
        group.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
