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
  sharded: two strong-scaling legs, {"config4", "config5_fp32"}: ONE config-4 tree
      (BASELINE configs[3]: branching 3, N = 10, 88,573 nodes, nx = 32, nu = 12, fp64) and
      ONE config-5 tree (configs[4]: branching 4, N = 9, 349,525 nodes, nx = 64, nu = 16,
      fp32) whose subtrees below the replicated top are sharded across the N GPUs
      (SURVEY.md 8(e)), with RCCL exchanges each iteration; CP iterations/s of that one tree
      (N = 1 is the unsharded solve, reported from the one-GPU legs below; both run k_cp5 and
      k_dy3 with its merged top, each entry names its kernels). At N > 1 each
      leg runs as N fresh child processes under a time limit, so that a failure there
      cannot take the line down.

torch is never imported: its wheel bundles a second ROCm runtime with the same soname
as the /opt/rocm one libraocp_hip.so links, and RCCL (dlopen'ed by the library) cannot
initialise next to it. Barriers and the max-over-ranks go through a socket group.

The JSON line also carries
  roofline: the part of the timed CP iteration with the larger device time (the kernel after
            the dynamics sweep -- the fused k_cp3 on the benchmark trees -- or the dynamics
            projection), timed with HIP events on the context's stream over a graph of
            back-to-back launches on a valid control block; algorithmic bytes per launch over
            active entries; peak 8 TB/s HBM3E (cache-resident at this size);
            its share of the step and the other part's figure next to it;
  kernels:  both parts of the iteration, named by the library's own selection;
  l_sweep:  L and L^T at config 2 (cache-resident), at config 4 and in fp32 at config 5 over
            rotating buffer sets larger than the 256 MiB Infinity Cache (the HBM regime);
  config4 / fp32_config5: BASELINE configs[3] (fp64, 88,573 nodes, nx = 32) and configs[4]
            (fp32, 349,525 nodes, nx = 64) on one GPU: CP it/s, kernels, roofline, L / L^T;
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


def kernel_bytes(cache, w=8):
    """Algorithmic bytes per launch: every input vector read once, every
    output written once, tables excluded. The CP iteration after the dynamics sweep:
    the fused k_cp3 reads p, z+, d and writes eta+ and the next half step (3|P| + 2|D|);
    the two-launch k_cpd* + k_cpp* also write and re-read xi2 and re-read p, z+, d
    (5|P| + 6|D|). The dynamics projection reads and writes x, u. The one
    launch of both (k_drc) reads the half step's x, u and writes the projected x+, u+, then
    runs the CP iteration with x+, u+ from LDS: 3|P| + 2|D| + (n nx + m nu)."""
    P, D = active_sizes(cache)
    pk = cache.packed
    xu = pk.n * pk.nx + pk.m * pk.nu
    return {"cp_fused": w * (3 * P + 2 * D), "cp_two": w * (5 * P + 6 * D),
            "dynamics": w * 2 * xu, "dyn_cp": w * (3 * P + 2 * D + xu), "L": w * (P + D)}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/<round>/traffic.json, written by tools/traffic.py from rocprofv3 FETCH_SIZE /
    WRITE_SIZE passes of this bench), or None. `kernel` may list several launches as
    "name xcount" terms joined by " + " (raocp_kernel_info of the dynamics projection):
    their per-launch traffic is summed."""
    import glob
    import re
    terms = []
    for t in kernel.split(" + "):
        m = re.fullmatch(r"(.*) x(\d+)", t.strip())
        terms.append((m.group(1), int(m.group(2))) if m else (t.strip(), 1))
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json")), reverse=True):
        try:
            ks = json.load(open(f))["kernels"]
        except Exception:
            continue
        # a profiled name may carry template arguments raocp_kernel_info leaves out (the box
        # pattern, the block size): "k_drc<20, 8, 2>" matches "k_drc<20, 8, 2, 1>"
        def find(name):
            if name in ks:
                return ks[name]
            stem = name[:-1] + ", " if name.endswith(">") else None
            hits = [v for k, v in ks.items() if stem and k.startswith(stem)]
            return hits[0] if len(hits) == 1 else None
        found = [(find(name), cnt) for name, cnt in terms]
        if all(v is not None for v, _ in found):
            return sum(cnt * v["traffic_bytes"] for v, cnt in found), os.path.relpath(f, ROOT)
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
    """One process of a sharded solve (config 4 fp64 or config 5 fp32; a child of rank 0, see
    spawn)."""
    import raocp.core as core
    from raocp.core._native import comm_unique_id, load_library
    from raocp.problems import build_problem, recipe_config
    load_library()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    group = SocketGroup(rank, world) if world > 1 else None
    recipe = recipe_config(args.shard_config, seed=0)
    cache = core.Cache(build_problem(recipe)[1], dtype=args.shard_dtype)
    nat = cache.native
    alpha = 0.999 / nat.step_size(rtol=1e-7 if args.shard_dtype == "float32" else 1e-14)
    if world > 1:
        nat.shard(rank, world)
        uid = group.bcast(comm_unique_id() if rank == 0 else b"")
        nat.comm_init(uid, rank, world)
    wall, dev_ms = timed_cp(nat, recipe["x0"], alpha, args.shard_steps, args.shard_warmup, group)
    if rank == 0:
        lo, hi = nat.shard_owned() if world > 1 else (None, None)
        print(json.dumps({"its": args.shard_steps / wall, "wall_s": wall, "device_ms": dev_ms, "steps": args.shard_steps,
                          "nodes": cache.packed.n, "owned_leaves_rank0": None if lo is None else int(hi[-1] - lo[-1]),
                          "cp_kernel": nat.kernel_info(10), "dynamics_kernels": nat.kernel_info(9)}),
              flush=True)
    if group:
        group.barrier()


# the strong-scaling legs: (config, dtype) — BASELINE configs[3] (config 4, fp64) and
# configs[4] (config 5 in fp32, "report 1/2/4/8-GPU scaling")
SHARD_LEGS = ((4, "float64"), (5, "float32"))


def leg_key(cfg, dtype):
    return f"config{cfg}" + ("_fp32" if dtype == "float32" else "")


def sharded_entry(args, world, cfg, dtype, steps, warmup):
    """One strong-scaling leg at N > 1: N fresh child processes (one per GPU) under a time
    limit, ONE tree whose subtrees below the replicated top are sharded across them."""
    desc = {"config": f"SURVEY.md 8(d) config {cfg} (BASELINE configs[{cfg - 1}]): "
                      "ONE tree, subtrees below the replicated top sharded across the GPUs",
            "dtype": "f32" if dtype == "float32" else "f64",
            "n_gpus": world, "steps": steps, "unit": "it/s", "scaling": "strong"}
    argv = ["--shard-leg", "--shard-config", str(cfg), "--shard-dtype", dtype, "--shard-steps", str(steps),
            "--shard-warmup", str(warmup)]
    out, rcs = spawn(world, argv, timeout=args.shard_timeout)
    line = [ln for ln in out.splitlines() if ln.startswith("{")]
    if any(rc != 0 for rc in rcs) or not line:
        desc.update({"value": None, "error": f"shard leg failed: return codes {rcs}"})
        return desc
    r = json.loads(line[-1])
    desc.update({"value": r["its"], "ms_per_step": 1e3 * r["wall_s"] / r["steps"], "nodes": r["nodes"],
                 "device_ms_per_step": r["device_ms"] / r["steps"],
                 "cp_kernel": r.get("cp_kernel"), "dynamics_kernels": r.get("dynamics_kernels"),
                 "exchanges": "per iteration: all-gather of the boundary roots' q rows (dynamics), all-gather of "
                              "two entries per root (k_cp5: s of the half step and eta+ of eta2) together with the "
                              "previous iteration's residual record (the stopping test runs one iteration late, so "
                              "the residual reduction rides on it)"
                              if world > 1 else None})
    return desc


def _rate(b, us):
    gbs = b / (us * 1e-6) / 1e9
    return {"us_per_launch": us, "bytes_per_launch": b, "achieved": gbs, "frac": gbs / HBM_PEAK_GBS}


def iteration_kernels(nat, cache, w, reps, dev_ms_per_step):
    """HIP-event times (graph of back-to-back launches on the context's stream, valid control
    block) of the two parts of a CP iteration: the dynamics projection (op 9: a chain of tier
    launches, reported as a whole) and the kernel(s) after it (op 10: the fused k_cp3, or
    k_cpd* + k_cpp*); kernel names from the library's own selection (raocp_kernel_info).
    The roofline names the part with the larger device time per iteration."""
    kb = kernel_bytes(cache, w)
    name_cp, name_dyn, name_one = nat.kernel_info(10), nat.kernel_info(9), nat.kernel_info(11)
    fused = name_cp.startswith(("k_cp3", "k_cp4", "k_cp5", "k_cp6"))
    t_cp = 1e3 * nat.op_bench(10, reps)
    t_dyn = 1e3 * nat.op_bench(9, max(1, reps // 4))
    # with a one-launch iteration (k_drc) the loop runs neither standalone part: they are
    # reported beside it (the RAOCP_DRC=0 loop's kernels), the roofline is the one launch's
    kernels = {"cp": dict(_rate(kb["cp_fused" if fused else "cp_two"], t_cp), kernel=name_cp,
                          in_cp_iteration=not name_one),
               "dynamics": dict(_rate(kb["dynamics"], t_dyn), kernel=name_dyn, in_cp_iteration=not name_one)}
    if name_one:
        t_one = 1e3 * nat.op_bench(11, reps)
        kernels["dynamics_cp"] = dict(_rate(kb["dyn_cp"], t_one), kernel=name_one, in_cp_iteration=True)
    dev_us = 1e3 * dev_ms_per_step
    for k in kernels.values():
        k["share_of_step"] = k["us_per_launch"] / dev_us if dev_us > 0 and k["in_cp_iteration"] else None
    dom = max((k for k in kernels if kernels[k]["in_cp_iteration"]), key=lambda k: kernels[k]["us_per_launch"])
    traffic, src = pmc_traffic(kernels[dom]["kernel"])
    roofline = {"bound": "hbm", "kernel": kernels[dom]["kernel"], "part": dom, "achieved": kernels[dom]["achieved"],
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": kernels[dom]["frac"], "traffic": traffic,
                "traffic_source": src, "bytes_per_launch": kernels[dom]["bytes_per_launch"],
                "us_per_launch": kernels[dom]["us_per_launch"], "share_of_step": kernels[dom]["share_of_step"],
                "other_part": {k: kernels[k]["kernel"] + f": {kernels[k]['us_per_launch']:.1f} us, frac "
                                                         f"{kernels[k]['frac']:.3f}" for k in kernels if k != dom}}
    return kernels, roofline


def op_pair(nat, cache, w, reps, nsets):
    """L / L^T (standalone operators): HIP events over a graph of back-to-back launches;
    nsets > 1 cycles over that many input / output buffer pairs (beyond the 256 MiB
    Infinity Cache for configs 4 and 5: every launch reads HBM)."""
    P, D = active_sizes(cache)
    b = w * (P + D)
    res = {}
    for op, key in ((0, "L"), (1, "L_transpose")):
        ms = nat.op_bench_rot(op, reps, nsets) if nsets > 1 else nat.op_bench(op, reps)
        res[key] = dict(_rate(b, 1e3 * ms), kernel=nat.kernel_info(op))
    res.update({"buffer_sets": nsets, "bytes_per_set": w * (P + D),
                "regime": "HBM (buffer sets beyond the 256 MiB Infinity Cache)" if nsets * b > 256 * 2 ** 20
                else "cache-resident"})
    return res


def config_leg(cfg, dtype, steps, warmup, reps, nsets):
    """One BASELINE config on this GPU: CP it/s of the timed loop, its kernels and roofline,
    L / L^T over rotating buffer sets."""
    import raocp.core as core
    from raocp.problems import build_problem, recipe_config
    r = recipe_config(cfg, seed=0)
    c = core.Cache(build_problem(r)[1], dtype=dtype)
    nat = c.native
    w = 4 if dtype == "float32" else 8
    alpha = 0.999 / nat.step_size(rtol=1e-7 if w == 4 else 1e-14)
    wall, dev_ms = timed_cp(nat, r["x0"], alpha, steps, warmup, None)
    kernels, roofline = iteration_kernels(nat, c, w, reps, dev_ms / steps)
    pk = c.packed
    leg = {"config": f"SURVEY.md 8(d) config {cfg} (BASELINE configs[{cfg - 1}]): {pk.n} nodes, nx={pk.nx}, nu={pk.nu}",
           "dtype": "f32" if w == 4 else "f64", "nodes": pk.n,
           "cp": {"value": steps / wall, "unit": "it/s", "steps": steps, "ms_per_step": 1e3 * wall / steps,
                  "device_ms_per_step": dev_ms / steps},
           "kernels": kernels, "roofline": roofline,
           "cp_kernel": nat.kernel_info(10), "dynamics_kernels": nat.kernel_info(9)}
    if nsets:
        leg["l_sweep"] = op_pair(nat, c, w, max(10, reps // 2), nsets)
    del c
    return leg


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
    ap.add_argument("--no-shard", action="store_true", help="skip the sharded strong-scaling legs (configs 4, 5)")
    ap.add_argument("--no-fp32", action="store_true", help="skip the fp32 config-5 leg")
    ap.add_argument("--fp32-steps", type=int, default=48)
    ap.add_argument("--shard-config", type=int, default=4, help=argparse.SUPPRESS)
    ap.add_argument("--shard-dtype", default="float64", help=argparse.SUPPRESS)
    ap.add_argument("--shard-steps", type=int, default=200)
    ap.add_argument("--shard-warmup", type=int, default=20)
    ap.add_argument("--shard-timeout", type=float, default=240.0)
    ap.add_argument("--rank-timeout", type=float, default=1500.0,
                    help="time limit of the rank processes bench.py --gpus N starts itself")
    ap.add_argument("--shard-leg", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    if args.shard_leg:
        return shard_leg(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # start the N rank processes (no GPU has been touched in this one)
        out, rcs = spawn(args.gpus, sys.argv[1:], timeout=args.rank_timeout)
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

    kernels, roofline = iteration_kernels(nat, cache, 8, args.op_reps, dev_ms / args.steps)
    # L / L^T at config 2 (standalone operators, not launched by the CP iteration)
    l_sweep = {"config2": op_pair(nat, cache, 8, args.op_reps, 1)}
    legs = {}
    if not args.no_hbm:
        legs["config4"] = config_leg(4, "float64", args.shard_steps, args.shard_warmup, 200, 3)
        l_sweep["config4"] = legs["config4"]["l_sweep"]
    fp32 = None
    if not args.no_fp32:
        legs["config5_fp32"] = fp32 = config_leg(5, "float32", args.fp32_steps, 2, 40, 2)
        l_sweep["config5_fp32"] = fp32["l_sweep"]

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
        "config4": legs.get("config4"),
        "fp32_config5": fp32,
    }
    if not args.no_shard:
        sharded = {}
        for cfg, dtype in SHARD_LEGS:
            steps, warmup = (args.shard_steps, args.shard_warmup) if dtype == "float64" else (args.fp32_steps, 2)
            key = leg_key(cfg, dtype)
            if world > 1:
                sharded[key] = sharded_entry(args, world, cfg, dtype, steps, warmup)
                continue
            # the N = 1 point: the same tree unsharded in this process (the leg measured above)
            leg = legs.get(key) or config_leg(cfg, dtype, steps, warmup, 40, 0)
            sharded[key] = {"config": f"SURVEY.md 8(d) config {cfg} (BASELINE configs[{cfg - 1}]): ONE tree, "
                                      "unsharded on 1 GPU (the N = 1 point of the strong-scaling leg)",
                            "dtype": leg["dtype"], "n_gpus": 1, "steps": steps, "unit": "it/s", "scaling": "strong",
                            "value": leg["cp"]["value"], "ms_per_step": leg["cp"]["ms_per_step"],
                            "device_ms_per_step": leg["cp"]["device_ms_per_step"], "nodes": leg["nodes"],
                            "cp_kernel": leg.get("cp_kernel"), "dynamics_kernels": leg.get("dynamics_kernels")}
        out["sharded"] = sharded
    if not args.no_cpu and world == 1:
        out["cpu_baseline"] = cpu_baseline(recipe, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    if group:
        group.barrier()
    return 0


if __name__ == "__main__":
    sys.exit(main())
