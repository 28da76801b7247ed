"""ctypes binding of libraocp_hip.so (C-ABI in include/raocp_hip.h).

This is the only way the Python layer computes anything on the hot path: there
is no CPU fallback. If the library is missing or no HIP device is usable, the
calls raise immediately (RuntimeError), so a run can never silently measure or
validate a non-GPU path.
"""
import ctypes
import os

import numpy as np

__all__ = ["load_library", "NativeContext", "RaocpError", "LIB_PATH", "EXPORTED_SYMBOLS", "comm_unique_id",
           "group_cp_run"]

LIB_PATH = os.environ.get("RAOCP_HIP_LIB", os.path.join(os.path.dirname(os.path.abspath(__file__)),
                                                           "libraocp_hip.so"))

RAOCP_DEVICE_PTR = 1
_ERR_NAN_IN_BOX = -4

EXPORTED_SYMBOLS = [
    "raocp_ctx_create", "raocp_ctx_destroy", "raocp_last_error", "raocp_sizes", "raocp_ell", "raocp_ell_t",
    "raocp_set_primal", "raocp_get_primal", "raocp_set_dual", "raocp_get_dual", "raocp_set_initial_state",
    "raocp_prox_f", "raocp_relax_s0", "raocp_project_on_dynamics", "raocp_project_on_kernel", "raocp_prox_gconj",
    "raocp_step_size", "raocp_cp_run", "raocp_cp_prepare", "raocp_cp_bench", "raocp_op_bench",
    "raocp_dual_scale", "raocp_dual_add_halves", "raocp_dual_project", "raocp_dual_moreau",
    "raocp_device_synchronize", "raocp_debug_dyn_stamps",
    "raocp_shard_setup", "raocp_shard_owned", "raocp_comm_unique_id", "raocp_comm_init", "raocp_group_cp_run",
    "raocp_reset_iterate", "raocp_kernel_info", "raocp_op_bench_rot",
]

_i32p = ctypes.POINTER(ctypes.c_int32)
_f64p = ctypes.POINTER(ctypes.c_double)


class TreeDesc(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("m", ctypes.c_int32), ("nx", ctypes.c_int32), ("nu", ctypes.c_int32),
                ("anc", _i32p), ("stage", _i32p), ("ch_start", _i32p), ("nch", _i32p)]


class ProblemDesc(ctypes.Structure):
    _fields_ = [("n_sq", ctypes.c_int32), ("n_sr", ctypes.c_int32), ("n_sp", ctypes.c_int32),
                ("sqrt_q", _f64p), ("sqrt_r", _f64p), ("sqrt_pf", _f64p),
                ("i_sq", _i32p), ("i_sr", _i32p), ("i_sp", _i32p),
                ("alpha_r", _f64p), ("cond", _f64p),
                ("n_box_nl", ctypes.c_int32), ("n_box_l", ctypes.c_int32),
                ("box_nl_lo", _f64p), ("box_nl_hi", _f64p), ("box_l_lo", _f64p), ("box_l_hi", _f64p),
                ("i_box_nl", _i32p), ("i_box_l", _i32p),
                ("n_a", ctypes.c_int32), ("n_b", ctypes.c_int32), ("n_k", ctypes.c_int32),
                ("A", _f64p), ("B", _f64p), ("K", _f64p), ("Rinv", _f64p), ("M", _f64p),
                ("i_a", _i32p), ("i_b", _i32p), ("i_k", _i32p), ("dtype", ctypes.c_int32)]

DTYPES = {"float64": 0, "float32": 1}


class RaocpError(RuntimeError):
    pass


_lib = None


def load_library():
    """Load libraocp_hip.so and declare prototypes. Raises if it was not built."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"HIP extension missing: {LIB_PATH} not found (build it: make -C raocp-toolbox_amd, "
                           f"or __graft_entry__.build())")
    lib = ctypes.CDLL(LIB_PATH)
    vp, c_int, c_double, c_i64p = ctypes.c_void_p, ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_int64)
    proto = {
        "raocp_ctx_create": (c_int, [ctypes.POINTER(TreeDesc), ctypes.POINTER(ProblemDesc), c_int,
                                     ctypes.POINTER(vp)]),
        "raocp_ctx_destroy": (None, [vp]),
        "raocp_last_error": (ctypes.c_char_p, []),
        "raocp_sizes": (c_int, [vp, c_i64p, c_i64p]),
        "raocp_ell": (c_int, [vp, vp, vp, c_int]),
        "raocp_ell_t": (c_int, [vp, vp, vp, c_int]),
        "raocp_set_primal": (c_int, [vp, vp, c_int]),
        "raocp_get_primal": (c_int, [vp, vp, c_int]),
        "raocp_set_dual": (c_int, [vp, vp, c_int]),
        "raocp_get_dual": (c_int, [vp, vp, c_int]),
        "raocp_set_initial_state": (c_int, [vp, vp]),
        "raocp_reset_iterate": (c_int, [vp]),
        "raocp_kernel_info": (c_int, [vp, c_int, ctypes.c_char_p, c_int]),
        "raocp_prox_f": (c_int, [vp, c_double]),
        "raocp_relax_s0": (c_int, [vp, c_double]),
        "raocp_project_on_dynamics": (c_int, [vp]),
        "raocp_project_on_kernel": (c_int, [vp]),
        "raocp_prox_gconj": (c_int, [vp, c_double]),
        "raocp_step_size": (c_int, [vp, _f64p, c_int, c_double]),
        "raocp_cp_run": (c_int, [vp, vp, c_int, c_double, c_double, ctypes.POINTER(c_int), ctypes.POINTER(c_int),
                                 vp, vp]),
        "raocp_cp_prepare": (c_int, [vp, vp, c_int, c_double]),
        "raocp_cp_bench": (c_int, [vp, vp, c_int, c_double, ctypes.POINTER(ctypes.c_float)]),
        "raocp_op_bench": (c_int, [vp, c_int, c_int, ctypes.POINTER(ctypes.c_float)]),
        "raocp_op_bench_rot": (c_int, [vp, c_int, c_int, c_int, ctypes.POINTER(ctypes.c_float)]),
        "raocp_dual_scale": (c_int, [vp, c_double]),
        "raocp_dual_add_halves": (c_int, [vp]),
        "raocp_dual_project": (c_int, [vp, c_int]),
        "raocp_dual_moreau": (c_int, [vp, c_double, vp]),
        "raocp_device_synchronize": (c_int, [c_int]),
        "raocp_debug_dyn_stamps": (c_int, [vp, vp, c_int]),
        "raocp_shard_setup": (c_int, [vp, c_int, c_int]),
        "raocp_shard_owned": (c_int, [vp, vp, vp, c_int]),
        "raocp_comm_unique_id": (c_int, [vp]),
        "raocp_comm_init": (c_int, [vp, vp, c_int, c_int]),
        "raocp_group_cp_run": (c_int, [vp, c_int, vp, c_int, c_double, c_double, ctypes.POINTER(c_int),
                                       ctypes.POINTER(c_int), vp, vp]),
    }
    for name, (res, args) in proto.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _default_device():
    for key in ("RAOCP_DEVICE", "LOCAL_RANK"):
        if key in os.environ:
            return int(os.environ[key])
    return 0


def device_synchronize(device=None):
    """hipDeviceSynchronize through libraocp_hip.so's own HIP runtime."""
    lib = load_library()
    rc = lib.raocp_device_synchronize(_default_device() if device is None else int(device))
    if rc != 0:
        raise RaocpError(lib.raocp_last_error().decode(errors="replace"))


def comm_unique_id():
    """128-byte RCCL unique id (call on one rank, share with the others)."""
    lib = load_library()
    out = np.zeros(128, dtype=np.uint8)
    rc = lib.raocp_comm_unique_id(_ptr(out))
    if rc != 0:
        raise RaocpError(lib.raocp_last_error().decode(errors="replace"))
    return out.tobytes()


def group_cp_run(contexts, x0, max_iters, tol, alpha):
    """CP loop over the shards of one process (contexts[r].shard(r, R) done), exchanging
    through device copies. Returns (status, error_cache, delta_error_cache) like cp_run."""
    lib = load_library()
    R = len(contexts)
    arr = (ctypes.c_void_p * R)(*[c._h for c in contexts])
    x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).reshape(-1))
    err = np.zeros((max_iters + 1, 3))
    derr = np.zeros((max_iters + 1, 3))
    status, iters = ctypes.c_int(), ctypes.c_int()
    rc = lib.raocp_group_cp_run(ctypes.cast(arr, ctypes.c_void_p), R, _ptr(x0), int(max_iters), float(tol), float(alpha),
                                ctypes.byref(status), ctypes.byref(iters), _ptr(err), _ptr(derr))
    if rc != 0:
        raise RaocpError(lib.raocp_last_error().decode(errors="replace"))
    k = iters.value
    return status.value, err[:k].copy(), derr[:k].copy()


class NativeContext:
    """One device context (raocp_ctx) holding a packed problem in HBM."""

    def __init__(self, packed, device=None, dtype="float64"):
        self._lib = load_library()
        self.dtype = np.dtype(dtype).name
        if self.dtype not in DTYPES:
            raise ValueError(f"dtype {dtype}: float64 or float32")
        self._packed = packed  # keep arrays alive while the descriptors point at them
        p = packed
        self.tree_desc = TreeDesc(p.n, p.m, p.nx, p.nu, *[a.ctypes.data_as(_i32p) for a in
                                                            (p.anc, p.stage, p.ch_start, p.nch)])
        f = lambda a: a.ctypes.data_as(_f64p)  # noqa: E731
        i = lambda a: a.ctypes.data_as(_i32p)  # noqa: E731
        self.prob_desc = ProblemDesc(
            p.sqrt_q.shape[0], p.sqrt_r.shape[0], p.sqrt_pf.shape[0], f(p.sqrt_q), f(p.sqrt_r), f(p.sqrt_pf),
            i(p.i_sq), i(p.i_sr), i(p.i_sp), f(p.alpha_r), f(p.cond),
            p.n_box_nl, p.n_box_l, f(p.box_nl_lo), f(p.box_nl_hi), f(p.box_l_lo), f(p.box_l_hi),
            i(p.i_box_nl), i(p.i_box_l),
            p.A.shape[0], p.B.shape[0], p.K.shape[0],
            f(p.A), f(p.B), f(p.K), f(p.Rinv), f(p.M), i(p.i_a), i(p.i_b), i(p.i_k), DTYPES[self.dtype])
        self.device = _default_device() if device is None else device
        h = ctypes.c_void_p()
        self._check(self._lib.raocp_ctx_create(ctypes.byref(self.tree_desc), ctypes.byref(self.prob_desc),
                                               self.device, ctypes.byref(h)))
        self._h = h
        P, D = ctypes.c_int64(), ctypes.c_int64()
        self._check(self._lib.raocp_sizes(self._h, ctypes.byref(P), ctypes.byref(D)))
        self.P, self.D = P.value, D.value

    def _check(self, rc):
        if rc == 0:
            return
        msg = self._lib.raocp_last_error().decode(errors="replace")
        if rc == _ERR_NAN_IN_BOX:
            raise ValueError(msg)
        raise RaocpError(f"libraocp_hip error {rc}: {msg}")

    def close(self):
        if getattr(self, "_h", None):
            self._lib.raocp_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def _vec(x, size):
        a = np.ascontiguousarray(np.asarray(x, dtype=np.float64).reshape(-1))
        if a.size != size:
            raise ValueError(f"vector of length {a.size}, expected {size}")
        return a

    def _require_l(self):
        err = getattr(self._packed, "l_error", None)
        if err:
            # what numpy raises in the reference when the cost and state sizes disagree (operators.py:33-36)
            raise ValueError(f"matmul: cost weights inconsistent with the dynamics ({err})")

    # ---- operators
    def ell(self, z, template=None):
        self._require_l()
        z = self._vec(z, self.P)
        out = np.zeros(self.D) if template is None else self._vec(template, self.D).copy()
        self._check(self._lib.raocp_ell(self._h, _ptr(z), _ptr(out), 0))
        return out

    def ell_t(self, eta, template=None):
        self._require_l()
        eta = self._vec(eta, self.D)
        out = np.zeros(self.P) if template is None else self._vec(template, self.P).copy()
        self._check(self._lib.raocp_ell_t(self._h, _ptr(eta), _ptr(out), 0))
        return out

    # ---- iterate
    def set_primal(self, z):
        z = self._vec(z, self.P)
        self._check(self._lib.raocp_set_primal(self._h, _ptr(z), 0))

    def get_primal(self):
        out = np.empty(self.P)
        self._check(self._lib.raocp_get_primal(self._h, _ptr(out), 0))
        return out

    def set_dual(self, e):
        e = self._vec(e, self.D)
        self._check(self._lib.raocp_set_dual(self._h, _ptr(e), 0))

    def get_dual(self):
        out = np.empty(self.D)
        self._check(self._lib.raocp_get_dual(self._h, _ptr(out), 0))
        return out

    def reset_iterate(self):
        """Zero the current primal / dual on the device (a fresh Cache's iterate)."""
        self._check(self._lib.raocp_reset_iterate(self._h))

    def kernel_info(self, op):
        """rocprofv3 name of the kernel the default selection launches for op (raocp_op_bench
        numbering: 0 L, 1 L^T, 2 / 6 the dual / primal CP kernels, 9 dynamics, 10 fused CP)."""
        buf = ctypes.create_string_buffer(256)
        self._check(self._lib.raocp_kernel_info(self._h, int(op), buf, 256))
        return buf.value.decode()

    def set_initial_state(self, x0):
        x0 = self._vec(x0, self._packed.nx)
        self._check(self._lib.raocp_set_initial_state(self._h, _ptr(x0)))

    # ---- prox operators on the current iterate
    def prox_f(self, alpha):
        self._check(self._lib.raocp_prox_f(self._h, float(alpha)))

    def relax_s0(self, alpha):
        self._check(self._lib.raocp_relax_s0(self._h, float(alpha)))

    def project_on_dynamics(self):
        self._check(self._lib.raocp_project_on_dynamics(self._h))

    def project_on_kernel(self):
        self._check(self._lib.raocp_project_on_kernel(self._h))

    def prox_gconj(self, alpha):
        self._check(self._lib.raocp_prox_gconj(self._h, float(alpha)))

    def dual_scale(self, alpha):
        self._check(self._lib.raocp_dual_scale(self._h, float(alpha)))

    def dual_add_halves(self):
        self._check(self._lib.raocp_dual_add_halves(self._h))

    def dual_project(self, which):
        self._check(self._lib.raocp_dual_project(self._h, int(which)))

    def dual_moreau(self, alpha, modified):
        modified = self._vec(modified, self.D)
        self._check(self._lib.raocp_dual_moreau(self._h, float(alpha), _ptr(modified)))

    # ---- solver
    def step_size(self, max_it=300, rtol=1e-14):
        self._require_l()
        lam = ctypes.c_double()
        self._check(self._lib.raocp_step_size(self._h, ctypes.byref(lam), int(max_it), float(rtol)))
        return lam.value

    def cp_run(self, x0, max_iters, tol, alpha, warm=False):
        """The CP loop on the device. warm=False starts from (x0 at node 0, zeros) / 0;
        warm=True from the context's current primal / dual (set_primal / set_dual), x0
        written into node 0's state, as the reference's chock continues from the cache."""
        self._require_l()
        x0 = self._vec(x0, self._packed.nx)
        if not warm:
            self.reset_iterate()
        err = np.zeros((max_iters + 1, 3))
        derr = np.zeros((max_iters + 1, 3))
        status, iters = ctypes.c_int(), ctypes.c_int()
        self._check(self._lib.raocp_cp_run(self._h, _ptr(x0), int(max_iters), float(tol), float(alpha),
                                           ctypes.byref(status), ctypes.byref(iters), _ptr(err), _ptr(derr)))
        k = iters.value
        return status.value, err[:k].copy(), derr[:k].copy()

    def cp_prepare(self, iters, x0=None, alpha=0.0):
        """Capture the CP graphs an `iters`-iteration cp_bench launches and, given x0, reset
        the iterate for that run (outside timing); cp_bench(None, iters, alpha) follows."""
        x0p = None if x0 is None else _ptr(self._vec(x0, self._packed.nx))
        self._check(self._lib.raocp_cp_prepare(self._h, x0p, int(iters), float(alpha)))

    def cp_bench(self, x0, iters, alpha):
        """Exactly `iters` CP iterations (tol = 0); x0=None: the run cp_prepare(iters, x0)
        set up. Returns device ms."""
        self._require_l()
        x0p = None if x0 is None else _ptr(self._vec(x0, self._packed.nx))
        ms = ctypes.c_float()
        self._check(self._lib.raocp_cp_bench(self._h, x0p, int(iters), float(alpha), ctypes.byref(ms)))
        return ms.value

    def debug_dyn_stamps(self, cap=128):
        out = np.zeros(cap, dtype=np.uint64)
        self._check(self._lib.raocp_debug_dyn_stamps(self._h, _ptr(out), int(cap)))
        return out

    # ---- subtree sharding (include/raocp_hip.h)
    def shard(self, rank, nranks):
        """Restrict this context to shard `rank` of `nranks` (owned subtrees + replicated top)."""
        self._check(self._lib.raocp_shard_setup(self._h, int(nranks), int(rank)))
        self.rank, self.nranks = int(rank), int(nranks)

    def shard_owned(self):
        """Owned node-id range [lo, hi) per stage 0..N."""
        N = int(self._packed.N)
        lo = np.zeros(N + 1, dtype=np.int32)
        hi = np.zeros(N + 1, dtype=np.int32)
        self._check(self._lib.raocp_shard_owned(self._h, _ptr(lo), _ptr(hi), N + 1))
        return lo, hi

    def comm_init(self, uid, rank, nranks):
        """Bind an RCCL communicator (uid: 128 bytes from comm_unique_id() on one rank)."""
        buf = np.frombuffer(bytes(uid), dtype=np.uint8).copy()
        self._check(self._lib.raocp_comm_init(self._h, _ptr(buf), int(nranks), int(rank)))

    def op_bench(self, op, reps):
        ms = ctypes.c_float()
        self._check(self._lib.raocp_op_bench(self._h, int(op), int(reps), ctypes.byref(ms)))
        return ms.value

    def op_bench_rot(self, op, reps, nsets):
        """L (0) / L^T (1) cycling over nsets buffer pairs (HBM-honest beyond 256 MiB)."""
        ms = ctypes.c_float()
        self._check(self._lib.raocp_op_bench_rot(self._h, int(op), int(reps), int(nsets), ctypes.byref(ms)))
        return ms.value
