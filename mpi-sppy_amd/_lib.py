"""ctypes binding of libphg.so (include/phg.h).

The library is built in-tree (``mpi-sppy_amd/libphg.so``, see ``__graft_entry__.build``).  There is
deliberately NO fallback: if the shared object is missing or no HIP device is present, importing
the engine's solver raises -- the product path never computes on the CPU.
"""
import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("PHG_LIB", os.path.join(_HERE, "libphg.so"))

i32p = C.POINTER(C.c_int32)
f64p = C.POINTER(C.c_double)


class PhgBatch(C.Structure):
    _fields_ = [
        ("S", C.c_int32), ("n", C.c_int32), ("m", C.c_int32), ("nnz", C.c_int32),
        ("rowptr", i32p), ("colidx", i32p), ("vals", f64p), ("c", f64p),
        ("col_lo", f64p), ("col_hi", f64p), ("row_lo", f64p), ("row_hi", f64p),
        ("obj_offset", f64p), ("sense", C.c_int32),
        ("N", C.c_int32), ("nonant_col", i32p), ("L", C.c_int32), ("nonant_level", i32p),
        ("nonant_pos", i32p), ("level_len", i32p), ("scen_node", i32p), ("n_nodes", C.c_int32),
        ("node_off", i32p), ("N_tot", C.c_int32), ("prob", f64p), ("prob_coeff", f64p),
        ("scen_global0", C.c_int32), ("S_global", C.c_int32), ("virt_nproc", C.c_int32),
        ("prob_coeff_var", f64p),
        ("vals_form", C.c_int32), ("n_delta", C.c_int32), ("delta_pos", i32p), ("delta_vals", f64p),
    ]


VALS_PER_SCENARIO, VALS_SHARED, VALS_DELTA = 0, 1, 2


class PhgOpts(C.Structure):
    _fields_ = [("eps_rel", C.c_double), ("max_iter", C.c_int32), ("check_every", C.c_int32),
                ("warm_start", C.c_int32), ("fix_nonants", C.c_int32), ("schedule", C.c_int32),
                ("beta_sufficient", C.c_double), ("beta_necessary", C.c_double),
                ("beta_artificial", C.c_double), ("primal_weight_theta", C.c_double),
                ("skip_if_conv_below", C.c_double), ("fix_tol", C.c_double), ("safe_bound", C.c_int32)]


(F_X, F_Y, F_XN, F_W, F_RHO, F_XBAR, F_XSQBAR, F_OBJ, F_BOUND, F_EVAL, F_KKT, F_FIXED, F_CONV_PART, F_OMEGA,
 F_Z, F_SMOOTH_P, F_SMOOTH_BETA, F_WARM) = range(18)
I_ITERS, I_STATUS, I_ORDER = 0, 1, 2

# every symbol include/phg.h declares, with its ctypes signature
SIGNATURES = {
    "phg_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "phg_destroy": (None, [C.c_void_p]),
    "phg_last_error": (C.c_char_p, []),
    "phg_set_stream": (C.c_int, [C.c_void_p, C.c_void_p]),
    "phg_set_presolve": (C.c_int, [C.c_void_p, C.c_int32]),
    "phg_conv_start": (C.c_int, [C.c_void_p, C.c_void_p]),
    "phg_conv_wait": (C.c_int, [C.c_void_p, C.POINTER(C.c_double)]),
    "phg_presolve_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_int32)]),
    "phg_sync": (C.c_int, [C.c_void_p]),
    "phg_set_layout": (C.c_int, [C.c_void_p, C.c_int32]),
    "phg_plan": (C.c_int, [C.POINTER(PhgBatch), i32p]),
    "phg_implied_bounds": (C.c_int, [C.POINTER(PhgBatch), f64p, f64p, i32p]),
    "phg_load_batch": (C.c_int, [C.c_void_p, C.POINTER(PhgBatch)]),
    "phg_set": (C.c_int, [C.c_void_p, C.c_int32, f64p]),
    "phg_get": (C.c_int, [C.c_void_p, C.c_int32, f64p]),
    "phg_get_i32": (C.c_int, [C.c_void_p, C.c_int32, i32p]),
    "phg_solve_results": (C.c_int, [C.c_void_p, i32p, i32p, f64p, f64p, f64p, f64p]),
    "phg_info": (C.c_int, [C.c_void_p, i32p]),
    "phg_solve": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32, C.POINTER(PhgOpts)]),
    "phg_node_sums": (C.c_int, [C.c_void_p, C.c_void_p]),
    "phg_apply_xbar": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "phg_conv_finish": (C.c_int, [C.c_void_p, C.c_void_p, f64p]),
    "phg_ph_update": (C.c_int, [C.c_void_p, f64p]),
    "phg_solve_summary": (C.c_int, [C.c_void_p, i32p]),
    "phg_set_smoothing": (C.c_int, [C.c_void_p, C.c_int32]),
    "phg_copy_from": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32]),
    "phg_fix_from": (C.c_int, [C.c_void_p, C.c_void_p, C.c_int32]),
    "phg_query": (C.c_int, [C.c_void_p, i32p]),
    "phg_eval_objective": (C.c_int, [C.c_void_p, C.c_int32, C.c_int32]),
    "phg_exchange_buffers": (C.c_int, [C.c_void_p, C.POINTER(C.c_void_p), C.POINTER(C.c_void_p)]),
    "phg_timing_reset": (C.c_int, [C.c_void_p, C.c_int32]),
    "phg_timing": (C.c_int, [C.c_void_p, C.c_int32, f64p, i32p, C.POINTER(C.c_int64)]),
    "phg_exchange_layout": (C.c_int, [C.c_void_p, i32p]),
    "phg_ph_head": (C.c_int, [C.c_void_p, C.c_void_p, C.c_double, C.c_int32]),
    "phg_solve_undo": (C.c_int, [C.c_void_p]),
    "phg_fold_partials": (C.c_int, [C.c_void_p, C.c_void_p]),
    "phg_set_fold": (C.c_int, [C.c_void_p, C.c_int32, i32p]),
    "phg_ph_step": (C.c_int, [C.c_void_p, C.c_double, C.c_int32, i32p]),
    "phg_mfma_info": (C.c_int, [C.c_void_p, i32p]),
    "phg_values_info": (C.c_int, [C.c_void_p, i32p]),
    "phg_local_info": (C.c_int, [C.c_void_p, i32p]),
    "phg_set_tail": (C.c_int, [C.c_void_p, C.c_int32, C.c_double, C.c_void_p]),
    "phg_tail_info": (C.c_int, [C.c_void_p, i32p]),
    "phg_set_col_bounds": (C.c_int, [C.c_void_p, f64p, f64p]),
    "phg_group_unique_id": (C.c_int, [C.c_void_p]),
    "phg_create_group": (C.c_int, [C.c_int32, C.c_int32, C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]),
    "phg_group_size": (C.c_int, [C.c_void_p, i32p]),
    "phg_group_allreduce": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64]),
    "phg_ph_exchange": (C.c_int, [C.c_void_p, C.c_void_p]),
    "phg_destroy_group": (None, [C.c_void_p]),
}

_lib = None


def load():
    """Load libphg.so and bind every exported symbol (raises if missing)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libphg.so not found at {LIB_PATH}: build it with "
                           "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback)")
    lib = C.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        if "PHG_LIB" in os.environ and not hasattr(lib, name):
            continue   # (an older build under A/B comparison: its missing entry points stay unbound)
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


class PhgError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        raise PhgError(load().phg_last_error().decode())


def as_f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


def as_i32(a):
    return np.ascontiguousarray(a, dtype=np.int32)


def ptr(a):
    if a is None:
        return None
    if a.dtype == np.float64:
        return a.ctypes.data_as(f64p)
    if a.dtype == np.int32:
        return a.ctypes.data_as(i32p)
    raise TypeError(a.dtype)


class PhgGroup:
    """An RCCL communicator owned by libphg.so (``phg_create_group``: one process per GPU,
    ``ncclCommInitRank``).  Collective over the ``nranks`` processes, which must share the 128-byte
    id of :meth:`unique_id` (made by one rank, broadcast by the caller)."""

    @staticmethod
    def unique_id():
        buf = (C.c_uint8 * 128)()
        check(load().phg_group_unique_id(buf))
        return bytes(buf)

    def __init__(self, nranks, rank, uid, device):
        if len(uid) != 128:
            raise ValueError("the group id is 128 bytes (PhgGroup.unique_id)")
        self.lib = load()
        g = C.c_void_p()
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        check(self.lib.phg_create_group(int(nranks), int(rank), buf, int(device), C.byref(g)))
        self.g = g
        self.nranks, self.rank, self.device = int(nranks), int(rank), int(device)

    def allreduce(self, handle, dev_ptr, count):
        """In-place SUM of ``count`` doubles at device address ``dev_ptr``, on ``handle``'s stream."""
        check(self.lib.phg_group_allreduce(self.g, handle, C.c_void_p(int(dev_ptr)), C.c_int64(int(count))))

    def size(self):
        """(ranks, this rank) of the communicator as RCCL reports them (``phg_group_size``:
        ``ncclCommCount``, ``ncclCommUserRank``)."""
        n = np.zeros(2, np.int32)
        check(self.lib.phg_group_size(self.g, ptr(n)))
        return int(n[0]), int(n[1])

    def ph_exchange(self, handle):
        """All-reduce the handle's own packed exchange buffer (``phg_ph_exchange``)."""
        check(self.lib.phg_ph_exchange(handle, self.g))

    def close(self):
        if self.g:
            self.lib.phg_destroy_group(self.g)
            self.g = None
