"""ctypes binding of libodesat_hip.so (include/odesat.h).

The product path: every call goes to the in-tree HIP library; there is no CPU fallback.  If the
library is missing, import of the integrator fails loudly with the build command to run.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libodesat_hip.so")  # the in-tree product library (use_library: A/B builds)
HEADER = os.path.join(os.path.dirname(_HERE), "include", "odesat.h")

ODESAT_OK, ODESAT_EINVAL, ODESAT_ENOMEM, ODESAT_EDEVICE, ODESAT_ESTATE = 0, -1, -2, -3, -4
ODESAT_F32, ODESAT_F64 = 0, 1
ODESAT_STOP_EACH, ODESAT_STOP_ANY, ODESAT_STOP_NONE = 0, 1, 2
ODESAT_SCHED_AUTO, ODESAT_SCHED_STEP_MAJOR, ODESAT_SCHED_CHUNK_MAJOR = 0, 1, 2
ODESAT_ALG_FUSED, ODESAT_ALG_TWOPASS, ODESAT_ALG_RESIDENT, ODESAT_ALG_ONCHIP = 0, 1, 2, 3
ODESAT_PART_CLAUSES, ODESAT_PART_VARIABLES, ODESAT_PART_CLAUSES_RS = 0, 1, 2
ODESAT_STEP_VARIABLE_ELIMINATION, ODESAT_STEP_BLOCKED_CLAUSE, ODESAT_UNSET = 0, 1, 2


class OdesatError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"odesat error {code}: {msg}")
        self.code = code


class Params(C.Structure):
    _fields_ = [("adaptive", C.c_int32), ("stop", C.c_int32), ("tol", C.c_double), ("dt", C.c_double),
                ("zeta", C.c_double), ("max_steps", C.c_int64), ("poll_interval", C.c_int32),
                ("dt_policy", C.c_int32)]


_P = C.c_void_p
_i64 = C.c_int64
_dp = C.POINTER(C.c_double)
_u8p = C.POINTER(C.c_uint8)
_i64p = C.POINTER(C.c_int64)
_i32p = C.POINTER(C.c_int32)
_fp = C.POINTER(C.c_float)

# name -> (restype, argtypes); kept in sync with include/odesat.h (tests/test_abi.py checks)
SIGNATURES = {
    "odesat_last_error": (C.c_char_p, []),
    "odesat_version": (C.c_char_p, []),
    "odesat_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "odesat_cnf_parse": (C.c_int, [C.c_char_p, C.c_size_t, C.POINTER(_P)]),
    "odesat_cnf_from_arrays": (C.c_int, [_i64, _i64, _i64p, _i64p, _u8p, C.POINTER(_P)]),
    "odesat_cnf_free": (None, [_P]),
    "odesat_cnf_varnum": (_i64, [_P]),
    "odesat_cnf_nclauses": (_i64, [_P]),
    "odesat_cnf_nliterals": (_i64, [_P]),
    "odesat_cnf_export": (C.c_int, [_P, _i64p, _i64p, _u8p]),
    "odesat_cnf_normalize": (C.c_int, [_P, C.POINTER(_P), _i64p, _i64p]),
    "odesat_cnf_evaluate": (C.c_int, [_P, _u8p, _i64]),
    "odesat_cnf_init_short_term_memory": (C.c_int, [_P, _dp]),
    "odesat_create": (_P, [C.c_int, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.c_char_p,
                           C.c_size_t]),
    "odesat_run": (C.c_int, [_P, C.POINTER(Params), C.c_int32, _fp, _fp, _fp, _fp, _fp, _fp, _i64p, _i64p]),
    "odesat_destroy": (None, [_P]),
    "odesat_stoch_create": (C.c_int, [C.c_int, _P, _i64, C.POINTER(_P)]),
    "odesat_stoch_destroy": (None, [_P]),
    "odesat_stoch_reset": (C.c_int, [_P, _i64, _i64]),
    "odesat_stoch_wave_width": (C.c_int, [_P]),
    "odesat_stoch_set_state": (C.c_int, [_P, _i64, _i64, _u8p, C.POINTER(C.c_uint64)]),
    "odesat_stoch_get_state": (C.c_int, [_P, _i64, _i64, _u8p, C.POINTER(C.c_uint64)]),
    "odesat_stoch_search": (C.c_int, [_P, C.c_uint64, _i64, _i64, C.c_int, C.c_int32, _i64p, _i64p]),
    "odesat_preprocess": (C.c_int, [_P, C.c_float, C.POINTER(_P), C.POINTER(_P)]),
    "odesat_trace_free": (None, [_P]),
    "odesat_trace_nsteps": (_i64, [_P]),
    "odesat_trace_step": (C.c_int, [_P, _i64, C.POINTER(C.c_int32), _i64p, _i64p, _i64p]),
    "odesat_trace_step_clauses": (C.c_int, [_P, _i64, _i64p, _i64p, _u8p]),
    "odesat_trace_apply": (C.c_int, [_P, _u8p, _i64]),
    "odesat_cnf_evaluate_assign": (C.c_int, [_P, _u8p, _i64]),
    "odesat_cnf_max_variable": (_i64, [_P]),
    "odesat_solver_create": (C.c_int, [C.c_int, _P, _i64, C.c_int, C.POINTER(_P)]),
    "odesat_solver_destroy": (None, [_P]),
    "odesat_solver_batch": (_i64, [_P]),
    "odesat_solver_varnum": (_i64, [_P]),
    "odesat_solver_nclauses": (_i64, [_P]),
    "odesat_solver_device_bytes": (_i64, [_P]),
    "odesat_set_state": (C.c_int, [_P, _i64, _i64, _dp, _dp, _dp]),
    "odesat_init_state": (C.c_int, [_P, C.c_uint64, _i64]),
    "odesat_get_state": (C.c_int, [_P, _i64, _i64, _dp, _dp, _dp]),
    "odesat_get_assignment": (C.c_int, [_P, _i64, _u8p]),
    "odesat_evaluate": (C.c_int, [_P, _u8p, _i64p]),
    "odesat_compute_derivatives": (C.c_int, [_P, C.c_double, _dp, _dp, _dp, _u8p]),
    "odesat_euler_step_fixed": (C.c_int, [_P, C.c_double, C.c_double, _u8p]),
    "odesat_euler_step": (C.c_int, [_P, C.c_double, _dp, C.c_double, _u8p]),
    "odesat_simulate": (C.c_int, [_P, C.POINTER(Params), _i64p, _i64p, _dp, _i64p]),
    "odesat_simulate_continue": (C.c_int, [_P, C.POINTER(Params), _i64p, _i64p, _dp, _i64p]),
    "odesat_synchronize": (C.c_int, [_P]),
    "odesat_checkpoint": (C.c_int, [_P]),
    "odesat_rollback": (C.c_int, [_P]),
    "odesat_profile_enable": (C.c_int, [_P, C.c_int]),
    "odesat_profile_read": (C.c_int, [_P, _dp, _i64p]),
    "odesat_clause_kernel_bytes": (_i64, [_P]),
    "odesat_set_chunk_replicas": (C.c_int, [_P, _i64]),
    "odesat_set_schedule": (C.c_int, [_P, C.c_int]),
    "odesat_set_algorithm": (C.c_int, [_P, C.c_int]),
    "odesat_get_algorithm": (C.c_int, [_P]),
    "odesat_group_width": (C.c_int, [_P]),
    "odesat_step_kernel": (C.c_char_p, [_P, C.c_int]),
    "odesat_set_experiment": (C.c_int, [C.c_char_p, _i64]),
    "odesat_get_experiment": (C.c_int, [C.c_char_p, _i64p]),
    "odesat_clear_experiments": (None, []),
    "odesat_experiment_knob": (C.c_int, [C.c_int, C.POINTER(C.c_char_p)]),
    "odesat_cv_layout": (C.c_int, [_i64, _i64, _i32p, _i32p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, _i32p,
                                   _i32p, _i32p, _i64p, _i64p]),
    "odesat_part_create": (C.c_int, [C.c_int, C.c_int, _i64, _i64, _i64, _i64p, _i64p, _u8p, _i64, _i64, _i64p,
                                     _i64p, _i64, C.POINTER(_P)]),
    "odesat_part_destroy": (None, [_P]),
    "odesat_part_device_bytes": (_i64, [_P]),
    "odesat_part_set_memories": (C.c_int, [_P, _dp, _dp]),
    "odesat_part_get_memories": (C.c_int, [_P, _dp, _dp]),
    "odesat_part_rhs": (C.c_int, [_P, _P, _P, C.c_double, C.c_double, C.c_int, C.c_int, _P]),
    "odesat_part_apply": (C.c_int, [_P, _P, _P, C.c_double, _P]),
    "odesat_part_reduce_apply": (C.c_int, [_P, _P, _P, _P, C.c_int, C.c_double, _P]),
    "odesat_part_reset": (C.c_int, [_P, _P]),
    "odesat_part_status": (C.c_int, [_P, _P, _P, C.c_int, C.c_int, _P, _i64p, _i64p, C.POINTER(C.c_int32)]),
}

_lib = None


def _adopt_torch_runtime():
    """One HIP runtime per process.  PyTorch ships its own libamdhip64 and loads it by file name; if
    this library (linked against the system libamdhip64.so.7) is loaded first, a later `import
    torch` brings a second runtime and torch then sees no GPU.  Loading torch's runtime first, by
    path and RTLD_GLOBAL (torch itself is not imported), makes both resolve to it in either import
    order.  ODESAT_HIP_RUNTIME=system keeps the system runtime (processes that never use torch)."""
    if os.environ.get("ODESAT_HIP_RUNTIME") == "system":
        return
    import importlib.util
    spec = importlib.util.find_spec("torch")
    if spec is None or not spec.origin:
        return
    d = os.path.join(os.path.dirname(spec.origin), "lib")
    for name in ("libhsa-runtime64.so", "libamdhip64.so"):
        p = os.path.join(d, name)
        if os.path.exists(p):
            C.CDLL(p, mode=C.RTLD_GLOBAL)


def use_library(path: str) -> None:
    """Measurement tooling only (scripts/build_variant.sh builds): load `path` instead of the in-tree
    library.  Must be called before the first call into the library; the product never calls it."""
    global LIB_PATH
    if _lib is not None and os.path.abspath(path) != os.path.abspath(LIB_PATH):
        raise RuntimeError(f"libodesat_hip already loaded from {LIB_PATH}")
    LIB_PATH = os.path.abspath(path)


def lib():
    """Load the in-tree libodesat_hip.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        _adopt_torch_runtime()
        if not os.path.exists(LIB_PATH):
            raise OdesatError(ODESAT_EDEVICE, f"{LIB_PATH} not built: run `make -C odesat_amd/csrc` "
                                              "or `python -c 'import __graft_entry__ as g; g.build()'`")
        L = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc):
    if isinstance(rc, int) and rc < 0:
        msg = lib().odesat_last_error()
        raise OdesatError(rc, msg.decode() if msg else "")
    return rc


def dptr(a):
    return None if a is None else a.ctypes.data_as(_dp)


def u8ptr(a):
    return None if a is None else a.ctypes.data_as(_u8p)


def i64ptr(a):
    return None if a is None else a.ctypes.data_as(_i64p)


def i32ptr(a):
    return None if a is None else a.ctypes.data_as(_i32p)


def cv_layout(lits, vst, nl, cpl, tsize, blk_cap, iters):
    """k_solo_cv's lane and block placement (include/odesat.h odesat_cv_layout; a host-only test hook):
    (slot_clause, slot_order, blk, cost_plain, cost_opt) for the 3-SAT literals lits[3 m] (var << 1 |
    neg) with variable-major term starts vst[n + 1]."""
    import numpy as np
    lits = np.ascontiguousarray(lits, np.int32)
    vst = np.ascontiguousarray(vst, np.int32)
    n, m = len(vst) - 1, len(lits) // 3
    sc = np.zeros(nl * cpl, np.int32)
    so = np.zeros(3 * nl * cpl, np.int32)
    blk = np.zeros(n + 1, np.int32)
    cp, co = C.c_int64(0), C.c_int64(0)
    check(lib().odesat_cv_layout(n, m, i32ptr(lits), i32ptr(vst), nl, cpl, tsize, blk_cap, iters, i32ptr(sc),
                                 i32ptr(so), i32ptr(blk), C.byref(cp), C.byref(co)))
    return sc, so.reshape(-1, 3), blk, cp.value, co.value


def set_experiment(key: str, value) -> None:
    """An experiment knob (include/odesat.h odesat_set_experiment): A/B variants and the
    parity tests' forced paths.  value None (or < 0) unsets it.  Read when a solver / partition / stoch
    context is created."""
    check(lib().odesat_set_experiment(key.encode(), -1 if value is None else int(value)))


def get_experiment(key: str):
    v = C.c_int64(0)
    check(lib().odesat_get_experiment(key.encode(), C.byref(v)))
    return None if v.value < 0 else v.value


def clear_experiments() -> None:
    lib().odesat_clear_experiments()


def experiment_knobs() -> list:
    out, i = [], 0
    name = C.c_char_p()
    while lib().odesat_experiment_knob(i, C.byref(name)) == ODESAT_OK:
        out.append(name.value.decode())
        i += 1
    return out


class experiments:
    """Context manager: `with experiments(WAVE=1, RES_NARROW=0): ...` sets the knobs and restores their
    previous values on exit."""

    def __init__(self, **knobs):
        self.knobs = knobs
        self.old = {}

    def __enter__(self):
        for k, v in self.knobs.items():
            self.old[k] = get_experiment(k)
            set_experiment(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.old.items():
            set_experiment(k, v)
        return False


def device_count() -> int:
    c = C.c_int(0)
    check(lib().odesat_device_count(C.byref(c)))
    return c.value
