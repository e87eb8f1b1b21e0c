"""ctypes binding of the C oracle (oracle/build/libodesat_oracle.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as
the checker / CPU baseline, never by odesat_amd.  Build with `make -C oracle` (or
__graft_entry__.build()).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libodesat_oracle.so")

_i64p = np.ctypeslib.ndpointer(np.int64, flags="C_CONTIGUOUS")
_i32p = np.ctypeslib.ndpointer(np.int32, flags="C_CONTIGUOUS")
_u8p = np.ctypeslib.ndpointer(np.uint8, flags="C_CONTIGUOUS")
_f64p = np.ctypeslib.ndpointer(np.float64, flags="C_CONTIGUOUS")
_f32p = np.ctypeslib.ndpointer(np.float32, flags="C_CONTIGUOUS")


class _Formula(C.Structure):
    _fields_ = [("varnum", C.c_int64), ("nclauses", C.c_int64), ("clause_ptr", C.c_void_p),
                ("var", C.c_void_p), ("neg", C.c_void_p)]


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        for p, R, Rp in (("oc64_", C.c_double, _f64p), ("oc32_", C.c_float, _f32p)):
            fp = C.POINTER(_Formula)
            getattr(L, p + "compute_derivatives").argtypes = [fp, Rp, Rp, Rp, Rp, Rp, Rp, R, C.POINTER(C.c_int64)]
            getattr(L, p + "compute_derivatives").restype = C.c_int
            getattr(L, p + "update_state").argtypes = [fp, Rp, Rp, Rp, Rp, Rp, Rp, R]
            getattr(L, p + "update_state").restype = None
            getattr(L, p + "max_error").argtypes = [fp, Rp, Rp, Rp, Rp, Rp, Rp]
            getattr(L, p + "max_error").restype = R
            getattr(L, p + "euler_step").argtypes = [fp, Rp, Rp, Rp, R, C.POINTER(R), R, C.POINTER(C.c_int64)]
            getattr(L, p + "euler_step").restype = C.c_int
            getattr(L, p + "euler_step_fixed").argtypes = [fp, Rp, Rp, Rp, R, R, C.POINTER(C.c_int64)]
            getattr(L, p + "euler_step_fixed").restype = C.c_int
            getattr(L, p + "simulate").argtypes = [fp, Rp, Rp, Rp, C.c_int, R, C.c_int, R, C.c_int64,
                                                   C.c_int, R, _u8p, C.POINTER(C.c_int), C.POINTER(R),
                                                   C.POINTER(C.c_int64)]
            getattr(L, p + "simulate").restype = C.c_int64
            getattr(L, p + "simulate_inter").argtypes = [fp, C.c_int64, Rp, Rp, Rp, C.c_int, R, C.c_int, R,
                                                         C.c_int64, C.c_int, R, C.c_int, _u8p,
                                                         C.POINTER(C.c_int64), Rp, C.POINTER(C.c_int64)]
            getattr(L, p + "simulate_inter").restype = C.c_int64
            getattr(L, p + "init_short_term_memory").argtypes = [fp, Rp]
            getattr(L, p + "init_short_term_memory").restype = None
            getattr(L, p + "default_zeta").argtypes = [fp]
            getattr(L, p + "default_zeta").restype = R
            getattr(L, p + "batch_run").argtypes = [fp, C.c_int64, Rp, Rp, Rp, C.c_int, R, R, C.c_int64, R,
                                                    C.c_int, _i64p, _i64p, Rp]
            getattr(L, p + "batch_run").restype = C.c_int64
        L.oc_init_voltages.argtypes = [C.c_uint64, C.c_int64, C.c_int64, C.c_int64, _f64p]
        L.oc_init_voltages.restype = None
        L.oc_hash3.argtypes = [C.c_uint64, C.c_uint64, C.c_uint64]
        L.oc_hash3.restype = C.c_uint64
        for p, Rp in (("oc64_", _f64p), ("oc32_", _f32p)):
            getattr(L, p + "run").argtypes = [C.c_int32, C.c_int32, _i32p, _i32p, C.c_void_p, C.c_int32, Rp, Rp, Rp,
                                              Rp, Rp, Rp, _i64p, _i64p]
            getattr(L, p + "run").restype = C.c_int
        _u64p = np.ctypeslib.ndpointer(np.uint64, flags="C_CONTIGUOUS")
        L.oc_stoch_hash.argtypes = [C.c_uint64] * 4
        L.oc_stoch_hash.restype = C.c_uint64
        L.oc_stoch_step.argtypes = [C.POINTER(_Formula), _u8p, _u64p, C.c_uint64, C.c_uint64, C.c_uint64, _u64p, _u64p]
        L.oc_stoch_step.restype = C.c_int
        L.oc_stoch_search.argtypes = [C.POINTER(_Formula), _u8p, _u64p, C.c_uint64, C.c_uint64, C.c_int64, _u64p,
                                      C.POINTER(C.c_int)]
        L.oc_stoch_search.restype = C.c_int64
        _lib = L
    return _lib


class Oracle:
    """The C oracle bound to one formula, at one precision ("f64" or "f32")."""

    def __init__(self, clause_ptr, var, neg, varnum, precision="f64"):
        self.clause_ptr = np.ascontiguousarray(clause_ptr, dtype=np.int64)
        self.var = np.ascontiguousarray(var, dtype=np.int32)
        self.neg = np.ascontiguousarray(neg, dtype=np.uint8)
        self.n = int(varnum)
        self.m = len(self.clause_ptr) - 1
        self._f = _Formula(self.n, self.m, self.clause_ptr.ctypes.data, self.var.ctypes.data,
                           self.neg.ctypes.data)
        self.p = "oc64_" if precision == "f64" else "oc32_"
        self.T = np.float64 if precision == "f64" else np.float32
        self.CR = C.c_double if precision == "f64" else C.c_float
        self.L = lib()

    def _fn(self, name):
        return getattr(self.L, self.p + name)

    def _a(self, x):
        return np.ascontiguousarray(x, dtype=self.T)

    def compute_derivatives(self, v, xs, xl, zeta):
        v, xs, xl = self._a(v), self._a(xs), self._a(xl)
        dv = np.empty(self.n, self.T)
        dxs = np.empty(self.m, self.T)
        dxl = np.empty(self.m, self.T)
        rf = C.c_int64(0)
        s = self._fn("compute_derivatives")(C.byref(self._f), v, xs, xl, dv, dxs, dxl, zeta, C.byref(rf))
        return dv, dxs, dxl, bool(s), rf.value

    def update_state(self, v, xs, xl, dv, dxs, dxl, dt):
        self._fn("update_state")(C.byref(self._f), v, xs, xl, self._a(dv), self._a(dxs), self._a(dxl), dt)

    def max_error(self, a, b):
        return self._fn("max_error")(C.byref(self._f), *[self._a(x) for x in a], *[self._a(x) for x in b])

    def euler_step_fixed(self, v, xs, xl, dt, zeta):
        return bool(self._fn("euler_step_fixed")(C.byref(self._f), v, xs, xl, dt, zeta, None))

    def euler_step(self, v, xs, xl, tol, dt, zeta):
        h = self.CR(dt)
        s = self._fn("euler_step")(C.byref(self._f), v, xs, xl, tol, C.byref(h), zeta, None)
        return bool(s), h.value

    def simulate(self, v, xs, xl, tol=None, dt=None, steps=0, zeta=None):
        """In place on (v, xs, xl).  Returns (steps_taken, sat, assignment, final_dt, r_fired)."""
        assign = np.zeros(self.n, np.uint8)
        sat = C.c_int(0)
        h = self.CR(0.0)
        rf = C.c_int64(0)
        t = self._fn("simulate")(C.byref(self._f), v, xs, xl, tol is not None, tol or 0.0,
                                 dt is not None, dt or 0.0, steps, zeta is not None, zeta or 0.0,
                                 assign, C.byref(sat), C.byref(h), C.byref(rf))
        if t < 0:
            raise ValueError("oracle simulate failed")
        return t, bool(sat.value), assign.astype(bool), h.value, rf.value

    def simulate_inter(self, v, xs, xl, tol=None, dt=None, steps=0, zeta=None, shared_dt=True):
        """v [B, n], xs/xl [B, m] in place.  Returns (steps, winner, assignment, dts)."""
        B = v.shape[0]
        assign = np.zeros(self.n, np.uint8)
        win = C.c_int64(-1)
        dts = np.zeros(B, self.T)
        t = self._fn("simulate_inter")(C.byref(self._f), B, v, xs, xl, tol is not None, tol or 0.0,
                                       dt is not None, dt or 0.0, steps, zeta is not None, zeta or 0.0,
                                       1 if shared_dt else 0, assign, C.byref(win), dts, None)
        if t < 0:
            raise ValueError("oracle simulate_inter failed")
        return t, win.value, assign.astype(bool), (dts[:1] if shared_dt else dts)

    def init_short_term_memory(self):
        xs = np.empty(self.m, self.T)
        self._fn("init_short_term_memory")(C.byref(self._f), xs)
        return xs

    # -- stoch.rs (stoch_oracle.c) --------------------------------------------------------------
    def stoch_step(self, v, xl, seed, replica, step):
        """One step in place on v (uint8[n]) and xl (uint64[m]); returns all-satisfied (or raises
        where the reference panics)."""
        tot = np.zeros(max(self.n, 1), np.uint64)
        uns = np.zeros(max(self.n, 1), np.uint64)
        r = self.L.oc_stoch_step(C.byref(self._f), v, xl, seed, replica, step, tot, uns)
        if r < 0:
            raise ValueError("a variable occurs in no clause (stoch.rs:70 panics)")
        return bool(r)

    def stoch_search(self, v, xl, seed, replica, steps):
        """search (stoch.rs:83-110) from (v, xl) in place, at most `steps` steps.
        Returns (steps_taken, sat)."""
        scratch = np.zeros(2 * max(self.n, 1), np.uint64)
        sat = C.c_int(0)
        t = self.L.oc_stoch_search(C.byref(self._f), v, xl, seed, replica, steps, scratch, C.byref(sat))
        if t < 0:
            raise ValueError("a variable occurs in no clause (stoch.rs:70 panics)")
        return int(t), bool(sat.value)

    def batch_run(self, v, xs, xl, adaptive, tol, dt, steps, zeta, nthreads=1):
        """Independent replicas, replica-major [B, n] / [B, m], in place."""
        B = v.shape[0]
        sat = np.zeros(B, np.int64)
        done = np.zeros(B, np.int64)
        dts = np.zeros(B, self.T)
        total = self._fn("batch_run")(C.byref(self._f), B, v, xs, xl, 1 if adaptive else 0, tol, dt, steps,
                                      zeta, nthreads, sat, done, dts)
        return total, sat, done, dts


def run(n, clause_ptr, lits, params, v0, xs0, xl0, precision="f32"):
    """SURVEY 8(b) one-call boundary on the CPU (oc64_run / oc32_run): states replica-innermost
    [n][B] / [m][B]; params = a ctypes struct with odesat_params' layout.  Returns
    (v, xs, xl, first_sat_step[B], steps_done[B])."""
    T = np.float64 if precision == "f64" else np.float32
    cp = np.ascontiguousarray(clause_ptr, np.int32)
    lt = np.ascontiguousarray(lits, np.int32) if len(lits) else np.zeros(1, np.int32)
    v0, xs0, xl0 = (np.ascontiguousarray(a, T) for a in (v0, xs0, xl0))
    m, B = len(cp) - 1, v0.shape[1]
    v, xs, xl = np.empty_like(v0), np.empty_like(xs0), np.empty_like(xl0)
    sat, done = np.zeros(B, np.int64), np.zeros(B, np.int64)
    fn = getattr(lib(), ("oc64_" if precision == "f64" else "oc32_") + "run")
    if fn(n, m, cp, lt, C.cast(C.byref(params), C.c_void_p), B, v0, xs0, xl0, v, xs, xl, sat, done) != 0:
        raise ValueError("oracle run failed")
    return v, xs, xl, sat, done


def init_voltages(seed, r0, B, n):
    out = np.empty((B, n), np.float64)
    lib().oc_init_voltages(seed, r0, B, n, out)
    return out
