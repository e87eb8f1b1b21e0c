"""The integrator -- the Python face of the reference's src/system.rs, running on the MI355X.

`Solver` is the batched device object (one per GPU).  The module-level functions mirror the
reference's public API (system.rs:6-11, 25, 93, 101, 111, 141, 156, 241, 362) with the same names,
argument meanings and return values, so callers and tests read like the reference's own code.
Every call goes through libodesat_hip.so; there is no CPU path.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _lib
from ._lib import ODESAT_F32, ODESAT_F64, ODESAT_STOP_ANY, ODESAT_STOP_EACH, ODESAT_STOP_NONE, check, lib
from .cnf import CNFFormula, init_short_term_memory

__all__ = ["State", "Solver", "compute_derivatives", "update_state", "max_error", "euler_step",
           "euler_step_fixed", "simulate", "simulate_inter", "init_short_term_memory",
           "ODESAT_STOP_EACH", "ODESAT_STOP_ANY", "ODESAT_STOP_NONE"]


@dataclass
class State:
    """system.rs:6-11: voltages v[n], short memory xs[m], long memory xl[m] (f64 host arrays)."""
    v: np.ndarray
    xs: np.ndarray
    xl: np.ndarray

    def copy(self):
        return State(self.v.copy(), self.xs.copy(), self.xl.copy())


def _dtype_code(dtype):
    if dtype in ("f32", "float32", np.float32, ODESAT_F32):
        return ODESAT_F32
    if dtype in ("f64", "float64", np.float64, ODESAT_F64):
        return ODESAT_F64
    raise ValueError(f"dtype must be f32 or f64, got {dtype!r}")


class Solver:
    """A normalised formula + `batch` replica states resident on one GPU (odesat_solver)."""

    def __init__(self, formula: CNFFormula, batch: int, dtype="f32", device: int = 0):
        h = C.c_void_p()
        check(lib().odesat_solver_create(int(device), formula.handle, int(batch), _dtype_code(dtype),
                                         C.byref(h)))
        self._h = h
        self.formula = formula
        self.batch = int(batch)
        self.n = formula.varnum
        self.m = formula.nclauses
        self.dtype = "f64" if _dtype_code(dtype) == ODESAT_F64 else "f32"

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().odesat_solver_destroy(self._h)
        self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def device_bytes(self) -> int:
        return int(lib().odesat_solver_device_bytes(self._h))

    # -- state ------------------------------------------------------------------------------------
    def set_state(self, v, xs, xl, r0: int = 0):
        """Replica-major f64 arrays [count, n] / [count, m] for replicas r0 .. r0+count-1."""
        v = np.ascontiguousarray(np.atleast_2d(v), np.float64)
        xs = np.ascontiguousarray(np.atleast_2d(xs), np.float64)
        xl = np.ascontiguousarray(np.atleast_2d(xl), np.float64)
        count = v.shape[0]
        if v.shape != (count, self.n) or xs.shape != (count, self.m) or xl.shape != (count, self.m):
            raise ValueError("state shapes do not match the formula")
        check(lib().odesat_set_state(self._h, r0, count, _lib.dptr(v), _lib.dptr(xs), _lib.dptr(xl)))

    def init_state(self, seed: int, replica0: int = 0):
        check(lib().odesat_init_state(self._h, C.c_uint64(seed), replica0))

    def get_state(self, r0: int = 0, count: int | None = None):
        count = self.batch - r0 if count is None else count
        v = np.zeros((count, self.n), np.float64)
        xs = np.zeros((count, max(self.m, 1)), np.float64)[:, : self.m].copy()
        xl = np.zeros_like(xs)
        check(lib().odesat_get_state(self._h, r0, count, _lib.dptr(v), _lib.dptr(xs) if self.m else None,
                                     _lib.dptr(xl) if self.m else None))
        return v, xs, xl

    def get_assignment(self, r: int) -> np.ndarray:
        out = np.zeros(self.n, np.uint8)
        check(lib().odesat_get_assignment(self._h, r, _lib.u8ptr(out)))
        return out.astype(bool)

    def evaluate(self):
        """evaluate_cnf (cnf.rs:246-264) of every replica's assignment on the device.  Returns
        (satisfied bool[B], the lowest satisfying replica or -1)."""
        sat = np.zeros(self.batch, np.uint8)
        first = C.c_int64(-1)
        check(lib().odesat_evaluate(self._h, _lib.u8ptr(sat), C.byref(first)))
        return sat.astype(bool), int(first.value)

    # -- single operations (system.rs:25, 111, 141) -----------------------------------------------
    def compute_derivatives(self, zeta: float):
        B = self.batch
        dv = np.zeros((B, self.n))
        dxs = np.zeros((B, max(self.m, 1)))
        dxl = np.zeros((B, max(self.m, 1)))
        allsat = np.zeros(B, np.uint8)
        check(lib().odesat_compute_derivatives(self._h, zeta, _lib.dptr(dv), _lib.dptr(dxs) if self.m else None,
                                               _lib.dptr(dxl) if self.m else None, _lib.u8ptr(allsat)))
        return dv, dxs[:, : self.m], dxl[:, : self.m], allsat.astype(bool)

    def euler_step_fixed(self, dt: float, zeta: float):
        allsat = np.zeros(self.batch, np.uint8)
        check(lib().odesat_euler_step_fixed(self._h, dt, zeta, _lib.u8ptr(allsat)))
        return allsat.astype(bool)

    def euler_step(self, tol: float, dt, zeta: float):
        h = np.ascontiguousarray(np.broadcast_to(np.asarray(dt, np.float64), (self.batch,))).copy()
        allsat = np.zeros(self.batch, np.uint8)
        check(lib().odesat_euler_step(self._h, tol, _lib.dptr(h), zeta, _lib.u8ptr(allsat)))
        return allsat.astype(bool), h

    # -- drivers -----------------------------------------------------------------------------------
    def simulate(self, *, adaptive=False, dt=0.01, tol=1e-3, zeta=None, max_steps=1000,
                 stop=ODESAT_STOP_EACH, poll_interval=0, resume=False, reuse=False):
        """Returns dict(first_sat_step[B], steps_done[B], dt[B], steps_run).  resume=True continues
        the previous run (odesat_simulate_continue): bookkeeping carries over, steps are numbered
        from the run's start.

        reuse=True: the result arrays are the solver's own, overwritten by the next reuse=True call,
        and the call allocates nothing on the host (the params, the arrays and their ctypes pointers
        are built once per solver).  A call's Python prologue otherwise allocates three arrays and
        six ctypes objects: ~8 us per call, and ~55 us on the first timed call after a warm-up
        (profiles/r04s_first_call.jsonl) -- 3-4 % of a 20-step config-2 launch."""
        if reuse:
            return self._simulate_reuse(adaptive, dt, tol, zeta, max_steps, stop, poll_interval, resume)
        p = _lib.Params(1 if adaptive else 0, int(stop), float(tol), float(dt),
                        -1.0 if zeta is None else float(zeta), int(max_steps), int(poll_interval), 0)
        B = self.batch
        sat = np.zeros(B, np.int64)
        done = np.zeros(B, np.int64)
        dts = np.zeros(B, np.float64)
        run = C.c_int64(0)
        fn = lib().odesat_simulate_continue if resume else lib().odesat_simulate
        check(fn(self._h, C.byref(p), _lib.i64ptr(sat), _lib.i64ptr(done), _lib.dptr(dts), C.byref(run)))
        return {"first_sat_step": sat, "steps_done": done, "dt": dts, "steps_run": run.value}

    def _simulate_reuse(self, adaptive, dt, tol, zeta, max_steps, stop, poll_interval, resume):
        cache = self.__dict__.get("_call")
        if cache is None:
            B = self.batch
            p = _lib.Params(0, 0, 0.0, 0.0, -1.0, 1, 0, 0)
            res = {"first_sat_step": np.zeros(B, np.int64), "steps_done": np.zeros(B, np.int64),
                   "dt": np.zeros(B, np.float64), "steps_run": 0}
            run = C.c_int64(0)
            args = (C.byref(p), _lib.i64ptr(res["first_sat_step"]), _lib.i64ptr(res["steps_done"]),
                    _lib.dptr(res["dt"]), C.byref(run))
            cache = self._call = (p, res, run, args, lib().odesat_simulate, lib().odesat_simulate_continue)
        p, res, run, args, fn, fn_cont = cache
        p.adaptive = 1 if adaptive else 0
        p.stop = int(stop)
        p.tol = float(tol)
        p.dt = float(dt)
        p.zeta = -1.0 if zeta is None else float(zeta)
        p.max_steps = int(max_steps)
        p.poll_interval = int(poll_interval)
        check((fn_cont if resume else fn)(self._h, *args))
        res["steps_run"] = run.value
        return res

    def synchronize(self):
        check(lib().odesat_synchronize(self._h))

    def checkpoint(self):
        """Device-side copy of every replica's state and bookkeeping (odesat_checkpoint)."""
        check(lib().odesat_checkpoint(self._h))

    def rollback(self):
        """Back to the last checkpoint (odesat_rollback)."""
        check(lib().odesat_rollback(self._h))

    def set_chunk_replicas(self, replicas: int):
        check(lib().odesat_set_chunk_replicas(self._h, int(replicas)))

    def set_schedule(self, schedule: int):
        """_lib.ODESAT_SCHED_AUTO / _STEP_MAJOR / _CHUNK_MAJOR (results are identical)."""
        check(lib().odesat_set_schedule(self._h, int(schedule)))

    def set_algorithm(self, alg: int):
        """_lib.ODESAT_ALG_FUSED / _TWOPASS / _RESIDENT (results are bit-identical)."""
        check(lib().odesat_set_algorithm(self._h, int(alg)))

    @property
    def algorithm(self) -> int:
        return check(lib().odesat_get_algorithm(self._h))

    def step_kernel(self, adaptive: bool = False) -> str:
        """The kernel simulate launches for fixed or adaptive steps (odesat_step_kernel)."""
        return lib().odesat_step_kernel(self._h, 1 if adaptive else 0).decode()

    @property
    def group_width(self) -> int:
        return check(lib().odesat_group_width(self._h))

    def profile(self, enable: bool):
        check(lib().odesat_profile_enable(self._h, 1 if enable else 0))

    def profile_read(self):
        ms = np.zeros(3)
        n = np.zeros(3, np.int64)
        check(lib().odesat_profile_read(self._h, _lib.dptr(ms), _lib.i64ptr(n)))
        return ms, n

    def clause_kernel_bytes(self) -> int:
        return int(lib().odesat_clause_kernel_bytes(self._h))


# ---------------------------------------------------------------------------------------------
# Reference-shaped functions (one replica, State in / out; f64 unless dtype says otherwise)
# ---------------------------------------------------------------------------------------------
def _one(formula, state: State, dtype):
    s = Solver(formula, 1, dtype)
    s.set_state(state.v[None], state.xs[None], state.xl[None])
    return s


def _load_back(s: Solver, state: State):
    v, xs, xl = s.get_state(0, 1)
    state.v[:] = v[0]
    state.xs[:] = xs[0]
    state.xl[:] = xl[0]


def compute_derivatives(y: State, formula: CNFFormula, zeta: float, dtype="f64"):
    """system.rs:25-91 -> (dy: State, allsat)."""
    with _one(formula, y, dtype) as s:
        dv, dxs, dxl, allsat = s.compute_derivatives(zeta)
    return State(dv[0], dxs[0], dxl[0]), bool(allsat[0])


def update_state(state: State, derivatives: State, dt: float, clause_nums: int):
    """system.rs:93-97 (host arithmetic on host arrays: the device fuses it into the step)."""
    eps = 0.001
    state.xs[:] = np.fmin(np.fmax(state.xs + dt * derivatives.xs, eps), 1.0 - eps)
    state.xl[:] = np.fmin(np.fmax(state.xl + dt * derivatives.xl, 1.0), 1e4 * float(clause_nums))
    state.v[:] = np.fmin(np.fmax(state.v + dt * derivatives.v, -1.0), 1.0)


def max_error(a: State, b: State) -> float:
    """system.rs:99-109 (NaN-seeded fold of f64::max)."""
    out = np.nan
    for x, y in ((a.v, b.v), (a.xs, b.xs), (a.xl, b.xl)):
        e = np.fmax.reduce(np.abs(x - y), initial=np.nan) if len(x) else np.nan
        out = np.fmax(out, e)
    return float(out)


def euler_step_fixed(state: State, formula: CNFFormula, dt: float, zeta: float, dtype="f64") -> bool:
    """system.rs:141-154 (state mutated in place)."""
    with _one(formula, state, dtype) as s:
        allsat = s.euler_step_fixed(dt, zeta)
        _load_back(s, state)
    return bool(allsat[0])


def euler_step(state: State, formula: CNFFormula, tolerance: float, dt: float, zeta: float, dtype="f64"):
    """system.rs:111-139 -> (allsat, new dt) (state mutated in place)."""
    with _one(formula, state, dtype) as s:
        allsat, h = s.euler_step(tolerance, dt, zeta)
        _load_back(s, state)
    return bool(allsat[0]), float(h[0])


_UNBOUNDED_CHUNK = 1 << 20


def simulate(state: State, formula: CNFFormula, tolerance=None, step_size=None, steps=None,
             learning_rate=None, dtype="f64"):
    """system.rs:156-239 -> Vec<bool> (state mutated in place).  steps=None runs until allsat, as the
    reference does (it never returns on an UNSAT formula)."""
    with _one(formula, state, dtype) as s:
        kw = dict(adaptive=step_size is None, dt=step_size or 0.01,
                  tol=1e-3 if tolerance is None else tolerance, zeta=learning_rate, stop=ODESAT_STOP_EACH)
        if steps is not None:
            if steps > 0:
                s.simulate(max_steps=steps, **kw)
        else:  # one run in bounded calls: dt and the step count carry over (system.rs:198-234)
            r = s.simulate(max_steps=_UNBOUNDED_CHUNK, **kw)
            while r["first_sat_step"][0] < 0:
                r = s.simulate(max_steps=_UNBOUNDED_CHUNK, resume=True, **kw)
        _load_back(s, state)
    return state.v > 0.0


def simulate_inter(states: list, formula: CNFFormula, tolerance=None, step_size=None, steps=None,
                   learning_rate=None, dtype="f64"):
    """system.rs:241-359 -> Vec<bool> of the first sat replica (else replica 0); states mutated.
    Declared deviation: the adaptive variant gives every replica its own dt (see include/odesat.h)."""
    B = len(states)
    with Solver(formula, B, dtype) as s:
        s.set_state(np.stack([x.v for x in states]), np.stack([x.xs for x in states]),
                    np.stack([x.xl for x in states]))
        kw = dict(adaptive=step_size is None, dt=step_size or 0.01,
                  tol=1e-3 if tolerance is None else tolerance, zeta=learning_rate, stop=ODESAT_STOP_ANY)
        if steps is None:
            r = s.simulate(max_steps=_UNBOUNDED_CHUNK, **kw)
            while not (r["first_sat_step"] >= 0).any():
                r = s.simulate(max_steps=_UNBOUNDED_CHUNK, resume=True, **kw)
        elif steps > 0:
            r = s.simulate(max_steps=steps, **kw)
        else:
            r = {"first_sat_step": np.full(B, -1)}
        v, xs, xl = s.get_state()
    for b, st in enumerate(states):
        st.v[:], st.xs[:], st.xl[:] = v[b], xs[b], xl[b]
    sat = np.flatnonzero(r["first_sat_step"] >= 0)
    # steps == 0: the reference's state_res starts all-true, so replica 0 is returned (:274, :353)
    pick = int(sat[0]) if len(sat) else 0
    return states[pick].v > 0.0
