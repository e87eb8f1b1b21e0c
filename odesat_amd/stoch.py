"""The discrete stochastic search of the reference's `stoch` command (stoch.rs:20-110), on the GPU.

The work runs in csrc/stoch.hip behind the C ABI (include/odesat.h, odesat_stoch_*); this module
marshals arrays.  `StochSearch` holds B independent replicas of a normalised formula; `search`
mirrors stoch.rs::search for one replica (v = false, xl = 1, step until every clause is satisfied).
The draw uses a counter RNG of (seed, replica, step, variable) instead of thread_rng (declared
deviation, include/odesat.h).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import ODESAT_STOP_EACH, ODESAT_STOP_NONE, check, lib
from .cnf import CNFFormula

__all__ = ["StochSearch", "search", "ODESAT_STOP_EACH", "ODESAT_STOP_NONE"]

_u64p = C.POINTER(C.c_uint64)


def _u64(a):
    return a.ctypes.data_as(_u64p)


class StochSearch:
    """B replicas of the stoch state (stoch.rs:8-12: v bool[n], xl u64[m]) on one GPU."""

    def __init__(self, formula: CNFFormula, batch: int, device: int = 0):
        h = C.c_void_p()
        check(lib().odesat_stoch_create(int(device), formula.handle, int(batch), C.byref(h)))
        self._h = h
        self.batch, self.n, self.m = int(batch), formula.varnum, formula.nclauses

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().odesat_stoch_destroy(self._h)
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
    def wave_width(self) -> int:
        """Replicas per workgroup of the one-wave-per-replica kernel, 0 on the 3-kernel path."""
        return int(lib().odesat_stoch_wave_width(self._h))

    def reset(self, r0: int = 0, count: int | None = None):
        count = self.batch - r0 if count is None else count
        check(lib().odesat_stoch_reset(self._h, r0, count))

    def set_state(self, v, xl, r0: int = 0):
        v = np.ascontiguousarray(np.atleast_2d(v), np.uint8)
        xl = np.ascontiguousarray(np.atleast_2d(xl), np.uint64)
        if v.shape[1] != self.n or xl.shape != (v.shape[0], self.m):
            raise ValueError("state shapes do not match the formula")
        check(lib().odesat_stoch_set_state(self._h, r0, v.shape[0], _lib.u8ptr(v), _u64(xl)))

    def get_state(self, r0: int = 0, count: int | None = None):
        count = self.batch - r0 if count is None else count
        v = np.zeros((count, self.n), np.uint8)
        xl = np.zeros((count, max(self.m, 1)), np.uint64)
        check(lib().odesat_stoch_get_state(self._h, r0, count, _lib.u8ptr(v), _u64(xl)))
        return v.astype(bool), xl[:, : self.m]

    def search(self, seed: int, max_steps: int, stop: int = ODESAT_STOP_EACH, replica0: int = 0,
               poll_interval: int = 0) -> dict:
        sat = np.zeros(self.batch, np.int64)
        done = np.zeros(self.batch, np.int64)
        check(lib().odesat_stoch_search(self._h, int(seed), int(replica0), int(max_steps), int(stop),
                                        int(poll_interval), _lib.i64ptr(sat), _lib.i64ptr(done)))
        return {"first_sat_step": sat, "steps_done": done}


def search(formula: CNFFormula, steps: int | None = None, seed: int = 42, device: int = 0) -> np.ndarray:
    """stoch.rs:83-110: one replica from v = false, xl = 1; `steps = None` runs until every clause is
    satisfied (in chunks of 2^16 steps).  Returns the boolean vector."""
    with StochSearch(formula, 1, device) as s:
        if steps is not None:
            if steps > 0:
                s.search(seed, steps)
        else:
            while s.search(seed, 1 << 16)["first_sat_step"][0] < 0:
                pass
        return s.get_state()[0][0]
