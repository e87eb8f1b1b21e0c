"""CNF preprocessing for `solve` -- the Python face of the reference's cnf.rs:317-840.

The work runs in the C++ implementation inside libodesat_hip.so (odesat_amd/csrc/preprocess.cpp,
C ABI in include/odesat.h); this module marshals formulas, traces and assignments.  Names follow
the reference: repeatedly_resolve_and_update (cnf.rs:833-840) returns the reduced formula and its
SimplificationTrace; calculate_trace (cnf.rs:501-519) fills in the eliminated variables.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import ODESAT_STEP_BLOCKED_CLAUSE, ODESAT_STEP_VARIABLE_ELIMINATION, ODESAT_UNSET, check, lib
from .cnf import CNFFormula

__all__ = ["SimplificationTrace", "repeatedly_resolve_and_update", "calculate_trace", "evaluate_cnf_assign",
           "ODESAT_STEP_VARIABLE_ELIMINATION", "ODESAT_STEP_BLOCKED_CLAUSE"]


class SimplificationTrace:
    """cnf.rs:560-578: the eliminations in the order they were made."""

    def __init__(self, handle):
        self._h = handle

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().odesat_trace_free(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None

    def __len__(self):
        return int(lib().odesat_trace_nsteps(self._h))

    def step(self, i: int):
        """(kind, var, [[(var, is_negated), ...], ...])."""
        kind, var, nc, nl = C.c_int32(), C.c_int64(), C.c_int64(), C.c_int64()
        check(lib().odesat_trace_step(self._h, i, C.byref(kind), C.byref(var), C.byref(nc), C.byref(nl)))
        cp = np.zeros(nc.value + 1, np.int64)
        v = np.zeros(max(nl.value, 1), np.int64)
        n = np.zeros(max(nl.value, 1), np.uint8)
        check(lib().odesat_trace_step_clauses(self._h, i, _lib.i64ptr(cp), _lib.i64ptr(v), _lib.u8ptr(n)))
        clauses = [[(int(v[s]), bool(n[s])) for s in range(cp[c], cp[c + 1])] for c in range(nc.value)]
        return int(kind.value), int(var.value), clauses

    def steps(self):
        return [self.step(i) for i in range(len(self))]


def repeatedly_resolve_and_update(formula: CNFFormula, desired_ratio: float):
    """Returns (reduced formula, trace); the input is not modified (the reference mutates its
    CNFFormulaSet in place and hands back the trace)."""
    out, tr = C.c_void_p(), C.c_void_p()
    check(lib().odesat_preprocess(formula.handle, float(desired_ratio), C.byref(out), C.byref(tr)))
    return CNFFormula(out), SimplificationTrace(tr)


def _to_tri(values: dict, top: int) -> np.ndarray:
    arr = np.full(max(top, 1), ODESAT_UNSET, np.uint8)
    for k, v in values.items():
        if 0 <= k < top:
            arr[k] = 1 if v else 0
    return arr


def _from_tri(arr: np.ndarray, values: dict) -> None:
    for k in np.flatnonzero(arr != ODESAT_UNSET):
        values[int(k)] = bool(arr[k])


def calculate_trace(assignments: dict, trace: SimplificationTrace, formula: CNFFormula | None = None) -> None:
    """cnf.rs:501-519, in place on {var: bool}.  `formula` (the unreduced input) only sizes the
    value array; without it the trace's own variables do."""
    top = max(assignments.keys(), default=-1)
    if formula is not None:
        top = max(top, int(lib().odesat_cnf_max_variable(formula.handle)))
    else:
        for _, var, clauses in trace.steps():
            top = max([top, var] + [v for c in clauses for v, _ in c])
    arr = _to_tri(assignments, top + 1)
    check(lib().odesat_trace_apply(trace._h, _lib.u8ptr(arr), len(arr)))
    _from_tri(arr, assignments)


def evaluate_cnf_assign(assignments: dict, formula: CNFFormula) -> bool:
    """cnf.rs:246-264 with its side effect on the map (unset variables read become false)."""
    top = max(max(assignments.keys(), default=-1), int(lib().odesat_cnf_max_variable(formula.handle))) + 1
    arr = _to_tri(assignments, top)
    r = check(lib().odesat_cnf_evaluate_assign(formula.handle, _lib.u8ptr(arr), len(arr)))
    _from_tri(arr, assignments)
    return bool(r)
