"""Formula loading and result helpers -- the Python face of the reference's src/cnf.rs.

Parsing, normalisation and evaluation run in the C++ loader of libodesat_hip.so
(odesat_amd/csrc/cnf.cpp, C ABI in include/odesat.h); this module only marshals arrays.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from ._lib import check, lib


class CNFFormula:
    """cnf.rs:53-57: clauses in file order as a CSR (clause_ptr, var, neg) plus `varnum`."""

    def __init__(self, handle):
        self._h = C.c_void_p(handle) if not isinstance(handle, C.c_void_p) else handle

    def __del__(self):
        h = getattr(self, "_h", None)
        if h is not None and h.value:
            try:
                lib().odesat_cnf_free(h)
            except Exception:  # interpreter shutdown
                pass
            self._h = None

    @property
    def handle(self):
        return self._h

    @property
    def varnum(self) -> int:
        return int(lib().odesat_cnf_varnum(self._h))

    @property
    def nclauses(self) -> int:
        return int(lib().odesat_cnf_nclauses(self._h))

    @property
    def nliterals(self) -> int:
        return int(lib().odesat_cnf_nliterals(self._h))

    def arrays(self):
        """(clause_ptr int64[m+1], var int64[L], neg uint8[L])."""
        m, L = self.nclauses, self.nliterals
        cp = np.zeros(m + 1, np.int64)
        var = np.zeros(max(L, 1), np.int64)
        neg = np.zeros(max(L, 1), np.uint8)
        check(lib().odesat_cnf_export(self._h, _lib.i64ptr(cp), _lib.i64ptr(var), _lib.u8ptr(neg)))
        return cp, var[:L], neg[:L]

    def clauses(self):
        """[[(variable, is_negated), ...], ...] (cnf.rs Literal fields)."""
        cp, var, neg = self.arrays()
        return [[(int(var[s]), bool(neg[s])) for s in range(cp[c], cp[c + 1])] for c in range(len(cp) - 1)]

    @classmethod
    def from_arrays(cls, clause_ptr, var, neg, varnum=None):
        cp = np.ascontiguousarray(clause_ptr, np.int64)
        v = np.ascontiguousarray(var, np.int64)
        n = np.ascontiguousarray(neg, np.uint8)
        h = C.c_void_p()
        check(lib().odesat_cnf_from_arrays(-1 if varnum is None else int(varnum), len(cp) - 1,
                                           _lib.i64ptr(cp), _lib.i64ptr(v) if len(v) else None,
                                           _lib.u8ptr(n) if len(n) else None, C.byref(h)))
        return cls(h)

    @classmethod
    def from_clauses(cls, clauses, varnum=None):
        ptr, var, neg = [0], [], []
        for c in clauses:
            for v, ng in c:
                var.append(v)
                neg.append(1 if ng else 0)
            ptr.append(len(var))
        return cls.from_arrays(ptr, var, neg, varnum)


def parse_dimacs_format(text) -> CNFFormula:
    """cnf.rs:138-172."""
    data = text.encode() if isinstance(text, str) else bytes(text)
    h = C.c_void_p()
    check(lib().odesat_cnf_parse(data, len(data), C.byref(h)))
    return CNFFormula(h)


def normalize_cnf_variables(formula: CNFFormula):
    """cnf.rs:206-219 with the ascending renaming.  Returns (var_mapping old->new, normalized)."""
    cp, var, _ = formula.arrays()
    names = np.zeros(max(len(np.unique(var)), 1), np.int64)
    k = C.c_int64(0)
    h = C.c_void_p()
    check(lib().odesat_cnf_normalize(formula.handle, C.byref(h), _lib.i64ptr(names), C.byref(k)))
    mapping = {int(names[i]): i for i in range(k.value)}
    return mapping, CNFFormula(h)


def evaluate_cnf(values: dict, formula: CNFFormula) -> bool:
    """cnf.rs:246-264: missing variables read false (and are inserted, as the reference does)."""
    _, var, _ = formula.arrays()
    top = int(max(var.max(initial=0), max(values.keys(), default=0))) + 1
    arr = np.zeros(top, np.uint8)
    for k, v in values.items():
        if 0 <= k < top:
            arr[k] = 1 if v else 0
    for v in np.unique(var):
        values.setdefault(int(v), False)
    return bool(check(lib().odesat_cnf_evaluate(formula.handle, _lib.u8ptr(arr), top)))


def map_values_by_indices(indices_map: dict, values) -> dict:
    """cnf.rs:301-315."""
    return {k: bool(values[i]) for k, i in indices_map.items() if i < len(values)}


def render_variable_map(values: dict) -> str:
    """cnf.rs:289-298; ascending variable order (the reference prints HashMap order)."""
    return "".join(f"{k} {1 if v else 0}\n" for k, v in sorted(values.items()))


def init_short_term_memory(formula: CNFFormula) -> np.ndarray:
    """system.rs:361-372."""
    xs = np.zeros(max(formula.nclauses, 1), np.float64)
    check(lib().odesat_cnf_init_short_term_memory(formula.handle, _lib.dptr(xs)))
    return xs[: formula.nclauses]
