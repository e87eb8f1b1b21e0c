"""Pure-Python restatement of the reference's DIMACS loader and result helpers (cnf.rs).

TEST INFRASTRUCTURE ONLY -- imported by tests/ as the checker for the product's C++ loader
(odesat_amd/csrc/cnf.cpp).  Parity status: no reference-executed outputs exist (Rust toolchain
absent), so this is pinned by the reference's own fixtures (tests/{small,easy,hard}.cnf, whose
shapes are asserted in tests/test_cnf.py) and by reading cnf.rs.

Deliberate, declared deviation shared with the product: the variable renaming of
normalize_cnf_variables (cnf.rs:206-219) iterates a HashSet, i.e. a random permutation per run;
here (and in the product) distinct variables are renamed in ascending order.
"""
from __future__ import annotations

import re

__all__ = [
    "DimacsError", "rust_lines", "parse_dimacs_format", "normalize_cnf_variables",
    "evaluate_cnf", "map_values_by_indices", "render_variable_map", "init_short_term_memory",
]


class DimacsError(ValueError):
    """Where the reference panics on `unwrap()` (cnf.rs:151,160)."""


_UINT = re.compile(r"^\+?[0-9]+$")
_INT = re.compile(r"^[+-]?[0-9]+$")
_WS = " \t\n\r\x0b\x0c"


def rust_lines(text: str) -> list[str]:
    """str::lines(): split on \\n, strip one trailing \\r per terminated line, no final empty line."""
    if text == "":
        return []
    parts = text.split("\n")
    terminated = [True] * (len(parts) - 1) + [False]
    if parts[-1] == "":
        parts.pop()
        terminated.pop()
    out = []
    for p, t in zip(parts, terminated):
        if t and p.endswith("\r"):
            p = p[:-1]
        out.append(p)
    return out


def _split_ws(line: str) -> list[str]:
    return [t for t in re.split(r"[ \t\n\r\x0b\x0c]+", line) if t]


def parse_dimacs_format(text: str):
    """cnf.rs:138-172.  Returns (clauses, varnum); clauses = [[(variable, is_negated), ...], ...]."""
    clauses: list[list[tuple[int, bool]]] = []
    varnum = None
    for line in rust_lines(text):
        if line.startswith("c"):  # :143
            continue
        if line.startswith("p cnf"):  # :146
            toks = _split_ws(line)
            if len(toks) < 3 or not _UINT.match(toks[2]):
                raise DimacsError(f"bad problem line: {line!r}")
            varnum = int(toks[2])
            continue
        lits = []
        for tok in _split_ws(line):  # :156-165
            if tok == "0":
                break
            if not _INT.match(tok):
                raise DimacsError(f"bad literal token {tok!r}")
            x = int(tok)
            if x < -(2**31) or x > 2**31 - 1:
                raise DimacsError(f"literal out of i32 range {tok!r}")
            lits.append((abs(x), x < 0))
        clauses.append(lits)  # an empty line is an empty clause (:167)
    if varnum is None:  # CNFFormula::new (cnf.rs:60-77)
        varnum = len({v for c in clauses for v, _ in c})
    return clauses, varnum


def normalize_cnf_variables(clauses, varnum):
    """cnf.rs:206-219 with the deterministic (ascending) renaming.  Returns (name_map, clauses)."""
    names = sorted({v for c in clauses for v, _ in c})
    name_map = {old: new for new, old in enumerate(names)}
    return name_map, [[(name_map[v], n) for v, n in c] for c in clauses]


def evaluate_cnf(values: dict, clauses) -> bool:
    """cnf.rs:246-264: a variable missing from the map reads (and is inserted as) false."""
    for c in clauses:
        ok = False
        for v, neg in c:
            val = values.setdefault(v, False)
            ok = ok or (not val if neg else val)
        if not ok:
            return False
    return True


def map_values_by_indices(indices_map: dict, values) -> dict:
    """cnf.rs:301-315."""
    return {k: bool(values[i]) for k, i in indices_map.items() if i < len(values)}


def render_variable_map(values: dict) -> str:
    """cnf.rs:289-298 ("{var} {0|1}\\n"); ascending order instead of HashMap order."""
    return "".join(f"{k} {1 if v else 0}\n" for k, v in sorted(values.items()))


def init_short_term_memory(clauses):
    """system.rs:361-372: +1 if the clause has a negated literal, else -1."""
    return [1.0 if any(n for _, n in c) else -1.0 for c in clauses]
