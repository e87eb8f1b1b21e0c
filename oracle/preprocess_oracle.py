"""Pure-Python restatement of the reference's CNF preprocessing (cnf.rs:317-840) and the trace that
rebuilds the eliminated variables (calculate_trace, cnf.rs:501-519).

TEST INFRASTRUCTURE ONLY -- imported by tests/ as the checker for the product's C++ implementation
(odesat_amd/csrc/preprocess.cpp).  Parity status: the reference ships no fixtures for this path and
cannot run here (no Rust toolchain), so this restatement is pinned by properties instead
(tests/test_preprocess.py): the reduced formula is satisfiable exactly when the input is, and the
trace turns every model of the reduced formula into a model of the input (brute force, small n).

Representation: a clause is a tuple of (variable, is_negated) pairs, sorted and de-duplicated --
the iteration order of BTreeSet<Literal> (Literal derives Ord on (variable, is_negated)), and tuple
comparison is BTreeSet<CNFClauseSet>'s order.  Every set the reference iterates is visited in
sorted order here.  The one deliberate deviation (shared with the product): min_ratio_resolvant
(cnf.rs:725-758) scans a HashSet, so ties go to a random variable per run; here candidates are
scanned in ascending order.
"""
from __future__ import annotations

import struct

__all__ = ["VE", "BCE", "preprocess", "calculate_trace", "evaluate_insert"]

VE, BCE = 0, 1  # SimplificationStep::{VariableElimination, BlockedClauseElimination} (cnf.rs:554-558)
U64 = (1 << 64) - 1


def _f32(x: float) -> float:
    return struct.unpack("f", struct.pack("f", x))[0]


def _f32_div(a: int, b: int) -> float:
    """`a as f32 / b as f32` (both usize)."""
    fa, fb = _f32(float(a)), _f32(float(b))
    if fb == 0.0:
        return float("nan") if fa == 0.0 else float("inf")
    return _f32(fa / fb)


def is_tautology(clause) -> bool:
    """cnf.rs:542-552."""
    s = set(clause)
    return any((v, not n) in s for v, n in clause)


def calculate_resolvents(index, clause, variable):
    """cnf.rs:403-443."""
    pos, neg = index[variable]
    other_clauses = neg if (variable, False) in clause else pos
    out = []
    for other in sorted(other_clauses):
        combined = set()
        contained = set()
        for v, n in clause:
            if v != variable:
                combined.add((v, n))
                contained.add((v, n))
        for v, n in other:
            if v != variable:
                if (v, not n) in contained:
                    combined.clear()
                    break
                combined.add((v, n))
        if combined:
            out.append(tuple(sorted(combined)))
    return out


def calculate_var_resolvents(index, variable):
    """cnf.rs:463-480."""
    res = set()
    for p in sorted(index[variable][0]):
        res.update(calculate_resolvents(index, p, variable))
    return res


def subsume_clauses(clauses: set):
    """cnf.rs:521-540 (in place)."""
    order = sorted(clauses)
    sets = [frozenset(c) for c in order]
    drop = []
    for c, sc in zip(order, sets):
        for d, sd in zip(order, sets):
            if c != d and sc >= sd:
                drop.append(c)
                break
    for c in drop:
        clauses.discard(c)


def is_blocked(clause, index):
    """cnf.rs:586-597."""
    for v, _ in clause:
        if all(is_tautology(r) for r in calculate_resolvents(index, clause, v)):
            return v
    return None


def eliminate_if_blocked(clause, clauses: set, index):
    """cnf.rs:599-629 -> (changed vars, step) or None."""
    var = is_blocked(clause, index)
    if var is None:
        return None
    changed = set()
    for v, n in clause:
        changed.add(v)
        pos, neg = index.setdefault(v, (set(), set()))
        (neg if n else pos).discard(clause)
    clauses.discard(clause)
    return changed, (BCE, var, [clause])


def eliminate_variable(state, index, variable, resolvents):
    """cnf.rs:632-722 -> (changed vars, modified positive clauses)."""
    if variable not in index:
        return set(), []
    opos, oneg = index.pop(variable)
    upd = set()
    for c in list(opos) + list(oneg):
        for v, _ in c:
            upd.add(v)
    for v in sorted(upd):
        if v in index:
            pos, neg = index[v]
            index[v] = ({c for c in pos if c not in opos and c not in oneg},
                        {c for c in neg if c not in opos and c not in oneg})
    for c in opos:
        state["clauses"].discard(c)
    for c in oneg:
        state["clauses"].discard(c)
    for r in resolvents:
        state["clauses"].add(r)
    state["varnum"] = (state["varnum"] - 1) & U64
    for r in resolvents:
        for v, n in r:
            pos, neg = index.setdefault(v, (set(), set()))
            (neg if n else pos).add(r)
    modified = {tuple(l for l in c if l != (variable, False)) for c in opos}
    return upd, sorted(modified)


def min_ratio_resolvant(cands, index, state, target):
    """cnf.rs:725-758 (ascending candidates)."""
    best, smallest = None, _f32(3.4028234663852886e38)
    for v in sorted(cands):
        if v not in index:
            continue
        pos, neg = index[v]
        res = {r for r in calculate_var_resolvents(index, v) if not is_tautology(r)}
        subsume_clauses(res)
        count = (len(state["clauses"]) - len(pos) - len(neg) + len(res)) & U64
        vars_ = (state["varnum"] - 1) & U64
        ratio = _f32_div(count, vars_)
        if ratio < smallest:
            smallest, best = ratio, (v, sorted(res))
    if smallest > _f32(target):
        return None
    return best


def preprocess(clauses, varnum: int, target_ratio: float):
    """convert_to_cnf_formula_set + repeatedly_resolve_and_update + convert_to_cnf_formula
    (cnf.rs:348-379, 760-840).  clauses: iterable of [(var, neg), ...].
    Returns (reduced clauses in set order, reduced varnum, trace steps [(kind, var, [clauses])])."""
    state = {"clauses": {tuple(sorted(set((int(v), bool(n)) for v, n in c))) for c in clauses},
             "varnum": int(varnum) & U64}
    index = {}
    for c in sorted(state["clauses"]):
        for v, n in c:
            pos, neg = index.setdefault(v, (set(), set()))
            (neg if n else pos).add(c)
    trace = []
    blocked = [c for c in sorted(state["clauses"]) if is_blocked(c, index) is not None]
    for c in blocked:
        r = eliminate_if_blocked(c, state["clauses"], index)
        if r is not None:
            trace.append(r[1])
    cands = set(index.keys())
    while True:
        pick = min_ratio_resolvant(cands, index, state, target_ratio)
        if pick is None:
            break
        var, res = pick
        changed, modified = eliminate_variable(state, index, var, res)
        trace.append((VE, var, modified))
        cands = set(changed)
        for r in res:
            got = eliminate_if_blocked(r, state["clauses"], index)
            if got is not None:
                trace.append(got[1])
                cands |= got[0]
    subsume_clauses(state["clauses"])
    return [list(c) for c in sorted(state["clauses"])], state["varnum"], trace


def evaluate_insert(values: dict, clauses) -> bool:
    """cnf.rs:246-287 evaluate_cnf / evaluate_cnf_set: unset variables read false and are inserted."""
    for c in clauses:
        ok = False
        for v, n in c:
            x = values.setdefault(v, False)
            ok = ok or (not x if n else x)
        if not ok:
            return False
    return True


def calculate_trace(values: dict, trace) -> None:
    """cnf.rs:501-519."""
    for kind, var, clauses in reversed(trace):
        if kind == VE:
            values[var] = not evaluate_insert(values, clauses)
        elif not evaluate_insert(values, clauses):
            values[var] = not values[var]
