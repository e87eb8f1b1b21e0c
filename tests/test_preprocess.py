"""CNF preprocessing (cnf.rs:317-840): the product's C++ (odesat_amd/csrc/preprocess.cpp, through
odesat_amd.preprocess) against the pure-Python restatement oracle/preprocess_oracle.py.

Parity: bit-for-bit equal reduced formulas (set order), varnums and traces, on the committed golden
cases (tests/golden/preprocess_golden.json, made by make_preprocess_golden.py from the reference's
fixtures) and on seeded random formulas that hit the edge cases the reference's code has (unit and
empty clauses, duplicate literals, tautologies, clashing units).  The reference has no fixtures for
this path and cannot run here, so the restatement itself is pinned by properties (brute force):
on k-SAT inputs (distinct variables per clause) every model of the reduced formula becomes a model
of the input through calculate_trace, and a satisfiable input never reduces to an unsatisfiable one.
"""
import itertools
import json
import os
import random

import numpy as np
import pytest

from odesat_amd import cnf
from odesat_amd._lib import ODESAT_UNSET, lib
from odesat_amd.preprocess import calculate_trace, evaluate_cnf_assign, repeatedly_resolve_and_update
from oracle import cnf_oracle as co
from oracle import preprocess_oracle as po

HERE = os.path.dirname(os.path.abspath(__file__))


def product(clauses, varnum, ratio):
    f = cnf.CNFFormula.from_clauses(clauses, varnum)
    g, tr = repeatedly_resolve_and_update(f, ratio)
    return g.clauses(), g.varnum, tr.steps(), tr


def as_lists(red, trace):
    return [list(c) for c in red], [(k, v, [list(c) for c in cs]) for k, v, cs in trace]


def edge_formula(seed):
    r = random.Random(seed)
    n = r.randint(1, 12)
    m = r.randint(0, 40)
    cl = []
    for _ in range(m):
        k = r.choice([0, 1, 1, 2, 3, 3, 4]) if r.random() < 0.3 else r.randint(1, 4)
        cl.append([(r.randint(1, n), r.random() < 0.5) for _ in range(k)])
    return cl, n, r.choice([1.0, 3.0, 4.5, 7.0, 20.0])


def ksat_formula(seed):
    r = random.Random(seed)
    n = r.randint(4, 13)
    m = r.randint(1, 5 * n)
    cl = [[(v, r.random() < 0.5) for v in r.sample(range(1, n + 1), min(n, r.choice([2, 3, 3, 4])))]
          for _ in range(m)]
    return cl, n, r.choice([3.0, 5.0, 7.0, 12.0])


def satisfies(clauses, a):
    return all(any(a.get(v, False) != ng for v, ng in c) for c in clauses)


def models(clauses, names):
    for bits in itertools.product([False, True], repeat=len(names)):
        a = dict(zip(names, bits))
        if satisfies(clauses, a):
            yield a


# --------------------------------------------------------------------------- golden + parity
def test_golden_fixtures():
    with open(os.path.join(HERE, "golden", "preprocess_golden.json")) as fh:
        cases = json.load(fh)
    assert len(cases) >= 5
    for case in cases:
        with open(os.path.join(HERE, "golden", case["fixture"] + ".cnf")) as fh:
            f = cnf.parse_dimacs_format(fh.read())
        g, tr = repeatedly_resolve_and_update(f, case["ratio"])
        exp_cl = [[(v, bool(n)) for v, n in c] for c in case["clauses"]]
        exp_tr = [(k, v, [[(a, bool(b)) for a, b in c] for c in cs]) for k, v, cs in case["trace"]]
        assert g.clauses() == exp_cl, case["fixture"]
        assert g.varnum == case["varnum"]
        assert tr.steps() == exp_tr


def test_oracle_reproduces_golden_small_case():
    """The restatement regenerates its committed vectors (fast cases; make_preprocess_golden.py
    regenerates all of them)."""
    with open(os.path.join(HERE, "golden", "preprocess_golden.json")) as fh:
        case = next(c for c in json.load(fh) if c["fixture"] == "small")
    with open(os.path.join(HERE, "golden", "small.cnf")) as fh:
        cl, varnum = co.parse_dimacs_format(fh.read())
    red, vn, trace = po.preprocess(cl, varnum, case["ratio"])
    assert [[[v, int(n)] for v, n in c] for c in red] == case["clauses"]
    assert vn == case["varnum"]
    assert [[k, v, [[[a, int(b)] for a, b in c] for c in cs]] for k, v, cs in trace] == case["trace"]


@pytest.mark.parametrize("seed", range(0, 240, 3))
def test_product_matches_oracle_edge_cases(seed):
    cl, n, ratio = edge_formula(seed)
    red, vn, steps, _ = product(cl, n, ratio)
    ored, ovn, otr = po.preprocess(cl, n, ratio)
    assert (red, steps) == as_lists(ored, otr)
    assert vn == ovn


def test_product_matches_oracle_uf_sized():
    from odesat_amd import workloads as wl
    var2, neg2 = wl.random_ksat(60, 256, 3, 11)
    cl = [[(int(v) + 1, bool(g)) for v, g in zip(a, b)] for a, b in zip(var2, neg2)]
    red, vn, steps, _ = product(cl, 60, 7.0)
    ored, ovn, otr = po.preprocess(cl, 60, 7.0)
    assert len(steps) > 5
    assert (red, steps) == as_lists(ored, otr) and vn == ovn


def test_empty_and_trivial_formulas():
    for cl, n in [([], 0), ([], 5), ([[]], 3), ([[(1, False)]], 1), ([[(1, False)], [(1, True)]], 1)]:
        red, vn, steps, _ = product(cl, n, 7.0)
        ored, ovn, otr = po.preprocess(cl, n, 7.0)
        assert (red, steps) == as_lists(ored, otr) and vn == ovn


def test_varnum_underflow_wraps_like_a_release_build():
    """usize arithmetic in min_ratio_resolvant / eliminate_variable (cnf.rs:741-742, :700)."""
    cl = [[(1, False), (2, False)], [(1, True), (3, False)]]
    red, vn, steps, _ = product(cl, 0, 1e30)
    ored, ovn, otr = po.preprocess(cl, 0, 1e30)
    assert (red, steps) == as_lists(ored, otr) and vn & po.U64 == ovn  # the ABI's int64 reads -1..


# --------------------------------------------------------------------------- properties
@pytest.mark.parametrize("seed", range(0, 160, 4))
def test_trace_rebuilds_models_of_the_input(seed):
    cl, n, ratio = ksat_formula(seed)
    red, _, _, tr = product(cl, n, ratio)
    names = sorted({v for c in cl for v, _ in c})
    rnames = sorted({v for c in red for v, _ in c})
    input_sat = any(True for _ in models(cl, names))
    reduced = list(itertools.islice(models(red, rnames), 32))
    if not input_sat:
        return  # the reference drops empty resolvents (cnf.rs:438), so UNSAT inputs may reduce to SAT ones
    assert reduced, "a satisfiable input reduced to an unsatisfiable formula"
    for a in reduced:
        got = dict(a)
        calculate_trace(got, tr)
        assert satisfies(cl, got)
        ref = dict(a)
        po.calculate_trace(ref, [(k, v, [tuple(c) for c in cs]) for k, v, cs in tr.steps()])
        assert got == ref


def test_calculate_trace_and_evaluate_insert_match_oracle():
    for seed in range(40):
        cl, n, ratio = edge_formula(1000 + seed)
        red, _, steps, tr = product(cl, n, ratio)
        r = random.Random(seed)
        base = {v: r.random() < 0.5 for c in red for v, _ in c if r.random() < 0.8}
        got, ref = dict(base), dict(base)
        calculate_trace(got, tr)
        po.calculate_trace(ref, [(k, v, [tuple(c) for c in cs]) for k, v, cs in steps])
        assert got == ref
        f = cnf.CNFFormula.from_clauses(cl, n)
        assert evaluate_cnf_assign(got, f) == po.evaluate_insert(ref, cl)
        assert got == ref  # the same variables were inserted


def test_abi_errors():
    import ctypes as C
    out, tr = C.c_void_p(), C.c_void_p()
    assert lib().odesat_preprocess(None, 7.0, C.byref(out), C.byref(tr)) < 0
    f = cnf.CNFFormula.from_clauses([[(5, False), (7, True)], [(5, True), (9, False)]], 9)
    g, t = repeatedly_resolve_and_update(f, 7.0)
    arr = np.full(3, ODESAT_UNSET, np.uint8)  # too short for variable 9
    from odesat_amd import _lib
    if len(t):
        assert lib().odesat_trace_apply(t._h, _lib.u8ptr(arr), 3) < 0
    assert lib().odesat_cnf_evaluate_assign(f.handle, _lib.u8ptr(arr), 3) < 0
    assert lib().odesat_cnf_max_variable(f.handle) == 9
