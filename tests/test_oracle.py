"""Pin the CPU oracle before trusting it (CPU only).

Parity status (see oracle/odesat_oracle.h): the Rust reference cannot run here, so the oracle is
pinned by (1) the hand-derived KATs in tests/golden/kat_small.json and (2) the golden vectors that
the independent numpy restatement wrote (tests/golden/make_golden.py), compared bit for bit.
"""
import json
import os

import numpy as np
import pytest

from oracle import np_oracle as npo
from oracle.oracle import Oracle, init_voltages
from odesat_amd import workloads as wl
from tests.common import FIXTURES, GOLDEN, golden, oracle_formula


def _oracle(f, prec):
    return Oracle(f.clause_ptr, f.var, f.neg, f.varnum, prec)


def _kat():
    with open(os.path.join(GOLDEN, "kat_small.json")) as fh:
        return json.load(fh)["cases"]


@pytest.mark.parametrize("case", _kat(), ids=lambda c: c["name"])
def test_hand_kat_small(case):
    f = oracle_formula("small")
    o = _oracle(f, "f64")
    v = np.array(case["v"], np.float64)
    xs = np.ones(f.m)
    xl = np.ones(f.m)
    dv, dxs, dxl, allsat, rfired = o.compute_derivatives(v, xs, xl, 0.001)
    assert allsat == case["allsat"]
    assert rfired == 0
    if "dv_renamed" in case:
        assert dv.tolist() == [eval(e) for e in case["dv_renamed"]]  # noqa: S307 (our own fixture)
        assert dxs.tolist() == [eval(e) for e in case["dxs"]]  # noqa: S307
        assert dxl.tolist() == [eval(e) for e in case["dxl"]]  # noqa: S307
    if "after_v" in case:
        sat = o.euler_step_fixed(v, xs, xl, case["dt"], 0.001)
        assert sat == case["allsat"]
        assert v.tolist() == [eval(e) for e in case["after_v"]]  # noqa: S307
        assert xs.tolist() == [eval(e) for e in case["after_xs"]]  # noqa: S307
        assert xl.tolist() == [eval(e) for e in case["after_xl"]]  # noqa: S307


def test_kat_survey_values():
    """SURVEY.md section 4 states the f64 literals of the v = 0 KAT."""
    assert 20.0 * (1.0 + 0.001) * (0.5 - 0.25) == 5.004999999999999
    assert 5.0 * (0.5 - 0.05) == 2.25
    assert 1.0 + 0.01 * 2.25 == 1.0225


@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
def test_c_oracle_matches_numpy_golden(name, prec, mode):
    g = golden(name)
    f = oracle_formula(name)
    assert np.array_equal(g["clause_ptr"], f.clause_ptr) and np.array_equal(g["var"], f.var)
    T = np.float64 if prec == "f64" else np.float32
    o = _oracle(f, prec)
    v0 = init_voltages(int(g["seed"]), 0, int(g["B"]), f.varnum)
    assert np.array_equal(v0, g["v0"])  # C counter RNG == numpy counter RNG
    key = f"{prec}_{mode}_"
    for b in range(int(g["B"])):
        v = v0[b].astype(T)
        xs = o.init_short_term_memory()
        xl = np.ones(f.m, T)
        kw = dict(dt=0.01) if mode == "fixed" else dict(tol=1e-3)
        t, sat, _, h, rfired = o.simulate(v, xs, xl, steps=int(g["steps"]), **kw)
        assert t == g[key + "steps"][b] and sat == g[key + "sat"][b]
        assert rfired == 0
        assert np.array_equal(v.view(np.uint8), g[key + "v"][b].view(np.uint8))
        assert np.array_equal(xs.view(np.uint8), g[key + "xs"][b].view(np.uint8))
        assert np.array_equal(xl.view(np.uint8), g[key + "xl"][b].view(np.uint8))
        if mode == "adaptive":
            assert T(h) == g[key + "dt"][b]


def test_easy_is_sat_hard_is_not():
    """Outcome KATs from the fixtures' own `c NOTE` lines (easy: satisfiable, hard: not)."""
    g = golden("easy")
    assert g["f64_fixed_sat"].all() and g["f64_adaptive_sat"].all()
    from oracle import cnf_oracle as co
    from tests.common import read
    cl, varnum = co.parse_dimacs_format(read("easy"))
    name_map, ncl = co.normalize_cnf_variables(cl, varnum)
    for b in range(int(g["B"])):
        vals = co.map_values_by_indices(name_map, g["f64_fixed_v"][b] > 0)
        assert co.evaluate_cnf(vals, cl)
    h = golden("hard")
    assert not h["f64_fixed_sat"].any()


def test_inter_semantics_vs_independent_runs():
    """simulate_inter (fixed step) == lock-step of independent simulate() runs: the first sat step
    over replicas is the minimum of the per-replica sat steps, and the winner is the lowest index."""
    f = oracle_formula("easy")
    o = _oracle(f, "f64")
    B = 4
    v0 = init_voltages(42, 0, B, f.varnum)
    xs0 = np.tile(o.init_short_term_memory(), (B, 1))
    xl0 = np.ones((B, f.m))
    v, xs, xl = v0.copy(), xs0.copy(), xl0.copy()
    t, win, assign, _ = o.simulate_inter(v, xs, xl, dt=0.01, steps=5000)
    g = golden("easy")
    steps = g["f64_fixed_steps"]
    assert t == steps.min()
    assert win == int(np.argmin(steps))
    # the winner's final state equals its independent run
    assert np.array_equal(v[win], g["f64_fixed_v"][win])


def test_shared_dt_differs_from_per_replica_dt():
    """Documents the declared deviation: adaptive inter threads one dt through the replicas."""
    f = oracle_formula("rand200")
    o = _oracle(f, "f64")
    B = 3
    v0 = init_voltages(42, 0, B, f.varnum)
    xs0 = np.tile(o.init_short_term_memory(), (B, 1))
    res = []
    for shared in (True, False):
        v, xs, xl = v0.copy(), xs0.copy(), np.ones((B, f.m))
        o.simulate_inter(v, xs, xl, tol=1e-3, steps=20, shared_dt=shared)
        res.append(v)
    assert not np.array_equal(res[0], res[1])


def test_rigidity_term_never_fires_from_valid_states():
    """with v in [-1, 1] the rigidity term R is identically zero."""
    var, neg = wl.random_ksat(300, 1300, 3, 11)
    cp, v_, n_ = wl.formula_arrays(var, neg)
    o = Oracle(cp, v_, n_, 300, "f64")
    v = init_voltages(7, 0, 1, 300)[0]
    xs = o.init_short_term_memory()
    xl = np.ones(1300)
    _, _, _, _, rfired = o.simulate(v, xs, xl, dt=0.05, steps=400)
    assert rfired == 0


def test_rigidity_term_can_fire_from_out_of_range_state():
    """...but a caller-supplied v outside [-1, 1] makes it fire on the first RHS, which is why the
    GPU kernels keep the term instead of dropping it."""
    f = npo.Formula.from_clauses([[(0, False), (1, False)]], 2)
    o = Oracle(f.clause_ptr, f.var, f.neg, 2, "f64")
    # values: 1-2 = -1 (min), 1-1.5 = -0.5; C = -0.5 == value of literal 2 -> R fires
    _, _, _, _, rfired = o.compute_derivatives(np.array([2.0, 1.5]), np.array([0.5]), np.array([1.0]), 0.1)
    assert rfired == 1
    dv_np, _, _, _, rf_np = npo.compute_derivatives(f, np.array([2.0, 1.5]), np.array([0.5]), np.array([1.0]), 0.1)
    dv_c = o.compute_derivatives(np.array([2.0, 1.5]), np.array([0.5]), np.array([1.0]), 0.1)[0]
    assert rf_np == 1 and np.array_equal(dv_np, dv_c)


def test_counter_rng_three_implementations_agree():
    from oracle.oracle import lib
    seeds = [(0, 0, 0), (42, 3, 17), (2**63 + 5, 2**40, 999_999)]
    for s, r, i in seeds:
        a = lib().oc_hash3(s, r, i)
        b = int(npo.hash3(s, r, i))
        c = int(wl.hash3(s, r, i))
        assert a == b == c
    v = init_voltages(9, 5, 3, 50)
    assert np.array_equal(v, npo.init_voltages(9, 5, 3, 50))
    assert v.min() >= -1.0 and v.max() < 1.0


def test_batch_run_equals_simulate_per_replica():
    f = oracle_formula("easy")
    for prec, T in (("f64", np.float64), ("f32", np.float32)):
        o = _oracle(f, prec)
        B = 4
        v = init_voltages(42, 0, B, f.varnum).astype(T)
        xs = np.tile(o.init_short_term_memory(), (B, 1))
        xl = np.ones((B, f.m), T)
        total, sat, done, _ = o.batch_run(v, xs, xl, False, 1e-3, 0.01, 2000, 0.001, nthreads=2)
        g = golden("easy")
        assert np.array_equal(done, g[f"{prec}_fixed_steps"])
        assert np.array_equal(sat, np.where(g[f"{prec}_fixed_sat"], done - 1, -1))
        assert np.array_equal(v, g[f"{prec}_fixed_v"])
