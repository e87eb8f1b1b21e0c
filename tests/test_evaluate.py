"""Batched evaluate_cnf on the device (odesat_evaluate) against the host check
(oracle/cnf_oracle.evaluate_cnf, cnf.rs:246-264) of every replica's assignment (v > 0,
system.rs:238), on every algorithm's state layout and both precisions.  Bar: identical booleans and
the same first satisfying replica (batch's pick, main.rs:302-307)."""
import itertools

import numpy as np
import pytest

from oracle import cnf_oracle as co
from odesat_amd import _lib, cnf
from odesat_amd.system import ODESAT_STOP_EACH, Solver
from tests.common import read

pytestmark = pytest.mark.gpu


def normalized(name):
    cl, varnum = co.parse_dimacs_format(read(name))
    _, ncl = co.normalize_cnf_variables(cl, varnum)
    _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(read(name)))
    return ncl, f


def host_check(s, ncl):
    sat = []
    for r in range(s.batch):
        a = s.get_assignment(r)
        sat.append(co.evaluate_cnf({i: bool(x) for i, x in enumerate(a)}, ncl))
    first = next((r for r, x in enumerate(sat) if x), -1)
    return np.array(sat), first


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_every_assignment_of_small(prec):
    """All 2^5 assignments of the reference's tests/small.cnf, as voltages of +-0.5."""
    ncl, f = normalized("small")
    n, m = f.varnum, f.nclauses
    bits = np.array(list(itertools.product([0, 1], repeat=n)), np.float64)
    v = np.where(bits > 0, 0.5, -0.5)
    B = len(v)
    with Solver(f, B, prec) as s:
        s.set_state(v, np.ones((B, m)), np.ones((B, m)))
        sat, first = s.evaluate()
        hs, hf = host_check(s, ncl)
    assert np.array_equal(sat, hs) and first == hf
    assert sat.any() and not sat.all()


@pytest.mark.parametrize("name", ["easy", "rand200"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("alg", ["RESIDENT", "FUSED", "TWOPASS", "ONCHIP"])
def test_after_simulation_matches_host(name, prec, alg):
    ncl, f = normalized(name)
    B = 70
    with Solver(f, B, prec) as s:
        code = getattr(_lib, "ODESAT_ALG_" + alg)
        if alg == "ONCHIP" and s.algorithm != code:
            pytest.skip("not ONCHIP-eligible")
        s.set_algorithm(code)
        s.init_state(3)
        s.simulate(dt=0.1, max_steps=300, stop=ODESAT_STOP_EACH)
        sat, first = s.evaluate()
        hs, hf = host_check(s, ncl)
    assert np.array_equal(sat, hs) and first == hf


def test_unsat_formula_has_no_satisfied_replica():
    ncl, f = normalized("hard")
    with Solver(f, 40, "f32") as s:
        s.init_state(1)
        s.simulate(dt=0.1, max_steps=100, stop=ODESAT_STOP_EACH)
        sat, first = s.evaluate()
    assert not sat.any() and first == -1
