"""The product's C++ DIMACS loader (libodesat_hip.so, cnf.rs replacement) vs the Python restatement
of cnf.rs:138-315 (oracle/cnf_oracle.py).  Host-only calls: runs on CPU."""
import numpy as np
import pytest

from oracle import cnf_oracle as co
from odesat_amd import cnf
from odesat_amd import workloads as wl
from odesat_amd._lib import OdesatError
from tests.common import FIXTURES, read


def _product(text):
    f = cnf.parse_dimacs_format(text)
    return f.clauses(), f.varnum


@pytest.mark.parametrize("name", FIXTURES)
def test_fixture_parse_matches(name):
    text = read(name)
    assert _product(text) == co.parse_dimacs_format(text)


def test_fixture_shapes():
    """Shapes stated by the fixtures' own headers (and SURVEY.md section 2 row 19)."""
    cl, n = _product(read("small"))
    assert n == 5 and [len(c) for c in cl] == [3, 4, 2]
    cl, n = _product(read("easy"))
    assert n == 100 and len(cl) == 160 and all(len(c) == 3 for c in cl)
    hard, _ = _product(read("hard"))
    diff = [i for i, (a, b) in enumerate(zip(cl, hard)) if a != b]
    assert diff == [2]  # file line 14: -30 35 -78 vs -30 35 78


EDGE_CASES = {
    "empty_line_is_empty_clause": "p cnf 3 2\n1 2 0\n\n-3 0\n",
    "no_header": "1 -2 0\n2 7 0\n",
    "comment_prefix_anywhere": "c hi\ncnf is a comment too\np cnf 4 1\n1 2 0\n",
    "crlf": "p cnf 3 2\r\n1 -3 0\r\n2 0\r\n",
    "no_trailing_newline": "p cnf 3 1\n1 2 3 0",
    "tokens_after_zero_ignored": "p cnf 3 1\n1 2 0 3 4\n",
    "clause_without_terminator": "p cnf 3 1\n1 2 3\n",
    "minus_zero_is_var_0": "p cnf 3 1\n1 -0 2 0\n",
    "plus_sign": "p cnf 3 1\n+1 -2 0\n",
    "lone_zero_line": "p cnf 2 2\n1 2 0\n0\n",
    "tabs": "p\tcnf 3 1\np cnf\t3 1\n1\t-2  3 0\n",
    "duplicate_literal": "p cnf 2 1\n1 1 -1 2 0\n",
    "second_header_wins": "p cnf 3 1\np cnf 9 1\n1 2 0\n",
    "final_cr_kept_out": "p cnf 2 1\n1 2 0\r\n",
}


@pytest.mark.parametrize("name", sorted(EDGE_CASES))
def test_edge_cases_match(name):
    text = EDGE_CASES[name]
    try:
        want = co.parse_dimacs_format(text)
    except co.DimacsError:
        with pytest.raises(OdesatError):
            _product(text)
        return
    assert _product(text) == want


@pytest.mark.parametrize("text", ["p cnf 3 1\n1 x 0\n", "p cnf\n1 0\n", "%\n0\n", "p cnf 3 1\n 1 2 0\nc\n c x\n",
                                  "p cnf 3 1\n99999999999 0\n", "p cnf -3 1\n1 0\n"])
def test_malformed_is_an_error_not_a_crash(text):
    """Where the reference panics (cnf.rs:151,160) the loader returns ODESAT_EINVAL."""
    with pytest.raises(co.DimacsError):
        co.parse_dimacs_format(text)
    with pytest.raises(OdesatError) as e:
        _product(text)
    assert e.value.code == -1


@pytest.mark.parametrize("name", FIXTURES)
def test_normalize_matches(name):
    text = read(name)
    f = cnf.parse_dimacs_format(text)
    mapping, nf = cnf.normalize_cnf_variables(f)
    cl, varnum = co.parse_dimacs_format(text)
    omap, ocl = co.normalize_cnf_variables(cl, varnum)
    assert mapping == omap
    assert nf.clauses() == ocl and nf.varnum == varnum


def test_normalize_sparse_names():
    f = cnf.parse_dimacs_format("p cnf 100 2\n7 -40 0\n-7 99 0\n")
    mapping, nf = cnf.normalize_cnf_variables(f)
    assert mapping == {7: 0, 40: 1, 99: 2}
    assert nf.clauses() == [[(0, False), (1, True)], [(0, True), (2, False)]]
    assert nf.varnum == 100


def test_evaluate_and_render():
    text = read("small")
    f = cnf.parse_dimacs_format(text)
    cl, _ = co.parse_dimacs_format(text)
    rng = np.random.default_rng(0)
    for _ in range(50):
        vals = {v: bool(rng.integers(2)) for v in (1, 2, 3, 4, 5) if rng.random() < 0.9}
        a, b = dict(vals), dict(vals)
        assert cnf.evaluate_cnf(a, f) == co.evaluate_cnf(b, cl)
        assert a == b  # missing variables inserted as false, as the reference does
    assert cnf.render_variable_map({3: True, 1: False}) == co.render_variable_map({3: True, 1: False}) == "1 0\n3 1\n"


def test_init_short_term_memory():
    f = cnf.parse_dimacs_format("p cnf 3 3\n1 2 0\n-1 2 0\n\n")
    assert cnf.init_short_term_memory(f).tolist() == [-1.0, 1.0, -1.0]


def test_generator_roundtrip_through_loader():
    var, neg = wl.random_ksat(50, 210, 3, 9)
    text = wl.to_dimacs(var, neg, 50)
    f = cnf.parse_dimacs_format(text)
    cp, v, n = f.arrays()
    assert np.array_equal(cp, np.arange(211) * 3)
    assert np.array_equal(v, var.reshape(-1)) and np.array_equal(n.astype(bool), neg.reshape(-1))
    assert co.parse_dimacs_format(text)[1] == 50


def test_generator_is_deterministic_and_distinct():
    a = wl.random_ksat(1000, 4200, 3, 1)
    b = wl.random_ksat(1000, 4200, 3, 1)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])
    s = np.sort(a[0], axis=1)
    assert not (s[:, 1:] == s[:, :-1]).any()
    assert a[0].min() >= 1 and a[0].max() <= 1000
    assert abs(a[1].mean() - 0.5) < 0.02


def test_committed_random_fixture_is_reproducible():
    var, neg = wl.random_ksat(200, 852, 3, 5)
    assert wl.to_dimacs(var, neg, 200, "random 3-SAT n=200 m=852 seed=5 (odesat_amd.workloads)") == read("rand200")
