"""The discrete stochastic search (stoch.rs:20-110): the C oracle (oracle/stoch_oracle.c) against an
independent pure-Python restatement, then the GPU (odesat_amd/csrc/stoch.hip, through the C ABI)
against the oracle.  Integer work, so the bar is bit-exact: v, xl, the sat step and the steps taken,
replica by replica.  The draw is the shared counter RNG (oc_stoch_hash; declared deviation from
thread_rng), so every comparison runs the same random stream."""
import numpy as np
import pytest

from oracle.oracle import Oracle, lib as oracle_lib
from odesat_amd import cnf
from tests.common import FIXTURES, oracle_formula, read

U64 = (1 << 64) - 1


def oracle_for(name):
    f = oracle_formula(name)
    return f, Oracle(f.clause_ptr, f.var, f.neg, f.varnum, "f64")


def py_step(f, v, xl, seed, replica, step):
    """stoch.rs:26-81, restated in plain Python from the source (independent of the C oracle)."""
    n, m = f.varnum, len(f.clause_ptr) - 1
    tot, uns = [0] * n, [0] * n
    all_sat = True
    for c in range(m):
        lits = range(f.clause_ptr[c], f.clause_ptr[c + 1])
        sat = any(bool(v[f.var[s]]) ^ bool(f.neg[s]) for s in lits)
        x = int(xl[c])
        x = max(max(x - 1, 0), 1) if sat else min(x + 20, U64)
        xl[c] = x
        for s in lits:
            tot[f.var[s]] = (tot[f.var[s]] + x) & U64
            if not sat:
                uns[f.var[s]] = (uns[f.var[s]] + x) & U64
        all_sat = all_sat and sat
    for i in range(n):
        if tot[i] == 0:
            raise ValueError("gen_range(1..=0) panics")
        h = oracle_lib().oc_stoch_hash(seed, replica, step, i)
        if 1 + ((h * tot[i]) >> 64) <= uns[i]:
            v[i] = 1 - v[i]
    return all_sat


# --------------------------------------------------------------------------------------- CPU
@pytest.mark.parametrize("name", ["easy", "rand200"])
def test_oracle_matches_python_restatement(name):
    f, o = oracle_for(name)
    v1 = np.zeros(o.n, np.uint8)
    xl1 = np.ones(o.m, np.uint64)
    v2, xl2 = [0] * o.n, [1] * o.m
    for k in range(25):
        a = o.stoch_step(v1, xl1, 7, 3, k)
        b = py_step(f, v2, xl2, 7, 3, k)
        assert a == b
        assert v1.tolist() == v2 and xl1.tolist() == xl2


def test_oracle_saturation_and_floor():
    f, o = oracle_for("small")
    v = np.zeros(o.n, np.uint8)
    xl = np.array([U64 - 5, 0, 1][: o.m], np.uint64)
    v2, xl2 = v.tolist(), [int(x) for x in xl]
    try:
        a = o.stoch_step(v, xl, 1, 0, 0)
    except ValueError:
        with pytest.raises(ValueError):
            py_step(f, v2, xl2, 1, 0, 0)
        return
    assert a == py_step(f, v2, xl2, 1, 0, 0)
    assert xl.tolist() == xl2
    assert all(int(x) >= 1 for x in xl)


def test_oracle_panics_on_a_variable_in_no_clause():
    o = Oracle(np.array([0, 2]), np.array([0, 1]), np.array([0, 1]), 3, "f64")  # variable 2 unused
    with pytest.raises(ValueError):
        o.stoch_step(np.zeros(3, np.uint8), np.ones(1, np.uint64), 0, 0, 0)


def test_oracle_search_stops_on_the_satisfying_step():
    f, o = oracle_for("easy")
    v = np.zeros(o.n, np.uint8)
    xl = np.ones(o.m, np.uint64)
    t, sat = o.stoch_search(v, xl, 11, 0, 20000)
    assert sat and 0 < t < 20000
    assign = {i: bool(v[i]) for i in range(o.n)}
    from oracle import cnf_oracle as co
    cl, varnum = co.parse_dimacs_format(read("easy"))
    _, ncl = co.normalize_cnf_variables(cl, varnum)
    assert co.evaluate_cnf(assign, ncl)


# --------------------------------------------------------------------------------------- GPU
def product_formula(name):
    _, g = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(read(name)))
    return g


# the two device paths: the one-wave-per-replica LDS kernel (default for formulas that fit) and
# the three-kernel HBM path (knob STOCH_WAVE = 0, the path large formulas take)
PATHS = {"wave": {}, "hbm": {"STOCH_WAVE": "0"}}


def set_path(xp, path):
    xp.delete("STOCH_WAVE")
    xp.delete("STOCH_WPW")
    for k, v in PATHS.get(path, {}).items():
        xp.set(k, v)
    if path.startswith("wpw"):
        xp.set("STOCH_WPW", path[3:])


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "hbm"])
@pytest.mark.parametrize("name", ["easy", "hard", "rand200"])
@pytest.mark.parametrize("B", [1, 37, 128])
def test_search_bitexact(name, B, path, xp):
    from odesat_amd.stoch import StochSearch
    set_path(xp, path)
    _, o = oracle_for(name)
    steps, seed = 300, 5
    with StochSearch(product_formula(name), B) as s:
        assert (s.wave_width > 0) == (path == "wave")
        r = s.search(seed, steps, replica0=100)
        gv, gxl = s.get_state()
    for b in range(B):
        v = np.zeros(o.n, np.uint8)
        xl = np.ones(o.m, np.uint64)
        t, sat = o.stoch_search(v, xl, seed, 100 + b, steps)
        assert np.array_equal(gv[b], v.astype(bool)) and np.array_equal(gxl[b], xl)
        assert r["steps_done"][b] == t
        assert r["first_sat_step"][b] == (t - 1 if sat else -1)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "hbm"])
def test_stop_none_and_chunked_calls(path, xp):
    """STOP_NONE keeps stepping after a satisfying step; two calls continue one RNG stream."""
    from odesat_amd.stoch import ODESAT_STOP_NONE, StochSearch
    set_path(xp, path)
    _, o = oracle_for("easy")
    with StochSearch(product_formula("easy"), 4) as s:
        s.search(9, 150, stop=ODESAT_STOP_NONE)
        s.search(9, 250, stop=ODESAT_STOP_NONE)
        gv, gxl = s.get_state()
    for b in range(4):
        v = np.zeros(o.n, np.uint8)
        xl = np.ones(o.m, np.uint64)
        for k in range(400):
            o.stoch_step(v, xl, 9, b, k)
        assert np.array_equal(gv[b], v.astype(bool)) and np.array_equal(gxl[b], xl)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "hbm"])
def test_set_state_roundtrip_and_errors(path, xp):
    from odesat_amd.stoch import StochSearch
    set_path(xp, path)
    _, o = oracle_for("rand200")
    rng = np.random.default_rng(0)
    v = rng.integers(0, 2, (3, o.n)).astype(np.uint8)
    xl = rng.integers(1, 1 << 40, (3, o.m)).astype(np.uint64)
    with StochSearch(product_formula("rand200"), 5) as s:
        s.set_state(v, xl, r0=1)
        gv, gxl = s.get_state(1, 3)
        assert np.array_equal(gv, v.astype(bool)) and np.array_equal(gxl, xl)
        r = s.search(4, 50, replica0=0)
        gv, gxl = s.get_state(1, 3)
    for b in range(3):
        vv, xx = v[b].copy(), xl[b].copy()
        t, sat = o.stoch_search(vv, xx, 4, 1 + b, 50)
        assert np.array_equal(gv[b], vv.astype(bool)) and np.array_equal(gxl[b], xx)
        assert r["steps_done"][1 + b] == t
    unused = cnf.CNFFormula.from_arrays([0, 2], [0, 1], [0, 1], varnum=3)
    from odesat_amd._lib import OdesatError
    with pytest.raises(OdesatError):
        StochSearch(unused, 1)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wpw1", "wpw2", "wpw4", "wpw8"])
def test_wave_workgroup_widths(path, xp):
    """WPW replicas share a workgroup's LDS topology; 37 replicas leave the last workgroup ragged."""
    from odesat_amd.stoch import StochSearch
    set_path(xp, path)
    _, o = oracle_for("rand200")
    B, steps, seed = 37, 200, 11
    with StochSearch(product_formula("rand200"), B) as s:
        assert s.wave_width == int(path[3:])
        r = s.search(seed, steps, poll_interval=17)
        gv, gxl = s.get_state()
    for b in range(B):
        v = np.zeros(o.n, np.uint8)
        xl = np.ones(o.m, np.uint64)
        t, sat = o.stoch_search(v, xl, seed, b, steps)
        assert np.array_equal(gv[b], v.astype(bool)) and np.array_equal(gxl[b], xl)
        assert r["steps_done"][b] == t
        assert r["first_sat_step"][b] == (t - 1 if sat else -1)


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "hbm"])
def test_saturating_memories(path, xp):
    """xl at the top of u64: +20 saturates (stoch.rs:50) and the u64 sums wrap, on both paths."""
    from odesat_amd.stoch import ODESAT_STOP_NONE, StochSearch
    set_path(xp, path)
    _, o = oracle_for("easy")
    rng = np.random.default_rng(3)
    B = 3
    v = rng.integers(0, 2, (B, o.n)).astype(np.uint8)
    xl = (np.uint64(U64) - rng.integers(0, 40, (B, o.m)).astype(np.uint64)).astype(np.uint64)
    with StochSearch(product_formula("easy"), B) as s:
        s.set_state(v, xl)
        s.search(2, 60, stop=ODESAT_STOP_NONE)
        gv, gxl = s.get_state()
    for b in range(B):
        vv, xx = v[b].copy(), xl[b].copy()
        for k in range(60):
            o.stoch_step(vv, xx, 2, b, k)
        assert np.array_equal(gv[b], vv.astype(bool)) and np.array_equal(gxl[b], xx)


@pytest.mark.gpu
def test_large_formula_takes_the_hbm_path(xp):
    from odesat_amd.stoch import StochSearch
    set_path(xp, "wave")
    n, m = 10_000, 42_000  # config 2's size: 9m + n bytes of state per replica exceed the LDS
    var = np.arange(3 * m) % n
    f = cnf.CNFFormula.from_arrays(np.arange(0, 3 * m + 1, 3), var, var % 2, varnum=n)
    with StochSearch(f, 8) as s:
        assert s.wave_width == 0
    with StochSearch(product_formula("rand200"), 1024) as s:
        assert s.wave_width >= 4  # 1024 replicas: four or more per workgroup still fill 256 CUs


def mixed_width_formula():
    """rand200 with every 5th clause cut to two literals and every 7th widened to four: the wave
    kernel's general (clause_ptr) form rather than its three-literal records."""
    f = oracle_formula("rand200")
    n = f.varnum
    cp, var, neg = [0], [], []
    for c in range(len(f.clause_ptr) - 1):
        lits = [(int(f.var[s]), int(f.neg[s])) for s in range(f.clause_ptr[c], f.clause_ptr[c + 1])]
        if c % 5 == 0:
            lits = lits[:2]
        if c % 7 == 0:
            extra = (lits[0][0] + 1) % n
            if all(x != extra for x, _ in lits):
                lits.append((extra, c % 2))
        var += [x for x, _ in lits]
        neg += [g for _, g in lits]
        cp.append(len(var))
    assert len(set(var)) == n
    return np.array(cp), np.array(var), np.array(neg, np.uint8), n


@pytest.mark.gpu
@pytest.mark.parametrize("path", ["wave", "hbm"])
def test_mixed_clause_widths(path, xp):
    from odesat_amd.stoch import StochSearch
    set_path(xp, path)
    cp, var, neg, n = mixed_width_formula()
    o = Oracle(cp, var, neg, n, "f64")
    B, steps, seed = 9, 250, 21
    with StochSearch(cnf.CNFFormula.from_arrays(cp, var, neg, varnum=n), B) as s:
        assert (s.wave_width > 0) == (path == "wave")
        r = s.search(seed, steps)
        gv, gxl = s.get_state()
    for b in range(B):
        v = np.zeros(n, np.uint8)
        xl = np.ones(o.m, np.uint64)
        t, sat = o.stoch_search(v, xl, seed, b, steps)
        assert np.array_equal(gv[b], v.astype(bool)) and np.array_equal(gxl[b], xl)
        assert r["steps_done"][b] == t
