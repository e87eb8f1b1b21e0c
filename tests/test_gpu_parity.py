"""GPU parity: the HIP integrator (through the C ABI) against the CPU oracle, on the same seeded
inputs.  Bar: BIT-EXACT states (v, xs, xl), sat steps and assignments, in f64 (the reference's
precision) and in f32 (vs the oracle's f32 restatement with the same operation order).  At
BASELINE.json's full size (n=10k, m=42k, B=1024) a subset of replicas is checked bit for bit and the
rest through size-independent properties.  f32-vs-f64 is compared with a stated tolerance."""
import numpy as np
import pytest

from oracle.oracle import Oracle, init_voltages
from odesat_amd import cnf
from odesat_amd import workloads as wl
from odesat_amd.system import (ODESAT_STOP_ANY, ODESAT_STOP_EACH, ODESAT_STOP_NONE, Solver, State,
                               compute_derivatives, euler_step, euler_step_fixed, simulate, simulate_inter)
from tests.common import FIXTURES, golden, oracle_formula, read

pytestmark = pytest.mark.gpu

T_OF = {"f64": np.float64, "f32": np.float32}


def same(a, b):
    """Bit-equal, except that NaN payloads may differ between the CPU and the GPU."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a[~na].view(np.uint64), b[~nb].view(np.uint64))


def product_formula(name):
    _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(read(name)))
    return f


def oracle_for(name, prec):
    f = oracle_formula(name)
    return f, Oracle(f.clause_ptr, f.var, f.neg, f.varnum, prec)


def init_states(o, B, seed=42, T=np.float64):
    v = init_voltages(seed, 0, B, o.n).astype(T)
    xs = np.tile(o.init_short_term_memory(), (B, 1)).astype(T)
    xl = np.ones((B, o.m), T)
    return v, xs, xl


# --------------------------------------------------------------------------- single RHS / step ---
@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("B", [1, 3, 64, 100])
def test_compute_derivatives_bitexact(name, prec, B):
    f, o = oracle_for(name, prec)
    T = T_OF[prec]
    v, xs, xl = init_states(o, B, T=T)
    with Solver(product_formula(name), B, prec) as s:
        s.init_state(42)
        gv, gxs, gxl = s.get_state()
        assert same(gv, v) and same(gxs, xs) and same(gxl, xl)  # device init == host oracle init
        dv, dxs, dxl, allsat = s.compute_derivatives(0.001)
    for b in range(B):
        odv, odxs, odxl, osat, _ = o.compute_derivatives(v[b], xs[b], xl[b], T(0.001))
        assert same(dv[b], odv) and same(dxs[b], odxs) and same(dxl[b], odxl)
        assert allsat[b] == osat


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_hand_kat_on_gpu(prec):
    import json
    import os
    from tests.common import GOLDEN
    cases = json.load(open(os.path.join(GOLDEN, "kat_small.json")))["cases"]
    T = T_OF[prec]
    f = product_formula("small")
    for case in cases:
        y = State(np.array(case["v"]), np.ones(3), np.ones(3))
        dy, allsat = compute_derivatives(y, f, 0.001, dtype=prec)
        assert allsat == case["allsat"]
        if "dv_renamed" in case and prec == "f64":
            assert dy.v.tolist() == [eval(e) for e in case["dv_renamed"]]  # noqa: S307
            assert dy.xs.tolist() == [eval(e) for e in case["dxs"]]  # noqa: S307
            assert dy.xl.tolist() == [eval(e) for e in case["dxl"]]  # noqa: S307
        if "after_v" in case:
            sat = euler_step_fixed(y, f, case["dt"], 0.001, dtype=prec)
            assert sat == case["allsat"]
            want = [T(eval(e)) for e in case["after_v"]]  # noqa: S307
            if prec == "f64":
                assert y.v.tolist() == want
                assert y.xs.tolist() == [eval(e) for e in case["after_xs"]]  # noqa: S307
                assert y.xl.tolist() == [eval(e) for e in case["after_xl"]]  # noqa: S307


@pytest.mark.parametrize("name", ["small", "easy", "rand200"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_single_steps_bitexact(name, prec):
    f, o = oracle_for(name, prec)
    T = T_OF[prec]
    B = 5
    v, xs, xl = init_states(o, B, T=T)
    with Solver(product_formula(name), B, prec) as s:
        s.init_state(42)
        for k in range(3):  # fixed
            allsat = s.euler_step_fixed(0.01, 0.001)
            for b in range(B):
                assert allsat[b] == o.euler_step_fixed(v[b], xs[b], xl[b], T(0.01), T(0.001))
        gv, gxs, gxl = s.get_state()
        assert same(gv, v) and same(gxs, xs) and same(gxl, xl)
        dts = np.full(B, 0.01)
        odt = [T(0.01)] * B
        for k in range(3):  # adaptive, per-replica dt
            allsat, dts = s.euler_step(1e-3, dts, 0.001)
            for b in range(B):
                sat, odt[b] = o.euler_step(v[b], xs[b], xl[b], T(1e-3), odt[b], T(0.001))
                assert allsat[b] == sat
                assert T(dts[b]) == T(odt[b])
        gv, gxs, gxl = s.get_state()
        assert same(gv, v) and same(gxs, xs) and same(gxl, xl)


def test_reference_shaped_functions():
    f = product_formula("easy")
    _, o = oracle_for("easy", "f64")
    v, xs, xl = init_states(o, 1)
    y = State(v[0].copy(), xs[0].copy(), xl[0].copy())
    sat, h = euler_step(y, f, 1e-3, 0.01, 0.001)
    osat, oh = o.euler_step(v[0], xs[0], xl[0], 1e-3, 0.01, 0.001)
    assert sat == osat and h == oh and same(y.v, v[0]) and same(y.xl, xl[0])


# ---------------------------------------------------------------------- whole trajectories ---
@pytest.mark.parametrize("name", FIXTURES)
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
def test_batch_trajectories_match_golden(name, prec, mode):
    """odesat_simulate(STOP_EACH) == the reference's sequential restart loop (main.rs:278-308):
    every replica runs to its own allsat (frozen after) or to the step limit, bit for bit."""
    g = golden(name)
    B, steps = int(g["B"]), int(g["steps"])
    with Solver(product_formula(name), B, prec) as s:
        s.init_state(int(g["seed"]))
        r = s.simulate(adaptive=mode == "adaptive", dt=0.01, tol=1e-3, max_steps=steps, stop=ODESAT_STOP_EACH,
                       poll_interval=7)
        v, xs, xl = s.get_state()
    key = f"{prec}_{mode}_"
    assert np.array_equal(r["steps_done"], g[key + "steps"])
    assert np.array_equal(r["first_sat_step"] >= 0, g[key + "sat"])
    assert np.array_equal(r["first_sat_step"][g[key + "sat"]], g[key + "steps"][g[key + "sat"]] - 1)
    assert same(v, g[key + "v"]) and same(xs, g[key + "xs"]) and same(xl, g[key + "xl"])
    if mode == "adaptive":
        assert np.array_equal(r["dt"].astype(T_OF[prec]), g[key + "dt"].astype(T_OF[prec]))


def test_easy_solves_and_evaluates():
    """End to end on the reference's SAT fixture: the GPU assignment satisfies the ORIGINAL formula."""
    text = read("easy")
    f = cnf.parse_dimacs_format(text)
    mapping, nf = cnf.normalize_cnf_variables(f)
    for prec in ("f64", "f32"):
        with Solver(nf, 8, prec) as s:
            s.init_state(7)
            r = s.simulate(dt=0.1, max_steps=5000, stop=ODESAT_STOP_EACH)
            winners = np.flatnonzero(r["first_sat_step"] >= 0)
            assert len(winners) > 0
            a = s.get_assignment(int(winners[0]))
        vals = cnf.map_values_by_indices(mapping, a)
        assert cnf.evaluate_cnf(vals, f)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_inter_fixed_matches_oracle(prec):
    """STOP_ANY == simulate_inter (fixed step): same stop step, winner and EVERY replica's state."""
    f, o = oracle_for("easy", prec)
    T = T_OF[prec]
    B = 6
    v, xs, xl = init_states(o, B, T=T)
    t, win, assign, _ = o.simulate_inter(v, xs, xl, dt=T(0.01), steps=4000)
    with Solver(product_formula("easy"), B, prec) as s:
        s.init_state(42)
        r = s.simulate(dt=0.01, max_steps=4000, stop=ODESAT_STOP_ANY, poll_interval=16)
        gv, gxs, gxl = s.get_state()
    sat = np.flatnonzero(r["first_sat_step"] >= 0)
    assert len(sat) and int(sat[0]) == win and r["first_sat_step"][win] == t - 1
    assert np.all(r["steps_done"] == t)
    assert same(gv, v) and same(gxs, xs) and same(gxl, xl)


def test_inter_adaptive_per_replica_dt_matches_oracle():
    """Declared deviation: adaptive STOP_ANY uses per-replica dt (oracle shared_dt=False)."""
    f, o = oracle_for("easy", "f64")
    B = 4
    v, xs, xl = init_states(o, B)
    t, win, _, dts = o.simulate_inter(v, xs, xl, tol=1e-3, steps=3000, shared_dt=False)
    with Solver(product_formula("easy"), B, "f64") as s:
        s.init_state(42)
        r = s.simulate(adaptive=True, tol=1e-3, max_steps=3000, stop=ODESAT_STOP_ANY)
        gv, gxs, gxl = s.get_state()
    assert int(np.flatnonzero(r["first_sat_step"] >= 0)[0]) == win
    assert same(gv, v) and same(gxs, xs) and same(gxl, xl) and same(r["dt"], dts)


def test_simulate_inter_function():
    f = product_formula("easy")
    _, o = oracle_for("easy", "f64")
    v, xs, xl = init_states(o, 3)
    states = [State(v[b].copy(), xs[b].copy(), xl[b].copy()) for b in range(3)]
    a = simulate_inter(states, f, step_size=0.01, steps=4000)
    t, win, assign, _ = o.simulate_inter(v, xs, xl, dt=0.01, steps=4000)
    assert np.array_equal(a, assign.astype(bool))
    y = State(v[0].copy(), xs[0].copy(), xl[0].copy())
    a1 = simulate(y, f, step_size=0.01, steps=50)
    assert a1.dtype == bool and a1.shape == (f.varnum,)


# ---------------------------------------------------------------------- edge cases ---------
EDGE = {
    "empty_clause": "p cnf 3 3\n1 -2 0\n\n2 3 0\n",
    "unit_clauses_inf": "p cnf 3 4\n1 0\n-1 0\n2 -3 0\n3 0\n",
    "duplicate_var_in_clause": "p cnf 3 2\n1 1 -2 0\n-1 2 2 3 0\n",
    "unused_variables": "p cnf 8 2\n1 -2 0\n2 3 0\n",
    "wide_clauses": "p cnf 7 3\n1 2 3 4 5 6 7 0\n-1 -2 -3 -4 -5 0\n6 -7 0\n",
    "all_positive": "p cnf 3 2\n1 2 3 0\n1 -2 3 0\n",
}


@pytest.mark.parametrize("name", sorted(EDGE))
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("B", [2, 70])
def test_edge_formulas(name, prec, B):
    text = EDGE[name]
    _, nf = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(text))
    cp, var, neg = nf.arrays()
    o = Oracle(cp, var, neg, nf.varnum, prec)
    T = T_OF[prec]
    v, xs, xl = init_states(o, B, seed=3, T=T)
    for b in range(B):
        o.simulate(v[b], xs[b], xl[b], dt=T(0.05), steps=40, zeta=T(0.01))
    with Solver(nf, B, prec) as s:
        s.init_state(3)
        s.simulate(dt=0.05, zeta=0.01, max_steps=40, stop=ODESAT_STOP_EACH)
        gv, gxs, gxl = s.get_state()
    assert same(gv, v) and same(gxs, xs) and same(gxl, xl)


@pytest.mark.parametrize("prec", ["f64", "f32"])
def test_out_of_range_initial_state_rigidity_term(prec):
    """v outside [-1, 1] makes the rigidity term fire (R != 0) on the first RHS; kept bit-exact."""
    _, nf = cnf.normalize_cnf_variables(cnf.parse_dimacs_format("p cnf 3 2\n1 2 0\n-2 3 0\n"))
    cp, var, neg = nf.arrays()
    o = Oracle(cp, var, neg, 3, prec)
    T = T_OF[prec]
    v = np.array([[2.0, 1.5, -3.0]], T)
    xs = np.array([[0.5, 0.25]], T)
    xl = np.array([[1.0, 3.0]], T)
    odv, odxs, odxl, _, rf = o.compute_derivatives(v[0], xs[0], xl[0], T(0.1))
    assert rf > 0
    with Solver(nf, 1, prec) as s:
        s.set_state(v, xs, xl)
        dv, dxs, dxl, _ = s.compute_derivatives(0.1)
    assert same(dv[0], odv) and same(dxs[0], odxs) and same(dxl[0], odxl)


def test_set_state_partial_range_and_readback():
    f = product_formula("rand200")
    rng = np.random.default_rng(1)
    with Solver(f, 130, "f64") as s:
        s.init_state(5)
        v0, xs0, xl0 = s.get_state()
        nv = rng.uniform(-1, 1, (7, f.varnum))
        s.set_state(nv, xs0[60:67], xl0[60:67], r0=60)
        v1, _, _ = s.get_state()
    assert same(v1[60:67], nv) and same(v1[:60], v0[:60]) and same(v1[67:], v0[67:])


def test_chunking_does_not_change_results():
    f = product_formula("rand200")
    out = []
    for chunk in (0, 64, 128):
        with Solver(f, 256, "f32") as s:
            s.set_chunk_replicas(chunk)
            s.init_state(11)
            s.simulate(dt=0.02, max_steps=30, stop=ODESAT_STOP_NONE)
            out.append(s.get_state())
    for o_ in out[1:]:
        for a, b in zip(out[0], o_):
            assert same(a, b)


# ------------------------------------------------------------------------ f32 vs f64 ---------
def test_f32_tracks_f64_on_short_horizon():
    """Tolerance (stated): after 20 fixed steps of dt=0.01 from identical f32-representable
    initial states, |v32 - v64| <= 1e-4 and |xl32 - xl64| <= 1e-4 * xl64 elementwise."""
    f = product_formula("rand200")
    res = {}
    for prec in ("f32", "f64"):
        with Solver(f, 16, prec) as s:
            s.init_state(2)
            v, xs, xl = s.get_state()
            s.set_state(v.astype(np.float32).astype(np.float64), xs, xl)
            s.simulate(dt=0.01, max_steps=20, stop=ODESAT_STOP_NONE)
            res[prec] = s.get_state()
    v32, xs32, xl32 = res["f32"]
    v64, xs64, xl64 = res["f64"]
    assert np.max(np.abs(v32 - v64)) <= 1e-4
    assert np.max(np.abs(xs32 - xs64)) <= 1e-4
    assert np.all(np.abs(xl32 - xl64) <= 1e-4 * xl64)


# ---------------------------------------------------------------- full size (BASELINE config 2) ---
@pytest.mark.parametrize("B,pair_off", [(1024, None), (1024, "0"), (256, None)])
def test_config2_full_size_subset_bitexact_and_properties(xp, B, pair_off):
    """n=10k, m=42k, B=1024 f32 for 12 steps: replicas {0, 517, 1023} bit-exact vs the oracle's f32
    restatement; every replica: v in [-1,1], xs in [eps, 1-eps], xl in [1, 1e4 m], finite.  The
    solver's wave-paired tiles (k_onchip<90, 1>) and the other pair offset (91 tiles: k_onchip<92, 0>).
    B = 256: BASELINE configs[1]'s own batch (one replica per CU, one round of workgroups), replicas
    {0, 127, 255}."""
    if pair_off is not None:
        xp.set("PAIR_OFF", pair_off)
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    o = Oracle(cp, v_, n_, c["n"], "f32")
    K = 12
    with Solver(f, B, "f32") as s:
        assert s.step_kernel(False) == "k_onchip"
        s.init_state(42)
        r = s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE)
        assert r["steps_run"] == K and np.all(r["steps_done"] == K)
        pick = [0, 517, 1023] if B == 1024 else [0, 127, 255]
        states = {b: s.get_state(b, 1) for b in pick}
        v, xs, xl = s.get_state()
    assert np.isfinite(v).all() and np.isfinite(xs).all() and np.isfinite(xl).all()
    assert v.min() >= -1 and v.max() <= 1
    eps = np.float32(0.001)
    assert xs.min() >= eps and xs.max() <= np.float32(1) - eps
    assert xl.min() >= 1 and xl.max() <= np.float32(1e4) * np.float32(c["m"])
    for b in pick:
        ov = init_voltages(42, b, 1, c["n"])[0].astype(np.float32)
        oxs = o.init_short_term_memory()
        oxl = np.ones(c["m"], np.float32)
        o.simulate(ov, oxs, oxl, dt=np.float32(0.01), steps=K, zeta=np.float32(0.001))
        gv, gxs, gxl = states[b]
        assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl)


def test_schedules_identical():
    """Step-major and chunk-major schedules give bit-identical states (replicas are independent)."""
    from odesat_amd import _lib
    f = product_formula("rand200")
    out = []
    for sched, chunk in ((_lib.ODESAT_SCHED_STEP_MAJOR, 64), (_lib.ODESAT_SCHED_CHUNK_MAJOR, 64),
                         (_lib.ODESAT_SCHED_CHUNK_MAJOR, 128), (_lib.ODESAT_SCHED_AUTO, 0)):
        for adaptive in (False, True):
            with Solver(f, 200, "f32") as s:
                s.set_chunk_replicas(chunk)
                s.set_schedule(sched)
                s.init_state(13)
                r = s.simulate(adaptive=adaptive, dt=0.05, max_steps=60, stop=ODESAT_STOP_EACH, poll_interval=5)
                out.append((adaptive, r["first_sat_step"], r["steps_done"], s.get_state()))
    base = {False: out[0], True: out[1]}
    for adaptive, sat, done, st in out:
        b = base[adaptive]
        assert np.array_equal(sat, b[1]) and np.array_equal(done, b[2])
        for x, y in zip(st, b[3]):
            assert same(x, y)


@pytest.mark.parametrize("name", ["rand200", "small"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("B", [3, 64, 130])
def test_algorithms_identical(name, prec, B, xp):
    """FUSED (variable-major recompute) and TWOPASS (contribution buffer) give bit-identical
    trajectories, including replicas frozen at different steps (STOP_EACH) and adaptive steps."""
    from odesat_amd import _lib
    f = product_formula(name)
    with Solver(f, B, prec) as s:
        default = s.algorithm
    # these formulas are small: RESIDENT as k_wave (one wave per replica, variable fold)
    assert default == _lib.ODESAT_ALG_RESIDENT
    # k_wave, the tile kernels (WAVE knob 0: RESIDENT, and ONCHIP for f32 3-SAT), FUSED, TWOPASS
    algs = [(_lib.ODESAT_ALG_RESIDENT, "1"), (_lib.ODESAT_ALG_RESIDENT, "0"), (_lib.ODESAT_ALG_FUSED, "1"),
            (_lib.ODESAT_ALG_TWOPASS, "1")]
    if prec == "f32" and name == "rand200":
        algs.append((_lib.ODESAT_ALG_ONCHIP, "0"))
    for adaptive in (False, True):
        out = []
        for alg, wave in algs:
            xp.set("WAVE", wave)
            xp.set("RES_NARROW", "0" if alg == _lib.ODESAT_ALG_ONCHIP else "1")  # ONCHIP: 512-lane tiles
            with Solver(f, B, prec) as s:
                s.set_algorithm(alg)
                s.init_state(21)
                r = s.simulate(adaptive=adaptive, dt=0.05, max_steps=80, stop=ODESAT_STOP_EACH, poll_interval=3)
                out.append((r["first_sat_step"], r["steps_done"], r["dt"], s.get_state()))
        xp.restore()
        for o in out[1:]:
            assert np.array_equal(out[0][0], o[0]) and np.array_equal(out[0][1], o[1])
            assert same(out[0][2], o[2])
            for x, y in zip(out[0][3], o[3]):
                assert same(x, y)


def _run_layout(xp, f, B, prec, width, **kw):
    from odesat_amd import _lib
    if width is None:
        xp.delete("GROUP_WIDTH")
    else:
        xp.set("GROUP_WIDTH", str(width))
    with Solver(f, B, prec) as s:
        alg, w = s.algorithm, s.group_width
        s.init_state(5)
        r = s.simulate(**kw)
        st = s.get_state()
    xp.delete("GROUP_WIDTH")
    return alg, w, r, st


@pytest.mark.parametrize("name", ["rand200", "small", "hard"])
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("width", [1, 2, 4, 8, 16, 32])
@pytest.mark.parametrize("mode", ["fixed-each", "fixed-any", "fixed-none", "adaptive-each", "adaptive-any"])
def test_resident_widths_match_fused_w64(xp, name, prec, width, mode):
    """RESIDENT with R = 1 .. 32 replicas per workgroup (LDS-resident voltages, tiled clause pass +
    ordered fold) == FUSED at group width 64: every stop policy, fixed and adaptive steps."""
    from odesat_amd import _lib
    f = product_formula(name)
    adaptive = mode.startswith("adaptive")
    stop = {"each": ODESAT_STOP_EACH, "any": ODESAT_STOP_ANY, "none": ODESAT_STOP_NONE}[mode.split("-")[1]]
    kw = dict(adaptive=adaptive, dt=0.05, tol=1e-3, max_steps=150, stop=stop, poll_interval=4)
    B = 37
    a1, w1, r1, s1 = _run_layout(xp, f, B, prec, width, **kw)
    a2, w2, r2, s2 = _run_layout(xp, f, B, prec, 64, **kw)
    # f32 3-SAT at R = 1: ONCHIP, unless the tile chain is narrow enough for one-wave tiles
    assert w1 == width and a1 in (_lib.ODESAT_ALG_RESIDENT, _lib.ODESAT_ALG_ONCHIP)
    assert (a2, w2) == (_lib.ODESAT_ALG_FUSED, 64)
    assert np.array_equal(r1["first_sat_step"], r2["first_sat_step"])
    assert np.array_equal(r1["steps_done"], r2["steps_done"]) and r1["steps_run"] == r2["steps_run"]
    assert same(r1["dt"], r2["dt"])
    for x, y in zip(s1, s2):
        assert same(x, y)


def test_small_instance_width_config3(xp):
    """Config 3 (n = 250): by default k_wave (one replica per wave); with the tile kernel the solver
    packs R replicas per workgroup (the largest R that still gives every CU a workgroup): B = 1024
    -> R = 4, B = 4096 -> R = 16.  Every trajectory equals FUSED's bit for bit on a replica subset."""
    from odesat_amd import _lib
    c = wl.CONFIGS["config3"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    for B, R, wave in ((1024, 1, "1"), (1024, 4, "0"), (4096, 16, "0")):
        xp.set("WAVE", wave)  # 1: k_wave (one replica per wave); 0: the tile kernel at width R
        with Solver(f, B, "f32") as s:
            xp.delete("WAVE")
            assert (s.algorithm, s.group_width) == (_lib.ODESAT_ALG_RESIDENT, R)
            s.init_state(42)
            r1 = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=40, stop=ODESAT_STOP_EACH, poll_interval=8)
            st1 = s.get_state(0, 70)
        with Solver(f, B, "f32") as s:
            s.set_algorithm(_lib.ODESAT_ALG_FUSED)
            s.init_state(42)
            r2 = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=40, stop=ODESAT_STOP_EACH, poll_interval=8)
            st2 = s.get_state(0, 70)
        assert np.array_equal(r1["first_sat_step"], r2["first_sat_step"]) and same(r1["dt"], r2["dt"])
        for x, y in zip(st1, st2):
            assert same(x, y)


def test_default_layout_is_resident_for_config2():
    from odesat_amd import _lib
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    # f32: the whole replica state fits on one CU (ONCHIP); f64: v and dv (160,000 B) fit in LDS
    # (RESIDENT; adaptive steps keep their full-step clone in HBM)
    for prec, alg in (("f32", _lib.ODESAT_ALG_ONCHIP), ("f64", _lib.ODESAT_ALG_RESIDENT)):
        with Solver(f, 1024, prec) as s:
            assert s.algorithm == alg and s.group_width == 1
            assert s.step_kernel(True) == ("k_onchip" if prec == "f32" else "k_resident")


def test_frozen_replicas_keep_state_across_buffer_flips():
    """A replica frozen by STOP_EACH keeps its exact state while the rest of its group steps on."""
    f = product_formula("easy")
    _, o = oracle_for("easy", "f64")
    B = 64
    with Solver(f, B, "f64") as s:
        s.init_state(42)
        r = s.simulate(dt=0.1, max_steps=3000, stop=ODESAT_STOP_EACH, poll_interval=1000)
        v, xs, xl = s.get_state()
    v0, xs0, xl0 = init_states(o, B)
    for b in range(0, B, 9):
        t, sat, _, _, _ = o.simulate(v0[b], xs0[b], xl0[b], dt=0.1, steps=3000)
        assert t == r["steps_done"][b] and sat == (r["first_sat_step"][b] >= 0)
        assert same(v[b], v0[b]) and same(xs[b], xs0[b]) and same(xl[b], xl0[b])


# ------------------------------------------------------------------ ONCHIP (onchip.hip) --------
def _instance(n, m, seed):
    var, neg = wl.random_ksat(n, m, 3, seed)
    cp, v_, n_ = wl.formula_arrays(var, neg)
    return cnf.CNFFormula.from_arrays(cp, v_, n_, n), (cp, v_, n_)


@pytest.mark.parametrize("stop", ["each", "any", "none"])
@pytest.mark.parametrize("pair_off", [None, "0", "1"])
def test_onchip_lds_tiles_match_resident_and_oracle(stop, xp, pair_off):
    """n=6000, m=33000 (ratio 5.5): 116 tiles, so ONCHIP keeps 96 tiles' memories in VGPRs and 20
    in LDS.  ONCHIP == RESIDENT (HBM-streamed memories) bit for bit on every stop policy, and
    replica 0 == the oracle's f32 restatement -- with the wave-paired tiles at either pair offset
    (ODESAT_PAIR_OFF; None = the solver's choice)."""
    if pair_off is not None:
        xp.set("PAIR_OFF", pair_off)
    from odesat_amd import _lib
    f, (cp, v_, n_) = _instance(6000, 33000, 5)
    pol = {"each": ODESAT_STOP_EACH, "any": ODESAT_STOP_ANY, "none": ODESAT_STOP_NONE}[stop]
    B, K = 6, 25
    out = []
    for alg in (_lib.ODESAT_ALG_ONCHIP, _lib.ODESAT_ALG_RESIDENT):
        with Solver(f, B, "f32") as s:
            s.set_algorithm(alg)
            s.init_state(9)
            r = s.simulate(dt=0.05, max_steps=K, stop=pol, poll_interval=10)
            out.append((r["first_sat_step"], r["steps_done"], s.get_state()))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    for x, y in zip(out[0][2], out[1][2]):
        assert same(x, y)
    o = Oracle(cp, v_, n_, 6000, "f32")
    ov = init_voltages(9, 0, 1, 6000)[0].astype(np.float32)
    oxs, oxl = o.init_short_term_memory(), np.ones(33000, np.float32)
    o.simulate(ov, oxs, oxl, dt=np.float32(0.05), steps=int(out[0][1][0]), zeta=np.float32(0.001))
    v, xs, xl = out[0][2]
    assert same(v[0], ov) and same(xs[0], oxs) and same(xl[0], oxl)


@pytest.mark.parametrize("path", ["onchip", "wave", "resident", "solo"])
def test_call_sequences_fold_and_mirror_match_fused(xp, path):
    """Round 4 (callio.hpp): the persistent kernels reset a call's bookkeeping themselves (STOP_NONE /
    STOP_EACH) and store STOP_NONE results straight into the pinned host buffers.  A sequence of calls
    that mixes every kind -- fresh STOP_NONE (reset + mirror), continued STOP_EACH, fresh STOP_ANY
    (k_begin_call), fresh adaptive STOP_EACH (reset, dt restarts at 0.01), a continued STOP_NONE (no
    mirror) -- returns the same results and states as FUSED (which never folds), call by call, with
    replicas freezing on easy.cnf.  The persistent path's calls take Solver.simulate's reuse=True
    path (the solver's own result arrays and params, rebuilt per call field by field).  Last, a fresh
    folded call, then the same solver switched to FUSED continuing it (resume=True, no k_begin_call):
    the folded begin leaves the bookkeeping FUSED reads as k_begin_call would."""
    from odesat_amd import _lib
    f = product_formula("easy")
    env = {"onchip": ("0", "0", "0"), "wave": ("1", "0", "0"), "resident": ("0", "1", "0"),
           "solo": ("1", "0", "1")}[path]
    xp.set("WAVE", env[0])
    xp.set("RES_NARROW", env[1])
    xp.set("SOLO", env[2])
    seq = [dict(stop=ODESAT_STOP_NONE, max_steps=40, resume=False),
           dict(stop=ODESAT_STOP_EACH, max_steps=900, resume=True),
           dict(stop=ODESAT_STOP_ANY, max_steps=900, resume=False),
           dict(stop=ODESAT_STOP_EACH, max_steps=300, resume=False, adaptive=True),
           dict(stop=ODESAT_STOP_NONE, max_steps=30, resume=True, adaptive=True)]
    B = 3 if path == "solo" else 40
    out = []
    for alg in (None, _lib.ODESAT_ALG_FUSED):
        runs = []
        with Solver(f, B, "f32") as s:
            s.set_algorithm(alg if alg is not None else
                            (_lib.ODESAT_ALG_ONCHIP if path == "onchip" else _lib.ODESAT_ALG_RESIDENT))
            kern = s.step_kernel(False)
            s.init_state(4)
            owned = None
            for kw in seq:
                r = s.simulate(dt=0.1, tol=1e-3, poll_interval=64, reuse=alg is None, **kw)
                if alg is None:  # reuse: the same arrays every call
                    assert owned is None or r["first_sat_step"] is owned
                    owned = r["first_sat_step"]
                runs.append(({k: np.copy(x) for k, x in r.items()}, s.get_state()))
            r = s.simulate(dt=0.1, stop=ODESAT_STOP_NONE, max_steps=25, poll_interval=64)  # folded (persistent)
            runs.append(({k: np.copy(x) for k, x in r.items()}, s.get_state()))
            s.set_algorithm(_lib.ODESAT_ALG_FUSED)
            r = s.simulate(dt=0.1, stop=ODESAT_STOP_EACH, max_steps=400, poll_interval=16, resume=True)
            runs.append(({k: np.copy(x) for k, x in r.items()}, s.get_state()))
        out.append((kern, runs))
    (k1, a), (k2, b) = out
    assert k2 == "k_step" and k1 == {"onchip": "k_onchip", "wave": "k_wave", "resident": "k_resident",
                                     "solo": "k_solo"}[path]
    for (ra, sa), (rb, sb) in zip(a, b):
        assert ra["steps_run"] == rb["steps_run"]
        assert np.array_equal(ra["first_sat_step"], rb["first_sat_step"])
        assert np.array_equal(ra["steps_done"], rb["steps_done"]) and same(ra["dt"], rb["dt"])
        for x, y in zip(sa, sb):
            assert same(x, y)
    assert (a[1][0]["first_sat_step"] >= 0).any()  # replicas froze on the way


def _deg0_formula():
    """40 variables: 0-31 in 60 distinct-variable 3-SAT clauses, variable 0 in the first 8 (degree 8,
    a full padded block: k_solo_cv runs only when no variable has more terms than SOLO_DPAD = 8),
    32-39 in none (degree 0)."""
    rng = np.random.default_rng(5)
    while True:
        var = np.zeros((60, 3), np.int64)
        for c in range(60):
            var[c] = (np.concatenate([[0], rng.choice(np.arange(1, 32), 2, replace=False)]) if c < 8
                      else rng.choice(np.arange(1, 32), 3, replace=False))
        if np.bincount(var.reshape(-1)).max() <= 8:
            break
    neg = (rng.random(180) < 0.5).astype(np.uint8)
    return np.arange(0, 181, 3, dtype=np.int64), var.reshape(-1), neg, 40


@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("shape,lanes", [("hard", 192), ("hard", 128), ("deg0", 64), ("deg0", 128)])
@pytest.mark.parametrize("adaptive", [False, True])
def test_solo_cv_matches_solo_fast_and_oracle(xp, adaptive, shape, lanes, prec):
    """k_solo_cv (round 5, wave.hpp: the clause slots hold their literals' voltages and fold them
    themselves) against k_solo_fast (knob SOLO_CV = 0) and the oracle, B = 1 over three calls of 300
    steps (continued): on hard.cnf (the criterion's formula) at one clause slot per lane (192 lanes) and
    at two (128: lanes 32-127 hold a slot past m, whose terms go to their sink words), and on a formula
    with a variable of degree 8 (a full padded block) and 8 variables of degree 0 starting at -0.0 /
    +0.0 / -1 / 1 / 0.25 / -0.5 (a taken step turns -0.0 into +0.0, as k_solo_fast's dv = +0 does) at
    64 and 128 lanes (m = 60: lanes past m)."""
    from odesat_amd import _lib
    T = T_OF[prec]
    if shape == "hard":
        fo, o = oracle_for("hard", prec)
        f = product_formula("hard")
        cp, n = fo.clause_ptr, fo.varnum
    else:
        cp, var, neg, n = _deg0_formula()
        f = cnf.CNFFormula.from_arrays(cp, var, neg, n)
        o = Oracle(cp, var, neg, n, prec)
    m = len(cp) - 1
    v0 = init_voltages(3, 0, 1, n)[0].astype(T)
    if shape == "deg0":
        v0[32:40] = np.array([-0.0, 0.0, -1.0, 1.0, -0.0, 0.25, -0.5, -0.0], T)
    xs0, xl0 = o.init_short_term_memory(), np.ones(m, T)
    out = []
    for cv in ("1", "0"):
        xp.set("WAVE", "1")
        xp.set("SOLO", "1")
        xp.set("SOLO_LANES", str(lanes))
        xp.set("SOLO_CV", cv)
        with Solver(f, 1, prec) as s:
            s.set_algorithm(_lib.ODESAT_ALG_RESIDENT)
            assert s.step_kernel(adaptive) == "k_solo"
            s.set_state(v0[None].astype(np.float64), xs0[None].astype(np.float64), xl0[None].astype(np.float64))
            runs = []
            for call in range(3):
                r = s.simulate(adaptive=adaptive, dt=0.01 if adaptive else 0.05, tol=1e-3, zeta=0.01,
                               max_steps=300, stop=ODESAT_STOP_EACH, poll_interval=300,
                               resume=call > 0)
                runs.append(({k: np.copy(x) for k, x in r.items()}, s.get_state()))
            out.append(runs)
    for (ra, sa), (rb, sb) in zip(*out):
        assert np.array_equal(ra["first_sat_step"], rb["first_sat_step"])
        assert np.array_equal(ra["steps_done"], rb["steps_done"]) and same(ra["dt"], rb["dt"])
        for x, y in zip(sa, sb):
            assert same(x, y)
    ov, oxs, oxl = v0.copy(), xs0.copy(), xl0.copy()
    ra, (gv, gxs, gxl) = out[0][-1]
    if adaptive:
        t, sat, _, h, _ = o.simulate(ov, oxs, oxl, tol=T(1e-3), dt=None, steps=900, zeta=T(0.01))
        assert same(ra["dt"][0], h)
    else:
        t, sat, _, h, _ = o.simulate(ov, oxs, oxl, dt=T(0.05), steps=900, zeta=T(0.01))
    assert ra["steps_done"][0] == t and (ra["first_sat_step"][0] >= 0) == bool(sat)
    assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl)
    if shape == "deg0" and t > 0:
        assert not np.signbit(gv[0][[32, 36, 39]]).any()  # -0.0 became +0.0


@pytest.mark.parametrize("adaptive", [False, True])
def test_onchip_long_launches_sat_and_freeze(xp, adaptive):
    """STOP_EACH over launches of many steps: replicas that satisfy easy.cnf freeze at their own
    step inside a launch (ONCHIP == k_wave == FUSED, states, sat steps and adaptive dt)."""
    from odesat_amd import _lib
    f = product_formula("easy")
    out = []
    for alg, wave in ((_lib.ODESAT_ALG_ONCHIP, "0"), (_lib.ODESAT_ALG_RESIDENT, "1"), (_lib.ODESAT_ALG_FUSED, "1")):
        xp.set("WAVE", wave)
        xp.set("RES_NARROW", "0")
        with Solver(f, 40, "f32") as s:
            s.set_algorithm(alg)
            if alg == _lib.ODESAT_ALG_ONCHIP:
                assert s.step_kernel(adaptive) == "k_onchip"
            s.init_state(4)
            r = s.simulate(adaptive=adaptive, dt=0.1, tol=1e-3, max_steps=3000, stop=ODESAT_STOP_EACH,
                           poll_interval=500)
            out.append((r["first_sat_step"], r["steps_done"], r["dt"], s.get_state()))
    assert (out[0][0] >= 0).any()
    for o in out[1:]:
        assert np.array_equal(out[0][0], o[0]) and np.array_equal(out[0][1], o[1]) and same(out[0][2], o[2])
        for x, y in zip(out[0][3], o[3]):
            assert same(x, y)


def test_onchip_split_barrier_timeout_fails_the_call(xp):
    """the adaptive k_onchip's split-barrier wait is bounded; a wait that gives up
    must fail the call (ODESAT_EDEVICE), not return dv updates that raced.  The experiment knob
    ONCHIP_POLL_LIMIT = 0 makes every wait not satisfied at its first poll give up (the product
    waits 2^22 polls).  A solver without the knob then runs the same call cleanly, and its replica 0
    equals the oracle's simulate (system.rs:111-139): the fault word was reset, no false report."""
    from odesat_amd import _lib
    n, m = 3000, 12600
    f, (cp, v_, n_) = _instance(n, m, 7)
    B, K = 256, 100
    xp.set("ONCHIP_POLL_LIMIT", 0)
    with Solver(f, B, "f32") as s:
        assert s.step_kernel(True) == "k_onchip"
        s.init_state(3)
        with pytest.raises(_lib.OdesatError, match="split-barrier") as ei:
            s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        assert ei.value.code == _lib.ODESAT_EDEVICE
    xp.delete("ONCHIP_POLL_LIMIT")
    with Solver(f, B, "f32") as s:
        s.init_state(3)
        r = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        gv, gxs, gxl = s.get_state(0, 1)
    o = Oracle(cp, v_, n_, n, "f32")
    ov = init_voltages(3, 0, 1, n)[0].astype(np.float32)
    oxs, oxl = o.init_short_term_memory(), np.ones(m, np.float32)
    t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=np.float32(1e-3), steps=K, zeta=np.float32(0.001))
    assert t == K and r["steps_done"][0] == K and same(np.float32(h), np.float32(r["dt"][0]))
    assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl)


@pytest.mark.parametrize("stop", ["each", "any", "none"])
def test_onchip_adaptive_matches_resident_and_oracle(stop, xp):
    """Adaptive steps on chip (k_onchip's adaptive variant: four voltage arrays in LDS, the clause
    memories in VGPRs, each pass its own code instance since round 5), at either pair offset and the
    tiler's own choice, == k_resident's adaptive step (knob ONCHIP_ADAPTIVE = 0) bit for bit on every
    stop policy, per-replica dt included, and replica 0 == the oracle's f32 simulate with tol 1e-3
    (system.rs:111-139, :204-234)."""
    from odesat_amd import _lib
    f, (cp, v_, n_) = _instance(3000, 12600, 5)
    pol = {"each": ODESAT_STOP_EACH, "any": ODESAT_STOP_ANY, "none": ODESAT_STOP_NONE}[stop]
    B, K = 6, 30
    out = []
    for ada, off in (("1", None), ("1", "0"), ("1", "1"), ("0", None)):
        xp.set("ONCHIP_ADAPTIVE", ada)
        xp.set("PAIR_OFF", off)
        with Solver(f, B, "f32") as s:
            assert s.algorithm == _lib.ODESAT_ALG_ONCHIP
            assert s.step_kernel(True) == ("k_onchip" if ada == "1" else "k_resident")
            s.init_state(9)
            r = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=pol, poll_interval=10)
            out.append((r, s.get_state()))
    r1, s1 = out[0]
    for r2, s2 in out[1:]:
        assert np.array_equal(r1["first_sat_step"], r2["first_sat_step"]) and np.array_equal(r1["steps_done"], r2["steps_done"])
        assert same(r1["dt"], r2["dt"])
        for x, y in zip(s1, s2):
            assert same(x, y)
    o = Oracle(cp, v_, n_, 3000, "f32")
    ov = init_voltages(9, 0, 1, 3000)[0].astype(np.float32)
    oxs, oxl = o.init_short_term_memory(), np.ones(12600, np.float32)
    t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=np.float32(1e-3), dt=None, steps=int(r1["steps_done"][0]),
                               zeta=np.float32(0.001))
    assert t == r1["steps_done"][0] and same(np.float32(h), np.float32(r1["dt"][0]))
    assert same(s1[0][0], ov) and same(s1[1][0], oxs) and same(s1[2][0], oxl)


@pytest.mark.parametrize("adaptive", [False, True])
@pytest.mark.parametrize("stop", ["each", "any", "none"])
def test_resident_f64_register_tiles_match_streaming_and_oracle(stop, adaptive, xp):
    """f64 steps keep the first RES_RC (fixed) / RES_RC_ADA (adaptive, VFG: with each tile's first-pass
    mn) tiles' memories in VGPRs for a launch (resident.hpp, round 4): == every tile streamed
    (knob RES_RC = 0) bit for bit on every stop policy -- fixed STOP_ANY launches write out of place and
    replay -- over a fresh call and a continued one (per-replica dt included), and replica 0 == the
    oracle's f64 simulate (system.rs:111-154).  The instances' tilings are deep enough (85+ tiles,
    tests/test_tiling.py's hook) for the register prefix (the host needs RC + 16); the adaptive one is
    large enough (n = 7 000) for the clone-in-HBM kernel.  Round 5: the default runs them on wave-paired
    tiles (resident.hpp PAIRS: a barrier after every second tile) at either pair offset; == plain tiles
    (knob RES_PAIRS = 0)."""
    from odesat_amd import _lib
    n, m = (7000, 29400) if adaptive else (3000, 12600)
    f, (cp, v_, n_) = _instance(n, m, 5)
    pol = {"each": ODESAT_STOP_EACH, "any": ODESAT_STOP_ANY, "none": ODESAT_STOP_NONE}[stop]
    B = 4 if adaptive else 6
    kw = dict(adaptive=True, tol=1e-3) if adaptive else dict(dt=0.05)
    out = []
    for rc, pairs, off in (("1", "1", None), ("1", "1", "0"), ("1", "1", "1"), ("1", "0", None), ("0", "0", None)):
        xp.set("RES_RC", rc)
        xp.set("RES_PAIRS", pairs)
        xp.set("PAIR_OFF", off)  # both pair offsets (PAIRS = 1, 2), and the tiler's own choice
        with Solver(f, B, "f64") as s:
            assert s.algorithm == _lib.ODESAT_ALG_RESIDENT and s.step_kernel(adaptive) == "k_resident"
            s.init_state(9)
            r1 = s.simulate(zeta=0.001, max_steps=13, stop=pol, poll_interval=13, **kw)
            r2 = s.simulate(zeta=0.001, max_steps=9, stop=pol, poll_interval=4, resume=True, **kw)
            out.append((r1, r2, s.get_state()))
    (a1, a2, sa) = out[0]
    for (b1, b2, sb) in out[1:]:
        for x, y in ((a1, b1), (a2, b2)):
            assert x["steps_run"] == y["steps_run"]
            assert np.array_equal(x["first_sat_step"], y["first_sat_step"]) and np.array_equal(x["steps_done"], y["steps_done"])
            assert same(x["dt"], y["dt"])
        for x, y in zip(sa, sb):
            assert same(x, y)
    o = Oracle(cp, v_, n_, n, "f64")
    ov = init_voltages(9, 0, 1, n)[0]
    oxs, oxl = o.init_short_term_memory(), np.ones(m)
    t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=1e-3 if adaptive else None, dt=None if adaptive else 0.05,
                               steps=int(a2["steps_done"][0]), zeta=0.001)
    assert t == a2["steps_done"][0]
    if adaptive:
        assert same(h, a2["dt"][0])
    assert same(sa[0][0], ov) and same(sa[1][0], oxs) and same(sa[2][0], oxl)


def test_onchip_adaptive_inter_after_out_of_range_set_state():
    """adaptive STOP_ANY (simulate_inter) on an ONCHIP solver whose caller state is
    out of range.  The first step runs RESIDENT's adaptive step in place (one step, nothing to
    replay), the rest k_onchip's multi-step launches with replay.  Every replica's state, dt and the
    stop equal the oracle's simulate_inter with per-replica dt (the declared deviation)."""
    from odesat_amd import _lib
    n, m = 3000, 12600
    f, (cp, v_, n_) = _instance(n, m, 5)
    o = Oracle(cp, v_, n_, n, "f32")
    B, K = 6, 40
    v, xs, xl = init_states(o, B, seed=9, T=np.float32)
    v[0, :50] *= 1.7        # voltages outside [-1, 1]
    xs[1, :40] = 0.0005      # short-term memories below the clamp
    xl[2, :30] = 0.5        # long-term memories below the clamp
    with Solver(f, B, "f32") as s:
        assert s.algorithm == _lib.ODESAT_ALG_ONCHIP and s.step_kernel(True) == "k_onchip"
        s.set_state(v.astype(np.float64), xs.astype(np.float64), xl.astype(np.float64))
        r = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_ANY, poll_interval=10)
        gv, gxs, gxl = s.get_state()
    t, win, _, dts = o.simulate_inter(v, xs, xl, tol=np.float32(1e-3), steps=K, zeta=np.float32(0.001),
                                      shared_dt=False)
    assert r["steps_run"] == t and np.all(r["steps_done"] == t)
    if win >= 0:
        assert int(np.flatnonzero(r["first_sat_step"] >= 0)[0]) == win
    assert same(gv, v) and same(gxs, xs) and same(gxl, xl) and same(r["dt"].astype(np.float32), dts)


@pytest.mark.parametrize("narrow", ["0", "1"])
@pytest.mark.parametrize("stop", ["each", "any", "none"])
def test_resident_adaptive_clone_in_hbm_matches_fused_and_oracle(stop, narrow, xp):
    """f64 at n = 7000: v and dv fill 112 KB of LDS and the full-step clone (56 KB more) does not
    fit, so adaptive steps run k_resident with the clone in HBM (VFG) instead of FUSED on the same
    one-replica layout.  VFG == FUSED (knob RES_VFG = 0) bit for bit on every stop policy, with
    full-width and one-wave tiles, per-replica dt included; replica 0 == the oracle's f64 simulate
    (system.rs:111-139)."""
    xp.set("RES_NARROW", narrow)
    f, (cp, v_, n_) = _instance(7000, 29400, 11)
    pol = {"each": ODESAT_STOP_EACH, "any": ODESAT_STOP_ANY, "none": ODESAT_STOP_NONE}[stop]
    B, K = 5, 30
    out = []
    for vfg in ("1", "0"):
        xp.set("RES_VFG", vfg)
        with Solver(f, B, "f64") as s:
            assert s.step_kernel(True) == ("k_resident" if vfg == "1" else "k_step")
            s.init_state(3)
            r = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=pol, poll_interval=10)
            out.append((r, s.get_state()))
    r1, s1 = out[0]
    for r2, s2 in out[1:]:
        assert np.array_equal(r1["first_sat_step"], r2["first_sat_step"]) and np.array_equal(r1["steps_done"], r2["steps_done"])
        assert same(r1["dt"], r2["dt"])
        for x, y in zip(s1, s2):
            assert same(x, y)
    o = Oracle(cp, v_, n_, 7000, "f64")
    ov = init_voltages(3, 0, 1, 7000)[0]
    oxs, oxl = o.init_short_term_memory(), np.ones(29400)
    t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=1e-3, dt=None, steps=int(r1["steps_done"][0]), zeta=0.001)
    assert t == r1["steps_done"][0] and same(h, r1["dt"][0])
    assert same(s1[0][0], ov) and same(s1[1][0], oxs) and same(s1[2][0], oxl)


@pytest.mark.parametrize("team", [None, "1", "2", "solo"])
@pytest.mark.parametrize("n,m,prec,wave_env,wpw", [(250, 1065, "f64", None, 2), (600, 2520, "f32", "1", 1)])
def test_wave_workgroup_widths(xp, n, m, prec, wave_env, wpw, team):
    """k_wave with 2 (config 3 in f64) and 1 (a larger instance, forced) replicas per workgroup
    equals FUSED bit for bit, fixed and adaptive -- with the automatic team (8 and 16 waves per
    replica) and with teams of 1 and 2 waves; and k_solo (one replica per workgroup, 4 clause slots
    per lane at m = 2520 with 640 lanes: the default 512 would need 5) on the same formulas."""
    xp.set("SOLO", "1" if team == "solo" else "0")
    if team == "solo":
        xp.set("SOLO_LANES", "640")
    if team not in (None, "solo"):
        xp.set("WAVE_TEAM", team)
    from odesat_amd import _lib
    var, neg = wl.random_ksat(n, m, 3, 7)
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, n)
    if wave_env is not None:
        xp.set("WAVE", wave_env)
    topo = m * 16 + (n + 1) * 4
    rep = ((2 * n + 3 * m + 3 * m) * (8 if prec == "f64" else 4) + 15) // 16 * 16
    assert (topo + 4 * rep > 159 * 1024) and (wpw == 1) == (topo + 2 * rep > 159 * 1024)
    for adaptive in (False, True):
        out = []
        for alg in (_lib.ODESAT_ALG_RESIDENT, _lib.ODESAT_ALG_FUSED):
            with Solver(f, 9, prec) as s:
                assert s.group_width == 1
                s.set_algorithm(alg)
                if alg == _lib.ODESAT_ALG_RESIDENT:
                    assert s.step_kernel(adaptive) == ("k_solo" if team == "solo" else "k_wave")
                s.init_state(11)
                r = s.simulate(adaptive=adaptive, dt=0.05, max_steps=40, stop=ODESAT_STOP_EACH, poll_interval=7)
                out.append((r, s.get_state()))
        assert np.array_equal(out[0][0]["first_sat_step"], out[1][0]["first_sat_step"])
        assert np.array_equal(out[0][0]["steps_done"], out[1][0]["steps_done"]) and same(out[0][0]["dt"], out[1][0]["dt"])
        for x, y in zip(out[0][1], out[1][1]):
            assert same(x, y)


@pytest.mark.parametrize("stop", [ODESAT_STOP_EACH, ODESAT_STOP_ANY, ODESAT_STOP_NONE])
@pytest.mark.parametrize("adaptive", [False, True])
def test_wave_teams_equal_fused(xp, stop, adaptive):
    """k_wave with one, two and four waves per replica (ODESAT_WAVE_TEAM) and k_solo with one, two
    and three waves (ODESAT_SOLO_LANES) equal FUSED bit for bit on easy.cnf, where replicas satisfy
    and freeze at their own steps inside long launches: a frozen replica's team keeps reaching the
    workgroup barriers of the others."""
    from odesat_amd import _lib
    f = product_formula("easy")
    out = []
    for alg, team in ((_lib.ODESAT_ALG_FUSED, "1"), (_lib.ODESAT_ALG_RESIDENT, "1"), (_lib.ODESAT_ALG_RESIDENT, "2"),
                      (_lib.ODESAT_ALG_RESIDENT, "4"), (_lib.ODESAT_ALG_RESIDENT, "solo64"),
                      (_lib.ODESAT_ALG_RESIDENT, "solo128"), (_lib.ODESAT_ALG_RESIDENT, "solo192")):
        xp.set("WAVE", "1")
        solo = team.startswith("solo")
        xp.set("SOLO", "1" if solo else "0")
        if solo:
            xp.set("SOLO_LANES", team[4:])
        else:
            xp.set("WAVE_TEAM", team)
        with Solver(f, 37, "f32") as s:
            s.set_algorithm(alg)
            if alg == _lib.ODESAT_ALG_RESIDENT:
                assert s.step_kernel(adaptive) == ("k_solo" if solo else "k_wave")
            s.init_state(6)
            r = s.simulate(adaptive=adaptive, dt=0.1, tol=1e-3, max_steps=1500, stop=stop, poll_interval=300)
            out.append((r, s.get_state()))
    assert (out[0][0]["first_sat_step"] >= 0).any()
    for r, st in out[1:]:
        assert np.array_equal(out[0][0]["first_sat_step"], r["first_sat_step"])
        assert np.array_equal(out[0][0]["steps_done"], r["steps_done"]) and same(out[0][0]["dt"], r["dt"])
        for x, y in zip(out[0][1], st):
            assert same(x, y)


@pytest.mark.parametrize("stop", [ODESAT_STOP_EACH, ODESAT_STOP_ANY, ODESAT_STOP_NONE])
@pytest.mark.parametrize("adaptive", [False, True])
def test_wave_partial_round_tail_launch(xp, stop, adaptive):
    """k_wave's partial last round as a launch of its own (round 6, knob WAVE_TAIL): B = 1100 on easy.cnf
    is one device round of 256 workgroups x 4 replicas plus 76 replicas, which now run after it at one
    replica per workgroup.  Replicas satisfy and freeze at their own steps inside 300-step launches, and
    STOP_ANY's stop word set in the first launch is read by the second: every state, sat step, step
    count and dt equals the single launch's (WAVE_TAIL = 0) and FUSED's."""
    from odesat_amd import _lib
    f = product_formula("easy")
    out = []
    for alg, tail in ((_lib.ODESAT_ALG_RESIDENT, None), (_lib.ODESAT_ALG_RESIDENT, "0"), (_lib.ODESAT_ALG_FUSED, None)):
        xp.set("WAVE", "1")
        xp.set("SOLO", "0")
        xp.set("WAVE_TAIL", tail)
        with Solver(f, 1100, "f32") as s:
            s.set_algorithm(alg)
            if alg == _lib.ODESAT_ALG_RESIDENT:
                assert s.step_kernel(adaptive) == "k_wave"
            s.init_state(6)
            r = s.simulate(adaptive=adaptive, dt=0.1, tol=1e-3, max_steps=1500, stop=stop, poll_interval=300)
            out.append((r, s.get_state()))
    assert (out[0][0]["first_sat_step"] >= 0).any()
    for r, st in out[1:]:
        assert np.array_equal(out[0][0]["first_sat_step"], r["first_sat_step"])
        assert np.array_equal(out[0][0]["steps_done"], r["steps_done"]) and same(out[0][0]["dt"], r["dt"])
        for x, y in zip(out[0][1], st):
            assert same(x, y)


def test_wave_partial_round_config3_vs_oracle(xp):
    """Config 3 (n = 250, m = 1065) at B = 1280: 1024 replicas in the main launch and 256 in the tail's
    (one replica per workgroup, 16-wave teams for fixed steps, 4 for adaptive).  20 adaptive steps equal
    the single launch's bit for bit, and replicas 0, 1023 (main) and 1024, 1279 (tail) equal the
    oracle's f32 simulate."""
    c = wl.CONFIGS["config3"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    B, K = 1280, 20
    out = []
    for tail in (None, "0"):
        xp.set("WAVE_TAIL", tail)
        with Solver(f, B, "f32") as s:
            assert s.step_kernel(True) == "k_wave"
            s.init_state(42)
            r = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_NONE)
            out.append((r, s.get_state()))
    (r1, s1), (r2, s2) = out
    assert np.all(r1["steps_done"] == K) and same(r1["dt"], r2["dt"])
    for x, y in zip(s1, s2):
        assert same(x, y)
    o = Oracle(cp, v_, n_, c["n"], "f32")
    for b in (0, 1023, 1024, 1279):
        ov = init_voltages(42, b, 1, c["n"])[0].astype(np.float32)
        oxs, oxl = o.init_short_term_memory(), np.ones(c["m"], np.float32)
        t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=np.float32(1e-3), dt=None, steps=K)
        assert t == K and same(np.float32(h), np.float32(r1["dt"][b]))
        assert same(s1[0][b], ov) and same(s1[1][b], oxs) and same(s1[2][b], oxl), f"replica {b}"
