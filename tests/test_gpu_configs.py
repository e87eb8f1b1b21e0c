"""BASELINE.json's configs at their real sizes, on the GPU, against the oracle:

  config 1  tests/easy.cnf, `odesat solve` (adaptive, tol 1e-3, -r 7): the CLI's assignment equals the
            f64 oracle's run of the same preprocessed formula and initial state, driven through
            several bounded calls (odesat_simulate_continue);
  config 2  n=10k m=42k f32 at the bench's horizon (200 steps): the f32 GPU against the f64 oracle --
            the north star's fp32 tolerance on (v, xs, xl) and the identical v > 0 assignment;
  config 3  uf250-style n=250 m=1065 seed 2, adaptive, B=1024 (k_wave): replicas bit-exact vs oc32;
  config 4  n=50k m=210k seed 3, B=1024 f32: replicas bit-exact vs oc32, every replica by property;
            inter (STOP_ANY) on the planted variant: the winner and the stop step;
  config 5  n=1M m=4.2M seed 4, one replica partitioned over 1, 2, 4 and 8 ranks (VARIABLES bit-exact;
            CLAUSES / CLAUSES_RS bit-exact at world 1, within a stated tolerance beyond) vs oc32's fixed
            steps; and the stop step of simulate on a planted instance of the same size at every world.
Subsets of replicas are checked bit for bit; the rest through size-independent properties (the
clamp ranges of system.rs:94-96, finiteness)."""
import os
import subprocess

import numpy as np
import pytest

from oracle.oracle import Oracle, init_voltages
from odesat_amd import cnf
from odesat_amd import workloads as wl
from odesat_amd.system import ODESAT_STOP_ANY, ODESAT_STOP_EACH, ODESAT_STOP_NONE, Solver

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def instance(name):
    c = wl.CONFIGS[name]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    return cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"]), (cp, v_, n_), c["n"], c["m"]


def assert_in_range(v, xs, xl, m):
    """system.rs:94-96 clamp ranges (f32 constants) and finiteness."""
    assert np.isfinite(v).all() and np.isfinite(xs).all() and np.isfinite(xl).all()
    assert v.min() >= -1 and v.max() <= 1
    eps = np.float32(0.001)
    assert xs.min() >= eps and xs.max() <= np.float32(1) - eps
    assert xl.min() >= 1 and xl.max() <= np.float32(1e4) * np.float32(m)


# ----------------------------------------------------------------------------------- config 4 ---
def test_config4_full_size_subset_bitexact_and_properties():
    f, (cp, v_, n_), n, m = instance("config4")
    o = Oracle(cp, v_, n_, n, "f32")
    B, K = 1024, 10
    pick = [0, 511, 1023]
    with Solver(f, B, "f32") as s:
        s.init_state(42)
        r = s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE)
        assert r["steps_run"] == K and np.all(r["steps_done"] == K)
        states = {b: s.get_state(b, 1) for b in pick}
        for r0 in range(0, B, 128):  # every replica, 128 at a time (0.5 GB of f64 per chunk)
            assert_in_range(*s.get_state(r0, 128), m)
    for b in pick:
        ov = init_voltages(42, b, 1, n)[0].astype(np.float32)
        oxs, oxl = o.init_short_term_memory(), np.ones(m, np.float32)
        o.simulate(ov, oxs, oxl, dt=np.float32(0.01), steps=K, zeta=np.float32(0.001))
        gv, gxs, gxl = states[b]
        assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl)


def test_config4_inter_winner_on_planted_instance():
    """simulate_inter (system.rs:278-294, 353-358) at config 4's size.  The instance is config 4's
    with a planted satisfying assignment x*.  Replica 700 starts at v = 0.6 x* (allsat at step 0:
    every clause has a literal with q v = 0.6 > 0.5, C = 0.2 < 0.25), replica 300 at 0.49 x* (not:
    C = 0.255), the rest random.  The lowest allsat index at the first allsat step is 700: every
    replica takes exactly that one step (the fixed step updates after the check, :148-152)."""
    c = wl.CONFIGS["config4"]
    n, m = c["n"], c["m"]
    var, neg, star = wl.planted_ksat(n, m, 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, n)
    o = Oracle(cp, v_, n_, n, "f32")
    sgn = np.where(star, 1.0, -1.0)
    B = 1024
    xs0 = o.init_short_term_memory().astype(np.float64)
    special = {300: 0.49 * sgn, 700: 0.6 * sgn}
    with Solver(f, B, "f32") as s:
        s.init_state(42)
        for b, v in special.items():
            s.set_state(v[None], xs0[None], np.ones((1, m)), r0=b)
        r = s.simulate(dt=0.01, max_steps=64, stop=ODESAT_STOP_ANY, poll_interval=16)
        pick = [0, 300, 700, 1023]
        states = {b: s.get_state(b, 1) for b in pick}
    sat = np.flatnonzero(r["first_sat_step"] >= 0)
    assert list(sat) == [700] and r["first_sat_step"][700] == 0
    assert np.all(r["steps_done"] == 1)
    for b in pick:
        ov = (special[b] if b in special else init_voltages(42, b, 1, n)[0]).astype(np.float32)
        oxs, oxl = o.init_short_term_memory(), np.ones(m, np.float32)
        allsat = o.euler_step_fixed(ov, oxs, oxl, np.float32(0.01), np.float32(0.001))
        assert allsat == (b == 700)
        gv, gxs, gxl = states[b]
        assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl)


# ----------------------------------------------------------------------------------- config 3 ---
@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_config3_wave_kernel_vs_oracle(prec):
    """Adaptive steps (tol 1e-3, dt0 0.01, per-replica dt), B = 1024, on k_wave (the default for
    this size): replicas {0, 511, 1023} bit-exact against the oracle's simulate, sat steps included."""
    from odesat_amd import _lib
    f, (cp, v_, n_), n, m = instance("config3")
    T = np.float32 if prec == "f32" else np.float64
    o = Oracle(cp, v_, n_, n, prec)
    B, K = 1024, 60
    pick = [0, 511, 1023]
    with Solver(f, B, prec) as s:
        assert s.algorithm == _lib.ODESAT_ALG_RESIDENT and s.group_width == 1  # k_wave
        s.init_state(42)
        r = s.simulate(adaptive=True, tol=1e-3, max_steps=K, stop=ODESAT_STOP_EACH, poll_interval=16)
        states = {b: s.get_state(b, 1) for b in pick}
    for b in pick:
        ov = init_voltages(42, b, 1, n)[0].astype(T)
        oxs, oxl = o.init_short_term_memory(), np.ones(m, T)
        t, sat, _, h, _ = o.simulate(ov, oxs, oxl, tol=T(1e-3), steps=K, zeta=T(0.001))
        assert r["steps_done"][b] == t and (r["first_sat_step"][b] >= 0) == sat
        assert T(r["dt"][b]) == T(h)
        gv, gxs, gxl = states[b]
        assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl)


# ----------------------------------------------------------------------------------- config 2 ---
F32_TOL = 1e-4  # stated fp32 tolerance at the bench horizon (profiles/r02_f32_vs_f64_horizon.txt)


def test_config2_f32_tracks_f64_reference_at_bench_horizon():
    """The north star's bar for the fp32 path: (v, xs, xl) within a stated fp32 tolerance of the
    reference's f64 trajectory and the SAME final boolean assignment (v > 0, system.rs:238), at the
    bench's horizon (200 fixed steps, B = 1024; the driver's 20-step run is inside it).  Both start
    from the f32-rounded initial voltages.  Measured horizon (oracle, same replicas): identical
    assignments through 300 steps, the first differing variable near step 500, decorrelated by
    ~1000 steps (chaotic divergence, ~x2 per 45 steps)."""
    f, (cp, v_, n_), n, m = instance("config2")
    o = Oracle(cp, v_, n_, n, "f64")
    B, K = 1024, 200
    pick = [0, 517, 1023]
    with Solver(f, B, "f32") as s:
        s.init_state(42)
        s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
        states = {b: s.get_state(b, 1) for b in pick}
    for b in pick:
        ov = init_voltages(42, b, 1, n)[0].astype(np.float32).astype(np.float64)
        oxs, oxl = o.init_short_term_memory(), np.ones(m)
        o.simulate(ov, oxs, oxl, dt=0.01, steps=K, zeta=0.001)
        gv, gxs, gxl = (x[0] for x in states[b])
        assert np.max(np.abs(gv - ov)) <= F32_TOL
        assert np.max(np.abs(gxs - oxs)) <= F32_TOL
        assert np.max(np.abs(gxl - oxl) / oxl) <= F32_TOL
        assert np.array_equal(gv > 0, ov > 0)


@pytest.mark.parametrize("leg,prec,adaptive,kernel", [
    ("adaptive", "f32", True, "k_onchip"),       # k_onchip<90, 1, true>
    ("f64", "f64", False, "k_resident"),         # short forms, 28 register tiles (§4.1)
    ("f64_adaptive", "f64", True, "k_resident"),  # VFG: the clone in HBM, 12 register tiles (§4.1)
])
def test_config2_bench_leg_kernels_bitexact(leg, prec, adaptive, kernel):
    """bench.py's `adaptive`, `f64` and `f64_adaptive` legs at the configuration they time: n=10k,
    m=42k, B=1024, the bench's call shape (a 5-step warm-up call, then a 15-step call, each ONE
    persistent launch, STOP_NONE).  The solver runs the kernel the leg names; replicas {0, 517, 1023}
    are bit-exact against the oracle's simulate of the same two calls (state, per-replica dt --
    restarting at 0.01 per call, system.rs:205 -- and step counts); every replica stays finite and in
    the clamp ranges (system.rs:94-96).  Reference: system.rs:111-139, :141-154, :204-234."""
    f, (cp, v_, n_), n, m = instance("config2")
    T = np.float32 if prec == "f32" else np.float64
    o = Oracle(cp, v_, n_, n, prec)
    B, calls = 1024, (5, 15)
    pick = [0, 517, 1023]
    with Solver(f, B, prec) as s:
        assert s.step_kernel(adaptive) == kernel
        s.init_state(42)
        rs = []
        for K in calls:
            r = s.simulate(adaptive=adaptive, dt=0.01, tol=1e-3, max_steps=K, poll_interval=K, stop=ODESAT_STOP_NONE)
            assert r["steps_run"] == K and np.all(r["steps_done"] == K)
            rs.append(r)
        states = {b: s.get_state(b, 1) for b in pick}
        eps = T(0.001)
        for r0 in range(0, B, 256):
            v, xs, xl = s.get_state(r0, 256)
            assert np.isfinite(v).all() and np.isfinite(xs).all() and np.isfinite(xl).all()
            assert v.min() >= -1 and v.max() <= 1
            assert xs.min() >= eps and xs.max() <= T(1) - eps
            assert xl.min() >= 1 and xl.max() <= T(1e4) * T(m)
        if adaptive:
            assert np.all(rs[-1]["dt"][:B] >= 2.0 ** -7) and np.all(rs[-1]["dt"][:B] <= 1e3)
    for b in pick:
        ov = init_voltages(42, b, 1, n)[0].astype(T)
        oxs, oxl = o.init_short_term_memory(), np.ones(m, T)
        for K, r in zip(calls, rs):
            if adaptive:
                t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=T(1e-3), steps=K, zeta=T(0.001))
                assert same(T(h), T(r["dt"][b])), (b, h, r["dt"][b])
            else:
                t, _, _, _, _ = o.simulate(ov, oxs, oxl, dt=T(0.01), steps=K, zeta=T(0.001))
            assert t == K and r["steps_done"][b] == K
        gv, gxs, gxl = states[b]
        assert same(gv[0], ov) and same(gxs[0], oxs) and same(gxl[0], oxl), b


# ----------------------------------------------------------------------------------- config 1 ---
def test_config1_cli_solve_easy_adaptive_matches_oracle(tmp_path):
    """`odesat solve -f easy.cnf` exactly as BASELINE states config 1 (adaptive step, tol 1e-3,
    -r 7, the reference's f64), run unbounded in bounded calls of 64 steps (the hidden --run-chunk flag) so the
    continue path carries dt and the step count across calls: the printed assignment equals the f64
    oracle's continuous run of the same preprocessed formula from the same initial state, mapped
    back through the same trace, and satisfies the input."""
    from odesat_amd import preprocess as pp
    path = os.path.join(ROOT, "tests", "golden", "easy.cnf")
    out = tmp_path / "easy.txt"
    binp = os.path.join(ROOT, "odesat_amd", "bin", "odesat")
    r = subprocess.run([binp, "solve", "-f", path, "-o", str(out), "--run-chunk", "64"], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    assert "Checking if solution vector satisfies formula: true" in r.stdout
    got = {}
    for line in out.read_text().strip().splitlines():
        a, b = line.split()
        got[int(a)] = b == "1"
    text = open(path).read()
    formula = cnf.parse_dimacs_format(text)
    reduced, trace = pp.repeatedly_resolve_and_update(formula, 7.0)
    mapping, norm = cnf.normalize_cnf_variables(reduced)
    ncp, nvar, nneg = norm.arrays()
    o = Oracle(ncp, nvar, nneg, norm.varnum, "f64")
    v = init_voltages(42, 0, 1, norm.varnum)[0]
    xs, xl = o.init_short_term_memory(), np.ones(norm.nclauses)
    t, sat, assign, _, _ = o.simulate(v, xs, xl, tol=1e-3, steps=1 << 22, zeta=None)
    assert sat and t > 64  # the run crossed several bounded calls
    vals = cnf.map_values_by_indices(mapping, assign)
    pp.calculate_trace(vals, trace, formula)
    assert pp.evaluate_cnf_assign(vals, formula)
    assert got == {k: bool(v) for k, v in vals.items()}


# ----------------------------------------------------------------------------------- config 5 ---
CLAUSES_TOL = 1e-5  # CLAUSES at world > 1 sums per-rank partial dv (reordered fold), max |dv| after 5 steps
# BASELINE configs[4] names an 8-way partition; every world up to it runs as ranks held by one process on
# the box's GPU (LocalComm + step_in_process: the collectives' sums and copies done in process)
PART_CASES = [("VARIABLES", 2), ("VARIABLES", 4), ("VARIABLES", 8), ("CLAUSES", 1), ("CLAUSES", 2),
              ("CLAUSES", 4), ("CLAUSES", 8), ("CLAUSES_RS", 1), ("CLAUSES_RS", 2), ("CLAUSES_RS", 4),
              ("CLAUSES_RS", 8)]


@pytest.fixture(scope="module")
def config5_random():
    """Config 5 (n = 1M, m = 4.2M, seed 4) and the oracle's 5 fixed steps of dt 0.01 from replica 0."""
    from odesat_amd.partition import default_zeta
    c = wl.CONFIGS["config5"]
    n, m = c["n"], c["m"]
    var, neg = wl.random_ksat(n, m, 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    del var, neg
    o = Oracle(cp, v_, n_, n, "f32")
    K, dt, zeta = 5, 0.01, default_zeta(n, m)
    v0 = init_voltages(42, 0, 1, n)[0].astype(np.float32)
    xs0 = o.init_short_term_memory()
    v, xs, xl = v0.copy(), xs0.copy(), np.ones(m, np.float32)
    for _ in range(K):
        o.euler_step_fixed(v, xs, xl, np.float32(dt), np.float32(zeta))
    return dict(cp=cp, var=v_, neg=n_, n=n, m=m, K=K, dt=dt, zeta=zeta, init=(v0, xs0, np.ones(m)), ref=(v, xs, xl))


def _run_partition(cfg, mode, world, steps, stop):
    from odesat_amd.partition import LocalComm, PartitionedSolver, step_in_process
    parts = [PartitionedSolver(cfg["cp"], cfg["var"], cfg["neg"], cfg["n"], mode, comm=LocalComm(r, world))
             for r in range(world)]
    try:
        for p in parts:
            p.set_state(*cfg["init"])
        for _ in range(steps):
            step_in_process(parts, cfg["dt"], cfg["zeta"], stop)
        return [(p.status(stop), p.get_state()) for p in parts]
    finally:
        for p in parts:
            p.close()


def _check_partition(cfg, mode, world, out, v, xs, xl):
    from odesat_amd.partition import VARIABLES
    for st, (gv, gxs, gxl, loc) in out:
        if mode == VARIABLES or world == 1:  # the reference's fold order on every rank: bit-exact
            assert np.array_equal(gv.astype(np.float32), v)
            assert np.array_equal(gxs.astype(np.float32), xs[loc]) and np.array_equal(gxl.astype(np.float32), xl[loc])
        else:  # CLAUSES / CLAUSES_RS: the ranks' partial sums reorder each dv fold
            assert np.max(np.abs(gv - v)) <= CLAUSES_TOL
            assert np.max(np.abs(gxs - xs[loc])) <= CLAUSES_TOL
            assert np.max(np.abs(gxl - xl[loc]) / xl[loc]) <= CLAUSES_TOL


@pytest.mark.parametrize("mode_name,world", PART_CASES)
def test_config5_partitioned_full_size_vs_oracle(config5_random, mode_name, world):
    """One replica of n = 1M, m = 4.2M split over `world` ranks (up to the 8 BASELINE names): VARIABLES
    bit-exact at every world (its spanning clauses duplicated: 33 % of the clauses per rank at world
    8), CLAUSES and CLAUSES_RS (reduce-scatter + all-gather) bit-exact at world 1 and within
    CLAUSES_TOL beyond, against oc32's fixed steps (system.rs:141-154), 5 steps of dt 0.01."""
    from odesat_amd import partition
    mode = getattr(partition, mode_name)
    cfg = config5_random
    out = _run_partition(cfg, mode, world, cfg["K"], stop=False)
    for st, _ in out:
        assert st["steps_done"] == cfg["K"] and st["first_sat_step"] == -1
    _check_partition(cfg, mode, world, out, *cfg["ref"])


@pytest.fixture(scope="module")
def config5_planted():
    """Config 5's size with a planted assignment x*: v0 = 0.6 x* except three variables flipped to
    -0.6 x*_i, xs0 per system.rs:361-372, fixed dt 0.1.  The oracle's simulate (system.rs:190-203)
    reaches its first allsat step T, takes that step's update and stops (T + 1 steps)."""
    c = wl.CONFIGS["config5"]
    n, m = c["n"], c["m"]
    var, neg, star = wl.planted_ksat(n, m, 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    del var, neg
    o = Oracle(cp, v_, n_, n, "f32")
    v0 = (np.float32(0.6) * np.where(star, 1.0, -1.0)).astype(np.float32)
    v0[[10, 500000, 999990]] *= -1
    xs0 = o.init_short_term_memory()
    v, xs, xl = v0.copy(), xs0.copy(), np.ones(m, np.float32)
    dt, zeta, cap = 0.1, 0.001, 200
    t, sat, _, _, _ = o.simulate(v, xs, xl, dt=np.float32(dt), steps=cap, zeta=np.float32(zeta))
    assert sat and 1 < t < cap  # (measured: T = 78, so t = 79 steps)
    return dict(cp=cp, var=v_, neg=n_, n=n, m=m, dt=dt, zeta=zeta, init=(v0, xs0, np.ones(m)), ref=(v, xs, xl),
                steps_run=t, cap=t + 10)


@pytest.mark.parametrize("mode_name,world", PART_CASES)
def test_config5_partitioned_stop_step_vs_oracle_simulate(config5_planted, mode_name, world):
    """The stop of simulate (system.rs:190-203: the first allsat step T, its update taken, nothing after)
    at config 5's size over `world` ranks: the device bookkeeping folds the previous step's collective
    result (CLAUSES: the all-reduced unsat count; VARIABLES / CLAUSES_RS: every block's flag slot), so
    every rank reports first_sat_step T and T + 1 steps done while the driver keeps stepping past it;
    the final state as in test_config5_partitioned_full_size_vs_oracle."""
    from odesat_amd import partition
    mode = getattr(partition, mode_name)
    cfg = config5_planted
    out = _run_partition(cfg, mode, world, cfg["cap"], stop=True)
    for st, _ in out:
        assert st["first_sat_step"] == cfg["steps_run"] - 1 and st["steps_done"] == cfg["steps_run"] and st["frozen"]
    _check_partition(cfg, mode, world, out, *cfg["ref"])
