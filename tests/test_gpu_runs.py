"""Runs that span several calls, launches, threads or processes -- all bit-exact against one plain
run or the oracle:
  * odesat_simulate_continue: an unbounded run (the reference's steps = None) in bounded calls keeps
    the reference's trajectory (adaptive dt and frozen replicas carry over), through the Python API,
    the one-call boundary odesat_run and the CLI;
  * STOP_ANY (simulate_inter) on the persistent kernels: multi-step launches with the replay at the
    first allsat step equal FUSED's lock-step run and the oracle;
  * odesat_checkpoint / odesat_rollback;
  * two solvers driven from two host threads at once (per-device kernel attributes);
  * the sharded drivers (odesat_amd/sharding.py) in two gloo processes on the box's GPU, and the CLI's
    --gpus: the same winner and per-replica states as one process over the same global replicas."""
import ctypes as C
import json
import os
import socket
import subprocess
import threading

import numpy as np
import pytest

from odesat_amd import _lib
from odesat_amd import cnf
from odesat_amd import workloads as wl
from odesat_amd.system import ODESAT_STOP_ANY, ODESAT_STOP_EACH, ODESAT_STOP_NONE, Solver
from oracle import oracle as orc
from tests.common import oracle_formula, read

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def same(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    return np.array_equal(na, nb) and np.array_equal(a[~na].view(np.uint64), b[~nb].view(np.uint64))


def product_formula(name):
    _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(read(name)))
    return f


def results_equal(r1, s1, r2, s2):
    assert np.array_equal(r1["first_sat_step"], r2["first_sat_step"])
    assert np.array_equal(r1["steps_done"], r2["steps_done"])
    assert same(r1["dt"], r2["dt"])
    for x, y in zip(s1, s2):
        assert same(x, y)


# ------------------------------------------------------------------------------- continue ---
@pytest.mark.parametrize("prec", ["f64", "f32"])
@pytest.mark.parametrize("adaptive", [False, True])
def test_continue_equals_one_call(prec, adaptive):
    """simulate(300) == simulate(100) + continue(100) + continue(100): states, run-relative sat
    steps, cumulative steps, adaptive dt; replicas frozen in an earlier call stay frozen."""
    f = product_formula("easy")
    kw = dict(adaptive=adaptive, dt=0.1, tol=1e-3, stop=ODESAT_STOP_EACH, poll_interval=9)
    with Solver(f, 24, prec) as s:
        s.init_state(42)
        r1 = s.simulate(max_steps=300, **kw)
        s1 = s.get_state()
    with Solver(f, 24, prec) as s:
        s.init_state(42)
        s.simulate(max_steps=100, **kw)
        s.simulate(max_steps=100, resume=True, **kw)
        r2 = s.simulate(max_steps=100, resume=True, **kw)
        s2 = s.get_state()
    assert (r1["first_sat_step"] >= 0).any()
    results_equal(r1, s1, r2, s2)


@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
@pytest.mark.parametrize("stop", [0, 1])
def test_run_abi_unbounded_in_small_chunks_matches_oracle(xp, mode, stop):
    """odesat_run with max_steps = 0 (None) forced into 7-step calls (knob RUN_CHUNK) equals the
    oracle's continuous run (oc32_run): adaptive dt is not reset between calls."""
    xp.set("RUN_CHUNK", "7")
    f = oracle_formula("easy")
    n, cp = f.varnum, np.asarray(f.clause_ptr, np.int32)
    lits = (np.asarray(f.var, np.int32) << 1) | np.asarray(f.neg, np.int32)
    B = 12
    o = orc.Oracle(f.clause_ptr, f.var, f.neg, n, "f32")
    v = orc.init_voltages(42, 0, B, n).astype(np.float32).T.copy()
    xs = np.tile(o.init_short_term_memory()[:, None], (1, B)).astype(np.float32)
    xl = np.ones((len(cp) - 1, B), np.float32)
    p = _lib.Params(1 if mode == "adaptive" else 0, stop, 1e-3, 0.1, -1.0, 0, 0, 0)
    L = _lib.lib()
    fp = lambda a: a.ctypes.data_as(C.POINTER(C.c_float))  # noqa: E731
    err = C.create_string_buffer(256)
    ctx = L.odesat_create(0, n, len(cp) - 1, cp.ctypes.data_as(C.POINTER(C.c_int32)),
                          lits.ctypes.data_as(C.POINTER(C.c_int32)), err, 256)
    assert ctx, err.value
    try:
        gv, gxs, gxl = np.empty_like(v), np.empty_like(xs), np.empty_like(xl)
        sat, done = np.zeros(B, np.int64), np.zeros(B, np.int64)
        _lib.check(L.odesat_run(ctx, C.byref(p), B, fp(v), fp(xs), fp(xl), fp(gv), fp(gxs), fp(gxl),
                                _lib.i64ptr(sat), _lib.i64ptr(done)))
    finally:
        L.odesat_destroy(ctx)
    ov, oxs, oxl, osat, odone = orc.run(n, cp, lits, p, v, xs, xl, "f32")
    assert odone.max() > 7  # several bounded calls
    assert np.array_equal(sat, osat) and np.array_equal(done, odone)
    assert np.array_equal(gv, ov) and np.array_equal(gxs, oxs) and np.array_equal(gxl, oxl)


# ---------------------------------------------------------------------- STOP_ANY replay ---
# (algorithm, WAVE knob, RES_NARROW knob, precision, adaptive)
REPLAY = [
    ("onchip", "0", "0", "f32", False),      # k_onchip, out-of-place launches
    ("wave", "1", "1", "f32", False),        # k_wave
    ("wave", "1", "1", "f64", True),         # k_wave adaptive (per-replica dt restored on replay)
    ("resident", "0", "0", "f64", False),    # k_resident fixed, 512-lane tiles
    ("resident", "0", "1", "f32", False),    # k_resident fixed, one-wave tiles
    ("resident", "0", "0", "f64", True),     # k_resident adaptive: one step per launch
]


@pytest.mark.parametrize("alg,wave,narrow,prec,adaptive", REPLAY)
def test_inter_multistep_launches_equal_lockstep(xp, alg, wave, narrow, prec, adaptive):
    """STOP_ANY with 500-step launches: the first allsat step falls inside a launch, the replicas
    that ran past it are replayed to it.  Same stop step, winner and EVERY replica's state as
    FUSED's one-launch-per-step run (and, fixed step, as the oracle's simulate_inter)."""
    f = product_formula("easy")
    B = 40
    kw = dict(adaptive=adaptive, dt=0.1, tol=1e-3, max_steps=6000, stop=ODESAT_STOP_ANY)
    xp.set("WAVE", wave)
    xp.set("RES_NARROW", narrow)
    with Solver(f, B, prec) as s:
        want = {"onchip": _lib.ODESAT_ALG_ONCHIP}.get(alg, _lib.ODESAT_ALG_RESIDENT)
        if s.algorithm != want:
            s.set_algorithm(want)
        s.init_state(4)
        r1 = s.simulate(poll_interval=500, **kw)
        s1 = s.get_state()
    xp.delete("WAVE")
    xp.delete("RES_NARROW")
    with Solver(f, B, prec) as s:
        s.set_algorithm(_lib.ODESAT_ALG_FUSED)
        s.init_state(4)
        r2 = s.simulate(poll_interval=500, **kw)
        s2 = s.get_state()
    sat = np.flatnonzero(r1["first_sat_step"] >= 0)
    assert len(sat) >= 1
    T = int(r1["first_sat_step"][sat].min())
    assert T % 500 != 499 and T > 0  # the stop fell inside a launch (a replay happened)
    assert np.all(r1["steps_done"] == T + 1)
    results_equal(r1, s1, r2, s2)
    if not adaptive:
        o = orc.Oracle(*(lambda g: (g.clause_ptr, g.var, g.neg, g.varnum))(oracle_formula("easy")), prec)
        Tt = np.float64 if prec == "f64" else np.float32
        v = orc.init_voltages(4, 0, B, o.n).astype(Tt)
        xs = np.tile(o.init_short_term_memory(), (B, 1))
        xl = np.ones((B, o.m), Tt)
        t, win, _, _ = o.simulate_inter(v, xs, xl, dt=Tt(0.1), steps=6000)
        assert t == T + 1 and win == int(sat[0])
        assert same(s1[0], v) and same(s1[1], xs) and same(s1[2], xl)


def test_set_state_ends_a_stopped_inter_run(xp):
    """a STOP_ANY run that stopped, then odesat_set_state with states outside ONCHIP's
    range.  set_state ends the run (and its stop word), so a continue runs its steps (it returned 0
    before) and does not mark the state in range; a fresh simulate then takes its first step on the
    clamping kernel.  Both equal the oracle's simulate_inter from the same states."""
    f = product_formula("easy")
    B = 40
    o = orc.Oracle(*(lambda g: (g.clause_ptr, g.var, g.neg, g.varnum))(oracle_formula("easy")), "f32")
    rng = np.random.default_rng(5)
    v = rng.uniform(-1.5, 1.5, (B, o.n)).astype(np.float32)
    xs = rng.uniform(-0.5, 1.5, (B, o.m)).astype(np.float32)
    xl = rng.uniform(0.5, 3.0, (B, o.m)).astype(np.float32)
    kw = dict(dt=0.1, max_steps=30, stop=ODESAT_STOP_ANY, poll_interval=30)
    xp.set("WAVE", "0")  # one replica per group, as ONCHIP needs (REPLAY above)
    xp.set("RES_NARROW", "0")
    with Solver(f, B, "f32") as s:
        s.set_algorithm(_lib.ODESAT_ALG_ONCHIP)
        s.init_state(4)
        r = s.simulate(dt=0.1, max_steps=6000, stop=ODESAT_STOP_ANY, poll_interval=500)
        assert (r["first_sat_step"] >= 0).any()
        s.set_state(v, xs, xl)
        rc = s.simulate(resume=True, **kw)
        sc = s.get_state()
        s.set_state(v, xs, xl)
        rf = s.simulate(**kw)
        sf = s.get_state()
    ov, oxs, oxl = v.copy(), xs.copy(), xl.copy()
    t, _, _, _ = o.simulate_inter(ov, oxs, oxl, dt=np.float32(0.1), steps=30)
    assert t > 0 and rc["steps_run"] == t and rf["steps_run"] == t
    for got in (sc, sf):
        assert same(got[0], ov) and same(got[1], oxs) and same(got[2], oxl)


def test_onchip_inter_at_config2_size_stop_none_equivalent():
    """Config 2's instance, B = 64, STOP_ANY in one 40-step launch with no replica satisfied: the same
    states as STOP_NONE (the out-of-place launch and its parity flip change nothing)."""
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    out = []
    for stop in (ODESAT_STOP_ANY, ODESAT_STOP_NONE):
        with Solver(f, 64, "f32") as s:
            assert s.algorithm == _lib.ODESAT_ALG_ONCHIP
            s.init_state(42)
            r = s.simulate(dt=0.01, max_steps=40, stop=stop, poll_interval=40)
            out.append((r, s.get_state()))
    assert np.all(out[0][0]["first_sat_step"] == -1)
    results_equal(out[0][0], out[0][1], out[1][0], out[1][1])


# ------------------------------------------------------------------- checkpoint / rollback ---
@pytest.mark.parametrize("prec", ["f32", "f64"])
def test_checkpoint_rollback_replays_identically(prec):
    f = product_formula("rand200")
    kw = dict(adaptive=prec == "f64", dt=0.05, tol=1e-3, stop=ODESAT_STOP_EACH, poll_interval=6)
    with Solver(f, 70, prec) as s:
        s.init_state(8)
        s.simulate(max_steps=30, **kw)
        s.checkpoint()
        ra = s.simulate(max_steps=40, resume=True, **kw)
        sa = s.get_state()
        s.rollback()
        rb = s.simulate(max_steps=40, resume=True, **kw)
        sb = s.get_state()
    results_equal(ra, sa, rb, sb)


def test_rollback_without_checkpoint_fails():
    with Solver(product_formula("small"), 2, "f32") as s:
        with pytest.raises(_lib.OdesatError):
            s.rollback()


# ------------------------------------------------------------------------- host threads ---
def test_two_solvers_from_two_threads():
    """include/odesat.h: one solver per GPU, each driven by its own host thread.  Two solvers (on
    devices 0 and 1 when there are two, else both on device 0) run concurrently -- an ONCHIP instance
    and a k_wave instance, both needing more than 64 KiB of dynamic LDS -- and equal their sequential
    runs bit for bit."""
    ndev = _lib.device_count()
    jobs = [("config2", 0, "f32"), ("rand200", 1 % ndev, "f64")]

    def formula(name):
        if name == "config2":
            c = wl.CONFIGS[name]
            var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
            cp, v_, n_ = wl.formula_arrays(var, neg)
            return cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
        return product_formula(name)

    forms = [formula(j[0]) for j in jobs]

    def run(i, out):
        with Solver(forms[i], 8, jobs[i][2], device=jobs[i][1]) as s:
            s.init_state(3)
            r = s.simulate(dt=0.01, max_steps=30, stop=ODESAT_STOP_NONE, poll_interval=10)
            out[i] = (r, s.get_state())

    seq = [None, None]
    for i in range(2):
        run(i, seq)
    par = [None, None]
    th = [threading.Thread(target=run, args=(i, par)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i in range(2):
        results_equal(seq[i][0], seq[i][1], par[i][0], par[i][1])


# --------------------------------------------------------------------- sharded drivers ---
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _shard_worker(rank, world, port, out, per, seed):
    import torch.distributed as td

    from odesat_amd import sharding
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    td.init_process_group("gloo", rank=rank, world_size=world)
    f = product_formula("easy")
    r0, cnt = sharding.shard_range(rank, world, per)
    res = {}
    with Solver(f, cnt, "f32", device=0) as s:
        s.init_state(seed, replica0=r0)
        win, _ = sharding.run_batch(td, s, r0, dt=0.1, max_steps=3000, poll_interval=100)
        res["batch"] = [win, s.get_state()[0].tolist()]
        s.init_state(seed, replica0=r0)
        (step, rep), ran = sharding.run_inter(td, s, r0, max_steps=6000, chunk=128, dt=0.1)
        res["inter"] = [step, rep, ran, s.get_state()[0].tolist(), s.get_state()[2].tolist()]
    with open(f"{out}.{rank}", "w") as fh:
        json.dump(res, fh)
    td.destroy_process_group()


def test_sharded_device_solvers_two_processes_match_one():
    """Two gloo ranks, each a device solver over its global replicas (sharing the box's GPU): batch
    picks the same lowest satisfying global index and leaves the same per-replica states as one
    process over all replicas; inter stops EVERY replica at the global first allsat step (the
    lagging rank rolls back and re-runs), same winner and states."""
    import tempfile

    import torch.multiprocessing as mp

    from odesat_amd import sharding
    world, per, seed = 2, 6, 13
    out = os.path.join(tempfile.mkdtemp(), "shard")
    mp.spawn(_shard_worker, args=(world, _free_port(), out, per, seed), nprocs=world, join=True)
    ranks = [json.load(open(f"{out}.{r}")) for r in range(world)]
    f = product_formula("easy")
    B = world * per
    with Solver(f, B, "f32") as s:
        s.init_state(seed)
        win, _ = sharding.run_batch(None, s, 0, dt=0.1, max_steps=3000, poll_interval=100)
        vb = s.get_state()[0]
        s.init_state(seed)
        (step, rep), ran = sharding.run_inter(None, s, 0, max_steps=6000, chunk=128, dt=0.1)
        vi, _, xli = s.get_state()
    assert win != sharding.NO_SAT and step != sharding.NO_SAT
    for r, res in enumerate(ranks):
        assert res["batch"][0] == win
        assert same(np.array(res["batch"][1]), vb[r * per:(r + 1) * per])
        assert res["inter"][:3] == [step, rep, ran]
        assert same(np.array(res["inter"][3]), vi[r * per:(r + 1) * per])
        assert same(np.array(res["inter"][4]), xli[r * per:(r + 1) * per])


def _planted_file(tmp_path, n=60, m=240, seed=9):
    var, neg, _ = wl.planted_ksat(n, m, 3, seed)
    p = tmp_path / "planted.cnf"
    p.write_text(wl.to_dimacs(var, neg, n))
    return p


@pytest.mark.parametrize("cmd", [("batch", "-n", "20000"), ("inter",)])
def test_cli_gpus_matches_one_gpu(tmp_path, cmd):
    """`odesat batch|inter --gpus 3` (shards sharing the box's GPU, the hidden --share-devices flag) prints the
    same result and assignment as --gpus 1 (replicas keep their global indices)."""
    p = _planted_file(tmp_path)
    binp = os.path.join(ROOT, "odesat_amd", "bin", "odesat")
    outs = []
    for g in ("1", "3"):
        r = subprocess.run([binp, cmd[0], "-f", str(p), *cmd[1:], "-b", "11", "-s", "0.1", "--seed", "5", "--gpus", g,
                            "--share-devices"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        outs.append(r.stdout)
    assert "satisfies formula: true" in outs[0]
    assert outs[0] == outs[1]
    if cmd[0] == "batch":  # main.rs:279-280 progress line ('\r' reads as a newline in text mode)
        assert "Running simulation 1." in outs[0]
