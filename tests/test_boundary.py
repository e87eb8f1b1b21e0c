"""The one-call boundary of SURVEY.md §8(b): odesat_create / odesat_run / odesat_destroy
(odesat_amd/csrc/run_abi.cpp) against the oracle's entry point with the same arguments
(oracle/oracle_body.inc, oc32_run).  States are replica-innermost f32 ([n][B], [m][B]); the bar is
bit-exact states, first sat steps and steps taken, for every stop policy, fixed and adaptive steps,
bounded and unbounded (max_steps = 0, the reference's None)."""
import ctypes as C

import numpy as np
import pytest

from odesat_amd import _lib
from oracle import oracle as orc
from tests.common import oracle_formula


def formula(name):
    f = oracle_formula(name)
    lits = (np.asarray(f.var, np.int32) << 1) | np.asarray(f.neg, np.int32)
    return f.varnum, np.asarray(f.clause_ptr, np.int32), lits, f


def initial(f, B, seed=42):
    o = orc.Oracle(f.clause_ptr, f.var, f.neg, f.varnum, "f32")
    v = orc.init_voltages(seed, 0, B, f.varnum).astype(np.float32).T.copy()          # [n][B]
    xs = np.tile(o.init_short_term_memory()[:, None], (1, B)).astype(np.float32)     # [m][B]
    xl = np.ones((len(f.clause_ptr) - 1, B), np.float32)
    return v, xs, xl


def params(adaptive, stop, max_steps, dt=0.05, dt_policy=0):
    return _lib.Params(adaptive, stop, 1e-3, dt, -1.0, max_steps, 0, dt_policy)


def test_oracle_run_matches_simulate():
    """The oracle's boundary entry equals its per-replica simulate (EACH) on a fixture."""
    n, cp, lits, f = formula("rand200")
    B = 5
    v, xs, xl = initial(f, B)
    ov, oxs, oxl, sat, done = orc.run(n, cp, lits, params(0, 0, 60), v, xs, xl, "f32")
    o = orc.Oracle(f.clause_ptr, f.var, f.neg, n, "f32")
    for b in range(B):
        vb, xsb, xlb = v[:, b].copy(), xs[:, b].copy(), xl[:, b].copy()
        t, s, _, _, _ = o.simulate(vb, xsb, xlb, dt=np.float32(0.05), steps=60)
        assert done[b] == t and sat[b] == (t - 1 if s else -1)
        assert np.array_equal(ov[:, b], vb) and np.array_equal(oxs[:, b], xsb) and np.array_equal(oxl[:, b], xlb)


def test_create_without_device_reports_error():
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    n, cp, lits, _ = formula("small")
    err = C.create_string_buffer(256)
    h = _lib.lib().odesat_create(0, n, len(cp) - 1, cp.ctypes.data_as(C.POINTER(C.c_int32)),
                                 lits.ctypes.data_as(C.POINTER(C.c_int32)), err, 256)
    assert not h and b"device" in err.value


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["easy", "rand200"])
@pytest.mark.parametrize("mode", ["fixed", "adaptive"])
@pytest.mark.parametrize("stop", [0, 1, 2])
@pytest.mark.parametrize("max_steps", [0, 80])
def test_run_bitexact_vs_oracle(name, mode, stop, max_steps):
    if max_steps == 0 and (stop == 2 or name == "rand200"):
        pytest.skip("unbounded runs need a stop policy and a formula the replicas solve quickly")
    n, cp, lits, f = formula(name)
    B = 24
    v, xs, xl = initial(f, B)
    p = params(1 if mode == "adaptive" else 0, stop, max_steps, dt=0.1 if max_steps == 0 else 0.05)
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
        bad = _lib.Params(1, 1, 1e-3, 0.05, -1.0, 10, 0, 1)  # the shared serial dt is the CPU's
        assert L.odesat_run(ctx, C.byref(bad), B, fp(v), fp(xs), fp(xl), None, None, None, None, None) < 0
    finally:
        L.odesat_destroy(ctx)
    ov, oxs, oxl, osat, odone = orc.run(n, cp, lits, p, v, xs, xl, "f32")
    assert np.array_equal(sat, osat) and np.array_equal(done, odone)
    assert np.array_equal(gv, ov) and np.array_equal(gxs, oxs) and np.array_equal(gxl, oxl)
