"""Size boundaries of the on-chip kernels (edge cases at their maximum sizes, round 6).

k_onchip keeps a replica's voltages and their sinks below the 16-bit LDS immediate DVC (onchip.hpp
MAX_N = 65 520 / 4 - 32 = 16 348 variables), and its adaptive step keeps four voltage arrays of
40 960 bytes, the first also holding the flags and the waves' error and pair words (ADA_MAX_N =
10 240 - 32 - 26 = 10 182).  At the largest n each kernel admits, and one variable past it -- where the
solver must fall back to k_resident -- every replica's state after a few steps equals the oracle's f32
restatement bit for bit (system.rs:111-154), and the two sides of the adaptive boundary agree with
k_resident's adaptive step run on the same instance (knob ONCHIP_ADAPTIVE = 0)."""
import numpy as np
import pytest

from odesat_amd import cnf
from odesat_amd import workloads as wl
from odesat_amd.system import ODESAT_STOP_NONE, Solver
from oracle.oracle import Oracle, init_voltages

pytestmark = pytest.mark.gpu

MAX_N = 65520 // 4 - 32            # onchip.hpp MAX_N
ADA_MAX_N = 40960 // 4 - 32 - 26   # onchip.hpp ADA_MAX_N (ADA_FLAGS = 2 + 3 * 8 waves)


def same(a, b):
    """Bit-equal as f64 (the f32 states widen exactly; no state here is NaN)."""
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return a.shape == b.shape and np.array_equal(a.view(np.uint64), b.view(np.uint64))


def _instance(n, m, seed):
    var, neg = wl.random_ksat(n, m, 3, seed)
    cp, v_, n_ = wl.formula_arrays(var, neg)
    return cnf.CNFFormula.from_arrays(cp, v_, n_, n), (cp, v_, n_)


def _oracle_states(cp, v_, n_, n, m, B, seed, steps, adaptive):
    o = Oracle(cp, v_, n_, n, "f32")
    out = []
    for b in range(B):
        ov = init_voltages(seed, b, 1, n)[0].astype(np.float32)
        oxs, oxl = o.init_short_term_memory(), np.ones(m, np.float32)
        t, _, _, h, _ = o.simulate(ov, oxs, oxl, tol=np.float32(1e-3) if adaptive else None,
                                   dt=None if adaptive else np.float32(0.05), steps=steps, zeta=np.float32(0.001))
        out.append((t, h, ov, oxs, oxl))
    return out


@pytest.mark.parametrize("n,kernel", [(MAX_N, "k_onchip"), (MAX_N + 1, "k_resident")])
def test_fixed_steps_at_the_onchip_size_limit(n, kernel):
    """Fixed steps at n = MAX_N (k_onchip, 62 tiles all in VGPRs) and MAX_N + 1 (k_resident)."""
    m, B, K = 30000, 3, 6
    f, (cp, v_, n_) = _instance(n, m, 7)
    with Solver(f, B, "f32") as s:
        assert s.step_kernel(False) == kernel
        s.init_state(11)
        r = s.simulate(dt=0.05, max_steps=K, stop=ODESAT_STOP_NONE, zeta=0.001)
        assert np.all(r["steps_done"] == K)
        v, xs, xl = s.get_state()
    for b, (t, _, ov, oxs, oxl) in enumerate(_oracle_states(cp, v_, n_, n, m, B, 11, K, False)):
        assert t == K
        assert same(v[b], ov) and same(xs[b], oxs) and same(xl[b], oxl), f"replica {b}"


@pytest.mark.parametrize("n,kernel", [(ADA_MAX_N, "k_onchip"), (ADA_MAX_N + 1, "k_resident")])
def test_adaptive_steps_at_the_onchip_size_limit(n, kernel, xp):
    """Adaptive steps (tol 1e-3, per-replica dt) at n = ADA_MAX_N (k_onchip's adaptive step, 89-90
    tiles) and ADA_MAX_N + 1 (k_resident's): == k_resident's adaptive step and == the oracle."""
    m, B, K = 42000, 2, 5
    f, (cp, v_, n_) = _instance(n, m, 7)
    res = []
    for ada in (None, "0"):
        xp.set("ONCHIP_ADAPTIVE", ada)
        with Solver(f, B, "f32") as s:
            assert s.step_kernel(True) == (kernel if ada is None else "k_resident")
            s.init_state(11)
            r = s.simulate(adaptive=True, dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_NONE, zeta=0.001)
            assert np.all(r["steps_done"] == K)
            res.append((r, s.get_state()))
    (r1, s1), (r2, s2) = res
    assert same(r1["dt"], r2["dt"]) and all(same(a, b) for a, b in zip(s1, s2))
    for b, (t, h, ov, oxs, oxl) in enumerate(_oracle_states(cp, v_, n_, n, m, B, 11, K, True)):
        assert t == K and same(np.float32(h), np.float32(r1["dt"][b]))
        assert same(s1[0][b], ov) and same(s1[1][b], oxs) and same(s1[2][b], oxl), f"replica {b}"
