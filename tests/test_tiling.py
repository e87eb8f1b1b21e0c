"""The wave-paired clause tiling of k_onchip (odesat_hip.hip pair_tiles), checked on
the CPU through the library's test hook odesat_debug_pair_tiles.  A tiling that let two waves touch
one dv entry inside a barrier interval would race on the GPU without failing reliably, so its
invariants are checked directly:
  * a tile holds at most 64 clauses per wave (8 waves, 512 slots);
  * a tile is var-disjoint, and every variable's tiles increase in the reference's clause order
    (system.rs:80's left fold, as for the plain tiles);
  * a clause in the same barrier interval -- tiles 2i - off, 2i + 1 - off -- as the previous clause of
    one of its variables is in that clause's wave (LDS operations of one wave complete in order)."""
import ctypes as C

import numpy as np
import pytest

from odesat_amd import _lib, cnf
from odesat_amd import workloads as wl


def pair_tiles(f, m, off):
    t = np.zeros(m, np.int32)
    w = np.zeros(m, np.int8)
    nt = C.c_int32(0)
    fn = _lib.lib().odesat_debug_pair_tiles
    fn.argtypes = [C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_void_p]
    _lib.check(fn(f._h, off, t.ctypes.data, w.ctypes.data, C.byref(nt)))
    return t, w, nt.value


def check_invariants(var, m, off, t, w, nt):
    assert nt == (int(t.max()) + 1 if m else 0)
    assert (w >= 0).all() and (w < 8).all()
    cnt = np.zeros((max(nt, 1), 8), np.int64)
    np.add.at(cnt, (t, w), 1)
    assert cnt.max(initial=0) <= 64
    iv = (t + off) // 2
    last = {}
    seen = {}
    for c in range(m):
        vs = set(var[c])
        for v in vs:
            key = (int(t[c]), v)
            assert key not in seen, f"tile {t[c]} holds variable {v} twice (clauses {seen.get(key)} and {c})"
            seen[key] = c
            p = last.get(v)
            if p is not None:
                assert t[p] < t[c], f"variable {v}: clause {c} (tile {t[c]}) not after clause {p} (tile {t[p]})"
                if iv[p] == iv[c]:
                    assert w[p] == w[c], f"clauses {p}, {c} share variable {v} inside interval {iv[c]} on waves {w[p]}, {w[c]}"
            last[v] = c


def formula(var, neg, n):
    cp, v_, n_ = wl.formula_arrays(np.asarray(var), np.asarray(neg))
    return cnf.CNFFormula.from_arrays(cp, v_, n_, n)


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("n,m,seed", [(50, 200, 1), (300, 1265, 2), (2000, 8400, 3), (20, 400, 4)])
def test_random_3sat_pair_tiling_invariants(n, m, seed, off):
    var, neg = wl.random_ksat(n, m, 3, seed)
    f = formula(var, neg, n)
    t, w, nt = pair_tiles(f, m, off)
    check_invariants((var - 1).tolist(), m, off, t, w, nt)


@pytest.mark.parametrize("off", [0, 1])
def test_star_and_repeated_variable_pair_tiling(off):
    # every clause holds variable 0 (one chain: one clause per tile), some a variable twice
    rng = np.random.default_rng(5)
    n, m = 40, 150
    var = np.stack([np.zeros(m, np.int64), rng.integers(1, n, m), rng.integers(1, n, m)], 1)
    neg = rng.integers(0, 2, (m, 3)).astype(bool)
    f = formula(var + 1, neg, n)
    t, w, nt = pair_tiles(f, m, off)
    check_invariants(var.tolist(), m, off, t, w, nt)
    assert nt >= m  # variable 0's clauses are a chain of m tiles


def test_config2_pair_tiling_depth():
    """config 2 (n = 10 000, m = 42 000) needs 91 tiles at offset 0, 90 at offset 1
    (the solver keeps offset 1: k_onchip<90, 1>, 46 barrier intervals)."""
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    f = formula(var, neg, c["n"])
    res = {}
    for off in (0, 1):
        t, w, nt = pair_tiles(f, c["m"], off)
        res[off] = nt
        check_invariants((var - 1).tolist(), c["m"], off, t, w, nt)
    assert res == {0: 91, 1: 90}


def test_empty_formula_and_bad_arguments():
    f = cnf.CNFFormula.from_arrays(np.zeros(1, np.int64), np.zeros(0, np.int64), np.zeros(0, np.uint8), 3)
    t, w, nt = pair_tiles(f, 0, 0)
    assert nt == 0
    with pytest.raises(Exception):
        pair_tiles(f, 0, 2)
