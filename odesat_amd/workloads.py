"""Seeded synthetic workloads (BASELINE.md "Inputs for configs 2-5").

Uniform random k-SAT: k distinct variables per clause, fair signs, written as DIMACS with no `%`
trailer (the reference's parser panics on SATLIB's `%` line, cnf.rs:160).  Every draw comes from the
same splitmix64 counter hash as the initial voltages, so an instance is a pure function of
(n, m, k, seed) on every machine.
"""
from __future__ import annotations

import numpy as np

# the configs of BASELINE.json (n, m, k, generator seed)
CONFIGS = {
    "config2": dict(n=10_000, m=42_000, k=3, seed=1),
    "config3": dict(n=250, m=1_065, k=3, seed=2),
    "config4": dict(n=50_000, m=210_000, k=3, seed=3),
    "config5": dict(n=1_000_000, m=4_200_000, k=3, seed=4),
}

_SIGN_SALT = 0x5A17_C0DE_0DE5_A7


def _mix64(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash3(seed, a, b):
    """oc_hash3 / the device init_voltage hash, vectorised (uint64 wrap-around arithmetic)."""
    with np.errstate(over="ignore"):
        h = _mix64(np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15))
        a = np.asarray(a, dtype=np.uint64)
        h = _mix64(h ^ (a * np.uint64(0xD1B54A32D192ED03) + np.uint64(0x632BE59BD9B4E019)))
        b = np.asarray(b, dtype=np.uint64)
        h = _mix64(h ^ (b * np.uint64(0x8CB92BA72F3D8DD7) + np.uint64(0x9E3779B97F4A7C15)))
    return h


def random_ksat(n: int, m: int, k: int = 3, seed: int = 1):
    """Returns (var [m, k] int64 in 1..n, neg [m, k] bool)."""
    if k > n:
        raise ValueError("k distinct variables need n >= k")
    c = np.arange(m, dtype=np.uint64)[:, None]
    j = np.arange(k, dtype=np.uint64)[None, :]
    var = (hash3(seed, c, j) % np.uint64(n)).astype(np.int64) + 1
    attempt = 1
    while True:
        srt = np.sort(var, axis=1)
        dup_rows = np.flatnonzero((srt[:, 1:] == srt[:, :-1]).any(axis=1))
        if len(dup_rows) == 0:
            break
        for col in range(1, k):  # redraw a column that repeats an earlier one
            rows = dup_rows[(var[dup_rows, col][:, None] == var[dup_rows, :col]).any(axis=1)]
            if len(rows):
                draw = hash3(seed, rows.astype(np.uint64), np.uint64(attempt * k + col))
                var[rows, col] = (draw % np.uint64(n)).astype(np.int64) + 1
        attempt += 1
    neg = (hash3(seed ^ _SIGN_SALT, c, j) >> np.uint64(63)).astype(bool)
    return var, neg


def to_dimacs(var, neg, n: int, comment: str | None = None) -> str:
    m, k = var.shape
    lits = np.where(neg, -var, var)
    head = f"c {comment}\n" if comment else ""
    body = "\n".join(" ".join(map(str, row)) + " 0" for row in lits.tolist())
    return f"{head}p cnf {n} {m}\n{body}\n"


def formula_arrays(var, neg):
    """Normalised 0-based CSR (clause_ptr, var, neg) for a dense instance (all of 1..n used or not,
    names are kept: variable i -> index i-1, which the ascending renaming reproduces when every
    variable occurs)."""
    m, k = var.shape
    return (np.arange(m + 1, dtype=np.int64) * k, (var - 1).reshape(-1).astype(np.int64),
            neg.reshape(-1).astype(np.uint8))


def init_voltages(seed: int, replica0: int, count: int, n: int) -> np.ndarray:
    """Initial voltages v ~ U[-1, 1) of replicas replica0 .. replica0+count-1 ([count, n] f64): the
    counter RNG the device uses (kernels.hpp init_voltage; main.rs:171 maps rand's f64 the same way,
    (u64 >> 11) * 2^-53 * 2 - 1)."""
    r = np.arange(replica0, replica0 + count, dtype=np.uint64)[:, None]
    i = np.arange(n, dtype=np.uint64)[None, :]
    h = hash3(seed, r, i)
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0) * 2.0 - 1.0


def planted_ksat(n: int, m: int, k: int = 3, seed: int = 1, plant_seed: int = 7):
    """random_ksat(n, m, k, seed) made satisfiable by a planted assignment: every clause that the
    assignment star (bool[n], star[i] = value of variable i+1; counter hash of plant_seed) falsifies
    gets the sign of one literal (position chosen by the hash) flipped.  Returns (var, neg, star)."""
    var, neg = random_ksat(n, m, k, seed)
    star = (hash3(plant_seed, np.arange(n, dtype=np.uint64), np.uint64(0)) >> np.uint64(63)).astype(bool)
    bad = np.flatnonzero(~(star[var - 1] != neg).any(axis=1))
    j = (hash3(plant_seed, bad.astype(np.uint64), np.uint64(1)) % np.uint64(k)).astype(np.int64)
    neg = neg.copy()
    neg[bad, j] = ~neg[bad, j]
    return var, neg, star
