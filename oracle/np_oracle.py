"""Independent numpy restatement of /root/reference/src/system.rs (f64 or f32).

TEST INFRASTRUCTURE ONLY.  Written separately from the C oracle (oracle/odesat_oracle.c) so the two
can cross-check each other bit for bit; it generates the committed golden fixtures
(tests/golden/make_golden.py).  Vectorised over clauses; the dv scatter uses np.add.at, which applies
the additions one index at a time in array order -- the reference's clause-ascending, literal-order
accumulation (system.rs:35,62,80).
"""
from __future__ import annotations

import numpy as np

ALPHA, BETA, GAMMA, DELTA, EPSILON = 5.0, 20.0, 0.25, 0.05, 0.001  # system.rs:19-23


class Formula:
    """Clause->literal CSR (file order).  var: 0-based normalised variables."""

    def __init__(self, clause_ptr, var, neg, varnum):
        self.clause_ptr = np.asarray(clause_ptr, dtype=np.int64)
        self.var = np.asarray(var, dtype=np.int64)
        self.neg = np.asarray(neg, dtype=bool)
        self.varnum = int(varnum)
        self.m = len(self.clause_ptr) - 1
        widths = np.diff(self.clause_ptr)
        self.K = int(widths.max()) if self.m else 0
        # padded [m, K] views (mask = slot exists)
        self.mask = np.arange(self.K)[None, :] < widths[:, None]
        idx = np.where(self.mask, self.clause_ptr[:-1, None] + np.arange(self.K)[None, :], 0)
        self.pvar = np.where(self.mask, self.var[idx] if len(self.var) else 0, 0)
        self.pneg = np.where(self.mask, self.neg[idx] if len(self.neg) else False, False)

    @classmethod
    def from_clauses(cls, clauses, varnum):
        ptr = [0]
        var, neg = [], []
        for c in clauses:
            for v, n in c:
                var.append(v)
                neg.append(bool(n))
            ptr.append(len(var))
        return cls(ptr, var, neg, varnum)


def compute_derivatives(f: Formula, v, xs, xl, zeta, dt=np.float64):
    """system.rs:25-91 -> (dv, dxs, dxl, allsat, r_fired)."""
    T = dt
    one, half = T(1.0), T(0.5)
    dv = np.zeros(f.varnum, dtype=T)
    mn = np.full(f.m, np.inf, dtype=T)
    second = np.full(f.m, np.inf, dtype=T)
    q = np.where(f.pneg, T(-1.0), T(1.0)).astype(T)
    vals = (one - q * v[f.pvar]).astype(T)  # [m, K]
    for j in range(f.K):  # :46-57 strict-< min / second-min, literal order
        val = vals[:, j]
        ok = f.mask[:, j]
        lt_min = ok & (val < mn)
        lt_sec = ok & ~lt_min & (val < second)
        second = np.where(lt_min, mn, np.where(lt_sec, val, second))
        mn = np.where(lt_min, val, mn)
    c_m = (half * mn).astype(T)  # :60
    sel = np.where(vals != mn[:, None], mn[:, None], second[:, None])
    g = ((half * q) * sel).astype(T)  # :64-70
    vi = v[f.pvar]
    r = np.where(c_m[:, None] == (one - q * vi), half * (q - vi), T(0.0)).astype(T)  # :73-77
    t1 = (xl[:, None] * xs[:, None]) * g
    t2 = ((one + T(zeta) * xl)[:, None] * (one - xs)[:, None]) * r
    contrib = (t1 + t2).astype(T)
    np.add.at(dv, f.pvar[f.mask], contrib[f.mask])  # :80 row-major = clause, then literal order
    dxs = (T(BETA) * (xs + T(EPSILON)) * (c_m - T(GAMMA))).astype(T)  # :84
    dxl = (T(ALPHA) * (c_m - T(DELTA))).astype(T)  # :85
    allsat = bool(np.all(c_m < T(GAMMA))) if f.m else True
    return dv, dxs, dxl, allsat, int(np.count_nonzero(r[f.mask]))


def update_state(f: Formula, v, xs, xl, dv, dxs, dxl, h):
    """system.rs:93-97 (in place)."""
    T = v.dtype.type
    xs[:] = np.fmin(np.fmax(xs + T(h) * dxs, T(EPSILON)), T(1.0) - T(EPSILON))
    xl[:] = np.fmin(np.fmax(xl + T(h) * dxl, T(1.0)), T(1e4) * T(f.m))
    v[:] = np.fmin(np.fmax(v + T(h) * dv, T(-1.0)), T(1.0))


def max_error(a, b):
    """system.rs:99-109: NaN-seeded fold of f64::max (np.fmax ignores NaN)."""
    T = a[0].dtype.type
    out = T(np.nan)
    for x, y in zip(a, b):
        e = np.fmax.reduce(np.abs(x - y), initial=T(np.nan)) if len(x) else T(np.nan)
        out = e if np.isnan(out) else (out if np.isnan(e) else max(out, e))
    return T(out)


def euler_step(f, v, xs, xl, tol, h, zeta):
    """system.rs:111-139 -> (allsat, new dt)."""
    T = v.dtype.type
    dv, dxs, dxl, allsat, _ = compute_derivatives(f, v, xs, xl, zeta, T)
    if not allsat:
        t = (v.copy(), xs.copy(), xl.copy())
        update_state(f, *t, dv, dxs, dxl, h)
        update_state(f, v, xs, xl, dv, dxs, dxl, T(0.5) * T(h))
        dv, dxs, dxl, _, _ = compute_derivatives(f, v, xs, xl, zeta, T)
        update_state(f, v, xs, xl, dv, dxs, dxl, T(0.5) * T(h))
        err = max_error(t, (v, xs, xl))
        with np.errstate(divide="ignore", invalid="ignore"):
            h = np.fmax(np.fmin(T(h) * np.sqrt(T(tol) / err), T(1e3)), T(2.0 ** -7))
    return allsat, T(h)


def euler_step_fixed(f, v, xs, xl, h, zeta):
    """system.rs:141-154."""
    T = v.dtype.type
    dv, dxs, dxl, allsat, _ = compute_derivatives(f, v, xs, xl, zeta, T)
    update_state(f, v, xs, xl, dv, dxs, dxl, h)
    return allsat


def default_zeta(f):
    d = f.m / f.varnum
    return 0.1 if d >= 6.0 else (0.01 if d >= 4.9 else 0.001)


def simulate(f, v, xs, xl, tol=None, dt=None, steps=0, zeta=None):
    """system.rs:156-239 with a bounded step count -> (steps_taken, sat, assignment, final dt)."""
    T = v.dtype.type
    z = default_zeta(f) if zeta is None else zeta
    tolv = 1e-3 if tol is None else tol
    h = T(0.01)
    for k in range(steps):
        if dt is not None:
            if euler_step_fixed(f, v, xs, xl, T(dt), z):
                return k + 1, True, v > 0, h
        else:
            sat, h = euler_step(f, v, xs, xl, tolv, h, z)
            if sat:
                return k + 1, True, v > 0, h
    return steps, False, v > 0, h


def init_short_term_memory(f, dtype=np.float64):
    """system.rs:361-372."""
    return np.where((f.pneg & f.mask).any(axis=1), 1.0, -1.0).astype(dtype)


# ---- counter RNG (same function as oracle/odesat_oracle.c oc_hash3 and the GPU) ----
_M64 = (1 << 64) - 1


def _mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def hash3(seed, replica, var):
    with np.errstate(over="ignore"):
        h = _mix64(np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15))
        r = np.asarray(replica, dtype=np.uint64)
        h = _mix64(h ^ (r * np.uint64(0xD1B54A32D192ED03) + np.uint64(0x632BE59BD9B4E019)))
        x = np.asarray(var, dtype=np.uint64)
        h = _mix64(h ^ (x * np.uint64(0x8CB92BA72F3D8DD7) + np.uint64(0x9E3779B97F4A7C15)))
    return h


def init_voltages(seed, r0, B, n):
    """[B, n] f64: (u64 >> 11) * 2^-53 * 2 - 1 (rand 0.8 Standard f64 mapping, main.rs:171)."""
    r = np.arange(r0, r0 + B, dtype=np.uint64)[:, None]
    i = np.arange(n, dtype=np.uint64)[None, :]
    u = (hash3(seed, r, i) >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)
    return u * 2.0 - 1.0
