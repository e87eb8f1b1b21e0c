"""Read the k_onchip stamp sums of a diagnostic build (scripts/build_variant.sh NAME -DONCHIP_STAMPS=1|2;
run with XP_LIB=expt/libNAME.so): per tile and wave, cycles waiting at the barrier vs working
before it (and, build 2, the dv read-modify-write at the tile's start).  Config 2, B = 256 (one round
of workgroups), one launch of STEPS steps.  Shares only: the stamps drain LDS operations."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import _lib, cnf, workloads as wl
from odesat_amd.system import ODESAT_STOP_NONE, Solver

c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
B, K = 256, int(os.environ.get("STEPS", "20"))
with Solver(f, B, "f32") as s:
    assert s.algorithm == _lib.ODESAT_ALG_ONCHIP
    s.init_state(42)
    s.simulate(dt=0.01, max_steps=1, stop=ODESAT_STOP_NONE)  # the first step of a call on a fresh state runs RESIDENT
    s.simulate(dt=0.01, max_steps=K, stop=ODESAT_STOP_NONE, poll_interval=K)
    s.synchronize()
    buf = np.zeros(4096 * 16 * 4, np.uint64)
    fn = _lib.lib().odesat_onchip_stamps
    fn.argtypes = [C.c_void_p, C.c_int]
    assert fn(buf.ctypes.data, buf.size) == 0
st = buf.reshape(4096, 16, 4)[:B, :8].astype(np.float64)
tiles = st[..., 3]
assert (tiles == tiles[0, 0]).all() and tiles[0, 0] > 0, np.unique(tiles)
per = st[..., :3] / tiles[..., None]  # [B, wave, (bar, work, rmw)] cycles per tile
tot = per[..., 0] + per[..., 1]
print(f"tiles per wave {tiles[0, 0]:.0f} ({K} steps); cycles per tile, mean over replicas:")
for w in range(8):
    print(f"  wave {w}: barrier {per[:, w, 0].mean():6.1f}  work {per[:, w, 1].mean():6.1f}"
          + (f" (of which dv RMW {per[:, w, 2].mean():6.1f})" if per[..., 2].any() else "")
          + f"  total {tot[:, w].mean():6.1f}")
print(f"all waves: barrier {per[..., 0].mean():.1f}  work {per[..., 1].mean():.1f}  rmw {per[..., 2].mean():.1f}"
      f"  min-barrier wave share of work {per[..., 1].max(axis=1).mean():.1f}")
