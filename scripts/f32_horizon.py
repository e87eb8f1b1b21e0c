import sys, numpy as np
sys.path.insert(0, '/root/repo')
from oracle.oracle import Oracle, init_voltages
from odesat_amd import workloads as wl
c = wl.CONFIGS["config2"]
var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
n, m = c["n"], c["m"]
o64 = Oracle(cp, v_, n_, n, "f64"); o32 = Oracle(cp, v_, n_, n, "f32")
reps = [0, 517, 1023]
B = len(reps)
v64 = np.stack([init_voltages(42, r, 1, n)[0] for r in reps]).astype(np.float32).astype(np.float64)
v32 = v64.astype(np.float32)
xs64 = np.tile(o64.init_short_term_memory(), (B, 1)); xs32 = xs64.astype(np.float32)
xl64 = np.ones((B, m)); xl32 = np.ones((B, m), np.float32)
done = 0
for K in [20, 50, 100, 200, 300, 500, 750, 1000, 1500, 2000]:
    k = K - done
    o64.batch_run(v64, xs64, xl64, False, 1e-3, 0.01, k, 0.001, nthreads=3)
    o32.batch_run(v32, xs32, xl32, False, 1e-3, 0.01, k, 0.001, nthreads=3)
    done = K
    dv = np.abs(v32 - v64).max(); dxs = np.abs(xs32 - xs64).max(); dxl = (np.abs(xl32 - xl64) / xl64).max()
    flips = [(int(((v32[b] > 0) != (v64[b] > 0)).sum())) for b in range(B)]
    near = [(int((np.abs(v64[b]) < 1e-3).sum())) for b in range(B)]
    print(K, f"dv={dv:.3g} dxs={dxs:.3g} dxl_rel={dxl:.3g} flips={flips} near0={near}", flush=True)
