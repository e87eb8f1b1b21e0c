"""Fixed workload for rocprofv3 counter passes: config-2 instance (CONFIG), B replicas, K fixed steps
(ADAPTIVE=1: adaptive steps, tol 1e-3) in one launch, DTYPE f32 / f64, ALG forces an algorithm."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402

B = int(os.environ.get("B", "1024"))
K = int(os.environ.get("STEPS", "20"))
CHUNK = int(os.environ.get("CHUNK", "0"))
SCHED = int(os.environ.get("SCHED", "0"))
c = wl.CONFIGS[os.environ.get("CONFIG", "config2")]
var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
cp, v_, n_ = wl.formula_arrays(var, neg)
f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
with Solver(f, B, os.environ.get("DTYPE", "f32")) as s:
    if CHUNK:
        s.set_chunk_replicas(CHUNK)
    s.set_schedule(SCHED)
    if "ALG" in os.environ:
        s.set_algorithm(int(os.environ["ALG"]))
    s.init_state(42)
    s.simulate(adaptive=os.environ.get("ADAPTIVE", "0") == "1", dt=0.01, tol=1e-3, max_steps=K, stop=ODESAT_STOP_NONE,
               poll_interval=K)  # one launch of K steps
    s.synchronize()
print("done", B, K, CHUNK, SCHED)
