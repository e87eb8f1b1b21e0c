import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from odesat_amd import cnf
from odesat_amd.system import ODESAT_STOP_NONE, Solver
_, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(open(os.path.join(ROOT, "tests/golden/hard.cnf")).read()))
for dt in ("f32", "f64"):
    with Solver(f, 1, dt) as s:
        s.init_state(42)
        s.simulate(dt=0.01, max_steps=2000, stop=ODESAT_STOP_NONE, poll_interval=2000)
        s.synchronize()
        t0 = time.perf_counter()
        s.simulate(dt=0.01, max_steps=2000, stop=ODESAT_STOP_NONE, poll_interval=2000)
        s.synchronize()
        print(dt, "alg", s.algorithm, "us/step", (time.perf_counter() - t0) / 2000 * 1e6, flush=True)
