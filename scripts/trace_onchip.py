"""Per-tile timeline of k_onchip (experiment build with -DONCHIP_TRACE, scripts/build_variant.sh TR).

  ODESAT_LIB=$PWD/expt/libTR.so python scripts/trace_onchip.py

Runs config 2 at B=1024 for one 50-step launch and prints, per wave of block 0, the mean cycles
(s_memtime) of each phase of a tile step over tiles 8..87 of the last step:
  read   = barrier -> dv reads returned;   work = -> back/front issued and every LDS op drained;
  wait   = -> barrier released.
"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from odesat_amd import _lib, cnf
    from odesat_amd import workloads as wl
    from odesat_amd.system import ODESAT_STOP_NONE, Solver
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], 3, c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    with Solver(f, 1024, "f32") as s:
        s.init_state(42)
        s.simulate(dt=0.01, max_steps=50, stop=ODESAT_STOP_NONE, poll_interval=50)
        s.simulate(dt=0.01, max_steps=50, stop=ODESAT_STOP_NONE, poll_interval=50)
        s.synchronize()
    L = _lib.lib()
    buf = np.zeros((8, 128, 4), np.uint64)
    L.onchip_trace_read.argtypes = [C.c_void_p]
    assert L.onchip_trace_read(buf.ctypes.data) == 0
    t = buf[:, 8:88, :].astype(np.int64)
    read = t[:, :, 1] - t[:, :, 0]
    work = t[:, :, 2] - t[:, :, 1]
    wait = t[:, :, 3] - t[:, :, 2]
    total = t[:, 1:, 0] - t[:, :-1, 0]
    print("wave  read  work  wait  tile(total)")
    for w in range(8):
        print(f"{w:4d} {read[w].mean():6.0f} {work[w].mean():6.0f} {wait[w].mean():6.0f} {total[w].mean():8.0f}")
    print("all ", f"{read.mean():6.0f} {work.mean():6.0f} {wait.mean():6.0f} {total.mean():8.0f}")
    print("percentiles of tile total:", np.percentile(total, [10, 50, 90]).round())
    np.save("gpurun_out/trace_onchip.npy", buf)


if __name__ == "__main__":
    main()
