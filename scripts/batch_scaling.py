"""One-GPU batch-scaling table (north_star: "near-linear batch scaling"): the headline
path's kernels timed at B in BATCHES with bench.py's own timing (time_gpu: warmup, then one call of
`steps` steps between device syncs; the kernel time from HIP events on the solver's stream), plus the
same call repeated back to back (steady state, the medians of the last half).
    python scripts/batch_scaling.py [--out profiles/r06_batch_scaling.jsonl] [--steps 20 --warmup 5]
Families: config 2 f32 fixed (k_onchip), config 2 f64 fixed (k_resident), config 3 f32 adaptive
(k_wave).  One JSON line per (family, B)."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

BATCHES = (64, 128, 256, 512, 768, 1024, 1280, 2048, 4096)
FAMILIES = (("config2", "f32", False), ("config2", "f64", False), ("config3", "f32", True))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--out", default=os.path.join(ROOT, "profiles", "r06_batch_scaling.jsonl"))
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--steady", type=int, default=6)
    p.add_argument("--batches", default=",".join(map(str, BATCHES)))
    p.add_argument("--families", default="", help="comma-separated config:dtype:mode, default all")
    p.add_argument("--knob", action="append", default=[], metavar="KEY=VALUE", help="experiment knob (A/B)")
    a = p.parse_args()
    import bench
    from odesat_amd import _lib
    for kv in a.knob:
        k, v = kv.split("=", 1)
        _lib.set_experiment(k.strip(), int(v))
    from odesat_amd.system import ODESAT_STOP_NONE, Solver
    fams = FAMILIES
    if a.families:
        fams = [(c, d, m == "adaptive") for c, d, m in (x.split(":") for x in a.families.split(","))]
    batches = [int(x) for x in a.batches.split(",")]
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "a") as fh:
        for config, dtype, adaptive in fams:
            c, _, _, _, f = bench.formula_of(config)
            for B in batches:
                t0 = time.time()
                with Solver(f, B, dtype, device=0) as s:
                    s.init_state(42)
                    wall, ms, launches, ran, (walls, kern) = bench.time_gpu(
                        s, a.steps, a.warmup, None, 0, True, ODESAT_STOP_NONE, adaptive, a.steady)
                    st = bench.steady_state(B, a.steps, walls, kern)
                    rec = {"config": config, "n": c["n"], "m": c["m"], "dtype": dtype,
                           "step": "adaptive tol 1e-3" if adaptive else "fixed dt 0.01", "batch": B,
                           "kernel": s.step_kernel(adaptive), "steps": ran, "warmup": a.warmup,
                           "value": B * ran / wall, "ms_per_step": wall * 1e3 / ran,
                           "kernel_us_per_step": ms[0] * 1e3 / ran,
                           "steady_value": st["value"], "steady_kernel_us_per_step": st["kernel_us_per_call"] / ran,
                           "knobs": a.knob,
                           "date": time.strftime("%Y-%m-%d %H:%M:%S")}
                fh.write(json.dumps(rec) + "\n")
                fh.flush()
                print(f"{config} {dtype} {'ada' if adaptive else 'fix'} B={B:5d} {rec['kernel']:10s} "
                      f"{rec['value'] / 1e6:8.3f} M/s  steady {rec['steady_value'] / 1e6:8.3f} M/s  "
                      f"kernel {rec['kernel_us_per_step']:8.1f} us/step  ({time.time() - t0:.1f} s)", flush=True)


if __name__ == "__main__":
    main()
