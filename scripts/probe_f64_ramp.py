"""Probe: why does the f64 leg's 20-step k_resident launch run ~25 % slower per step
than a 200-step one?  Two candidate causes: the GPU's clocks ramping under sustained HBM load (power
management) or first-touch / TLB cost of a fresh solver's buffers.  The probe separates them:

  A  fresh solver (the bench's shape: a 5-step warm-up launch), then 10 back-to-back 20-step launches;
  B  the same solver after 1.5 s idle, then 4 more back-to-back launches (buffers already touched:
     a slow first launch here is a clock effect, not first touch);
  C  a second fresh solver right after B (hot GPU, untouched buffers: a fast first launch here rules
     first touch out);
  D  after 1.5 s idle, 60 launches of 4 f64 steps (the ramp's time course, ~1 ms resolution);
  E  after 1.5 s idle, 60 launches of 4 steps of the f32 headline kernel (k_onchip: compute-bound,
     the state on the CU -- does a kernel that barely touches HBM ramp too?);
  F  after 1.5 s idle, ~100 ms of k_onchip launches, then D's f64 launches (does compute load prime
     the memory-bound kernel?).

Each launch: HIP-event kernel time (the solver's stream) and the host time window.  A sampler thread
reads the current DPM levels (sysfs pp_dpm_sclk / pp_dpm_mclk / pp_dpm_fclk, the '*' line) every
~2 ms; each launch reports the levels seen inside its window.  One JSON line per launch, then a
summary line."""
import glob
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import tooling  # noqa: E402  (XP_LIB / XP_KNOBS: a variant build and experiment knobs)
tooling.apply()
from odesat_amd import cnf  # noqa: E402
from odesat_amd import workloads as wl  # noqa: E402
from odesat_amd.system import ODESAT_STOP_NONE, Solver  # noqa: E402


def dpm_files():
    out = {}
    for card in sorted(glob.glob("/sys/class/drm/card*/device")):
        if os.path.exists(os.path.join(card, "pp_dpm_mclk")):
            for k in ("sclk", "mclk", "fclk", "socclk"):
                p = os.path.join(card, f"pp_dpm_{k}")
                if os.access(p, os.R_OK):
                    out[k] = p
            break
    return out


def current(path):
    try:
        with open(path) as fh:
            for line in fh:
                if line.rstrip().endswith("*"):
                    return line.split(":", 1)[1].strip().rstrip("*").strip()
    except OSError:
        return None
    return None


class Sampler(threading.Thread):
    def __init__(self, files, period=0.002):
        super().__init__(daemon=True)
        self.files, self.period, self.samples, self.stop = files, period, [], False

    def run(self):
        while not self.stop:
            t = time.perf_counter()
            self.samples.append((t, {k: current(p) for k, p in self.files.items()}))
            time.sleep(self.period)

    def levels(self, t0, t1):
        seen = {}
        for t, d in self.samples:
            if t0 <= t <= t1:
                for k, v in d.items():
                    seen.setdefault(k, {}).setdefault(v, 0)
                    seen[k][v] += 1
        return seen


def main():
    c = wl.CONFIGS["config2"]
    var, neg = wl.random_ksat(c["n"], c["m"], c["k"], c["seed"])
    cp, v_, n_ = wl.formula_arrays(var, neg)
    f = cnf.CNFFormula.from_arrays(cp, v_, n_, c["n"])
    files = dpm_files()
    print(json.dumps({"dpm_files": files}), flush=True)
    smp = Sampler(files)
    smp.start()
    dtype = os.environ.get("DTYPE", "f64")
    steps = int(os.environ.get("STEPS", "20"))
    rows = []

    def launch(s, phase, i):
        s.profile(True)
        s.synchronize()
        t0 = time.perf_counter()
        s.simulate(dt=0.01, max_steps=steps, stop=ODESAT_STOP_NONE, poll_interval=steps)
        s.synchronize()
        t1 = time.perf_counter()
        ms, _ = s.profile_read()
        s.profile(False)
        row = {"phase": phase, "i": i, "kernel_us": round(ms[0] * 1e3, 1), "us_per_step": round(ms[0] * 1e3 / steps, 2),
               "wall_us": round((t1 - t0) * 1e6, 1), "levels": smp.levels(t0, t1)}
        rows.append(row)
        print(json.dumps(row), flush=True)

    with Solver(f, 1024, dtype) as s:
        s.init_state(42)
        s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
        for i in range(10):
            launch(s, "A_fresh_back_to_back", i)
        s.synchronize()
        t = time.perf_counter()
        time.sleep(1.5)
        print(json.dumps({"idle_levels": smp.levels(t + 1.0, t + 1.5)}), flush=True)
        for i in range(4):
            launch(s, "B_after_idle", i)
    with Solver(f, 1024, dtype) as s:
        s.init_state(7)
        s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
        for i in range(4):
            launch(s, "C_fresh_hot", i)
    def series(s, phase, k, count):
        out = []
        for i in range(count):
            s.profile(True)
            s.simulate(dt=0.01, max_steps=k, stop=ODESAT_STOP_NONE, poll_interval=k)
            ms, _ = s.profile_read()
            s.profile(False)
            out.append(round(ms[0] * 1e3 / k, 2))
        row = {"phase": phase, "steps_per_launch": k, "us_per_step": out}
        print(json.dumps(row), flush=True)
        return row

    with Solver(f, 1024, "f64") as s64, Solver(f, 1024, "f32") as s32:
        s64.init_state(42)
        s32.init_state(42)
        s64.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
        s32.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE, poll_interval=5)
        s64.synchronize()
        time.sleep(1.5)
        series(s64, "D_f64_after_idle", 4, 60)
        time.sleep(1.5)
        series(s32, "E_onchip_after_idle", 4, 60)
        time.sleep(1.5)
        series(s32, "F_onchip_primer", 4, 30)
        series(s64, "F_f64_after_onchip", 4, 60)
    smp.stop = True
    summ = {}
    for r in rows:
        summ.setdefault(r["phase"], []).append(r["us_per_step"])
    print(json.dumps({"summary_us_per_step": summ}), flush=True)


if __name__ == "__main__":
    main()
