"""Probe: which HIP runtime a process ends up with when torch and libodesat_hip.so are both loaded,
in either order (one subprocess per order)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

P1 = r"""
import sys; sys.path.insert(0, %r)
import torch
print("torch avail", torch.cuda.is_available(), torch.version.hip)
x = torch.ones(4, device="cuda")
from odesat_amd import _lib, cnf
from odesat_amd.system import Solver, ODESAT_STOP_NONE
print("lib devices", _lib.device_count())
_, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format("p cnf 3 2\n1 -2 3 0\n-1 2 3 0\n"))
with Solver(f, 4, "f32") as s:
    s.init_state(1); s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE)
print("solver ok", float(x.sum()))
maps = [l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l]
print(sorted(set(maps)))
""" % ROOT

P2 = r"""
import sys; sys.path.insert(0, %r)
from odesat_amd import _lib, cnf
from odesat_amd.system import Solver, ODESAT_STOP_NONE
print("lib devices", _lib.device_count())
_, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format("p cnf 3 2\n1 -2 3 0\n-1 2 3 0\n"))
with Solver(f, 4, "f32") as s:
    s.init_state(1); s.simulate(dt=0.01, max_steps=5, stop=ODESAT_STOP_NONE)
import torch
print("torch avail", torch.cuda.is_available())
maps = [l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l]
print(sorted(set(maps)))
x = torch.ones(4, device="cuda")
print("torch ok", float(x.sum()))
""" % ROOT

for name, src in (("torch-first", P1), ("lib-first", P2)):
    r = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=180)
    print("==", name, "rc", r.returncode)
    print(r.stdout[-2000:])
    print(r.stderr[-1500:])
