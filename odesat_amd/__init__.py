"""odesat_amd -- MI355X-native drop-in for odesat's per-step ODE integrator (src/system.rs) and its
DIMACS loader (src/cnf.rs), as hand-written gfx950 HIP kernels behind a C ABI (include/odesat.h).
"""
from ._lib import (ODESAT_F32, ODESAT_F64, ODESAT_STOP_ANY, ODESAT_STOP_EACH, ODESAT_STOP_NONE,  # noqa: F401
                   OdesatError, device_count)

__version__ = "0.1.0"
