"""Measurement tooling only (scripts/, never the product): the variant library and the experiment
knobs a measurement script runs with.

  XP_LIB=expt/libNAME.so            load that build (scripts/build_variant.sh) instead of the in-tree one
  XP_KNOBS="WAVE=1,SOLO_LANES=256"  odesat_set_experiment for each knob (include/odesat.h)

libodesat_hip.so itself reads no environment variable: a script calls apply() before its first call into
the library, and the values are recorded in its output by knobs()."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

TERMS = {"region": 0, "ell": 1, "slot": 2}


def parse_knobs(text):
    out = {}
    for item in (text or "").split(","):
        item = item.strip()
        if not item:
            continue
        k, v = item.split("=", 1)
        k, v = k.strip(), v.strip()
        out[k] = TERMS[v] if k == "PART_TERMS" and v in TERMS else int(v)
    return out


def apply(lib_path=None, knobs=None):
    """Load the variant library (XP_LIB or lib_path) and set the knobs (XP_KNOBS and `knobs`)."""
    from odesat_amd import _lib
    path = lib_path or os.environ.get("XP_LIB")
    if path:
        _lib.use_library(path)
    for k, v in {**parse_knobs(os.environ.get("XP_KNOBS")), **(knobs or {})}.items():
        _lib.set_experiment(k, v)


def knobs():
    """The knobs in effect and the library loaded (for a script's JSON output)."""
    from odesat_amd import _lib
    set_ = {}
    for k in _lib.experiment_knobs():
        v = _lib.get_experiment(k)
        if v is not None:
            set_[k] = v
    return {"lib": os.path.relpath(_lib.LIB_PATH, ROOT), "knobs": set_}
