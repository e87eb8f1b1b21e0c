"""Shared helpers for the test-suite (fixture loading)."""
import os

import numpy as np

from oracle import cnf_oracle as co
from oracle import np_oracle as npo

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FIXTURES = ("small", "easy", "hard", "rand200")


def read(name):
    with open(os.path.join(GOLDEN, name if name.endswith(".cnf") else name + ".cnf")) as fh:
        return fh.read()


def oracle_formula(name):
    """Normalised npo.Formula of a fixture via the Python loader restatement."""
    cl, varnum = co.parse_dimacs_format(read(name))
    _, ncl = co.normalize_cnf_variables(cl, varnum)
    return npo.Formula.from_clauses(ncl, varnum)


def golden(name):
    return np.load(os.path.join(GOLDEN, f"{name}_golden.npz"))
