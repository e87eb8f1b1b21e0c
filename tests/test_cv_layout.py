"""k_solo_cv's lane and LDS block placement (odesat_amd/csrc/cv_layout.cpp, the odesat_cv_layout test
hook; no device): every clause on exactly one slot with its own literals, distinct blocks inside the
area, and a bank-conflict model cost no higher than the plain layout's -- lower on the criterion's
hard.cnf.  The GPU side (tests/test_gpu_parity.py::test_solo_cv_matches_solo_fast_and_oracle) runs the
kernel on these layouts bit-exact against k_solo_fast and the oracle."""
import numpy as np
import pytest

from odesat_amd import _lib, cnf
from tests.common import read


def _arrays(name):
    _, f = cnf.normalize_cnf_variables(cnf.parse_dimacs_format(read(name)))
    cp, var, neg = f.arrays()
    assert (np.diff(cp) == 3).all()
    lits = (np.asarray(var, np.int64) << 1 | np.asarray(neg, np.int64)).astype(np.int32)
    deg = np.bincount(np.asarray(var), minlength=f.varnum)
    vst = np.concatenate([[0], np.cumsum(deg)]).astype(np.int32)
    return lits, vst


CAP = {8: (4096 - 512) // 10, 4: (8192 - 512) // 12}  # wave.hpp solo_cv_blk_cap


@pytest.mark.parametrize("nl,cpl", [(192, 1), (256, 1), (128, 2)])
@pytest.mark.parametrize("tsize", [8, 4])
def test_layout_is_a_placement_and_cuts_conflicts(nl, cpl, tsize):
    lits, vst = _arrays("hard")
    n, m = len(vst) - 1, len(lits) // 3
    sc, so, blk, plain, opt = _lib.cv_layout(lits, vst, nl, cpl, tsize, CAP[tsize], 20000)
    assert sorted(sc[sc >= 0].tolist()) == list(range(m))  # every clause on exactly one slot
    for s in np.nonzero(sc >= 0)[0]:
        assert sorted(so[s].tolist()) == [0, 1, 2]
    assert len(set(blk.tolist())) == n + 1 and blk.min() >= 0 and blk.max() < CAP[tsize]
    assert opt <= plain and opt < 0.9 * plain, (plain, opt)
    # the plain layout (no search): clause s on slot s, literals as given, block v for variable v
    sc0, so0, blk0, p0, o0 = _lib.cv_layout(lits, vst, nl, cpl, tsize, CAP[tsize], 0)
    assert p0 == o0 == plain
    assert (sc0[:m] == np.arange(m)).all() and (sc0[m:] == -1).all() and (blk0 == np.arange(n + 1)).all()
    assert (so0 == np.arange(3)).all()


def test_layout_rejects_bad_arguments():
    lits, vst = _arrays("hard")
    with pytest.raises(_lib.OdesatError):
        _lib.cv_layout(lits, vst, 100, 1, 8, CAP[8], 10)  # lanes not a multiple of 64
    with pytest.raises(_lib.OdesatError):
        _lib.cv_layout(lits, vst, 64, 1, 8, CAP[8], 10)  # m = 160 clauses on 64 slots
