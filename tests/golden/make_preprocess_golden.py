"""Generate tests/golden/preprocess_golden.json (run from the repo root:
`python tests/golden/make_preprocess_golden.py`).

Expected outputs come from oracle/preprocess_oracle.py (the pure-Python restatement of cnf.rs:317-840),
on the reference's own fixtures tests/{small,easy,hard}.cnf and rand200.cnf, at the `solve` default
ratio 7 (main.rs:150-154) and at 4.5.  Per case: the reduced formula (set order), its varnum and the
trace [(kind, var, clauses)], each clause as [[var, negated], ...].
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from oracle import cnf_oracle as co  # noqa: E402
from oracle import preprocess_oracle as po  # noqa: E402

CASES = [("small", 7.0), ("easy", 7.0), ("hard", 7.0), ("rand200", 7.0), ("easy", 4.5)]


def enc(clauses):
    return [[[int(v), int(n)] for v, n in c] for c in clauses]


def main():
    out = []
    for name, ratio in CASES:
        with open(os.path.join(HERE, name + ".cnf")) as fh:
            cl, varnum = co.parse_dimacs_format(fh.read())
        red, vn, trace = po.preprocess(cl, varnum, ratio)
        out.append({"fixture": name, "ratio": ratio, "varnum": vn, "clauses": enc(red),
                    "trace": [[k, v, enc(cs)] for k, v, cs in trace]})
    with open(os.path.join(HERE, "preprocess_golden.json"), "w") as fh:
        json.dump(out, fh, separators=(",", ":"))


if __name__ == "__main__":
    main()
