"""Per-pass PMC shares of k_onchip's adaptive step, from scripts/gpu_r06c.sh's part C:
three builds of the same launch (scripts/prof_step.py, ADAPTIVE=1, config 2, B = 1024, 20 steps):
the product (full), ONCHIP_ADA_SKIP=1 (no pass 2) and ONCHIP_ADA_SKIP=2 (no pass 1).  Pass 2's share of
a counter = full - skip1, pass 1's = full - skip2 (the rest: the voltage phases and the dt update).
    python scripts/pass_counters.py <dir of pmc_<tag>_onchipctl, ..._adaskip1, ..._adaskip2> <tag> [out.json]
Counters are per launch (max over the run's dispatches of k_onchip), in millions."""
import collections
import csv
import glob
import json
import os
import sys


def counters(root, kern="k_onchip"):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                per[r["Counter_Name"]][r.get("Dispatch_Id", "0")] += float(r["Counter_Value"])
    return {k: max(v.values()) / 1e6 for k, v in per.items()}


def main():
    d, tag = sys.argv[1], sys.argv[2]
    full, s1, s2 = (counters(os.path.join(d, f"pmc_{tag}_{v}")) for v in ("onchipctl", "adaskip1", "adaskip2"))
    out = {"full": full, "no_pass2": s1, "no_pass1": s2, "pass2": {}, "pass1": {}, "rest": {}}
    for k in sorted(full):
        if k in s1 and k in s2:
            out["pass2"][k] = full[k] - s1[k]
            out["pass1"][k] = full[k] - s2[k]
            out["rest"][k] = full[k] - out["pass1"][k] - out["pass2"][k]
    for k in sorted(out["pass2"]):
        print(f"{k:24s} full {full[k]:10.2f}  pass1 {out['pass1'][k]:10.2f}  pass2 {out['pass2'][k]:10.2f}  "
              f"rest {out['rest'][k]:10.2f}")
    if len(sys.argv) > 3:
        with open(sys.argv[3], "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
