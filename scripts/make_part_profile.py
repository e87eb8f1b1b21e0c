"""PMC profile of the partitioned single-instance step (config 5, partition.hip) at world 1:
profiles/profile_k_part_config5.json, read by bench.py's partition_config5 leg for roofline.traffic.

Every step launches each per-rank kernel once (k_part_status, k_part_clause3, k_part_var and, for
CLAUSES, k_part_apply), so a kernel's counters averaged over its dispatches are its per-step figures.
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; the gfx950 FETCH_SIZE correction,
MI355X_MICROARCH.md), each counter from its own --pmc pass (scripts/pmc.sh with
PROG=scripts/bench_partition.py, eager launches: --graph 0).

usage: python scripts/make_part_profile.py <out.json> <partition>:<pmc dir> [<partition>:<pmc dir> ...]
"""
import collections
import csv
import glob
import json
import re
import sys


def per_kernel(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            mt = re.search(r"k_part\w*", r["Kernel_Name"])
            if mt is None:
                continue
            short = mt.group(0)
            vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in vals.items():
        c = {n: sum(v) / len(v) for n, v in d.items()}
        row = {n: c[n] for n in ("FETCH_SIZE", "WRITE_SIZE", "TCC_HIT_sum", "TCC_MISS_sum") if n in c}
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            row["hbm_bytes"] = 2.0 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
        if "TCC_HIT_sum" in c and "TCC_MISS_sum" in c and c["TCC_HIT_sum"] + c["TCC_MISS_sum"] > 0:
            row["l2_hit_rate"] = c["TCC_HIT_sum"] / (c["TCC_HIT_sum"] + c["TCC_MISS_sum"])
        row["dispatches"] = max(len(v) for v in d.values())
        out[k] = row
    return out


def main():
    out = sys.argv[1]
    res = {"kernel": "k_part", "config": "config5", "world": 1, "partitions": {},
           "note": "per step (one dispatch of each kernel per step): HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE "
                   "(gfx950 FETCH_SIZE correction), one --pmc pass per counter group, kernel trace only, eager "
                   "launches (--graph 0); world 1: every clause on the one rank"}
    for a in sys.argv[2:]:
        part, d = a.split(":", 1)
        ks = per_kernel(d)
        tot = sum(k.get("hbm_bytes", 0.0) for k in ks.values())
        res["partitions"][part] = {"kernels": ks, "hbm_bytes_per_step": tot}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
