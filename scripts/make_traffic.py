"""Per-step HBM traffic of the dominant kernel from a pmc.sh run (profiles/traffic_<tag>.json).

FETCH_SIZE / WRITE_SIZE are in KiB per launch.  On gfx950 FETCH_SIZE tallies 128-byte EA read
requests at 64 B, so it reports half the bytes read (MI355X_MICROARCH.md, HBM/rocprofv3 section):
reads = 2 x FETCH_SIZE.  WRITE_SIZE needs no correction.  prof_step.py runs ONE launch of STEPS
steps (the persistent kernels' launch = poll interval = STEPS), so per step = per launch / STEPS.

usage: python scripts/make_traffic.py <pmc dir> <kernel substring> <batch> <steps> <dtype> <config> <out.json>
"""
import collections
import csv
import glob
import json
import sys

root, kern, batch, steps, dtype, config, out = sys.argv[1:8]
vals = collections.defaultdict(list)
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kern in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
fetch_kb = sum(vals["FETCH_SIZE"]) / len(vals["FETCH_SIZE"])
write_kb = sum(vals["WRITE_SIZE"]) / len(vals["WRITE_SIZE"])
reads = 2.0 * fetch_kb * 1024
writes = write_kb * 1024
steps = int(steps)
res = {
    "kernel": kern, "batch": int(batch), "dtype": dtype, "config": config, "steps_per_launch": steps,
    "fetch_size_kib_per_launch": fetch_kb, "write_size_kib_per_launch": write_kb,
    "hbm_read_bytes_per_launch": reads, "hbm_write_bytes_per_launch": writes,
    "hbm_bytes_per_launch": reads + writes,
    "hbm_bytes_per_step": (reads + writes) / steps,
    "note": "reads = 2 x FETCH_SIZE (gfx950 tallies 128-B requests at 64 B); separate --pmc passes, "
            "kernel-trace only",
}
for k in ("TCC_HIT_sum", "TCC_MISS_sum", "TCC_EA0_RDREQ_sum", "TCC_EA0_WRREQ_sum"):
    if vals.get(k):
        res[k] = sum(vals[k]) / len(vals[k])
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
