"""Calibrate rocprofv3's HBM byte counters on gfx950 (VERDICT r4 "Next #2"): scripts/micro/fetch_calib
moves a known number of bytes per dispatch in each access shape the product kernels use; this script
divides each counter-derived byte figure by that number.

usage: python scripts/fetch_calib_report.py <run.jsonl> <pmc dir with p*/run_counter_collection.csv> <out.json>

Byte figures per dispatch (KiB counters x 1024, request counters x their size):
  fetch_size       FETCH_SIZE (rocprofv3's derived counter: BUBBLE x 128 + other x 64 + 32B x 32)
  write_size       WRITE_SIZE
  rdreq_sized      RDREQ_128B x 128 + (RDREQ - RDREQ_128B - RDREQ_32B) x 64 + RDREQ_32B x 32: every
                   L2 -> fabric read request at its own size
  rdreq_dram       RDREQ_DRAM x 64 (requests destined for DRAM; 32 B ones at 32)
Each ratio = figure / the dispatch's known bytes.  A ratio of 1 for the cold 1 GiB shapes means the
figure counts HBM bytes for that shape; the warm 64 MiB re-read tells whether Infinity-Cache hits are
counted (ratio ~1 again) or excluded (~0).
"""
import collections
import csv
import glob
import json
import sys


def dispatches(pmc_dir):
    """{dispatch order index among non-runtime kernels: {counter: value}} merged over the passes."""
    per_pass = []
    for f in sorted(glob.glob(f"{pmc_dir}/p*/run_counter_collection.csv")):
        rows = collections.OrderedDict()
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"].startswith("__amd_rocclr"):
                continue
            d = int(r["Dispatch_Id"])
            rows.setdefault(d, {"kernel": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
        per_pass.append([rows[k] for k in sorted(rows)])
    n = min(len(p) for p in per_pass)
    out = []
    for i in range(n):
        merged = {}
        for p in per_pass:
            merged.update(p[i])
        out.append(merged)
    return out


def main():
    runs = [json.loads(x) for x in open(sys.argv[1]) if x.startswith("{")]
    disp = dispatches(sys.argv[2])
    if len(disp) != len(runs):
        raise SystemExit(f"{len(disp)} counted dispatches vs {len(runs)} runs")
    res = []
    for run, c in zip(runs, disp):
        if run["name"] == "flush":
            continue
        known = run["bytes"]
        fig = {}
        if "FETCH_SIZE" in c:
            fig["fetch_size"] = c["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in c:
            fig["write_size"] = c["WRITE_SIZE"] * 1024
        if all(k in c for k in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_128B_sum", "TCC_EA0_RDREQ_32B_sum")):
            r, r128, r32 = c["TCC_EA0_RDREQ_sum"], c["TCC_EA0_RDREQ_128B_sum"], c["TCC_EA0_RDREQ_32B_sum"]
            fig["rdreq_sized"] = 128 * r128 + 64 * (r - r128 - r32) + 32 * r32
        if all(k in c for k in ("TCC_EA0_RDREQ_DRAM_sum", "TCC_EA0_RDREQ_DRAM_32B_sum")):
            d, d32 = c["TCC_EA0_RDREQ_DRAM_sum"], c["TCC_EA0_RDREQ_DRAM_32B_sum"]
            fig["rdreq_dram"] = 64 * (d - d32) + 32 * d32
        raw = {k: v for k, v in c.items() if k != "kernel"}
        res.append({"name": run["name"], "note": run["note"], "known_bytes": known, "us": run["us"],
                    "GBps": run["GBps"], "kernel": c["kernel"], "counters": raw,
                    "ratio": {k: v / known for k, v in fig.items()}})
    out = {"what": "rocprofv3 byte counters / known bytes per access shape on MI355X (scripts/micro/fetch_calib.hip)",
           "shapes": res}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    for s in res:
        print(f"{s['name']:18s} {s['GBps']:8.1f} GB/s  " +
              "  ".join(f"{k}={v:.3f}" for k, v in sorted(s["ratio"].items())))


if __name__ == "__main__":
    main()
