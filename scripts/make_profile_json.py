"""PMC profile of one persistent kernel as fixed-per-launch + per-step fits (profiles/profile_<kernel>.json),
read by bench.py for roofline.traffic and, for k_onchip, the VALU-issue roofline.

A launch of k steps costs F + k * P of a counter: the state crosses HBM once per launch (F) and the
per-step traffic (P) is ~0 for k_onchip, the clause memories for k_resident.  Two launch sizes k1 < k2
(scripts/prof_step.py runs ONE launch of STEPS steps) give P = (c2 - c1) / (k2 - k1), F = c1 - k1 P.
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KiB -> bytes; on gfx950 FETCH_SIZE tallies 128-B read requests
at 64 B, MI355X_MICROARCH.md HBM section); each counter comes from its own --pmc pass, kernel trace only.

usage: python scripts/make_profile_json.py <kernel substring> <batch> <dtype> <config> <out.json> [mode=adaptive]
           k1:<dir> k2:<dir>
       (each dir holds the p*/run_counter_collection.csv of scripts/pmc.sh; mode defaults to fixed)
"""
import collections
import csv
import glob
import json
import sys


def counters(root, kern):
    vals = collections.defaultdict(list)
    for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
        for r in csv.DictReader(open(f)):
            if kern in r["Kernel_Name"]:
                vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    kern, batch, dtype, config, out = sys.argv[1:6]
    mode = "fixed"
    pts = []
    for a in sys.argv[6:]:
        if a.startswith("mode="):
            mode = a[5:]
            continue
        k, d = a.split(":", 1)
        c = counters(d, kern)
        pt = {"steps": int(k), "fetch_size_kib": c["FETCH_SIZE"], "write_size_kib": c["WRITE_SIZE"]}
        pt["hbm_bytes"] = 2.0 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
        for name in ("SQ_INSTS_VALU", "SQ_WAVES", "GRBM_GUI_ACTIVE", "SQ_INSTS_SALU", "SQ_INSTS_LDS"):
            if name in c:
                pt[name] = c[name]
        pts.append(pt)
    pts.sort(key=lambda p: p["steps"])
    p1, p2 = pts[0], pts[-1]
    dk = p2["steps"] - p1["steps"]

    def fit(key):
        per = (p2[key] - p1[key]) / dk
        return p1[key] - p1["steps"] * per, per

    res = {"kernel": kern, "batch": int(batch), "dtype": dtype, "config": config, "mode": mode, "points": pts}
    res["hbm_bytes_fixed"], res["hbm_bytes_per_step"] = fit("hbm_bytes")
    if all("SQ_INSTS_VALU" in p for p in (p1, p2)):
        res["valu_insts_fixed"], res["valu_insts_per_step"] = fit("SQ_INSTS_VALU")
    if all("SQ_INSTS_LDS" in p for p in (p1, p2)):
        res["lds_insts_fixed"], res["lds_insts_per_step"] = fit("SQ_INSTS_LDS")
    if all("GRBM_GUI_ACTIVE" in p for p in (p1, p2)):  # busy GPU cycles, summed over the 8 XCDs
        res["grbm_cycles_fixed"], res["grbm_cycles_per_step"] = fit("GRBM_GUI_ACTIVE")
    res["note"] = ("per launch of k steps: fixed + k * per_step; HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 "
                   "FETCH_SIZE correction), one --pmc pass per counter group, kernel trace only")
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
