"""Average each PMC counter per kernel (and per launch) over a pmc.sh output directory."""
import collections
import csv
import glob
import sys

root = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{root}/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)", "anon").split("(")[0].replace("void ", "")
        agg[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(agg.items()):
    if any(x in k for x in ("k_step", "k_clause", "k_variable", "k_status", "k_resident", "k_onchip")):
        n = len(next(iter(d.values())))
        print(k, "launches=%d" % n)
        for c, v in sorted(d.items()):
            print("   %-28s %14.4g" % (c, sum(v) / len(v)))
