"""Average PMC counters per traj_kernel dispatch from tools/pmc.sh output."""
import collections
import csv
import glob
import sys

out = sys.argv[1]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{out}/pass*/p_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if "traj_kernel" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(acc):
    v = acc[k]
    print(f"{k:40s} n={len(v):3d} mean={sum(v)/len(v):.4g}")
