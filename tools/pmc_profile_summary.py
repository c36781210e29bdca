"""Means per dispatch of the trajectory kernel that ran, from a tools/profile_round.sh directory.

    python tools/pmc_profile_summary.py PROFILE_DIR STEPS_PER_LAUNCH [LABEL] > profiles/rNN/cX/pmc_summary.txt

Pathline launches dispatch both instantiations (the cooperative and the plain one, the other exits at
once): the one that ran is the traj_kernel with the longest average in the stats pass.  Besides the
counters' means it prints per wave-step instruction counts (SQ_INSTS_* / SQ_WAVES / steps) and the busy
fractions (TD over 256 CUs, VALU / SALU / LDS over 1024 SIMDs, per XCD-cycle of GRBM_GUI_ACTIVE).
"""
import collections
import csv
import glob
import sys

out, steps = sys.argv[1], float(sys.argv[2])
label = sys.argv[3] if len(sys.argv) > 3 else out
stats = [r for f in glob.glob(f"{out}/stats/*kernel_stats.csv") for r in csv.DictReader(open(f))
         if "traj_kernel" in r["Name"]]
ran = max(stats, key=lambda r: float(r["AverageNs"]))
name = ran["Name"]
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{out}/*/*counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"] == name:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(f"# {label}: {name}, {ran['Calls']} dispatches of {float(ran['AverageNs']) / 1e6:.1f} ms on average "
      f"(rocprofv3 stats); counter means per dispatch of that kernel")
m = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(acc):
    print(f"{k:40s} n={len(acc[k]):3d} mean={m[k]:.4g}")
w = m.get("SQ_WAVES")
if w:
    ws = w * steps
    f64 = sum(m.get(f"SQ_INSTS_VALU_{o}_F64", 0.0) for o in ("ADD", "MUL", "FMA"))
    print(f"# per wave-step ({steps:g} steps): VALU {m.get('SQ_INSTS_VALU', 0) / ws:.1f} (FP64 add/mul/fma "
          f"{f64 / ws:.1f}), SALU {m.get('SQ_INSTS_SALU', 0) / ws:.1f}, VMEM {m.get('SQ_INSTS_VMEM_RD', 0) / ws:.2f}, "
          f"LDS {m.get('SQ_INSTS_LDS', 0) / ws:.1f}")
g = m.get("GRBM_GUI_ACTIVE")
if g:
    cyc = g / 8.0
    parts = []
    if "TD_TD_BUSY_sum" in m:
        parts.append(f"TD busy {m['TD_TD_BUSY_sum'] / 256.0 / cyc:.3f}")
    for c, n in (("SQ_ACTIVE_INST_VALU", "VALUBusy"), ("SQ_ACTIVE_INST_SCA", "SALUBusy"), ("SQ_ACTIVE_INST_LDS", "LDSBusy")):
        if c in m:
            parts.append(f"{n} {m[c] * 4.0 / 1024.0 / cyc:.3f}")
    print("# " + ", ".join(parts))
