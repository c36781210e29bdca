"""Summarise a rocprofv3 PC-sampling CSV (round 6): samples per instruction of one kernel, with the
stochastic sampler's issue / stall fields when present.

    python3 tools/pcsamp_summary.py RAW_DIR OUT.txt [KERNEL_SUBSTRING]

The raw CSV (hundreds of MB) stays on the GPU box; OUT.txt holds the header, per-field value counts,
and the top instructions by samples (offset, text, samples, share, and the stall reasons of the
samples at that instruction).
"""
import collections
import csv
import glob
import sys

raw, out = sys.argv[1], sys.argv[2]
ksub = sys.argv[3] if len(sys.argv) > 3 else None
files = sorted(glob.glob(f"{raw}/**/*pc_sampling*.csv", recursive=True)) or \
    sorted(glob.glob(f"{raw}/**/*.csv", recursive=True))
lines = []
kern_col = None
for f in files:
    with open(f, newline="") as fh:
        rd = csv.DictReader(fh)
        cols = rd.fieldnames or []
        lines.append(f"# {f}: columns {cols}")
        if not any("nstruction" in c for c in cols):
            continue
        key_cols = [c for c in cols if c in ("Code_Object_Offset", "Inst_Index", "Instruction", "Code_Object_Id")]
        cat_cols = [c for c in cols if any(t in c for t in ("Stall", "Issued", "Inst_Type", "Wave_Count", "Hw_Id"))
                    and "Id" not in c[-3:]]
        kern_col = next((c for c in cols if c in ("Kernel_Name", "Kernel-Name", "Dispatch_Kernel_Name")), None)
        per = collections.Counter()
        text = {}
        stall = collections.defaultdict(collections.Counter)
        cats = collections.defaultdict(collections.Counter)
        total = 0
        for r in rd:
            if ksub and kern_col and ksub not in r.get(kern_col, ""):
                continue
            k = tuple(r.get(c, "") for c in key_cols)
            per[k] += 1
            total += 1
            text[k] = r.get("Instruction", "") + ("  ;" + r["Instruction_Comment"] if r.get("Instruction_Comment") else "")
            for c in cat_cols:
                cats[c][r.get(c, "")] += 1
            sr = [r.get(c, "") for c in cat_cols if "Stall" in c]
            if sr:
                stall[k]["/".join(sr)] += 1
        lines.append(f"# samples {total}; key {key_cols}; categorical {cat_cols}")
        for c, cnt in cats.items():
            lines.append(f"# {c}: " + ", ".join(f"{v}={n} ({n / max(total, 1):.3f})" for v, n in cnt.most_common(24)))
        lines.append(f"{'samples':>8} {'share':>6}  key | instruction | stall reasons")
        for k, n in per.most_common(400):
            st = ", ".join(f"{v}:{m}" for v, m in stall[k].most_common(4)) if k in stall else ""
            lines.append(f"{n:8d} {n / max(total, 1):6.4f}  {'/'.join(k[:2])} | {text[k][:90]} | {st}")
open(out, "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:40]))
