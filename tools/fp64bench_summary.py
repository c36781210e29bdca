"""SIMD-cycles per wave64 instruction for each tools/fp64bench.hip kernel (round 6 class-price table).

    python3 tools/fp64bench_summary.py OUTDIR > profiles/r06/fp64bench/summary.txt

price = (GRBM_GUI_ACTIVE / 8 XCDs) x 1024 SIMDs / SQ_INSTS_VALU of the dispatch (the asm instruction
dominates: 8 chains x 2048 iterations per lane, against ~60 setup instructions); VALUBusy and the
dual-issue fraction beside it; the SQ_INSTS_VALU_* class the instruction landed in from the counters.
"""
import collections
import csv
import glob
import json
import sys

out = sys.argv[1]
times = {}
for line in open(f"{out}/times.jsonl"):
    if line.startswith("{"):
        d = json.loads(line)
        times[d["kernel"]] = d
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{out}/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "fb_kernel<" not in k:
            continue
        op = k.split("fb_kernel<")[1].split(">")[0]
        vals[op][r["Counter_Name"]].append(float(r["Counter_Value"]))
# one dispatch per kernel per pass; counters taken in both passes (GRBM_GUI_ACTIVE, SQ_WAVES) are averaged
rows = {op: {c: sum(v) / len(v) for c, v in d.items()} for op, d in vals.items()}
classes = ("FMA_F64", "ADD_F64", "MUL_F64", "TRANS_F64", "INT32", "INT64", "CVT", "FMA_F32", "TRANS_F32")
print(f"{'kernel':18s} {'class(asm)':10s} {'counted as':12s} {'SIMD-cyc/inst':>13s} {'VALUBusy':>8s} {'dual':>6s} {'ms':>8s}")
for op, t in times.items():
    r = rows.get(op, {})
    g, n = r.get("GRBM_GUI_ACTIVE"), r.get("SQ_INSTS_VALU")
    if not g or not n:
        print(f"{op:18s} {t['class']:10s} (no counters)")
        continue
    cyc = g / 8.0
    price = cyc * 1024.0 / n
    busy = r.get("SQ_ACTIVE_INST_VALU", 0.0) * 4.0 / 1024.0 / cyc
    dual = r.get("SQ_ACTIVE_INST_VALU2", 0.0) * 4.0 / 1024.0 / cyc
    counted = [c for c in classes if r.get(f"SQ_INSTS_VALU_{c}", 0.0) > 0.5 * n]
    print(f"{op:18s} {t['class']:10s} {','.join(counted) or '-':12s} {price:13.2f} {busy:8.3f} {dual:6.3f} {t['ms']:8.3f}")
