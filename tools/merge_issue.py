"""Merge the trajectory kernel's issue-pipe occupancy (tools/pmc_issue.sh) into a workload's record of
profiles/pmc_traffic.json (written by tools/make_traffic.py for the same engine build).

    python tools/merge_issue.py ISSUE_DIR WORKLOAD_KEY profiles/pmc_traffic.json

Fractions are per SIMD cycle, from the pass's own dispatches (so independent of how many launches ran):
  valu_busy = sum SQ_ACTIVE_INST_VALU x 4 / 1024 SIMDs / (sum GRBM_GUI_ACTIVE / 8 XCDs)
(rocprof's VALUBusy; SQ_ACTIVE_INST_* count quad-cycles per wave, so overlapping waves of one SIMD can
push the ANY figure past 1 -- VALU, SALU and LDS stay below it), likewise salu_busy and lds_busy.
The record's instruction-count model, from its own SQ_INSTS counts, is added by make_traffic.py
(valu_issue_model)."""
import csv, glob, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

src, key, dst = sys.argv[1], sys.argv[2], sys.argv[3]
tot = {}
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "traj_kernel" in r["Kernel_Name"]:
            tot[r["Counter_Name"]] = tot.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
cyc = tot["GRBM_GUI_ACTIVE"] / 8.0
frac = lambda c: tot[c] * 4.0 / 1024.0 / cyc  # noqa: E731
recs = json.load(open(dst))
bid = bench.engine_build_id()
hit = [r for r in recs if r.get("workload") == key and r.get("engine_build") == bid]
if not hit:
    raise SystemExit(f"no record for {key} on engine build {bid}: run tools/make_traffic.py first")
hit[0].update(valu_busy=frac("SQ_ACTIVE_INST_VALU"), salu_busy=frac("SQ_ACTIVE_INST_SCA"),
              lds_busy=frac("SQ_ACTIVE_INST_LDS"), issue_profile=src)
json.dump(recs, open(dst, "w"), indent=1)
print(json.dumps({k: hit[0][k] for k in ("workload", "valu_busy", "salu_busy", "lds_busy")}))
