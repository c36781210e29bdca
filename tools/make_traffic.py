"""Merge one workload's HBM bytes per traj_kernel launch into profiles/pmc_traffic.json
(a list of records keyed by workload) from a profile run's fetch/ and write/ passes.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE (KiB) counts half the
bytes of 16-B-per-lane reads, so bytes = 2 x FETCH_SIZE (the raw value is kept
beside it); WRITE_SIZE (KiB) is taken as is.  Both are L2 memory-side counters
(Infinity-Cache hits included).  Each record carries the engine build id
(bench.engine_build_id: source + flags hash) it was measured on; bench.py uses
a record only for that build.

Usage: python tools/make_traffic.py PROFILE_DIR WORKLOAD_KEY profiles/pmc_traffic.json UNITS [LABEL]
UNITS = how many of bench.py's timed units (roofline.timed_unit: a launch, or a config-2
segment of overlapping part x chunk launches) the profiled run executed; the record's
bytes_per_unit = all traj_kernel bytes of the run / UNITS.
"""
import csv, glob, json, os, statistics, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
out = sys.argv[1]; workload = sys.argv[2]; dst = sys.argv[3]
units_arg = sys.argv[4]  # a number, or "dispatches" (the bench's timed unit is one launch)
label = sys.argv[5] if len(sys.argv) > 5 else out
def total(counter, d):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"{out}/{d}/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if "traj_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(v), len(v)
def total_any(counter):
    v = [float(r["Counter_Value"]) for f in glob.glob(f"{out}/pmc/**/*counter_collection.csv", recursive=True)
         for r in csv.DictReader(open(f)) if "traj_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return sum(v), len(v)
fetch, nf = total("FETCH_SIZE", "fetch")
write, nw = total("WRITE_SIZE", "write")
units = float(nf) if units_arg == "dispatches" else float(units_arg)
rec = dict(workload=workload, engine_build=bench.engine_build_id(), profile=label,
           fetch_size_kib_total=fetch, write_size_kib_total=write, dispatches=[nf, nw], units=units,
           bytes_per_unit=(2.0 * fetch + write) * 1024.0 / units,
           note="bytes_per_unit = (2*FETCH_SIZE + WRITE_SIZE)*1024 summed over the run's traj_kernel dispatches / units "
                "(gfx950 FETCH_SIZE correction)")
# FP64 VALU work of the same run (tools/profile_r02.sh's second counter pass), if present:
# wave-instructions x 64 lanes, an FMA counted as 2 flops
add, na = total_any("SQ_INSTS_VALU_ADD_F64")
mul, nm = total_any("SQ_INSTS_VALU_MUL_F64")
fma, nfm = total_any("SQ_INSTS_VALU_FMA_F64")
if na and nm and nfm:
    rec["fp64_flops_per_unit"] = 64.0 * (add + mul + 2.0 * fma) / units
valu, nv = total_any("SQ_INSTS_VALU")
# the memory-return view (tools/pmc_td.sh counters in the profile's td/ pass): vector-L1 tag accesses
# (64 B each: tools/membench.hip, mb_l1_x4), L1 -> L2 read requests (128 B each) and TD busy cycles
tcp, nt = total("TCP_TOTAL_CACHE_ACCESSES_sum", "td")
tcc, _ = total("TCP_TCC_READ_REQ_sum", "td")
tdb, _ = total("TD_TD_BUSY_sum", "td")
grbm, ng = total("GRBM_GUI_ACTIVE", "td")
if nt:
    rec["tcp_accesses_per_unit"] = tcp / units
    rec["l1_to_l2_requests_per_unit"] = tcc / units
    if grbm > 0:
        rec["td_busy"] = (tdb / 256.0) / (grbm / 8.0)
        if nv and na and nm and nfm:
            # VALU issue model: every wave64 VALU instruction holds its SIMD 4 cycles -- measured on MI355X for
            # FP64 fma / add / mul and for 32-bit integer add / xor alike, 4.1-4.2 SIMD-cycles each at ~97%
            # VALUBusy (tools/fp64bench.hip, profiles/r05/fp64bench/); against 1024 SIMDs x the cycles.  (Round
            # 4's model priced non-FP64 instructions at 2 cycles, from the FP32 rate, and undercounted.)
            f64 = add + mul + fma
            rec["valu_issue_model"] = 4.0 * valu / units / (1024.0 * grbm / units / 8.0)
            rec["valu_issue_model_fp64_only"] = 4.0 * f64 / units / (1024.0 * grbm / units / 8.0)
            # round 6 class prices (tools/fp64bench.hip, profiles/r06/fp64bench): FP64 transcendental seeds (rcp / rsq /
            # sqrt) hold the SIMD 16 cycles, FP32 ones 8, every other VALU instruction 4 -- the transcendental fractions
            # of the VALU count come from the profile's mix/ pass (SQ_INSTS_VALU_TRANS_F64 / _F32 over SQ_INSTS_VALU)
            mv = [float(r["Counter_Value"]) for f in glob.glob(f"{out}/mix/**/*counter_collection.csv", recursive=True)
                  for r in csv.DictReader(open(f)) if "traj_kernel" in r["Kernel_Name"]
                  and r["Counter_Name"] in ("SQ_INSTS_VALU",)]
            t64, _ = total("SQ_INSTS_VALU_TRANS_F64", "mix")
            t32, _ = total("SQ_INSTS_VALU_TRANS_F32", "mix")
            if mv and sum(mv) > 0:
                rec["valu_trans_f64_frac"] = t64 / sum(mv)
                rec["valu_trans_f32_frac"] = t32 / sum(mv)
# the profiled box and the rocprofv3 kernel-trace average of the kernel that ran (stats pass), so the bench line
# can state which box its PMC cycles came from next to its own launch time
if os.path.exists(f"{out}/host.txt"):
    rec["profile_host"] = open(f"{out}/host.txt").read().strip()
st = [r for f in glob.glob(f"{out}/stats/*kernel_stats.csv") for r in csv.DictReader(open(f)) if "traj_kernel" in r["Name"]]
if st:
    # a timed unit may run several instantiations (RK4 since round 6: the hand-off kernel, then the cooperative one
    # resuming the waves it handed over; the one the selection flag skips exits at once): the unit's time is their
    # sum, named after the longest (each instantiation is dispatched once per launch: per-call averages add up)
    ran = max(st, key=lambda r: float(r["AverageNs"]))
    rec["profile_kernel"] = ran["Name"]
    calls = float(ran["Calls"])
    rec["profile_avg_launch_ms"] = sum(float(r["TotalDurationNs"]) for r in st) / calls / 1e6
    rec["profile_kernels_ms"] = {r["Name"]: float(r["TotalDurationNs"]) / calls / 1e6 for r in st}
recs = []
if os.path.exists(dst):
    old = json.load(open(dst))
    recs = [r for r in (old if isinstance(old, list) else [old]) if r.get("workload") != workload]
recs.append(rec)
json.dump(recs, open(dst, "w"), indent=1)
print(json.dumps(rec))
