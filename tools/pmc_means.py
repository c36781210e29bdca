"""Per-dispatch means of one trajectory kernel's counters over rocprofv3 pass directories, plus the
stall decomposition (round 6, tools/pmc_stall.sh):

    python3 tools/pmc_means.py OUTDIR "traj_kernel<7, true, false, true>" STEPS_PER_LAUNCH

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles per wave (MI355X_MICROARCH.md, the
s_memtime row); GRBM_GUI_ACTIVE is summed over the 8 XCDs.  Fractions of wave time: waiting for anything
(SQ_WAIT_ANY), waiting to issue (SQ_WAIT_INST_ANY: the wave has an instruction but it cannot go --
dependency or arbitration), issuing (SQ_ACTIVE_INST_ANY).  Per-SIMD busy: VALU, dual-issue VALU2, SALU.
Latency: SQ_INST_LEVEL_{LDS,VMEM} / SQ_INSTS_{LDS,VMEM_RD} = mean cycles an instruction is in flight.
"""
import collections
import csv
import glob
import sys

out, kname, steps = sys.argv[1], sys.argv[2], float(sys.argv[3])
acc = collections.defaultdict(list)
for f in sorted(glob.glob(f"{out}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if r["Kernel_Name"].startswith(kname):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(v) / len(v) for k, v in acc.items()}
print(f"# {kname}: counter means per dispatch ({out})")
for k in sorted(m):
    print(f"{k:32s} n={len(acc[k]):3d} mean={m[k]:.4g}")
w = m.get("SQ_WAVES")
cyc = m.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
if w and "SQ_WAVE_CYCLES" in m:
    wc = m["SQ_WAVE_CYCLES"]
    print(f"# wave lifetime {4 * wc / w:.4g} cycles, {4 * wc / w / steps:.1f} cycles per wave-step; fractions of wave time: "
          + ", ".join(f"{n} {m[c] / wc:.3f}" for c, n in (("SQ_WAIT_ANY", "wait_any"), ("SQ_WAIT_INST_ANY", "wait_inst_any"),
                                                        ("SQ_ACTIVE_INST_ANY", "issue_any"), ("SQ_WAIT_INST_LDS", "wait_inst_lds"))
                      if c in m))
    if cyc:
        print(f"# resident waves per SIMD {4 * wc / 1024.0 / cyc:.2f}")
if w and "SQ_IFETCH" in m:
    print(f"# instruction fetches per wave-step {m['SQ_IFETCH'] / w / steps:.1f}")
if "SQC_ICACHE_HITS" in m and "SQC_ICACHE_MISSES" in m:
    h, mi = m["SQC_ICACHE_HITS"], m["SQC_ICACHE_MISSES"]
    print(f"# instruction cache: hits {h:.4g}, misses {mi:.4g}, miss rate {mi / max(h + mi, 1):.4f}"
          + (f", misses per wave-step {mi / w / steps:.2f}" if w else ""))
if cyc:
    parts = [f"{n} {m[c] * 4.0 / 1024.0 / cyc:.3f}" for c, n in (("SQ_ACTIVE_INST_VALU", "VALUBusy"),
             ("SQ_ACTIVE_INST_VALU2", "VALU2 (dual issue)"), ("SQ_ACTIVE_INST_SCA", "SALUBusy")) if c in m]
    if parts:
        print("# per SIMD: " + ", ".join(parts))
for lvl, n in (("SQ_INST_LEVEL_LDS", "SQ_INSTS_LDS"), ("SQ_INST_LEVEL_VMEM", "SQ_INSTS_VMEM_RD")):
    if lvl in m and m.get(n):
        print(f"# {lvl} / {n} = {m[lvl] / m[n]:.1f} (mean in-flight cycles per instruction, level units)")
