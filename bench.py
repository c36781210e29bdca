#!/usr/bin/env python3
"""Benchmark: particle-steps/sec of the MI355X trajectory hot path.

Default workload (BASELINE.json configs[2], the largest config that fits one GPU): EC30to60-class
mesh (synthetic, ~236k ocean cells, 60 levels), 1e7 particles per GPU, "layer 10" (mid-depth of
0-based layer 10), dt = 60 s, 7-day pathline as 7 chained daily snapshot pairs (the reference's
MOPSPathline.run, tutorial/pyMOPSAPI.py:1396-1531; mops_amd/chain.py), each pair's duration from the
snapshots' timestamps.  One bench "step" = the whole 7-day chain: per pair the seed location
(hinted by each particle's cell after pair 0), locality order, 1440 integration steps, the line
assembly + NaN cleanup, and -- for N > 1 -- an RCCL gather to rank 0 of the pair's record slab
(every particle's trajectory records, with seeds and slot ids; ``--gather records``: an all-gather)
over xGMI on a side stream, overlapped with the next pair.  ``--gpus N`` without a launcher starts the N ranks itself.

``--config 2``: BASELINE configs[1] -- 1e6 particles/GPU, depth 800 m, dt 120 s, 1-day streamline
(720 Euler steps), records gathered after every call for N > 1.

``--config 4``: BASELINE configs[3] -- oRRS18to6-class mesh (3.5M ocean cells, 80 levels), 1e7
particles in total sharded over the ranks (strong scaling), depth 20 m, dt 120 s, 30-day pathline
over 31 daily snapshots generated and derived in HBM inside the timed region (2 fields resident,
~75 GB each).

``--config 5``: BASELINE configs[4] -- same mesh, 1.25e7 Gaussian-seeded (Gulf-of-Mexico box)
particles per GPU (weak scaling, 1e8 on 8 GPUs), dt 60 s, 12 calendar-month pairs (Jan..Dec =
365 days = 525 600 steps, daily records; ``--pairs k`` runs the first k months).

Inputs (mesh, fields, seeds) are resident in HBM before the timed region.
Rank 0 prints one JSON line (driver contract).
"""
from __future__ import annotations

import argparse
import json
import socket
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=None, help="timed steps (default per config: 3; config 5: 1)")
    p.add_argument("--warmup", type=int, default=None, help="untimed steps (default per config: 1; config 5: 0)")
    p.add_argument("--particles", type=int, default=1_000_000, help="particles per GPU")
    p.add_argument("--freq", type=int, default=158, help="icosahedral frequency (158 -> ~236k ocean cells)")
    p.add_argument("--levels", type=int, default=60)
    p.add_argument("--depth", type=float, default=800.0)
    p.add_argument("--dt", type=int, default=120)
    p.add_argument("--duration", type=int, default=86400)
    p.add_argument("--record", type=int, default=3600)
    p.add_argument("--method", choices=["euler", "rk4"], default="euler")
    p.add_argument("--mode", choices=["streamline", "pathline"], default="streamline",
                   help="config 2 only: pathline = two snapshots (front/back) on the config-2 mesh")
    p.add_argument("--config", type=int, choices=[2, 3, 4, 5], default=3,
                   help="BASELINE.json config: 3 = 1e7-particle 7-day chained pathline at layer 10, dt 60 s (default: "
                        "the largest single-GPU config); 2 = 1e6-particle 1-day streamline; 4 = oRRS18to6-class "
                        "1e7-particle 30-day pathline (strong scaling); 5 = oRRS18to6-class 1.25e7 Gaussian "
                        "particles/GPU, 12 calendar-month pairs (weak scaling)")
    p.add_argument("--pairs", type=int, default=None,
                   help="configs 3/4/5: snapshot pairs (defaults 7 daily / 30 daily / 12 monthly)")
    p.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                   help="collective backend for N > 1 (nccl = RCCL over xGMI; gloo only to rehearse the multi-rank "
                        "path on one GPU with MOPS_BENCH_ONE_DEVICE=1)")
    p.add_argument("--segment", type=int, default=0,
                   help="integration steps per kernel launch (config 2: whole record periods, 0 = the whole "
                        "run; chains: 0 = launches of 3 simulated days with a locality re-sort between them)")
    p.add_argument("--parts", type=int, default=2,
                   help="config 2: particle parts on their own streams (ParticleSet.advance_pipelined)")
    p.add_argument("--chunks", type=int, default=6,
                   help="config 2: step chunks per part and segment (shorter launches whose tails overlap)")
    p.add_argument("--gather", choices=["root", "records", "checkpoint"], default="root",
                   help="N > 1, the trajectory collection at every checkpoint (the end of a config-2 call, the end "
                        "of each chained pair): 'root' (default) = every rank's record slab + seeds + slot ids "
                        "gathered to rank 0 (SURVEY 8e's Gather to rank 0: each sender over its own xGMI link), "
                        "'records' = the same all-gathered to every rank (distributed.RecordGather mode 'all'); "
                        "both overlapped with the next call / pair.  DESIGN.md section 7 models both: at config 3 "
                        "and 8 ranks a ring all-gather moves 7 x 11.5 GB per rank per pair (~0.53 s against a "
                        "0.5 s pair), the gather 11.5 GB per link (~75 ms).  'checkpoint' = only every particle's "
                        "final state (position, depth, death, id) / the pair's continuation points")
    p.add_argument("--deliver", choices=["host", "none"], default="host",
                   help="config 3, N = 1: also time the chain with every pair's lines delivered to pinned host "
                        "memory (chain.HostLineSink: a copy stream overlapped with the next pair), as the reference "
                        "returns them to its caller -> the line's host_delivery block (value stays device-resident)")
    p.add_argument("--topography", choices=["sigma", "zlevel"], default="sigma",
                   help="config 2: synthetic vertical grid (synth.make_snapshot): 'zlevel' = MPAS-O z-levels with "
                        "partial bottom cells and zero-thickness inactive levels")
    p.add_argument("--defer-lines", action="store_true",
                   help="configs 3-5: assemble each pair's lines on a side stream beside the next pair "
                        "(PathlineChain.run(defer_lines=True); not with record gathers). Off by default: measured "
                        "neutral (config 3 3838/3846 vs 3829 ms, config 4 3119 vs 3120 ms per 6 pairs) -- the "
                        "assembly's blocks take LDS and CU slots from the LDS-limited trajectory launch")
    p.add_argument("--side-cus", type=int, default=0,
                   help="configs 4/5: CUs reserved for a side stream that generates and derives snapshot p+2 while "
                        "pair p computes on the others (three field buffers); -1 = the same on an unmasked side "
                        "stream (its kernels share every CU with the trajectory launch); 0 = off (two buffers, derivation "
                        "between pairs, the default: measured slower, DESIGN.md section 3.3)")
    p.add_argument("--compact", choices=["auto", "on", "off"], default="auto",
                   help="config 2: re-sort each particle part with its dead particles last between step chunks "
                        "(ParticleSet.compact); auto = on for RK4 (quirk Q1 kills half the particles in a day)")
    p.add_argument("--finalize", choices=["parts", "after"], default="parts",
                   help="config 2: assemble each particle part's lines on its own stream after its last chunk "
                        "(parts, overlapping the other parts' final waves) or all lines once every part is done")
    p.add_argument("--compact-priority", action="store_true",
                   help="run the compaction re-sorts on high-priority streams (experiment)")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample length")
    return p.parse_args(argv)


STEPS_DEFAULT = {2: (3, 1), 3: (3, 1), 4: (2, 1), 5: (1, 0)}  # (steps, warmup)


def apply_config_defaults(args):
    """Fill the options left at their config-2 defaults with the chosen config's values (and the
    per-config steps / warmup)."""
    if args.config in (3, 4, 5):
        d = vars(argparse.Namespace(mode="streamline", particles=1_000_000, dt=120, duration=86400, record=3600,
                                    method="euler", depth=800.0, freq=158, levels=60))
        for k, v in {3: CONFIG3, 4: CONFIG4, 5: CONFIG5}[args.config].items():
            if getattr(args, k) == d[k]:
                setattr(args, k, v)
        if args.pairs is None:
            args.pairs = PAIRS_DEFAULT[args.config]
    st, wu = STEPS_DEFAULT[args.config]
    if args.steps is None:
        args.steps = st
    if args.warmup is None:
        args.warmup = wu
    return args


def all_gather_flat(dist, out, inp, backend):
    from mops_amd.distributed import all_gather_flat as agf
    agf(dist, out, inp, backend)


def make_seeds(n: int, rank: int) -> np.ndarray:
    """Uniform on |lat| < 70 deg, rejected on land; one shard per rank."""
    from mops_amd import synth
    seeds = synth.uniform_band_seeds(int(n * 1.25) + 64, seed=12345 + rank)
    r = np.linalg.norm(seeds, axis=1)
    lat = np.arcsin(seeds[:, 2] / r); lon = np.arctan2(seeds[:, 1], seeds[:, 0])
    return seeds[~synth._land_mask(lat, lon, "continents")][:n]


def make_gaussian_seeds(n: int, rank: int) -> np.ndarray:
    """Config 5: truncated Gaussian in the Gulf-of-Mexico box, ocean only; one draw per rank."""
    from mops_amd import synth
    out = []
    have = 0
    k = 0
    while have < n:
        s = synth.gaussian_box_seeds(int((n - have) * 1.6) + 64, seed=2024 + 1000 * rank + k)
        r = np.linalg.norm(s, axis=1)
        lat = np.arcsin(s[:, 2] / r); lon = np.arctan2(s[:, 1], s[:, 0])
        s = s[~synth._land_mask(lat, lon, "continents")]
        out.append(s); have += len(s); k += 1
    return np.concatenate(out)[:n]


def engine_build_id() -> str:
    """Identity of the engine build (mops_amd/_build_id.py: sources, headers, hipcc flags, ROCm
    release -- the id stamped into libmops_traj.so); tools/make_traffic.py stamps every PMC entry
    with it, so a changed kernel never inherits another build's measured traffic."""
    from mops_amd import _build_id
    return _build_id.build_id()


PEAK_FP64_TFLOPS = 78.6  # MI355X FP64 vector (spec; half of the guide's 157.3 TF FP32 vector rate)
# vector-L1 / texture-data return: 64 B per clock per CU (measured: tools/membench.hip mb_l1_x4 moves 64 B per
# TD-busy cycle at 97% TD busy, 38.0 TB/s chip-wide; one TCP tag access = 64 B), x 256 CUs x 2.4 GHz
PEAK_L1_RETURN_GBS = 64.0 * 256 * 2.4
L1_MEASURED_GBS = 38.0e3


def measured_entry(key: str):
    """profiles/pmc_traffic.json's entry for this workload if it was measured on this engine build.
    Returns (entry or None, provenance string)."""
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc_path):
        return None, "no profiles/pmc_traffic.json"
    try:
        pm = json.load(open(pmc_path))
    except (OSError, ValueError) as e:
        return None, f"unreadable profiles/pmc_traffic.json: {e}"
    bid = engine_build_id()
    for e in (pm if isinstance(pm, list) else [pm]):
        if e.get("workload") != key:
            continue
        if e.get("engine_build") != bid:
            return None, f"stale: the PMC entry for {key} was measured on engine build {e.get('engine_build')}, not {bid}"
        return e, (f"profiles/pmc_traffic.json[{key}] (rocprofv3 PMC passes per timed unit, engine build {bid}, "
                   f"{e.get('profile', '?')})")
    return None, f"no PMC entry for {key}"


def measured_traffic(key: str):
    """Per-launch DRAM bytes of this workload from profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE/WRITE_SIZE
    passes merged by tools/make_traffic.py), only if they were measured on this kernel build.
    Returns (bytes or None, provenance string)."""
    pmc_path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(pmc_path):
        return None, "no profiles/pmc_traffic.json"
    try:
        pm = json.load(open(pmc_path))
    except (OSError, ValueError) as e:
        return None, f"unreadable profiles/pmc_traffic.json: {e}"
    bid = engine_build_id()
    for e in (pm if isinstance(pm, list) else [pm]):
        if e.get("workload") != key:
            continue
        if e.get("engine_build") != bid:
            return None, f"stale: the PMC entry for {key} was measured on engine build {e.get('engine_build')}, not {bid}"
        return float(e["bytes_per_unit"]), (f"profiles/pmc_traffic.json[{key}] (rocprofv3 2*FETCH_SIZE + WRITE_SIZE "
                                             f"per timed unit, engine build {bid}, {e.get('profile', '?')})")
    return None, f"no PMC entry for {key}"


def _entry_of(key_or_entry):
    """(entry, provenance) for a workload key (this build's PMC entry only) or an entry given directly."""
    if isinstance(key_or_entry, dict):
        return key_or_entry, f"PMC entry {key_or_entry.get('workload')} (engine build {key_or_entry.get('engine_build')})"
    return measured_entry(key_or_entry)


# independent v_fma_f64 chains on all 1024 SIMDs (tools/fp64bench.hip, profiles/r05/fp64bench/times.jsonl): the
# sustained clock under FP64 load is ~2.0 GHz, below the 2.4 GHz of the vendor's 78.6 TF
MEASURED_FP64_FMA_TFLOPS = 61.8


def fp64_block(key, unit_s: float):
    """The FP64 vector-issue view of the same unit: PMC-counted FP64 add/mul/fma work over its time, against
    the FP64 vector peak (the path's arithmetic is FP64 scalar geometry; no MFMA applies)."""
    e, src = _entry_of(key)
    fl = e.get("fp64_flops_per_unit") if e else None
    if fl is None:
        return {"achieved": None, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": None, "source": src}
    ach = fl / unit_s / 1e12
    return {"achieved": ach, "peak": PEAK_FP64_TFLOPS, "unit": "TFLOP/s", "frac": ach / PEAK_FP64_TFLOPS,
            "measured_peak": MEASURED_FP64_FMA_TFLOPS, "frac_of_measured": ach / MEASURED_FP64_FMA_TFLOPS,
            "flops_per_unit": fl, "source": src + " SQ_INSTS_VALU_{ADD,MUL,FMA}_F64 x 64 lanes (fma = 2); "
                                                  "measured_peak: tools/fp64bench.hip fb_fma (profiles/r05/fp64bench)"}


def l1_block(key, unit_s: float):
    """The memory-return view that binds the gather kernels: bytes the vector L1 returned to the lanes
    (TCP_TOTAL_CACHE_ACCESSES x 64 B, rocprofv3) over the unit's time, against the TD return peak."""
    e, src = _entry_of(key)
    acc = e.get("tcp_accesses_per_unit") if e else None
    if acc is None or e.get("td_busy") is None:
        return {"achieved": None, "peak": PEAK_L1_RETURN_GBS, "unit": "GB/s", "frac": None, "source": src}
    td = e["td_busy"]
    tag = acc * 64.0 / unit_s / 1e9
    # frac: the TD's measured busy fraction.  achieved: the return rate that busy fraction carries at the
    # 64 B/clk/CU peak.  The tag-access rate (64 B per TCP access) is exact for coalesced 16-B lanes
    # (tools/membench.hip mb_l1_x4) and an upper bound for scattered ones (config 4: above the peak).
    return {"achieved": td * PEAK_L1_RETURN_GBS, "peak": PEAK_L1_RETURN_GBS, "peak_measured": L1_MEASURED_GBS,
            "unit": "GB/s", "frac": td, "td_busy": td, "tag_rate_gbs": tag, "tag_rate_frac": tag / PEAK_L1_RETURN_GBS,
            "l1_to_l2_bytes_per_unit": (e.get("l1_to_l2_requests_per_unit") or 0.0) * 128.0,
            "source": src + " frac = TD_TD_BUSY_sum / 256 CUs over GRBM_GUI_ACTIVE / 8 XCDs; tag_rate = "
                      "TCP_TOTAL_CACHE_ACCESSES_sum x 64 B over the launch time (upper bound for scattered lanes)"}


# SIMD cycles a wave64 VALU instruction holds, by class (tools/fp64bench.hip, profiles/r06/fp64bench/summary.txt:
# SIMD-cycles per instruction x VALUBusy): FP64 rcp / rsq / sqrt seeds 16, FP32 transcendentals 8, every other VALU
# instruction 4 -- FP64 add / mul / fma, compares, selects, conversions, 64-bit integer, VOP3 forms alike (VOP2
# v_mov_b32 / v_add_u32 / v_xor_b32 / v_fma_f32 can dual-issue: 2 cycles in pairs, SQ_ACTIVE_INST_VALU2)
VALU_CYC = 4.0
VALU_CYC_TRANS_F64 = 16.0
VALU_CYC_TRANS_F32 = 8.0


def valu_block(key):
    """The VALU-issue view: how much of the SIMDs' cycles the kernel's vector instructions hold, from the same
    profile.  Round 6 prices them by class (VALU_CYC*: 4 cycles, FP64 transcendental seeds 16, FP32 ones 8) with
    the transcendental fractions of the profile's class mix; it reconciles with rocprof's VALUBusy
    (SQ_ACTIVE_INST_VALU, tools/merge_issue.py), which counts the same cycles.  Entries without a class mix keep
    the flat 4-cycle count (`priced` False).  As a roofline: achieved = frac of the peak 1.0 (every SIMD issuing
    a VALU instruction every cycle)."""
    e, src = _entry_of(key)
    if not e or e.get("valu_issue_model") is None:
        return {"frac": None, "source": src}
    flat = e["valu_issue_model"]  # 4 cycles x SQ_INSTS_VALU / (1024 SIMDs x cycles)
    t64, t32 = e.get("valu_trans_f64_frac"), e.get("valu_trans_f32_frac")
    priced = t64 is not None and t32 is not None
    frac = flat * (1.0 + (VALU_CYC_TRANS_F64 / VALU_CYC - 1.0) * t64 + (VALU_CYC_TRANS_F32 / VALU_CYC - 1.0) * t32) \
        if priced else flat
    return {"achieved": frac, "peak": 1.0, "frac": frac, "priced": priced, "flat_4_cycle_frac": flat,
            "valu_trans_f64_frac": t64, "valu_trans_f32_frac": t32,
            "valu_busy": e.get("valu_busy"), "salu_busy": e.get("salu_busy"),
            "lds_busy": e.get("lds_busy"), "unit": "fraction of SIMD cycles",
            "source": src + " SQ_INSTS_VALU priced by class: 4 SIMD-cycles per wave64 instruction, FP64 transcendental "
                      "16, FP32 transcendental 8 (tools/fp64bench.hip, profiles/r06/fp64bench), over 1024 SIMDs x "
                      "GRBM_GUI_ACTIVE / 8; valu_busy = SQ_ACTIVE_INST_VALU x 4 / 1024 / (GRBM_GUI_ACTIVE / 8)"}


def limiter_kind(l1: dict, valu: dict) -> str:
    """The roof that binds, from the counters (the rule limiter_text states): "l1_return" (TD >= 80% busy, or
    clearly busier than the VALU), "valu_issue" (VALUBusy clearly above TD), else the busier of the two;
    "hbm" when the PMC entry has neither view."""
    td, vf = l1.get("td_busy"), valu.get("frac")
    if td is None or vf is None:
        return "hbm"
    vb = valu.get("valu_busy") or vf
    if td >= 0.8 or td > vb + 0.1:
        return "l1_return"
    if vb > td + 0.1:
        return "valu_issue"
    return "l1_return" if td >= vb else "valu_issue"


def limiter_text(l1: dict, valu: dict) -> str:
    td, vf = l1.get("td_busy"), valu.get("frac")
    if td is not None and vf is not None:
        vb = valu.get("valu_busy") or vf  # (the count model undercounts, VALUBusy overlaps waves: compare with the latter)
        if td >= 0.8 or td > vb + 0.1:
            return (f"texture-data return of the per-lane gathers: TD {td:.0%} busy (l1_return); VALU issue "
                    f"{vf:.0%} of SIMD cycles by instruction count, VALUBusy {vb:.0%} (valu_issue) -- DESIGN.md section 3")
        if vb > td + 0.1:
            return (f"VALU issue: the FP64 geometry's instructions hold {vf:.0%} of SIMD cycles by count "
                    f"(rocprof VALUBusy {vb:.0%}); TD {td:.0%} busy, DRAM far below its peak -- DESIGN.md section 3")
        return (f"TD return and VALU issue together: TD {td:.0%} busy, VALU {vf:.0%} of SIMD cycles by instruction "
                f"count (VALUBusy {vb:.0%}); DRAM far below its peak -- DESIGN.md section 3")
    return ("not DRAM: the texture-data return of the per-lane gathers (l1_return) together with FP64 VALU "
            "issue and gather latency at 3 waves/SIMD (DESIGN.md section 3)")


def bench_host() -> str:
    """This run's box: host name + the GPU's uuid and PCI address from the device properties (no subprocess: a
    process that has initialised the GPU must not start programs), as tools/profile_round.sh records the profiled
    box's (the container host name alone is not unique)."""
    ident = ""
    try:
        import torch
        pr = torch.cuda.get_device_properties(torch.cuda.current_device())
        ident = f" gpu {pr.uuid} pci {pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}"
    except Exception:  # (no GPU: the CPU tests)
        pass
    return socket.gethostname() + ident


def roofline_block(kernel: str, avg_kernel_s: float, psteps_per_launch: float, B: float, traffic_key: str,
                   per: str = "launch") -> dict:
    """The bench line's roofline: HBM GB/s MEASURED by rocprofv3 PMC counters (per launch) over the
    kernel's HIP-event launch time, against the 8 TB/s peak.  The SURVEY 8(d) bytes model is reported
    beside it, not as the roofline: it charges a full zTop column and no cross-particle reuse, so its
    rate exceeds the HBM peak -- the kernel is bound by gather latency and FP64 issue, not by DRAM."""
    traffic, src = measured_traffic(traffic_key)  # bytes per `per` unit
    achieved = traffic / avg_kernel_s / 1e9 if traffic is not None else None
    alg = B * psteps_per_launch / avg_kernel_s / 1e9
    hbm = {"achieved": achieved, "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": (achieved / PEAK_HBM_GBS) if achieved is not None else None, "traffic": traffic, "source": src}
    l1, valu = l1_block(traffic_key, avg_kernel_s), valu_block(traffic_key)
    kind = limiter_kind(l1, valu)
    top = {"hbm": hbm, "l1_return": l1, "valu_issue": valu}[kind]
    return {
        # top level = the HBM view, as BASELINE's metric defines the roofline (achieved DRAM GB/s over the 8 TB/s
        # peak).  No workload here is DRAM-bound: the roof that binds, chosen
        # from the counters (limiter_kind), is named separately in binding_roof / binding_frac.
        "bound": "hbm",
        "achieved": achieved,
        "peak": PEAK_HBM_GBS,
        "unit": "GB/s",
        "frac": hbm["frac"],
        "binding_roof": kind,
        "binding_frac": top.get("frac"),
        "binding_unit": top.get("unit"),
        "traffic": traffic,
        "traffic_source": src,
        "hbm": hbm,
        "limiter": limiter_text(l1, valu),
        "valu_issue": valu,
        "fp64_valu": fp64_block(traffic_key, avg_kernel_s),
        "l1_return": l1,
        "traffic_correction": ("bytes = 2 x FETCH_SIZE + WRITE_SIZE: the gfx950 factor 1/2 holds for this kernel's "
                               "scattered 80-B record reads too (tools/membench.hip: 4 GiB streamed -> FETCH_SIZE "
                               "0.500 of the bytes; 2^25 random 80-B records, one per 128-B line -> 2 x FETCH_SIZE "
                               "= 1.03 x the lines), DESIGN.md section 3.2"),
        "kernel": kernel,
        "timed_unit": per,
        "particle_steps_per_launch": psteps_per_launch,
        "avg_launch_ms": avg_kernel_s * 1e3,
        "bench_host": bench_host(),
        # the PMC entry's box and its rocprofv3 launch average: the counters' cycles are that box's, the rate above is
        # this run's (box-to-box spread ~3%)
        "pmc_host": (measured_entry(traffic_key)[0] or {}).get("profile_host"),
        "pmc_avg_launch_ms": (measured_entry(traffic_key)[0] or {}).get("profile_avg_launch_ms"),
        "algorithmic_model": {
            "bytes_per_particle_step": B,
            "gbs": alg,
            "source": "SURVEY.md 8(d): one compulsory stencil fetch per particle-step, full zTop column (8*nv*L)",
            "note": ("a model of what a reuse-free implementation would fetch; the engine reads one level-pair "
                     "record per vertex and lanes share stencils through L1/L2, so this rate is not a DRAM rate "
                     "and may exceed the HBM peak"),
        },
    }


def algorithmic_bytes_per_pstep(nv: float, L: int, S: int = 1) -> float:
    """one compulsory fetch of the particle's cell stencil per step."""
    return (4 + 4 * nv + 4 * nv + 24 * nv + 24 * (nv + 1) + S * (8 * nv * L + 2 * 24 * nv + 2 * 8 * nv) + 32)


CONFIG3 = dict(mode="pathline", particles=10_000_000, dt=60, duration=86400, record=3600, method="euler")
# (configs 3-5: `duration` is the daily snapshot spacing; config 5's snapshots are monthly -- each pair's
# duration comes from its calendar month, chain_timestamps)
# oRRS18to6 class: frequency-608 icosahedral dual (3.7M cells, 3.5M after the land cull), 80 levels
CONFIG4 = dict(mode="pathline", particles=10_000_000, dt=120, duration=86400, record=3600, method="euler",
               depth=20.0, freq=608, levels=80)
CONFIG5 = dict(mode="pathline", particles=12_500_000, dt=60, duration=30 * 86400, record=86400,
               method="euler", depth=20.0, freq=608, levels=80)
PAIRS_DEFAULT = {3: 7, 4: 30, 5: 12}


def chain_timestamps(config: int, pairs: int, spacing: int = 86400) -> list:
    """MPAS xtime of the chain's snapshots: daily from 0001-01-01 (configs 3/4), or the first day of
    each month from January 0001 (config 5: calendar-month pairs, MOPSPathline._month_pairs_forward);
    the chain derives each pair's simulationDuration from them (chain.pair_gaps)."""
    from mops_amd import chain
    if config == 5:
        mp = chain.month_pairs_forward(1, 1, 1 + (pairs // 12) + 1, 12)[:pairs]
        if len(mp) != pairs:
            raise ValueError("month pairs")
        return chain.month_timestamps(mp)
    from datetime import datetime, timedelta
    t0 = datetime(1, 1, 1)
    return [(t0 + timedelta(seconds=spacing * i)).strftime("%Y-%m-%d_%H:%M:%S").rjust(19, "0")
            for i in range(pairs + 1)]


def layer_mid_depth(mesh, layer: int = 10) -> float:
    """"fixed layer 10" = mid-depth of 0-based layer 10."""
    return 0.5 * (float(mesh.refBottomDepth[layer - 1]) + float(mesh.refBottomDepth[layer]))


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(gpus: int, argv, port: int) -> list:
    """The one-process-per-GPU launch of this script for ``--gpus N`` (N > 1) when no launcher set
    WORLD_SIZE: torch.distributed.run with N local ranks over 127.0.0.1, the same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]


def check_world(gpus: int, world: int) -> None:
    if world != gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started {world} rank(s) (WORLD_SIZE); "
                         "run `python bench.py --gpus N` alone (it starts the ranks itself) or under "
                         "torch.distributed.run with --nproc-per-node N")


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # no launcher: start the N ranks as child processes (before anything touches the GPU; never
        # exec) and exit with their status -- rank 0 prints the line
        import subprocess
        sys.exit(subprocess.run(launcher_command(args.gpus, sys.argv[1:], free_port())).returncode)
    check_world(args.gpus, int(os.environ.get("WORLD_SIZE", "1")))
    apply_config_defaults(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MOPS_BENCH_ONE_DEVICE") == "1":  # rehearsal: every rank on device 0
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    from mops_amd import synth
    from mops_amd.distributed import RecordGather
    from mops_amd.engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig

    mesh = synth.make_mesh(args.freq, n_levels=args.levels)
    if args.config == 3:
        args.depth = layer_mid_depth(mesh, 10)
    if args.config in (3, 4, 5):
        return main_chain(args, mesh, dev, world, rank)
    snap = synth.make_snapshot(mesh, timestep=0, topography=args.topography)
    dmesh = DeviceMesh.from_mesh(mesh)
    dfield = DeviceField.from_snapshot(dmesh, snap)
    pathline = args.mode == "pathline"
    dback = (DeviceField.from_snapshot(dmesh, synth.make_snapshot(mesh, timestep=1, phase=0.35,
                                                                  topography=args.topography))
             if pathline else None)
    seeds = make_seeds(args.particles, rank)
    n = seeds.shape[0]
    cfg = TrajectoryConfig(deltaT=args.dt, simulationDuration=args.duration, recordT=args.record, depth=args.depth,
                           method=1 if args.method == "euler" else 0)
    ps = ParticleSet(dmesh, seeds, args.depth, cfg, device=dev)
    seed_cells = ps.original(ps.cell).cpu().numpy()
    period = ps.record_period(pathline=pathline)
    n_steps = cfg.n_steps
    # launches: the whole run as one segment (every launch re-reads the particle state and
    # re-loads each particle's cell stencil: 30-step launches cost 6% at config 2)
    seg = args.segment if args.segment > 0 else n_steps
    seg = max(period, (seg // period) * period)  # whole record periods per launch
    bounds = list(range(0, n_steps, seg)) + [n_steps]
    segments = [(bounds[i], bounds[i + 1]) for i in range(len(bounds) - 1)]
    compute = torch.cuda.Stream(dev)
    comm = torch.cuda.Stream(dev)
    part_streams = [torch.cuda.Stream(dev) for _ in range(max(1, args.parts))]
    gather_records = world > 1 and args.gather in ("records", "root")
    collector = ckpt = gathered_ckpt = None
    if world > 1 and gather_records:
        # every call's record slab + seeds + slot ids, gathered on `comm` while the next call computes
        collector = RecordGather(dist, ps, world, backend=args.backend, comm_stream=comm,
                                 mode="root" if args.gather == "root" else "all")
    elif world > 1:
        ckpt = torch.empty((6, n), dtype=torch.float64, device=dev)  # x, y, z, depth, death step, slot id
        gathered_ckpt = torch.empty((world, 6, n), dtype=torch.float64, device=dev)

    kernel_ms = []
    finalize_ms = []  # line assembly + NaN cleanup per call
    lines_out = [None]  # the last call's finalized lines (kept alive until the next call)
    compact = args.compact == "on" or (args.compact == "auto" and args.method == "rk4")
    dispatch_ms = []  # per traj_kernel launch (HIP events on its part stream): what rocprofv3 averages
    ev_ckpt = [None]  # comm-stream event of the last checkpoint gather

    def one_call(timed: bool, pset=None):
        """One StreamLine call on this rank's shard (device resident); ``pset``: another ParticleSet
        of the same seeds (the RK4 companion line)."""
        ps_ = pset if pset is not None else ps
        with torch.cuda.stream(compute):
            ps_.reset(depth=args.depth)
            dmesh.locate(ps_.seeds.data_ptr(), ps_.cell.data_ptr(), n, stream=compute)  # seeds in slot order
            ps_.reorder(stream=compute)
            for (s0, s1) in segments:
                # the segment's trajectory launches: particle parts on their own streams, each in
                # step chunks, so one part's final partial round of waves overlaps the others' work
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(compute)
                for st in part_streams:
                    st.wait_event(e0)
                nch = max(1, round(args.chunks * (s1 - s0) / n_steps))
                ps_.advance_pipelined(dfield, dback, s0, s1, part_streams, nch,
                                     timing=dispatch_ms if timed else None,
                                     compact=compact or (pset is not None and args.compact != "off"),
                                     compact_priority=args.compact_priority)
                for st in part_streams:
                    j = torch.cuda.Event(); j.record(st); compute.wait_event(j)
                e1.record(compute)
                if timed:
                    kernel_ms.append((e0, e1))
                if (s0, s1) == segments[-1]:
                    # the reference's StreamLine ends by assembling the lines (FinalizeTrajectoryLines +
                    # RemoveNaN, MPASOVisualizerKernels.cpp:1005-1014), part of every call: each particle
                    # part's lines on its own stream, overlapping the other parts' final waves
                    fin = []
                    if args.finalize == "parts":
                        lines_out[0] = ps_.finalize(pathline, streams=part_streams, timing=fin)
                        for st in part_streams:
                            j = torch.cuda.Event(); j.record(st); compute.wait_event(j)
                    else:
                        lines_out[0] = ps_.finalize(pathline, stream=compute, timing=fin)
                    if timed:
                        finalize_ms.append(fin)
            # (every re-sort and compaction of the call is done: the slot ids, seeds and records below are
            # in one consistent slot order -- ADVICE r3: ids gathered right after the first sort went stale
            # once the compactions permuted the slots)
            if world > 1 and pset is None:
                if gather_records:
                    collector.collect(ps_, compute)  # records + seeds + ids; ps_ moves to the spare slab
                else:  # the checkpoint: every particle's final state (+ its slot id) on every rank
                    if ev_ckpt[0] is not None:  # the previous call's checkpoint gather has read ckpt
                        compute.wait_event(ev_ckpt[0])
                    ckpt[0].copy_(ps_.x); ckpt[1].copy_(ps_.y); ckpt[2].copy_(ps_.z)
                    ckpt[3].copy_(ps_.depth); ckpt[4].copy_(ps_.death); ckpt[5].copy_(ps_.ids)
                    done = torch.cuda.Event()
                    done.record(compute)
                    comm.wait_event(done)
                    with torch.cuda.stream(comm):
                        all_gather_flat(dist, gathered_ckpt.view(-1), ckpt.view(-1), args.backend)
                        ev_ckpt[0] = torch.cuda.Event()
                        ev_ckpt[0].record(comm)
        compute.synchronize()
        # the gathers overlap the next call's compute (events order the buffers); the timed region's
        # closing device synchronize waits for the last one

    for _ in range(args.warmup):
        one_call(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_call(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()

    # attempted particle-steps (a step counts once its velocity evaluation ran)
    death = ps.death.to(torch.int64)
    attempted = torch.where(death < 0, torch.full_like(death, n_steps), death + 1).sum().item()
    dead = int((death >= 0).sum().item())
    # the north star's integrator on the same workload, timed after the Euler line (N = 1 only;
    # not part of `value`, which is the reference's default integrator, MPASOVisualizer.h:99)
    rk4 = None
    if world == 1 and args.method == "euler" and not pathline and os.environ.get("MOPS_BENCH_NO_RK4") != "1":
        cfg4 = TrajectoryConfig(deltaT=args.dt, simulationDuration=args.duration, recordT=args.record,
                                depth=args.depth, method=0)
        ps4 = ParticleSet(dmesh, seeds, args.depth, cfg4, device=dev)
        torch.cuda.synchronize()  # its locate + locality order ran on the current stream, not `compute`
        one_call(False, ps4)
        torch.cuda.synchronize()
        t4 = time.perf_counter()
        one_call(False, ps4)
        torch.cuda.synchronize()
        el4 = time.perf_counter() - t4
        d4 = ps4.death.to(torch.int64)
        att4 = torch.where(d4 < 0, torch.full_like(d4, n_steps), d4 + 1).sum().item()
        rk4 = {"value": att4 / el4, "unit": "particle-steps/s", "ms_per_call": el4 * 1e3,
               "dead_fraction": float((d4 >= 0).sum().item()) / max(n, 1),
               "dead_particle_compaction": args.compact != "off",
               "note": "same workload integrated with RK4 (four evaluations per step in the step's start "
                       "cell, quirk Q1), one timed call after the Euler line; not part of value"}
        del ps4
    kms = [a.elapsed_time(b) for (a, b) in kernel_ms]
    avg_kernel_s = (sum(kms) / len(kms)) / 1e3 if kms else float("nan")
    dms = [a.elapsed_time(b) for (a, b) in dispatch_ms]
    stats = torch.tensor([elapsed, float(attempted), float(n), float(dead)], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        mx = stats.clone(); dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone(); dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed = mx[0].item()
        attempted_all, n_all, dead_all = sm[1].item(), sm[2].item(), sm[3].item()
    else:
        attempted_all, n_all, dead_all = float(attempted), float(n), float(dead)

    value = attempted_all * args.steps / elapsed
    nv_mean = float(np.mean(mesh.nEdgesOnCell.astype(np.float64)))
    B = algorithmic_bytes_per_pstep(nv_mean, mesh.nVertLevels, 2 if pathline else 1)
    psteps_per_launch = attempted / len(segments)
    roof = roofline_block(f"traj_kernel<7,{str(pathline).lower()},{str(args.method == 'euler').lower()}> "
                          f"({args.mode} {args.method})", avg_kernel_s, psteps_per_launch, B,
                          f"ec30to60_{args.mode}_{args.method}_{args.particles}_seg{seg}_p{args.parts}c{args.chunks}",
                          per=f"segment ({args.parts} particle parts x {args.chunks} step chunks = "
                              f"{args.parts * args.chunks} overlapping traj_kernel launches)")
    roof["dispatches_per_unit"] = len(dms) / max(1, args.steps * len(segments))
    roof["avg_dispatch_ms"] = (sum(dms) / len(dms)) if dms else None  # = rocprofv3's traj_kernel average
    fms = [sum(a.elapsed_time(b) for (a, b) in call) for call in finalize_ms]  # part launches per call
    finalize_avg = (sum(fms) / len(fms)) if fms else None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        back_snap = (synth.make_snapshot(mesh, timestep=1, phase=0.35, topography=args.topography)
                     if pathline else None)
        cpu = cpu_baseline(mesh, snap, back_snap, seeds, seed_cells, args, n_steps)

    print_prof_counters()
    if rank == 0:
        line = {
            "metric": "particle-steps/sec",
            "value": value,
            "unit": "particle-steps/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (icosahedral-dual Voronoi mesh, analytic flow; no MPAS files offline)",
            "config": {
                "workload": (f"EC30to60-class {args.mode} (BASELINE config 2), {n:.0e} particles/GPU, depth "
                             f"{args.depth:g} m, dt {args.dt} s, {args.duration / 86400:g} day"),
                "cells": mesh.nCells, "vertices": mesh.nVertices, "levels": mesh.nVertLevels,
                "particles_per_gpu": n, "particles_total": int(n_all), "integration_steps": n_steps,
                "records": ps.K, "method": args.method, "parallelism": f"particle-shard x{world}",
                "topography": args.topography,
                "record_gather": record_gather_text(world, args, per="call", K=ps.K, collector=collector),
                "record_gather_plan": (collector.plan(compute_s_per_checkpoint=elapsed / args.steps)
                                       if collector is not None else None),
            },
            "nominal_particle_steps_per_call": n_all * n_steps,
            "attempted_particle_steps_per_call": attempted_all,
            "dead_fraction": dead_all / max(n_all, 1),
            "finalize": {"ms_per_call": finalize_avg, "mode": args.finalize,
                         "share_of_step": (finalize_avg / (elapsed / args.steps * 1e3)) if finalize_avg else None,
                         "what": "line assembly + NaN cleanup on device (assemble_clean_kernel, or assemble_kernel + "
                                 "remove_nan_kernel past 24 records), inside every timed call as in the reference's "
                                 "StreamLine: one launch per particle part on its stream (ms_per_call sums them), "
                                 "overlapping the other parts' final waves"},
            "dead_particle_compaction": compact,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if rk4 is not None:
            line["rk4_companion"] = rk4
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def record_gather_text(world: int, args, per: str, K: int, collector=None) -> str:
    """What the N > 1 line collects (the bench line states it)."""
    if world == 1:
        return "none (one rank: its lines are assembled on the device every " + per + ")"
    be = "rccl" if args.backend == "nccl" else "gloo"
    if args.gather in ("records", "root"):
        if args.gather == "root":
            txt = (f"{be} gather to rank 0 at every {per} of each rank's record slab ({K} records x 48 B per particle, "
                   "in slot order) + seeds + slot ids (distributed.RecordGather mode 'root'): rank 0 holds every "
                   "particle's trajectory records, overlapped with the next " + per)
        else:
            txt = (f"{be} all_gather at every {per} of each rank's record slab ({K} records x 48 B per particle, in "
                   "slot order) + seeds + slot ids (distributed.RecordGather): every rank holds every particle's "
                   "trajectory records, overlapped with the next " + per)
        if collector is not None:
            txt += f"; {collector.bytes_per_rank / max(1, collector.checkpoints) / 1e9:.3f} GB sent per rank per {per}"
            if collector.chunk < collector.shape[0]:
                txt += (f", in chunks of {collector.chunk} records through a {collector.gathered.numel() * 8 / 1e9:.1f} GB "
                        "ring (the whole gathered slab does not fit beside the fields)")
        return txt
    return (f"{be} all_gather at every {per} of the final state / continuation points (+ slot ids); records stay "
            "sharded on their rank")


def print_prof_counters():
    """Event counters of an experiment build (-DMOPS_PROF, MOPS_PROF_SECTIONS=1) to stderr."""
    if os.environ.get("MOPS_PROF_SECTIONS") == "1":
        import ctypes
        from mops_amd import _lib
        buf = (ctypes.c_uint64 * 16)()
        _lib.load().mops_debug_prof(buf)
        print("prof counters lane-steps, lane walks, lane loads, wave-steps, wave-steps walking, wave-steps loading, "
              "coop wave-steps, coop groups, cells per wave-step (sum), (cell, hint) groups (sum), wave-steps with "
              "<= 2 cells, with <= 2 groups, wave-steps, lane-steps the neighbour table kept, RK4 hand-offs (waves), of them outside a hexagon:",
              list(buf), file=sys.stderr)


def main_chain(args, mesh, dev, world, rank):
    """BASELINE configs 3-5: chained snapshot-pair pathlines (MOPSPathline.run semantics, mops_amd/chain.py),
    each pair's simulationDuration from the snapshots' timestamps (daily for configs 3/4, calendar months
    for config 5).

    config 3: 1e7 particles/GPU, "layer 10", dt 60 s, 7 daily pairs; all 8 derived snapshots are resident in
    HBM before the timed region.  configs 4/5: oRRS18to6-class mesh; each snapshot is generated and derived in
    HBM inside the timed region (mops_field_create_device), two fields resident.  One bench step = the whole
    chain (seed locate per pair, every integration step, per-pair line assembly on device, and for N > 1 an
    RCCL all-gather of each pair's record slab + seeds + slot ids, overlapped with the next pair)."""
    import torch
    import torch.distributed as dist
    from mops_amd import synth
    from mops_amd.chain import PathlineChain, pair_gaps
    from mops_amd.distributed import RecordGather, max_shard, shard_bounds
    from mops_amd.engine import DeviceField, DeviceMesh

    n_snap = args.pairs + 1
    stamps = chain_timestamps(args.config, args.pairs, spacing=args.duration)
    gaps = pair_gaps(stamps)
    dmesh = DeviceMesh.from_mesh(mesh)
    snaps = None
    if args.config == 3:
        snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.35 * t) for t in range(n_snap)]
        fields = [DeviceField.from_snapshot(dmesh, s) for s in snaps]
        chain = PathlineChain(dmesh, lambda i, stream: fields[i], n_snap, timestamps=stamps, device=dev,
                              own_fields=False)
    else:
        from mops_amd.synth_device import DeviceFieldRecycler, DeviceSnapshotSource
        src = DeviceSnapshotSource(mesh, dev)
        recycler = DeviceFieldRecycler(dmesh, src)
        side_cus = args.side_cus or 0
        overlap = None
        if side_cus != 0 and n_snap > 2:
            from mops_amd.chain import cu_split_streams
            if side_cus > 0:
                compute_masked, overlap = cu_split_streams(dev, side_cus)
            else:
                compute_masked, overlap = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
            recycler.side = overlap  # snapshot generation runs there too
        # the field buffers (2, or 3 with the overlap stream) are allocated before the timed region
        # (hipMalloc of ~75 GB each is setup); every snapshot a call uses is still generated and
        # derived inside it
        bufs = [recycler(i, torch.cuda.current_stream(dev).cuda_stream) for i in range(3 if overlap else 2)]
        for b in bufs:
            recycler.release(b)
        del bufs
        torch.cuda.synchronize()
        chain = PathlineChain(dmesh, recycler, n_snap, timestamps=stamps,
                              device=dev, own_fields=True, prefetch=False, overlap_stream=overlap)
        chain.overlap_stream_cus = side_cus
    if args.config == 4:  # strong scaling: 1e7 particles in total, one contiguous shard per rank
        allseeds = make_seeds(args.particles, 0)
        lo, hi = shard_bounds(len(allseeds), rank, world)
        seeds = allseeds[lo:hi]
        n_pad = max_shard(len(allseeds), world)
        del allseeds
    else:
        seeds = make_gaussian_seeds(args.particles, rank) if args.config == 5 else make_seeds(args.particles, rank)
        n_pad = seeds.shape[0]
    n = seeds.shape[0]
    compute = torch.cuda.Stream(dev)
    if args.config in (4, 5) and chain.overlap_stream is not None:
        compute = compute_masked  # the trajectory launches leave the side stream's CUs free
    comm = torch.cuda.Stream(dev)
    if world > 1 and args.config != 4:  # weak scaling: every rank must hold the same particle count
        t = torch.tensor([n, -n], dtype=torch.int64, device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        if int(t[0].item()) != -int(t[1].item()):
            raise SystemExit("bench.py: ranks drew different particle counts")
    gather_records = world > 1 and args.gather in ("records", "root")
    defer_lines = args.defer_lines and not gather_records  # (RecordGather reads the pair's slab in on_pair)
    gathered = torch.empty((world, n_pad, 3), dtype=torch.float64, device=dev) if world > 1 else None
    send = torch.zeros((n_pad, 3), dtype=torch.float64, device=dev) if world > 1 else None
    collector = [None]
    timing = []

    t_start = [time.perf_counter()]

    def on_pair(p, last, ps):
        if rank == 0 and (args.pairs > 7 or world > 1):  # progress for long chains and multi-rank runs (stderr)
            print(f"[bench] pair {p + 1}/{args.pairs} enqueued at {time.perf_counter() - t_start[0]:.1f} s",
                  file=sys.stderr, flush=True)
        if gather_records:  # the pair's trajectory records (+ seeds, slot ids) on every rank
            if collector[0] is None:
                # the ring of gathered records must fit beside the fields (config 5 at 8 ranks gathers 149 GB
                # per pair: chunks of records through a bounded ring, RecordGather(max_bytes))
                free, _ = torch.cuda.mem_get_info(dev)
                budget = int(0.6 * (free - 2 * ps.records.numel() * 8))
                collector[0] = RecordGather(dist, ps, world, backend=args.backend, comm_stream=comm,
                                            max_bytes=max(budget, 1 << 30),
                                            mode="root" if args.gather == "root" else "all")
            collector[0].collect(ps, compute)
        elif world > 1:  # checkpoint: every rank gets the continuation points of all shards
            done = torch.cuda.Event(); done.record(compute)
            comm.wait_event(done)
            last.record_stream(comm)
            with torch.cuda.stream(comm):
                send[:n].copy_(last)
                all_gather_flat(dist, gathered.view(-1), send.view(-1), args.backend)

    on_pair.reads_records = gather_records  # (PathlineChain.run refuses defer_lines with a record-reading on_pair)
    seeds_dev = torch.as_tensor(np.ascontiguousarray(seeds, dtype=np.float64), device=dev)  # resident before timing

    def one_call(timed):
        res = chain.run(seeds_dev, depth=args.depth, method=1 if args.method == "euler" else 0, delta_t=args.dt,
                        record_t=args.record, keep_lines=False, compute_stream=compute, on_pair=on_pair,
                        timing=timing if timed else None, segment_steps=args.segment if args.segment else -1,
                        record_stride=n_pad, defer_lines=defer_lines, compact_chunks=RK4_COMPACT_CHUNKS)
        compute.synchronize(); comm.synchronize()
        return res

    if rank == 0:
        print(f"[bench] config {args.config}: setup done, {args.warmup} warmup + {args.steps} timed chains",
              file=sys.stderr, flush=True)
    for _ in range(args.warmup):
        one_call(False)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    attempted = 0
    for k in range(args.steps):
        attempted += int(one_call(True)["attempted"].item())
        if rank == 0:
            print(f"[bench] timed chain {k + 1}/{args.steps} done at {time.perf_counter() - t0:.1f} s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    print_prof_counters()
    kms = [a.elapsed_time(b) for (a, b) in timing]
    avg_kernel_s = (sum(kms) / len(kms)) / 1e3
    stats = torch.tensor([elapsed, float(attempted), float(n)], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
    if world > 1:
        mx = stats.clone(); dist.all_reduce(mx, op=dist.ReduceOp.MAX)
        sm = stats.clone(); dist.all_reduce(sm, op=dist.ReduceOp.SUM)
        elapsed, attempted_all, n_all = mx[0].item(), sm[1].item(), sm[2].item()
    else:
        attempted_all, n_all = float(attempted), float(n)
    n_steps = sum(g // args.dt for g in gaps)
    value = attempted_all / elapsed
    nv_mean = float(np.mean(mesh.nEdgesOnCell.astype(np.float64)))
    B = algorithmic_bytes_per_pstep(nv_mean, mesh.nVertLevels, 2)
    launches_per_call = len(timing) / args.steps
    psteps_per_launch = attempted / args.steps / launches_per_call
    mesh_class = "EC30to60" if args.config == 3 else "oRRS18to6"
    from mops_amd.chain import REORDER_SECONDS
    seg_key = args.segment if args.segment > 0 else min(gaps[0] // args.dt, REORDER_SECONDS // args.dt)
    kname = (f"traj_kernel<7,true,true,true|false> (pathline euler: the cooperative-tile instantiation where the "
             f"launch's sampled cells per wave are <= 6, else the plain one; both dispatched, the other exits at once)"
             if args.method == "euler" else "traj_kernel<7,true,false> (pathline rk4)")
    key_tail = f"seg{seg_key}" if args.method == "euler" else f"compact{RK4_COMPACT_CHUNKS}"  # (RK4: compaction)
    roof = roofline_block(kname,
                          avg_kernel_s, psteps_per_launch, B,
                          f"{mesh_class.lower()}_chain{args.config}_{args.method}_{args.particles}_{key_tail}")
    # the north star's integrator (and the reference caller's default, MOPSPathline.run(method="rk4"),
    # tutorial/pyMOPSAPI.py:1396) on the same chain, timed after the Euler line (N = 1; not part of value)
    rk4 = deliver = None
    companions = os.environ.get("MOPS_BENCH_NO_RK4") != "1" and os.environ.get("MOPS_BENCH_NO_COMPANIONS") != "1"
    if world == 1 and args.method == "euler" and args.config == 3 and companions:
        rk4 = chain_rk4_companion(args, chain, seeds_dev, compute, n, n_pad, gaps, B, mesh_class)
    if world == 1 and args.method == "euler" and args.config == 3 and companions and args.deliver == "host":
        deliver = chain_host_delivery(args, chain, seeds_dev, compute, n, n_pad, gaps, elapsed / args.steps)
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        seed_cells = dmesh_locate_host(dmesh, seeds, dev)
        if snaps is None:  # configs 4/5: the first pair's snapshots, built on the host for the oracle
            snaps = [synth.make_snapshot(mesh, timestep=t, phase=0.35 * t) for t in range(2)]
        cpu = cpu_baseline(mesh, snaps[0], snaps[1], seeds, seed_cells, args, gaps[0] // args.dt,
                           duration=gaps[0])
    days = sum(gaps) / 86400
    if args.config == 3:
        workload = (f"EC30to60-class chained pathline (BASELINE config 3), {n:.0e} particles/GPU, layer 10 "
                    f"({args.depth:.1f} m), dt {args.dt} s, {days:g} days = {args.pairs} daily pairs")
    elif args.config == 4:
        workload = (f"oRRS18to6-class chained pathline (BASELINE config 4), {int(n_all):.0e} particles in total "
                    f"({n} on this rank), depth {args.depth:g} m, dt {args.dt} s, {days:g} days = {args.pairs} "
                    "daily pairs, snapshots generated + derived in HBM inside the timed region")
    else:
        workload = (f"oRRS18to6-class chained pathline (BASELINE config 5), {n:.3g} Gaussian Gulf-of-Mexico particles"
                    f"/GPU, depth {args.depth:g} m, dt {args.dt} s, "
                    + (f"all {args.pairs} calendar-month pairs of the year ({days:g} days)" if args.pairs >= 12 else
                       f"the first {args.pairs} calendar-month pair(s) of the year ({days:g} days; a bounded "
                       "sample of the 12)")
                    + ", snapshots generated + derived in HBM inside the timed region")
    if rank == 0:
        line = {
            "metric": "particle-steps/sec", "value": value, "unit": "particle-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong" if args.config == 4 else "weak", "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (icosahedral-dual Voronoi mesh, analytic flow phase-shifted per snapshot)",
            "config": {
                "workload": workload,
                "cells": mesh.nCells, "vertices": mesh.nVertices, "levels": mesh.nVertLevels,
                "particles_per_gpu": n, "particles_total": int(n_all), "integration_steps": n_steps,
                "snapshot_times": [stamps[0], stamps[-1]], "pair_seconds": sorted(set(gaps)),
                "records_per_pair": sorted({g // args.record for g in gaps}), "record_t": args.record,
                "method": args.method, "parallelism": f"particle-shard x{world}",
                "snapshot_overlap": (
                    ((f"snapshot p+2 generated + derived on a {chain.overlap_stream_cus}-CU side stream"
                      if chain.overlap_stream_cus > 0 else "snapshot p+2 generated + derived on an unmasked side stream")
                     + " during pair p (3 field buffers)") if chain.overlap_stream is not None else
                    "snapshot p+2 generated on a side stream beside pair p's launches, derived after pair p"
                    if args.config in (4, 5) else "none (every snapshot derived before the timed region)"),
                "line_assembly": ("each pair's lines assembled on a side stream beside the next pair (second record "
                                  "slab; the continuation points from mops_traj_last_points)" if defer_lines else
                                  "each pair's lines assembled before the next pair starts"),
                "record_gather": record_gather_text(world, args, per="pair", K=max(g // args.record for g in gaps),
                                                    collector=collector[0]),
                "record_gather_plan": (collector[0].plan(compute_s_per_checkpoint=elapsed / args.steps / args.pairs)
                                       if collector[0] is not None else None)},
            "nominal_particle_steps_per_call": n_all * n_steps,
            "attempted_particle_steps_per_call": attempted_all / args.steps,
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if rk4 is not None:
            line["rk4_companion"] = rk4
        if deliver is not None:
            line["host_delivery"] = deliver
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def chain_host_delivery(args, chain, seeds_dev, compute, n, n_pad, gaps, plain_s_per_chain):
    """The caller-shaped rate: the same Euler chain with every pair's lines delivered to pinned
    host memory, as the reference's API returns them (MOPSApp.cpp:254-337 vector<TrajectoryLine>;
    bindings.cpp:383-455 list[dict]; MOPSPathline.run's per-pair accumulation, pyMOPSAPI.py:1497-1518).
    chain.HostLineSink stages each pair's lines on the device and moves them over PCIe on a copy stream while
    the next pair computes.  One untimed and one timed chain; exposed_d2h_ms_per_pair = (this chain - the
    line's device-resident chain) / pairs."""
    import torch
    from mops_amd.chain import HostLineSink
    K = max(g // args.record for g in gaps)
    t_alloc = time.perf_counter()
    sink = HostLineSink(n, K, compute.device)
    alloc_s = time.perf_counter() - t_alloc

    def run(timed):
        res = chain.run(seeds_dev, depth=args.depth, method=1, delta_t=args.dt, record_t=args.record,
                        keep_lines=False, compute_stream=compute, on_lines=sink,
                        segment_steps=args.segment if args.segment else -1, record_stride=n_pad,
                        compact_chunks=RK4_COMPACT_CHUNKS)
        compute.synchronize()
        sink.synchronize()
        return res

    run(False)
    sink.d2h_events.clear()
    sink.pairs = 0
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = run(True)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    att = float(res["attempted"].item())
    st = sink.d2h_stats()
    pairs = len(gaps)
    return {"value": att / el, "unit": "particle-steps/s", "ms_per_chain": el * 1e3,
            "exposed_d2h_ms_per_pair": (el - plain_s_per_chain) * 1e3 / pairs,
            "d2h_bytes_per_pair": st["bytes"] / pairs, "d2h_ms_per_pair": st["ms"] / pairs, "d2h_gbs": st["gbs"],
            "pinned_host_bytes": sum(v.numel() * v.element_size() for b in sink.hostbufs for v in b.values()),
            "setup_s": alloc_s,
            "note": ("the line's Euler chain with every pair's lines {points, velocity, temperature, salinity} + row "
                     "ids delivered to pinned host buffers (chain.HostLineSink: a device staging copy on the compute "
                     "stream, then PCIe on a copy stream overlapped with the next pair; two buffer sets, a caller "
                     "consumes each pair before the one two pairs later arrives); value = attempted particle-steps / "
                     "s including the last pair's copy; not part of the line's value, which keeps the lines in HBM")}


RK4_COMPACT_CHUNKS = 6  # PathlineChain.run's default: launches per pair with a dead-particle compaction between


def chain_rk4_companion(args, chain, seeds_dev, compute, n, n_pad, gaps, B, mesh_class):
    """The same chain integrated with RK4 (MOPSPathline.run's default integrator): one untimed and one
    timed chain, dead-particle compaction between RK4_COMPACT_CHUNKS launches per pair (quirk Q1 kills a
    particle at its first cell crossing; a pair's dead particles restart the next pair at their lastPoint).
    Reports attempted and nominal particle-steps, each pair's dead fraction and the RK4 kernel's roofline."""
    import torch
    timing4 = []
    n_steps = sum(g // args.dt for g in gaps)

    def run4(timed):
        deads = []

        def on4(p, last, ps):
            with torch.cuda.stream(compute):
                deads.append((ps.death >= 0).sum())
        res = chain.run(seeds_dev, depth=args.depth, method=0, delta_t=args.dt, record_t=args.record,
                        keep_lines=False, compute_stream=compute, on_pair=on4, timing=timing4 if timed else None,
                        segment_steps=args.segment if args.segment else -1, record_stride=n_pad,
                        compact=True, compact_chunks=RK4_COMPACT_CHUNKS)
        compute.synchronize()
        return res, deads

    run4(False)
    torch.cuda.synchronize()
    t4 = time.perf_counter()
    res4, deads = run4(True)
    torch.cuda.synchronize()
    el4 = time.perf_counter() - t4
    att4 = float(res4["attempted"].item())
    kms = [a.elapsed_time(b) for (a, b) in timing4]
    avg_s = (sum(kms) / len(kms)) / 1e3
    roof = roofline_block("traj_kernel<7,true,false,true|false> (pathline rk4: the cooperative-tile instantiation "
                          "where the launch's sampled cells per wave are <= 6, else the plain one)",
                          avg_s, att4 / len(kms), B,
                          f"{mesh_class.lower()}_chain{args.config}_rk4_{args.particles}_compact{RK4_COMPACT_CHUNKS}")
    roof["launches_per_chain"] = len(kms)
    return {"value": att4 / el4, "unit": "particle-steps/s", "ms_per_chain": el4 * 1e3,
            "attempted_particle_steps_per_chain": att4, "nominal_particle_steps_per_chain": float(n) * n_steps,
            "dead_fraction_per_pair": [float(d.item()) / max(n, 1) for d in deads],
            "dead_particle_compaction": f"{RK4_COMPACT_CHUNKS} launches per pair, live particles compacted between",
            "kernel_ms_per_chain": sum(kms),
            "roofline": roof,
            "note": ("the same 7-pair chain integrated with RK4 (MOPSPathline.run's default, four evaluations per step "
                     "in the step's start cell, quirk Q1: a particle dies at its first cell crossing and restarts "
                     "the next pair at its lastPoint), one timed chain after the Euler line; value = attempted "
                     "particle-steps / s; not part of the line's value")}


def dmesh_locate_host(dmesh, seeds, dev):
    import torch
    s = torch.as_tensor(np.ascontiguousarray(seeds, dtype=np.float64), device=dev)
    c = torch.empty((s.shape[0],), dtype=torch.int32, device=dev)
    dmesh.locate(s.data_ptr(), c.data_ptr(), int(s.shape[0]))
    torch.cuda.synchronize()
    return c.cpu().numpy()


CPU_CALIBRATION = os.path.join(ROOT, "profiles", "r04", "cpu_calibration.json")


def cpu_calibration(threads: int):
    """The port's speed relative to the reference's own TBB path (tools/calibrate_cpu.py: the port timed on the
    survey's probe shape in the build container, against the survey's timings of the reference built there),
    for the thread count closest to ``threads``."""
    try:
        cal = json.load(open(CPU_CALIBRATION))
    except (OSError, ValueError):
        return None
    runs = [r for r in cal.get("runs", []) if r.get("method") == "euler"]
    if not runs:
        return None
    r = min(runs, key=lambda r: abs(r["threads"] - threads))
    return {"port_over_reference": r["port_speed_over_reference"], "threads": r["threads"],
            "source": f"profiles/r04/cpu_calibration.json (tools/calibrate_cpu.py): the port {r['port_us_per_nominal_pstep']:.3f} "
                      f"vs the reference {r['reference_us_per_pstep_survey']:.3f} us per particle-step, Euler streamline, "
                      f"{cal['mesh']['cells']} cells x {cal['mesh']['levels']} levels, {cal['particles']} particles, "
                      f"{r['threads']} threads (SURVEY.md section 6 probe); the Euler ratio is applied to the pathline "
                      "sample (the survey timed no reference pathline)"}


def cpu_baseline(mesh, snap, back_snap, seeds, cells, args, n_steps, duration=None):
    """The CPU oracle (port of the TBB path) on this host's cores, bounded sample; with the calibration
    against the reference's own timings, the reference-equivalent rate beside it."""
    try:
        from oracle import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": f"oracle unavailable: {e}"}
    duration = args.duration if duration is None else int(duration)
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1)
    threads = max(1, min(threads, os.cpu_count() or 1))
    derived = O.preprocess(mesh, snap)
    back = O.preprocess(mesh, back_snap) if back_snap is not None else None
    euler = args.method == "euler"
    # calibrate on a small sample, then size the timed sample to ~cpu_seconds
    n0 = min(4000 if n_steps <= 20000 else 500, len(seeds))
    t = time.perf_counter()
    O.run(mesh, derived, back, seeds[:n0], depth=args.depth, delta_t=args.dt, duration=duration,
          record_t=args.record, euler=euler, cells=cells[:n0], n_threads=threads, finalize=False)
    rate = n0 * n_steps / max(time.perf_counter() - t, 1e-6)
    n1 = int(min(len(seeds), max(n0, rate * args.cpu_seconds / n_steps)))
    t = time.perf_counter()
    out = O.run(mesh, derived, back, seeds[:n1], depth=args.depth, delta_t=args.dt, duration=duration,
                record_t=args.record, euler=euler, cells=cells[:n1], n_threads=threads, finalize=False)
    dt = time.perf_counter() - t
    death = out["death"].astype(np.int64)
    attempted = np.where(death < 0, n_steps, death + 1).sum()
    value = float(attempted / dt)
    res = {"value": value, "unit": "particle-steps/s", "cores": threads, "kind": "port",
           "sample": f"{n1} of the same seeds x {n_steps} steps ({'pathline' if back is not None else 'streamline'} "
                     f"{args.method}, the first pair's snapshots), same mesh/fields, OpenMP schedule(dynamic,16) over "
                     f"particles; {dt:.1f} s"}
    cal = cpu_calibration(threads)
    if cal is not None:
        res["calibration"] = cal
        res["reference_equivalent_value"] = value / cal["port_over_reference"]
    return res


if __name__ == "__main__":
    main()
