"""Wave-lifetime / occupancy diagnostic for traj_kernel (perf experiments only).

Needs a -DMOPS_WAVE_STAMPS variant (tools/build_variant.sh stamps -DMOPS_WAVE_STAMPS)
selected with MOPS_TRAJ_LIB.  Runs the bench's config-2 call once (warm) and once with
per-slot stamps, then prints: the occupancy API's resident blocks per CU, the launch
span, wave lifetime quantiles, resident waves per SIMD over time, and the tail (time
from the 50th/90th/99th percentile wave end to the last).  Writes the per-wave table to
OUT (npz).  Usage: python tools/wave_stamps.py OUT.npz [bench args...]
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from mops_amd import _lib, synth  # noqa: E402
from mops_amd.engine import DeviceField, DeviceMesh, ParticleSet, TrajectoryConfig  # noqa: E402


def main():
    out = sys.argv[1]
    sys.argv = [sys.argv[0]] + sys.argv[2:]
    args = bench.parse()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    mesh = synth.make_mesh(args.freq, n_levels=args.levels)
    dmesh = DeviceMesh.from_mesh(mesh)
    dfield = DeviceField.from_snapshot(dmesh, synth.make_snapshot(mesh, timestep=0, topography=args.topography))
    pathline = args.mode == "pathline"
    dback = (DeviceField.from_snapshot(dmesh, synth.make_snapshot(mesh, timestep=1, phase=0.35, topography=args.topography))
             if pathline else None)
    seeds = bench.make_seeds(args.particles, 0)
    n = seeds.shape[0]
    cfg = TrajectoryConfig(deltaT=args.dt, simulationDuration=args.duration, recordT=args.record, depth=args.depth,
                           method=1 if args.method == "euler" else 0)
    ps = ParticleSet(dmesh, seeds, args.depth, cfg, device=dev)
    lib = _lib.load()
    lib.mops_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_void_p]
    occ = (ctypes.c_int * 4)()
    stamps = torch.zeros((n, 8), dtype=torch.int64, device=dev)

    info = {}

    def call():
        ps.reset(depth=args.depth)
        dmesh.locate(ps.seeds.data_ptr(), ps.cell.data_ptr(), n)
        ps.reorder()
        info["cell0"] = ps.cell.cpu().numpy().copy()
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record()
        ps.advance(dfield, dback, 0, cfg.n_steps)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1)

    assert lib.mops_debug_stamps(None, 0, occ) == 0
    warm = call()
    assert lib.mops_debug_stamps(ctypes.c_void_p(stamps.data_ptr()), n, None) == 0
    ms = call()
    assert lib.mops_debug_stamps(None, 0, None) == 0
    s = stamps.cpu().numpy().astype(np.int64)
    nw = (n + 63) // 64
    pad = nw * 64 - n
    st = np.concatenate([s, np.repeat(s[-1:], pad, 0)]) if pad else s
    st = st.reshape(nw, 64, 8)
    start = st[:, :, 0].min(1); end = st[:, :, 1].max(1)
    hw = st[:, 0, 2]; xcc = st[:, 0, 3] & 0xF
    simd = (hw >> 4) & 3; cu = (hw >> 8) & 0xF; sa = (hw >> 12) & 1; se = (hw >> 13) & 7
    t0 = start.min()
    start_us = (start - t0) / 100.0; end_us = (end - t0) / 100.0  # 100 MHz ticks -> us
    life = end_us - start_us
    span = end_us.max()
    print(f"occupancy API blocks(64 thr)/CU: SE {occ[0]} SR {occ[1]} PE {occ[2]} PR {occ[3]}")
    print(f"launch ms (events): warm {warm:.2f}, stamped {ms:.2f}; stamped span {span / 1e3:.2f} ms; waves {nw}")
    q = np.quantile(life, [0, 0.1, 0.5, 0.9, 0.99, 1.0]) / 1e3
    print("wave lifetime ms q0/10/50/90/99/100:", " ".join(f"{x:.2f}" for x in q))
    qs = np.quantile(start_us, [0.5, 0.9, 0.99, 1.0]) / 1e3
    print("wave start ms q50/90/99/100:", " ".join(f"{x:.2f}" for x in qs))
    qe = np.quantile(end_us, [0.5, 0.9, 0.99]) / 1e3
    print("wave end ms q50/90/99:", " ".join(f"{x:.2f}" for x in qe), f"last {span / 1e3:.2f}")
    simd_key = ((xcc * 8 + se) * 2 + sa) * 16 * 4 + cu * 4 + simd
    nsimd = len(np.unique(simd_key))
    grid = np.linspace(0, span, 41)[:-1] + span / 80
    res = [(np.sum((start_us <= t) & (end_us > t))) / max(nsimd, 1) for t in grid]
    print(f"distinct SIMDs seen {nsimd}; resident waves/SIMD at 40 instants:", " ".join(f"{r:.2f}" for r in res))
    busy = np.sum(life) / (nsimd * span)
    print(f"mean resident waves/SIMD over the span {busy:.2f}")
    per_slot = {}
    for k, a, b in zip(simd_key, start_us, end_us):
        per_slot.setdefault(k, []).append((a, b))
    maxconc = []
    for k, iv in per_slot.items():
        ev = sorted([(a, 1) for a, b in iv] + [(b, -1) for a, b in iv], key=lambda x: (x[0], x[1]))
        c = m = 0
        for _, d in ev:
            c += d; m = max(m, c)
        maxconc.append(m)
    print("max concurrent waves per SIMD: distribution", np.bincount(maxconc).tolist())
    cnt = s[:, 4:8].copy()
    names = ["walks", "loads", "fast misses", "levels read"]
    cnt[:, 3] &= 0xFFFFFFFF
    scans = s[:, 7] >> 32
    wave_cnt = np.concatenate([cnt, np.repeat(cnt[-1:], pad, 0)]).reshape(nw, 64, 4) if pad else cnt.reshape(nw, 64, 4)
    slow = np.argsort(life)[::-1][:20]
    print("per lane-step means, all lanes:", {k: round(float(cnt[:, i].sum()) / (n * cfg.n_steps), 4) for i, k in enumerate(names)},
          "bracket_scan calls/lane", round(float(scans.mean()), 3))
    sl = np.concatenate([np.arange(64 * w, min(64 * w + 64, n)) for w in slow])
    print("per lane-step means, 20 slowest waves:", {k: round(float(cnt[sl, i].sum()) / (len(sl) * cfg.n_steps), 4) for i, k in enumerate(names)},
          "bracket_scan calls/lane", round(float(scans[sl].mean()), 3))
    print("max over lanes in each slow wave of (walks, loads, misses, levels):")
    for w in slow[:10]:
        print("  wave", w, wave_cnt[w].max(0).tolist(), "sum", wave_cnt[w].sum(0).tolist())
    np.savez_compressed(out, cnt=s[:, 4:8], start_us=start_us, end_us=end_us, hw=hw, xcc=xcc, ids=ps.ids.cpu().numpy(),
                        cell0=info["cell0"], cell1=ps.cell.cpu().numpy(), death=ps.death.cpu().numpy(),
                        depth1=ps.depth.cpu().numpy(), seeds=ps.seeds.cpu().numpy())
    for w in slow:
        sl = slice(64 * w, min(64 * w + 64, n))
        c0 = info["cell0"][sl]; c1 = ps.cell[sl].cpu().numpy(); dd = ps.death[sl].cpu().numpy()
        print(f"slow wave {w}: life {life[w] / 1e3:.2f} ms start {start_us[w] / 1e3:.2f}; cells0 {len(set(c0))} "
              f"moved {(c0 != c1).sum()} dead {(dd >= 0).sum()}")


if __name__ == "__main__":
    main()
