"""Time the per-snapshot derivation chain (mops_field_rebuild_device) on an oRRS18to6-class mesh.

Every snapshot of a configs-4/5 chain is generated and derived in HBM between pairs
(DeviceFieldRecycler): cell zTop, ENU -> xyz velocity, cell -> vertex barycentric interpolation
(zTop, velocity, vertical velocity), the level-pair records and the fast-path words.  This times
the chain alone (HIP events around each rebuild); run it under `rocprofv3 --kernel-trace --stats`
for the per-kernel split.

    python tools/derive_bench.py [--freq 608] [--levels 80] [--reps 5]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--freq", type=int, default=608)
    ap.add_argument("--levels", type=int, default=80)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from mops_amd import synth
    from mops_amd.engine import DeviceMesh
    from mops_amd.synth_device import DeviceSnapshotSource, device_field_factory
    t = time.perf_counter()
    mesh = synth.make_mesh(a.freq, n_levels=a.levels, edges=False)
    print(f"mesh {mesh.nCells} cells {mesh.nVertices} vertices in {time.perf_counter() - t:.1f} s", file=sys.stderr)
    dev = torch.device("cuda", 0)
    dm = DeviceMesh.from_mesh(mesh)
    src = DeviceSnapshotSource(mesh, dev)
    f = device_field_factory(dm, src)(0, torch.cuda.current_stream(dev).cuda_stream)
    raw = src.make(timestep=1, phase=0.35)
    torch.cuda.synchronize()
    s = torch.cuda.current_stream(dev)
    ms = []
    for _ in range(a.reps):
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        e0.record(s)
        f.rebuild_from_device(raw, timestep=1, stream=s.cuda_stream)
        e1.record(s)
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    V, C, L = mesh.nVertices, mesh.nCells, mesh.nVertLevels
    # compulsory HBM bytes of the chain: raw reads, cell intermediates, vertex arrays, records
    b = 8 * (C * L * 3 + C + C * (L + 1)          # thick, zonal, meridional, bottom, w (raw, read)
             + C * L * 2 + C * L * 3 * 2           # cell zTop write+read, cell velocity write+read
             + V * L + V * L * 3 + V * (L + 1)     # vertex zTop / velocity / w written
             + (V * L + V * L * 3 + V * (L + 1))   # ... and read by the record build
             + (V * (L - 1) * 10)                  # level-pair records written
             + V * L)                              # zTop read by the fast-path words
    print(json.dumps({"freq": a.freq, "cells": C, "vertices": V, "levels": L, "rebuild_ms": ms,
                      "best_ms": min(ms), "compulsory_gb": b / 1e9, "compulsory_gbs_at_best": b / 1e6 / min(ms)}))


if __name__ == "__main__":
    main()
