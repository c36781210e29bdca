"""Diagnostic: distinct cells per 64-slot wave after ParticleSet's locality order (config-3 seeds)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import importlib.util
    import torch
    from mops_amd import synth
    from mops_amd.engine import DeviceMesh, ParticleSet, TrajectoryConfig
    spec = importlib.util.spec_from_file_location("b", os.path.join(os.path.dirname(os.path.dirname(
        os.path.abspath(__file__))), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    mesh = synth.make_mesh(158, n_levels=60)
    dm = DeviceMesh.from_mesh(mesh)
    seeds = b.make_seeds(n, 0)
    cfg = TrajectoryConfig(deltaT=60, simulationDuration=86400, recordT=3600, depth=100.0, method=1)
    ps = ParticleSet(dm, seeds, 100.0, cfg)
    torch.cuda.synchronize()
    c = ps.cell.cpu().numpy()
    w = c[: len(c) // 64 * 64].reshape(-1, 64)
    d = np.array([len(np.unique(r)) for r in w])
    print("waves", len(w), "distinct cells per wave: mean", d.mean(), "hist", np.bincount(d)[:12].tolist())
    print("cells monotone-run fraction", float(np.mean(np.diff(c) == 0)))
    print("first wave cells", w[0].tolist())
    ids = ps.ids.cpu().numpy()
    print("ids is a permutation", bool(np.array_equal(np.sort(ids), np.arange(len(ids)))))


if __name__ == "__main__":
    main()
