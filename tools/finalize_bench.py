"""Time mops_traj_finalize (line assembly + NaN cleanup) alone, slot order vs. a random slot -> line map.

The bench's finalize writes each slot's line at ids[slot]; after the locality re-sort that map is a
random permutation, so the line writes land scattered (one P*24-B run per line and array).  This
separates the kernel's own cost from the scatter's:

    python tools/finalize_bench.py [--n 1000000] [--K 6] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1_000_000)
    ap.add_argument("--K", type=int, nargs="+", default=[6, 24])
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import torch
    from mops_amd import _lib as L
    lib = L.load()
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev)
    g.manual_seed(1)
    n = a.n
    out = []
    for K in a.K:
        P = K + 1
        seeds = torch.rand((n, 3), dtype=torch.float64, device=dev, generator=g)
        rec = torch.rand((K, 6, n), dtype=torch.float64, device=dev, generator=g)
        pts = torch.empty((n, P, 3), dtype=torch.float64, device=dev)
        vel = torch.empty_like(pts)
        tmp = torch.empty((n, P), dtype=torch.float64, device=dev)
        sal = torch.empty_like(tmp)
        last = torch.empty((n, 3), dtype=torch.float64, device=dev)
        perm = torch.randperm(n, device=dev, generator=g).to(torch.int32)
        s = torch.cuda.current_stream(dev)
        for name, ids in (("identity", None), ("random", perm)):
            ms = []
            for _ in range(a.reps + 1):
                e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
                e0.record(s)
                L.check(lib.mops_traj_finalize(n, K, C.c_void_p(seeds.data_ptr()), C.c_void_p(rec.data_ptr()), n, 0,
                                               None if ids is None else C.c_void_p(ids.data_ptr()),
                                               C.c_void_p(pts.data_ptr()), C.c_void_p(vel.data_ptr()),
                                               C.c_void_p(tmp.data_ptr()), C.c_void_p(sal.data_ptr()),
                                               C.c_void_p(last.data_ptr()), C.c_void_p(s.cuda_stream)),
                        "mops_traj_finalize")
                e1.record(s)
                torch.cuda.synchronize()
                ms.append(e0.elapsed_time(e1))
            ms = ms[1:]
            nbytes = 8 * n * (3 + 6 * K + 3 * P * 2 + 2 * P + 3) + (4 * n if ids is not None else 0)
            out.append({"K": K, "map": name, "ms": ms, "best_ms": min(ms), "gbs_at_best": nbytes / 1e6 / min(ms)})
            print(json.dumps(out[-1]), flush=True)


if __name__ == "__main__":
    main()
