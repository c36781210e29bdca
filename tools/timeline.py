"""GPU busy time and idle gaps of one bench call from a rocprofv3 kernel trace.

    python tools/timeline.py OUTDIR/stats [--calls N] [--gap-us 10]

Reads the kernel_trace.csv under OUTDIR, merges the kernels of all streams into
busy intervals, and reports for the last N calls (a call starts at each
`locate_kernel` dispatch that follows a traj_kernel) the wall span, the busy
union, and every idle gap longer than --gap-us with the kernels either side.
"""
import argparse
import csv
import glob


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--calls", type=int, default=2)
    ap.add_argument("--gap-us", type=float, default=10.0)
    a = ap.parse_args()
    rows = []
    for f in glob.glob(f"{a.dir}/**/*kernel_trace.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if r[2].startswith("locate_kernel")
              and any(x[2].startswith("void traj_kernel") for x in rows[max(0, i - 40):i])]
    if not starts:
        starts = [0]
    bounds = starts[-a.calls:] + [len(rows)]
    for c in range(len(bounds) - 1):
        seg = rows[bounds[c]:bounds[c + 1]]
        t0 = seg[0][0]
        busy, gaps, cur_s, cur_e, prev = 0, [], seg[0][0], seg[0][1], seg[0][2]
        for s, e, n in seg[1:]:
            if s > cur_e:
                busy += cur_e - cur_s
                if (s - cur_e) / 1e3 > a.gap_us:
                    gaps.append(((cur_e - t0) / 1e3, (s - cur_e) / 1e3, prev, n))
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
            prev = n
        busy += cur_e - cur_s
        span = (cur_e - t0) / 1e3
        print(f"call {c}: {len(seg)} kernels, span {span:.1f} us, busy {busy / 1e3:.1f} us, idle {span - busy / 1e3:.1f} us")
        for at, g, p, n in gaps:
            print(f"   gap {g:8.1f} us at {at:9.1f}  after {p:48s} before {n}")


if __name__ == "__main__":
    main()
