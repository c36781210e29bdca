"""Golden vectors for the chain's pair schedule and per-pair gaps, made by the reference's own code.

Runs in the build container only (it reads /root/reference, which the GPU box does not have).
``tutorial/pyMOPSAPI.py`` imports ``pyMOPS`` and ``cartopy`` at module level, so it is not imported:
the three pure-Python static methods of ``MOPSPathline`` the chain follows are taken out of its syntax
tree and executed alone --

* ``_month_pairs_forward``  (tutorial/pyMOPSAPI.py:1236-1257)
* ``_month_pairs_backward`` (tutorial/pyMOPSAPI.py:1259-1279)
* ``_time_gap_seconds``     (tutorial/pyMOPSAPI.py:1285-1295)

-- over forward and backward month ranges and MPAS xtime pairs (with the NUL / blank padding of a
netCDF char variable), and the results are written to ``tests/golden/month_pairs.json``.
``tests/test_chain_schedule.py`` checks ``mops_amd.chain`` against that file.

    python tests/golden/make_month_pairs.py
"""
import ast
import json
import os
from datetime import datetime

REF = "/root/reference/tutorial/pyMOPSAPI.py"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "month_pairs.json")
WANT = ("_month_pairs_forward", "_month_pairs_backward", "_time_gap_seconds")


def reference_functions():
    tree = ast.parse(open(REF).read(), REF)
    cls = next(n for n in tree.body if isinstance(n, ast.ClassDef) and n.name == "MOPSPathline")
    funcs = []
    for n in cls.body:
        if isinstance(n, ast.FunctionDef) and n.name in WANT:
            n.decorator_list = []  # @staticmethod: plain functions here
            funcs.append(n)
    mod = ast.Module(body=funcs, type_ignores=[])
    ns = {"datetime": datetime}
    exec(compile(mod, REF, "exec"), ns)
    return {k: ns[k] for k in WANT}


def main():
    f = reference_functions()
    fwd_ranges = [(1, 1, 2, 1), (1, 1, 1, 12), (18, 1, 20, 12), (1, 3, 3, 12), (5, 11, 6, 2), (7, 6, 7, 6),
                  (7, 6, 7, 5), (1, 12, 2, 1)]
    bwd_ranges = [(2, 1, 1, 1), (20, 12, 18, 1), (3, 12, 1, 3), (6, 2, 5, 11), (7, 6, 7, 6), (7, 5, 7, 6),
                  (2, 1, 1, 12)]
    stamps = ["0001-01-01_00:00:00", "0001-02-01_00:00:00", "0001-03-01_00:00:00", "0004-02-01_00:00:00",
              "0004-03-01_00:00:00", "0100-02-01_00:00:00", "0100-03-01_00:00:00", "2000-02-01_00:00:00",
              "2000-03-01_00:00:00", "0018-07-15_06:30:00", "0018-07-16_00:00:00"]
    padded = [("0001-01-02_00:00:00" + "\x00" * 45, "0001-01-01_00:00:00" + " " * 45),
              ("  0001-12-01_00:00:00  ", "0002-01-01_00:00:00\x00junk")]
    gaps = []
    for a in stamps:
        for b in stamps:
            gaps.append({"t1": a, "t2": b, "seconds": f["_time_gap_seconds"](a, b)})
    for a, b in padded:
        gaps.append({"t1": a, "t2": b, "seconds": f["_time_gap_seconds"](a, b)})
    out = {
        "source": "tutorial/pyMOPSAPI.py MOPSPathline._month_pairs_forward/_backward (:1236-1279), "
                  "_time_gap_seconds (:1285-1295), executed alone (tests/golden/make_month_pairs.py)",
        "forward": [{"args": list(r), "pairs": f["_month_pairs_forward"](*r)} for r in fwd_ranges],
        "backward": [{"args": list(r), "pairs": f["_month_pairs_backward"](*r)} for r in bwd_ranges],
        "gaps": gaps,
    }
    json.dump(out, open(OUT, "w"), indent=1)
    print(f"wrote {OUT}: {len(out['forward'])} forward, {len(out['backward'])} backward ranges, {len(gaps)} gaps")


if __name__ == "__main__":
    main()
