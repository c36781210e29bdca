"""bench.py's roofline views from the committed PMC entries (profiles/pmc_traffic.json): every fraction is a
measured busy fraction in [0, 1], and the limiter names the unit the counters show binding -- VALU issue for
the cooperative config-3 kernel, the TD return for config 4, both together for config 2's streamline.  Skipped when the entries were measured on another
engine build (bench.py then reports them as stale, never as this build's)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

C3 = "ec30to60_chain3_euler_10000000_seg1440"
C4 = "orrs18to6_chain4_euler_10000000_seg720"
C2 = "ec30to60_streamline_euler_1000000_seg720_p2c6"


def _entry(bench, key):
    e, src = bench.measured_entry(key)
    if e is None:
        pytest.skip(src)
    return e


@pytest.mark.parametrize("key,launch_s,unit", [(C3, 0.530, "VALU issue"), (C4, 0.481, "texture-data return"),
                                               (C2, 0.0247, "TD return and VALU issue")])
def test_roofline_views_are_busy_fractions(key, launch_s, unit):
    import bench
    _entry(bench, key)
    l1, valu, fp = bench.l1_block(key, launch_s), bench.valu_block(key), bench.fp64_block(key, launch_s)
    for name, frac in (("l1_return", l1["frac"]), ("valu_issue", valu["frac"]), ("fp64_valu", fp["frac"])):
        assert frac is not None and 0.0 < frac <= 1.0, (name, frac)
    assert l1["achieved"] <= l1["peak"]
    assert 0.0 < valu["valu_busy"] <= 1.0
    assert bench.limiter_text(l1, valu).startswith(unit)
