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


def _entries_of_build(build):
    import json
    pm = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    return {e["workload"]: e for e in pm if e.get("engine_build") == build}


# the round-4 profiles (engine build 20548e0a, profiles/r04/c{2,5}) and the round-5 final build's
# (profiles/r05/c3, c4, which replaced their round-4 entries): the counter-chosen roof of each
R04 = "20548e0af4c5f230"


@pytest.mark.parametrize("key,kind", [(C3, "valu_issue"), (C4, "l1_return"), (C2, "l1_return"),
                                      ("orrs18to6_chain5_euler_12500000_seg4320", "valu_issue")])
def test_roofline_bound_is_the_counter_chosen_limiter(key, kind, monkeypatch):
    """The line's roofline.binding_roof names the roof the counters show binding (bench.limiter_kind) -- VALU
    issue for the cooperative configs 3/5 kernel, the TD return for config 4 (and config 2, where TD is the
    busier of the two) -- with binding_frac that view's; the top-level bound / achieved / peak / frac are the
    HBM view BASELINE's metric defines (a consumer reading roofline.frac gets the HBM fraction)."""
    import bench
    ents = _entries_of_build(R04)
    ents.update(_entries_of_build(bench.engine_build_id()))
    if key not in ents:
        pytest.skip(f"no round-4 or current-build PMC entry {key}")
    e = ents[key]
    l1, valu = bench.l1_block(e, 0.5), bench.valu_block(e)
    assert bench.limiter_kind(l1, valu) == kind
    # roofline_block over the same entry (measured_entry / measured_traffic answer with it)
    monkeypatch.setattr(bench, "measured_entry", lambda k: (e, "test"))
    monkeypatch.setattr(bench, "measured_traffic", lambda k: (float(e["bytes_per_unit"]), "test"))
    r = bench.roofline_block("k", 0.5, 1e10, 3660.0, key)
    assert r["binding_roof"] == kind
    view = r[kind]
    assert (r["binding_frac"], r["binding_unit"]) == (view["frac"], view["unit"])
    assert 0.0 < r["binding_frac"] <= 1.0
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and r["peak"] == bench.PEAK_HBM_GBS
    assert (r["achieved"], r["frac"]) == (r["hbm"]["achieved"], r["hbm"]["frac"])
    assert r["hbm"]["unit"] == "GB/s" and r["hbm"]["peak"] == bench.PEAK_HBM_GBS
    assert r["hbm"]["frac"] == pytest.approx(e["bytes_per_unit"] / 0.5 / 1e9 / bench.PEAK_HBM_GBS)
    if kind == "valu_issue":
        assert r["limiter"].startswith("VALU issue")
    else:
        assert "TD" in r["limiter"]


def test_priced_valu_issue_reconciles_with_valu_busy():
    """the VALU roof priced by instruction class (round 6, tools/fp64bench.hip: 4 SIMD-cycles per
    wave64 VALU instruction, 16 for the FP64 rcp / rsq / sqrt seeds, 8 for FP32 transcendentals) on the round-5
    config-3 entry and its committed class mix (profiles/r05/c3/valu_mix.txt: 23.1 FP64 and 2.7 FP32
    transcendentals of 1152.3 VALU per wave-step).  The flat 4-cycle count read 0.860; the priced count agrees
    with rocprof's independent VALUBusy (SQ_ACTIVE_INST_VALU) to 1%, which the flat one does not."""
    import bench
    e = _entries_of_build("c0f7b27a249dcf83").get(C3)
    if e is None or e.get("valu_trans_f64_frac") is None:
        pytest.skip("no round-5 config-3 entry with a class mix")
    v = bench.valu_block(e)
    assert v["priced"] and v["flat_4_cycle_frac"] == pytest.approx(0.8596, abs=1e-3)
    assert v["frac"] == pytest.approx(v["flat_4_cycle_frac"] * (1 + 3 * 23.1 / 1152.3 + 2.7 / 1152.3), rel=1e-12)
    assert abs(v["frac"] - e["valu_busy"]) < 0.01 < abs(v["flat_4_cycle_frac"] - e["valu_busy"])
    assert bench.VALU_CYC_TRANS_F64 == 16.0 and bench.VALU_CYC_TRANS_F32 == 8.0 and bench.VALU_CYC == 4.0


def test_bench_host_starts_no_program(monkeypatch):
    """The line names its box (host + GPU uuid / PCI address) without starting a program: a process that has
    initialised the GPU must not exec (round 6 first called rocm-smi, a python script, from the bench)."""
    import subprocess
    import bench

    def _refuse(*a, **k):
        raise AssertionError("bench_host started a program")
    monkeypatch.setattr(subprocess, "run", _refuse)
    monkeypatch.setattr(subprocess, "Popen", _refuse)
    h = bench.bench_host()
    assert isinstance(h, str) and h
