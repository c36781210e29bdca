"""Instruction mix between the "@@MARK <id>" comments of a -DMOPS_ISA_MARKS assembly build.

    hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -DMOPS_ISA_MARKS -Iinclude \
          --cuda-device-only -S -o marks.s mops_amd/csrc/mops_engine.hip
    python tools/isa_marks.py marks.s [--kernel _Z11traj_kernelILi7ELb0ELb1EEv8TrajArgs] [--dump 400:410]

For each marker, the instructions from it to the next marker in layout order (cold blocks the
compiler placed in between are counted too -- use --dump to read a region), split into FP64
VALU, other VALU, SALU, VMEM, LDS, SMEM and branches.  Only a counting aid: the markers are
volatile asm and may move the surrounding code a little.
"""
import argparse
import collections
import re


def classify(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        if re.search(r"_f64\b|_f64_e|_f64$", op) and not op.startswith(("v_cmp", "v_cmpx", "v_cvt")):
            return "valu_f64"
        if op.startswith(("v_cmp", "v_cmpx")):
            return "valu_cmp"
        if op.startswith("v_cndmask"):
            return "valu_cndmask"
        if op.startswith(("v_mov", "v_accvgpr")):
            return "valu_mov"
        return "valu_other"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "smem"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_swappc")):
        return "branch"
    if op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_sleep", "s_sched", "s_setprio")):
        return "wait"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--kernel", default="_Z11traj_kernelILi7ELb0ELb1EEv8TrajArgs")
    ap.add_argument("--dump", default=None, help="FROM:TO marker ids: print that region")
    a = ap.parse_args()
    lines = open(a.asm).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(a.kernel + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].startswith(".Lfunc_end"))
    regions = []  # (marker id, [instructions])
    cur = ["entry", []]
    for l in lines[start:end]:
        m = re.search(r"@@MARK (0x[0-9a-fA-F]+|\d+)", l)
        if m:
            regions.append(cur)
            cur = [str(int(m.group(1), 0)), []]
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            if t.endswith(":") and not t.startswith(";"):
                cur[1].append("LABEL " + t)
            continue
        cur[1].append(t.split(";")[0].strip())
    regions.append(cur)
    keys = ["valu_f64", "valu_cmp", "valu_cndmask", "valu_mov", "valu_other", "salu", "vmem", "lds", "smem",
            "branch", "wait"]
    print("%-8s %6s " % ("from", "instr") + " ".join("%8s" % k[:8] for k in keys) + "  labels")
    for rid, ins in regions:
        real = [x for x in ins if not x.startswith("LABEL")]
        c = collections.Counter(classify(x) for x in real)
        nl = sum(1 for x in ins if x.startswith("LABEL"))
        print("%-8s %6d " % (rid, len(real)) + " ".join("%8d" % c.get(k, 0) for k in keys) + "  %d" % nl)
    if a.dump:
        f, t = a.dump.split(":")
        on = False
        for rid, ins in regions:
            if rid == f:
                on = True
            if rid == t:
                break
            if on:
                print("==== MARK", rid)
                for x in ins:
                    print("   ", x)


if __name__ == "__main__":
    main()
