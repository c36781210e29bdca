import json, sys
for v in sys.argv[1:]:
    try:
        d = json.loads(open(f"gpurun_out/var_{v}.log").read().strip().splitlines()[-1])
        print(f"{v:10s} {d['value']:.4e} p-steps/s  launch {d['roofline']['avg_launch_ms']:.3f} ms")
    except Exception as e:
        print(v, "ERR", e)
