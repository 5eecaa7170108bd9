"""Summarise gpurun_out/perf_*.json and kchain.jsonl (tools/gpu_perf.sh)."""
import glob
import json
from collections import defaultdict

for f in sorted(glob.glob("gpurun_out/perf_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f, round(d["value"]), "steady", round(d["steady_state"]["value"]),
          [(r["entry"][11:], round(r["avg_us"], 1)) for r in d["window"]["top"]])
try:
    rows = [json.loads(line) for line in open("gpurun_out/kchain.jsonl")]
    agg = defaultdict(list)
    for r in rows[1:-1]:
        if "call" in r:
            agg[r["call"]].append(r["us"])
        else:
            print("  ", r)
    print("chain floor", round(rows[0]["us"], 2), "window", round(rows[-1]["window_us"], 1))
    for k, v in agg.items():
        print(f"  {k:28s} x{len(v):2d} {sum(v) / len(v):6.2f} us")
except FileNotFoundError:
    pass
