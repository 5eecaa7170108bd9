#!/bin/bash
# Summarise gpurun_out after tools/gpu_iter.sh
tail -2 gpurun_out/t_iter.log
for f in gpurun_out/b_*.log; do python - "$f" <<'PY'
import json, sys
l = [x for x in open(sys.argv[1]) if x.startswith('{')]
if l:
    d = json.loads(l[-1]); r = d['roofline']
    print(sys.argv[1].split('/')[-1], round(d['value']), d['unit'], round(d['ms_per_step'], 4), r['kernel'], round(r['avg_us'], 1), round(r['frac'], 3))
PY
done
for t in "$@"; do python - "$t" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(f"gpurun_out/prof_{sys.argv[1]}/run_kernel_stats.csv")))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("profile", sys.argv[1])
for r in rows[:12]:
    print(f'{int(r["Calls"]):7d} {float(r["AverageNs"])/1000:9.2f} {100*float(r["TotalDurationNs"])/tot:5.1f}%  {r["Name"].split("(")[0][:60]}')
PY
done
