#!/bin/bash
# GPU box, end of round 2 (second session): the whole -m gpu suite, smoke(),
# the default bench line + its rocprofv3 kernel-trace summary + the two PMC
# traffic passes + the config-5 line (tools/gpu_r02_final.sh), then the
# multi-sample lines and the 2-rank gloo rehearsal.  Usage: TAG
set -o pipefail
tag=${1:-r02final2}
bash tools/gpu_r02_final.sh $tag || exit $?
for spec in "cora 8" "cora 16" "citeseer 16"; do
  set -- $spec
  timeout -k 10 300 python bench.py --dataset $1 --samples $2 --steps 100 --warmup 10 --no-cpu-baseline \
    > gpurun_out/s_${1}_$2_$tag.json 2> gpurun_out/s_${1}_$2_$tag.err || exit $?
done
bash tools/gpu_multirank.sh || exit $?
