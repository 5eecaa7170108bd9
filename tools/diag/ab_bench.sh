#!/bin/bash
# A/B of library builds on the bench workloads: LDSGNN_LIB selects the build.
set -o pipefail
mkdir -p gpurun_out
for lib in lds-gnn_amd/ldsgnn/libldsgnn.so lds-gnn_amd/ldsgnn/libldsgnn_b1.so; do
  for ds in cora cora-synthetic; do
    LDSGNN_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline --dataset $ds --steps 100 > gpurun_out/ab_$(basename $lib .so)_$ds.json 2>/dev/null || exit $?
  done
done
