set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/t_engine.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/b_s1.log 2>&1 || exit $?
for S in 4 8 16; do timeout -k 10 200 python bench.py --no-cpu-baseline --samples $S > gpurun_out/b_s$S.log 2>&1 || exit $?; done
timeout -k 10 200 python bench.py --no-cpu-baseline --samples 16 --dataset citeseer > gpurun_out/b_cite16.log 2>&1 || exit $?
