set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/xth_tests.log 2>&1 || exit $?
timeout -k 10 200 python bench.py --samples 8 --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/xth_s8.json 2> gpurun_out/xth_s8.err || exit $?
