set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_config5_gpu.py -x -q -k "theta" --timeout 300 --timeout-method thread > gpurun_out/t_tg.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 200 > gpurun_out/tg_s1.json 2> gpurun_out/tg_s1.err || exit $?
timeout -k 10 300 python bench.py --samples 8 --steps 100 --no-cpu-baseline > gpurun_out/tg_s8.json 2> gpurun_out/tg_s8.err || exit $?
timeout -k 10 300 python bench.py --samples 16 --dataset citeseer --steps 100 --no-cpu-baseline > gpurun_out/tg_cs16.json 2> gpurun_out/tg_cs16.err || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_tgc -o run -- \
  python3 bench.py --samples 8 --no-cpu-baseline --no-breakdown --steps 20 --warmup 10 > gpurun_out/pmc_tgc.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmc_tgd -o run -- \
  python3 bench.py --no-cpu-baseline --no-breakdown --steps 20 --warmup 10 > gpurun_out/pmc_tgd.log 2>&1 || exit $?
