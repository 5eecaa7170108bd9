set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "bitmask_agg or spmm_blocked" > gpurun_out/bitagg_test.log 2>&1 && \
timeout -k 10 180 python -u tools/spmm_config5.py > gpurun_out/bitagg_c5.json 2> gpurun_out/bitagg_c5.err && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bitagg -o bitagg -- python3 tools/spmm_config5.py > gpurun_out/bitagg_prof.log 2>&1
echo EXIT $?
