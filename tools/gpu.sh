#!/bin/bash
# One launcher for every GPU-box step (replaces the round-1/2 per-session
# tools/gpu_*.sh copies).  Each step runs under its own time limit; the first
# failing step ends the script (no GPU work after a failure).
#
#   tools/gpu.sh TAG STEP [STEP ...]
#
# Steps (outputs under gpurun_out/, named with TAG):
#   tests      the whole -m gpu suite                       tests_TAG.log
#   smoke      __graft_entry__.smoke()                      smoke_TAG.log
#   bench      the default bench line (Cora, S = 1)          bench_TAG.json
#   prof       rocprofv3 kernel-trace summary of the bench   prof_TAG/
#   profnb     the same with --no-breakdown (per-window kernel shares)  profnb_TAG/
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the bench   pmc_TAG_{fetch,write}/
#   pmc5       FETCH_SIZE / WRITE_SIZE passes of the config-5 line pmc5_TAG_{fetch,write}/
#   config5    synthetic N = 20 000 line + its kernel trace c5_bench_TAG.json, c5_prof_TAG/
#   c5cpu      the config-5 line with its CPU baseline       c5_cpu_TAG.json
#   samples    Cora S = 8 / 16, Citeseer S = 16 lines        s_<ds>_<S>_TAG.json
#   scpu       the Citeseer S = 16 line with its CPU baseline s_cpu_TAG.json
#   perrank    N > 1 per-rank window on one GPU (S = 8, no-op exchange), S = 8 local, T1 (S = 64)
#   accuracy   LDS τ = 5 fused engine, 10 seeds, Cora + Citeseer acc_<ds>_tau5_TAG.jsonl
#   acc20      the same at τ = 20 (report.pdf's setting)          acc_<ds>_tau20_TAG.jsonl
#   acc5e      Citeseer τ = 5 on the drop-in autograd path, 3 seeds acc_citeseer_tau5_eager_TAG.jsonl
#   multirank  2 ranks on the card over gloo (N > 1 path)    bench_2rank_gloo_TAG*.log
#   spmmt      the CSR-SpMM kernel tests                     spmmt_TAG.log
#   spmm5      config-5 CSR-SpMM kernels + kernel trace + PMC spmm5_TAG.json, spmm5_prof_TAG/, spmm5_pmc_TAG_*/
#   xtpair     W0 products one vs two samples per wave (Citeseer S = 16, Cora S = 16 / 8) xp_<ds>_<S>_<mode>_TAG.json
set -o pipefail
tag=${1:?usage: tools/gpu.sh TAG STEP...}
shift
mkdir -p gpurun_out
export TMPDIR=/tmp
O=gpurun_out
run() {  # seconds, then the command; stdout/stderr redirected by the caller
    local t=$1
    shift
    timeout -k 10 "$t" "$@"
}
for step in "$@"; do
    echo "[gpu.sh] $step $(date +%T)"
    case $step in
    tests)
        run 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
            > $O/tests_$tag.log 2>&1 || exit $? ;;
    smoke)
        run 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$tag.log 2>&1 || exit $? ;;
    bench)
        run 300 python bench.py > $O/bench_$tag.json 2> $O/bench_$tag.err || exit $? ;;
    prof)
        run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$tag -o run -- \
            python3 bench.py --no-cpu-baseline --steps 100 > $O/prof_$tag.log 2>&1 || exit $? ;;
    profnb)  # the same without the window breakdown (its prefix replays inflate the early calls' counts)
        run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profnb_$tag -o run -- \
            python3 bench.py --no-cpu-baseline --no-breakdown --steps 200 > $O/profnb_$tag.log 2>&1 || exit $? ;;
    pmc)
        for c in FETCH_SIZE WRITE_SIZE; do
            lc=$(echo $c | cut -d_ -f1 | tr 'A-Z' 'a-z')
            run 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc_${tag}_$lc -o run -- \
                python3 bench.py --no-cpu-baseline --no-breakdown --steps 50 --warmup 10 \
                > $O/pmc_${tag}_$lc.log 2>&1 || exit $?
        done ;;
    pmc5)
        for c in FETCH_SIZE WRITE_SIZE; do
            lc=$(echo $c | cut -d_ -f1 | tr 'A-Z' 'a-z')
            run 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/pmc5_${tag}_$lc -o run -- \
                python3 bench.py --dataset synthetic20k --no-cpu-baseline --no-breakdown --steps 10 --warmup 5 \
                > $O/pmc5_${tag}_$lc.log 2>&1 || exit $?
        done ;;
    config5)
        run 400 python -u bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline \
            > $O/c5_bench_$tag.json 2> $O/c5_bench_$tag.err || exit $?
        run 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c5_prof_$tag -o run -- \
            python3 bench.py --dataset synthetic20k --steps 10 --warmup 5 --no-cpu-baseline --no-breakdown \
            > $O/c5_prof_$tag.log 2>&1 || exit $? ;;
    c5cpu)
        run 900 python -u bench.py --dataset synthetic20k --steps 10 --warmup 5 --cpu-steps 1 \
            > $O/c5_cpu_$tag.json 2> $O/c5_cpu_$tag.err || exit $? ;;
    xtpair)
        for spec in "citeseer 16 1" "citeseer 16 2" "cora 16 1" "cora 16 2" "cora 8 1" "cora 8 2"; do
            set -- $spec
            run 300 python bench.py --dataset $1 --samples $2 --xt-pair $3 --steps 100 --warmup 10 --no-cpu-baseline \
                > $O/xp_${1}_$2_$3_$tag.json 2> $O/xp_${1}_$2_$3_$tag.err || exit $?
        done ;;
    samples)
        for spec in "cora 8" "cora 16" "citeseer 16"; do
            set -- $spec
            run 300 python bench.py --dataset $1 --samples $2 --steps 100 --warmup 10 --no-cpu-baseline \
                > $O/s_${1}_$2_$tag.json 2> $O/s_${1}_$2_$tag.err || exit $?
        done ;;
    perrank)  # the N > 1 per-rank window on one GPU (no-op exchange, S = 8) beside T1 (S = 64 alone)
        run 300 python bench.py --samples 8 --exchange noop --steps 100 --warmup 10 --no-cpu-baseline \
            > $O/perrank_s8_$tag.json 2> $O/perrank_s8_$tag.err || exit $?
        run 300 python bench.py --samples 8 --steps 100 --warmup 10 --no-cpu-baseline --no-breakdown \
            > $O/perrank_s8_local_$tag.json 2> $O/perrank_s8_local_$tag.err || exit $?
        run 300 python bench.py --samples 64 --steps 50 --warmup 10 --no-cpu-baseline --no-breakdown \
            > $O/perrank_t1_s64_$tag.json 2> $O/perrank_t1_s64_$tag.err || exit $? ;;
    scpu)
        run 400 python bench.py --dataset citeseer --samples 16 --steps 100 --warmup 10 \
            > $O/s_cpu_$tag.json 2> $O/s_cpu_$tag.err || exit $? ;;
    accuracy)
        for ds in cora citeseer; do
            run 600 python -u tools/accuracy_run.py --dataset $ds --seeds 10 --tau 5 --fused \
                > $O/acc_${ds}_tau5_$tag.jsonl 2> $O/acc_${ds}_tau5_$tag.err || exit $?
        done ;;
    acc20)  # the report's setting (tau = 20), 10 seeds, fused engine
        for ds in cora citeseer; do
            run 900 python -u tools/accuracy_run.py --dataset $ds --seeds 10 --tau 20 --fused \
                > $O/acc_${ds}_tau20_$tag.jsonl 2> $O/acc_${ds}_tau20_$tag.err || exit $?
        done ;;
    acc5e)  # tau = 5 Citeseer through the drop-in autograd path (not the fused engine), first 3 seeds
        run 900 python -u tools/accuracy_run.py --dataset citeseer --seeds 3 --tau 5 \
            > $O/acc_citeseer_tau5_eager_$tag.jsonl 2> $O/acc_citeseer_tau5_eager_$tag.err || exit $? ;;
    multirank)
        run 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
            --master-port 29517 bench.py --gpus 2 --backend gloo --steps 50 --warmup 10 --no-cpu-baseline \
            > $O/bench_2rank_gloo_$tag.log 2>&1 || exit $?
        run 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
            --master-port 29518 bench.py --gpus 2 --backend gloo --samples 8 --steps 50 --warmup 10 \
            --no-cpu-baseline > $O/bench_2rank_gloo_s8_$tag.log 2>&1 || exit $? ;;
    spmmt)  # the CSR-SpMM kernel tests alone (kernels + config 5)
        run 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_config5_gpu.py -k "spmm or bitmask" -x -v \
            --timeout 240 --timeout-method thread > $O/spmmt_$tag.log 2>&1 || exit $? ;;
    spmm5)
        run 200 python tools/spmm_config5.py > $O/spmm5_$tag.json 2> $O/spmm5_$tag.err || exit $?
        run 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/spmm5_prof_$tag -o run -- \
            python3 tools/spmm_config5.py > $O/spmm5_prof_$tag.log 2>&1 || exit $?
        for c in FETCH_SIZE WRITE_SIZE; do
            lc=$(echo $c | cut -d_ -f1 | tr 'A-Z' 'a-z')
            run 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $O/spmm5_pmc_${tag}_$lc -o run -- \
                python3 tools/spmm_config5.py > $O/spmm5_pmc_${tag}_$lc.log 2>&1 || exit $?
        done
        # instruction mix and issue stalls per kernel (one pass: 8 SQ counters)
        run 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY \
            SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVES --kernel-trace --output-format csv \
            -d $O/spmm5_sq_$tag -o run -- python3 tools/spmm_config5.py > $O/spmm5_sq_$tag.log 2>&1 || exit $? ;;
    *)
        echo "unknown step $step" >&2
        exit 2 ;;
    esac
done
echo "[gpu.sh] done $(date +%T)"
