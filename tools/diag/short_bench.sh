set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/short.jsonl
for a in "--graph-windows 4" "--graph-windows 1" "--graph-windows 4" "--graph-windows 1" "--graph-windows 4 --warmup 20"; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-breakdown $a | sed "s/^{/{\"args\": \"$a\", /" >> gpurun_out/short.jsonl || exit $?
done
