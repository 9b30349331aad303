set -o pipefail
mkdir -p gpurun_out/lin
for b in 512 1024 2048 4096; do
  HGD_ROWGEMM_BLOCKS=$b timeout -k 10 120 python scripts/bench_linear.py --rows 69716 31668 > gpurun_out/lin/b$b.jsonl 2>&1 || exit 1
done
grep -h hgd gpurun_out/lin/*.jsonl
