#!/bin/bash
# Round-4 measurement batch on one MI355X (records under gpurun_out/r04_batch/<tag>):
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r04_batch.sh <tag>'
#   1. the GPU tests touched this round (p2p, objects, sharded, graph step, plugins, sampler);
#   2. the CPU keep-mask draw at 1..16 threads (scripts/bench_cpu_mask.py);
#   3. the HCCF step variants, keep-mask on 1 thread and on the default split;
#   4. the peer transport's data path priced locally (scripts/bench_p2p_price.py);
#   5. k_splitk_x3p barrier vs queue form (HGD_X3P_QUEUE): weight-gradient microbench at the
#      Amazon (144,242 x 128) and Yelp (69,716 x 64) shapes, and the LocalAware step.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-run}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r04 batch] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
lscpu | grep -E "Model name|^CPU\(s\)|Thread|MHz" > $O/lscpu.txt; nproc >> $O/lscpu.txt
timeout -k 10 900 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_objects.py \
    tests/test_gpu_linear.py tests/test_gpu_native_host.py tests/test_gpu_sharded_encoders.py tests/test_gpu_graph_step.py \
    tests/test_gpu_plugins.py tests/test_sampler.py -x -v -rw --timeout 300 --timeout-method thread \
    > $O/pytest.txt 2>&1 && echo "pytest ok" && \
timeout -k 10 300 python -u scripts/bench_cpu_mask.py > $O/cpu_mask.jsonl 2>&1 && echo "cpu mask ok" && \
timeout -k 10 300 python -u scripts/bench_hccf.py --variants hgd_cpu_mask,hgd_device_mask,hgd_graph \
    > $O/hccf.jsonl 2>&1 && echo "hccf ok" && \
HGD_CPU_RNG_THREADS=1 timeout -k 10 300 python -u scripts/bench_hccf.py --variants hgd_cpu_mask \
    > $O/hccf_rng1.jsonl 2>&1 && echo "hccf rng1 ok" && \
timeout -k 10 300 python -u scripts/bench_p2p_price.py > $O/p2p_price.json 2>&1 && echo "p2p price ok" && \
for q in 0 1; do
  HGD_X3P_QUEUE=$q timeout -k 10 120 python scripts/bench_linear.py --rows 144242 --dim 128 \
      --cases bwd_weight_hgd bwd_weight_mask_hgd > $O/x3p_q${q}_d128.jsonl 2>&1 && \
  HGD_X3P_QUEUE=$q timeout -k 10 120 python scripts/bench_linear.py --rows 69716 --dim 64 \
      --cases bwd_weight_hgd bwd_weight_mask_hgd > $O/x3p_q${q}_d64.jsonl 2>&1 && \
  HGD_X3P_QUEUE=$q timeout -k 10 200 python scripts/bench_local_aware.py > $O/la_q$q.jsonl 2>&1 \
    || exit 1
  echo "x3p queue=$q ok"
done
rc=$?
grep -h -E "passed|failed|AccumulateGrad" $O/pytest.txt | tail -3
echo "rc=$rc"
exit $rc
