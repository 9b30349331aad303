#!/bin/bash
# Round 5: the masked hop's kept weights by one multiply with 1 / keep (keep a power of two)
# against the IEEE division (HGD_MASK_DIV=1): bitwise tests, then the Yelp-shaped hop A/B/A/B.
#   gpurun --timeout 600 -- 'bash scripts/gpu_r05_div.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-div}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_masked_pair.py -x -q --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
for div in 1 0 1 0; do
  HGD_MASK_DIV=$div timeout -k 10 120 python -u scripts/bench_masked_hop.py > $O/hop_div$div.$RANDOM.json 2>&1 || exit 1
done && \
HGD_MASK_DIV=1 timeout -k 10 200 python -u scripts/bench_hccf.py --variants hgd_graph_ref_adam > $O/hccf_div1.jsonl 2>&1 && \
HGD_MASK_DIV=0 timeout -k 10 200 python -u scripts/bench_hccf.py --variants hgd_graph_ref_adam > $O/hccf_div0.jsonl 2>&1 && \
echo "div ok"
