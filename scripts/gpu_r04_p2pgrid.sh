#!/bin/bash
# Round 4: the peer exchange's kernels at 256 workgroups (the new default, two / four loads per
# thread in flight) against 1024 / 2048 (round 3's grids): the p2p GPU tests, then the local
# pricing at each grid (HGD_P2P_GRID). Records under gpurun_out/r04_batch/<tag>.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-p2pgrid}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_native_host.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
for g in 256 1024; do
  HGD_P2P_GRID=$g timeout -k 10 200 python -u scripts/bench_p2p_price.py > $O/price_g$g.json 2>&1 \
      || exit 1
done
rc=$?
echo "rc=$rc"
exit $rc
