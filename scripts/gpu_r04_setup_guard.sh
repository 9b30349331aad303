#!/bin/bash
# Round 4: the peer exchange's set-up calls on helper threads with a deadline (sharded.P2PExchange,
# HGD_P2P_SETUP_TIMEOUT_S). On one MI355X, records under gpurun_out/r04_batch/<tag>:
#   1. the p2p GPU tests and the native host's 2-rank p2p conv (set-up now off the main thread);
#   2. bench.py --gpus 2 --transport auto at d = 256 with 1 M items (8 slots of 256 MB per rank),
#      gloo standing in for RCCL (one device): the probe must run the peer exchange and pass;
#   3. the same with the slots in ONE 4 GiB segment (HGD_P2P_SEGMENT_MB=4096: the allocation whose
#      IPC open never returns on ROCm 7.2): the open must hit its 45 s deadline on both ranks, the
#      probe keep RCCL, the run print its line and both ranks exit (os._exit past the stuck call).
#   gpurun --timeout 900 -- 'bash scripts/gpu_r04_setup_guard.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r04_batch/${1:-guard}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[guard] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
SMALL="--gpus 2 --users 1000000 --items 1000000 --edges 10000000 --dim 256 --steps 2 --warmup 1
       --check --no-cpu-baseline --pmc off --transport auto"
timeout -k 10 300 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_native_host.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 && tail -1 $O/pytest.txt && \
HGD_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py $SMALL > $O/auto_ok.json \
    2> $O/auto_ok.err && echo "auto ok" && \
HGD_DIST_BACKEND=gloo HGD_P2P_SEGMENT_MB=4096 HGD_P2P_SETUP_TIMEOUT_S=45 HGD_STALL_DUMP_S=240 \
    timeout -k 10 400 python -u bench.py $SMALL > $O/auto_stuck.json 2> $O/auto_stuck.err && \
echo "auto stuck-open ok"
rc=$?
grep -h '^\[bench rank' $O/auto_stuck.err 2>/dev/null | tail -12
echo "rc=$rc"
exit $rc
