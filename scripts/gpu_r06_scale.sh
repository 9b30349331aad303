#!/bin/bash
# Round 6: bench.py --gpus N with the driver's default flags, N ranks rehearsed on ONE MI355X
# (gloo standing in for RCCL), checking the first timed step after the barrier on every rank
# (check.first_step); then the rehearsal hook that corrupts rank 1's kept first step, which must
# fail the run (exit 1) with check.first_step.failed_ranks == [1].
# Records under gpurun_out/r06_scale/<tag>.
#   gpurun --timeout 1100 -- 'bash scripts/gpu_r06_scale.sh <tag> [8 4 2]'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_scale/${1:-a}
shift
mkdir -p $O
NS=${@:-8 2}
( while sleep 45; do echo "[r06 scale] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
show() {
  python - "$1" <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
c = r.get("check") or {}
print(r["n_gpus"], r["value"], r.get("transport"), "check", c.get("ok"), "first_step",
      c.get("first_step"), "probe", r.get("transport_probe"))
PY
}
for n in $NS; do
  HGD_DIST_BACKEND=gloo timeout -k 10 500 python bench.py --gpus $n > $O/n$n.json 2> $O/n$n.err \
      || exit 1
  show $O/n$n.json || exit 1
done
# the hook: rank 1's first step corrupted after timing; the line must fail
HGD_DIST_BACKEND=gloo HGD_BENCH_CORRUPT_FIRST_STEP=1 timeout -k 10 500 python bench.py --gpus 2 \
    > $O/n2_corrupt_first.json 2> $O/n2_corrupt_first.err
rc=$?
echo "corrupt-first-step run exit status: $rc (expected 1)"
show $O/n2_corrupt_first.json || exit 1
[ $rc -eq 1 ] || exit 1
echo "rc=0"
