#!/bin/bash
# Round 6: the staging round trip of the first-step fault in 8 processes, each Ms block
# snapshotted before its producer: a torch matmul producer (no libhgd call), libhgd's hop,
# and the hop with the producing stream drained on the host (the library's gloo ordering).
# Records under gpurun_out/r06_seq/<tag>.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r06_seq7.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r06_seq/${1:-h}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r06 seq7] $(date +%T) $(ls -t $O | head -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
rt() {  # name, extra args
  timeout -k 10 240 python -u scripts/diag/diag_stream_order.py --mode chunks --roundtrip \
      --rt-consumers clone --procs 8 "${@:2}" > $O/$1.jsonl 2> $O/$1.err && \
  python - $O/$1.jsonl <<'PY'
import json, sys
tot = {}
for l in open(sys.argv[1]):
    if "] {" not in l or '"mode"' in l:
        continue
    for k, v in json.loads(l.split("] ", 1)[1]).items():
        t = tot.setdefault(k, [0, 0])
        t[0] += v["steps"]
        t[1] += v["steps_wrong"]
print(sys.argv[1], {k: f"{w} wrong of {n} process-steps" for k, (n, w) in tot.items()})
PY
}
rt mm_prior --producer mm --trials 60 --prior && \
rt hgd_prior --producer hgd --trials 60 --prior && \
rt hgd_prior_drained --producer hgd --trials 60 --prior --drain
rc=$?
echo "rc=$rc"
exit $rc
