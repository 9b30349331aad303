#!/bin/bash
# Round 5: the N > 1 bench with its DEFAULT flags (check on, --transport auto) rehearsed on ONE
# MI355X (VERDICT r4 "next" 3): N ranks share the device, gloo stands in for RCCL (RCCL needs
# one device per rank; HGD_DIST_BACKEND is an environment knob, not a flag). The line must carry
# `check` (every rank's Y / dX rows against the single-GPU conv of the global graph) and
# `transport_probe`. Records under gpurun_out/r05/<tag>.
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r05_d.sh <tag>'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/${1:-d}
mkdir -p $O
export TMPDIR=/tmp
( while sleep 45; do echo "[r05 d] $(date +%T) $(grep -h '^\[bench rank 0' $O/*.err 2>/dev/null | tail -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
for n in ${REH_N:-4}; do
  t0=$SECONDS
  HGD_DIST_BACKEND=gloo timeout -k 10 900 \
      python bench.py --gpus $n --steps 2 --warmup 1 > $O/n${n}.json 2> $O/n${n}.err
  rc=$?
  echo "n=$n rc=$rc wall=$((SECONDS - t0)) s" | tee $O/n${n}.wall
  [ $rc -eq 0 ] || { grep '^\[bench rank' $O/n${n}.err | tail -20; tail -5 $O/n${n}.err; exit $rc; }
  python - $O/n${n}.json <<'PY'
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print({k: r.get(k) for k in ("n_gpus", "value", "transport", "check")})
print(r.get("transport_probe"))
assert r["check"]["ok"] and sum(x["nnz"] for x in r["ranks"]) == r["config"]["edges"]
PY
done
