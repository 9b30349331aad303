#!/bin/bash
# Multi-rank rehearsals of the strong-scaling bench on ONE MI355X (VERDICT r2 "next" 2a): N ranks
# share the device, the exchange runs over gloo (RCCL needs one device per rank) or the direct
# peer transport (hgd_p2p over same-device IPC, gloo for setup). Each run is `bench.py --check`:
# Σ per-rank nnz must equal the global graph's 99,999,492 and every rank's Y / dX rows must match
# the single-GPU conv of the global graph at 1e-5 · conv(|x|). Correctness, not speed: gloo
# stages every all-reduce through host memory. Records under gpurun_out/r03_scale/.
#   gpurun --timeout 1200 -- 'bash scripts/gpu_scale_rehearsal.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r03_scale
mkdir -p $O
export TMPDIR=/tmp
# progress line for the runner while a rehearsal runs silently (each step has its own limit)
( while sleep 50; do echo "[rehearsal] $(date +%T) running: $(grep -h '^\[bench rank' $O/$(cat $O/current 2>/dev/null).err 2>/dev/null | tail -1)"; done ) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
run() {  # name, time limit, bench args...
  local name=$1 lim=$2
  shift 2
  echo "[rehearsal] $name: bench.py $*"
  echo $name > $O/current
  timeout -k 10 "$lim" python bench.py --check --no-cpu-baseline --pmc off \
    "$@" > $O/$name.json 2> $O/$name.err || { echo "FAILED rc=$? $name"; grep '^\[bench rank' $O/$name.err | tail -20; tail -5 $O/$name.err; exit 1; }
  python - "$O/$name.json" <<'EOF'
import json, sys
line = [l for l in open(sys.argv[1]) if l.startswith("{")][-1]
r = json.loads(line)
nnz = sum(x["nnz"] for x in r["ranks"])
print(f"  n={r['n_gpus']} d={r['config']['emb_dim']} transport={r['transport']} "
      f"sum_nnz={nnz} edges={r['config']['edges']} check={r['check']}")
assert nnz == r["config"]["edges"] == 99_999_492 and r["check"]["ok"]
EOF
  [ $? -eq 0 ] || exit 1
}
# gloo stages each all-reduce through host TCP (21 s per step at N = 4, d = 64:
# profiles/r03_scale/bench_strong_4ranks_gloo_d64_check.json; N = 8 at d = 256 reached "warm" at
# 7.4 s, profiles/r03_scale/gloo_n8_d256.phases.txt). The default runs use the peer transport
# (same sharding, same check; gloo only for setup): since round 4 its slots are exposed in
# <= 1 GiB segments, and d = 256 runs at N = 4 and 8 (profiles/r04_scale/).
STEPS="--steps ${REH_STEPS:-1} --warmup ${REH_WARMUP:-1}"
for spec in ${REH_RUNS:-"p2p:4:64 p2p:8:64 p2p:4:256 p2p:8:256"}; do
  IFS=: read tr n d <<< "$spec"
  extra=""
  [ "$tr" = p2p ] && extra="--transport p2p"
  HGD_DIST_BACKEND=gloo run ${tr}_n${n}_d${d} ${REH_LIMIT:-420} --gpus $n --dim $d $extra $STEPS
done
echo "[rehearsal] all ok"
