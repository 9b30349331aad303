#!/bin/bash
# Round 5: bench.py --gpus N with the driver's default flags, N ranks rehearsed on ONE MI355X
# (gloo standing in for RCCL), at the last HEAD. Records under gpurun_out/r05/scale_head.
#   gpurun --timeout 900 -- 'bash scripts/gpu_r05_scale_head.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/r05/scale_head
mkdir -p $O
for n in 8 4 2; do
  HGD_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus $n > $O/n$n.json 2> $O/n$n.err || exit 1
  python - $O/n$n.json <<'PY' || exit 1
import json, sys
r = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(r["n_gpus"], r["value"], r["transport"], r["check"]["ok"], r.get("transport_probe"), r.get("transport_fallback"))
PY
done
