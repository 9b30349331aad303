#!/bin/bash
# Round 5: the default-flag N > 1 bench rehearsed at N = 2 and 8 on ONE MI355X (gloo in place of
# RCCL; see scripts/gpu_r05_d.sh). gpurun --timeout 1200 -- 'bash scripts/gpu_r05_j.sh <tag>'
cd "$GRAFT_REPO_ROOT" || exit 1
REH_N="2 8" bash scripts/gpu_r05_d.sh ${1:-j}
