#!/bin/bash
# Round 6: the 8-process staging round trip (gpu_r06_seq6.sh) then the N-rank rehearsal with the
# first-step check (gpu_r06_scale.sh). One call, the first failure ends it.
#   gpurun --timeout 1200 -- 'bash scripts/gpu_r06_combo1.sh'
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_r06_seq6.sh g && bash scripts/gpu_r06_scale.sh a 8 2
