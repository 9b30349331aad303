#!/bin/bash
# One build -> measure iteration: selected GPU tests, then the small-kernel rocprof profile.
# usage: gpu_iter.sh <tag> <pytest file/-k args...>
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
tag=$1; shift
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider "$@" \
  > gpurun_out/$tag/pytest.log 2>&1 || { tail -40 gpurun_out/$tag/pytest.log; exit 1; }
tail -2 gpurun_out/$tag/pytest.log
bash scripts/gpu_small.sh $tag/small
