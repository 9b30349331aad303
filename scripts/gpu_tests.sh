#!/bin/bash
# The whole GPU suite (one pytest process), log under gpurun_out/.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 400 --timeout-method thread \
  -p no:cacheprovider "$@" > gpurun_out/pytest_all.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_all.log
exit $rc
