#!/bin/bash
# The round-end checks on one MI355X: the whole GPU suite, smoke(), the N=1 headline bench and
# the carrier benches (HCCF training step, ED-HNN block). Logs under gpurun_out/round/.
#   gpurun --timeout 1200 -- 'bash scripts/gpu_round.sh'
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/round
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  -p no:cacheprovider > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python scripts/bench_hccf.py > $O/hccf.jsonl 2>&1 || { tail -20 $O/hccf.jsonl; exit 1; }
grep variant $O/hccf.jsonl
timeout -k 10 300 python scripts/bench_edhnn.py > $O/edhnn.jsonl 2>&1 || { tail -20 $O/edhnn.jsonl; exit 1; }
grep variant $O/edhnn.jsonl
