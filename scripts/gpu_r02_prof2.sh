#!/bin/bash
# Profiles of the secondary paths (sharded encoder at N=1, HCCF step) + PMC reruns.
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r02_prof2
mkdir -p $OUT
timeout -k 10 300 python scripts/bench_sharded_encoder.py --model local_aware > $OUT/sharded_la.json 2> $OUT/sharded_la.err || { tail -20 $OUT/sharded_la.err; exit 1; }
cat $OUT/sharded_la.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/sharded_trace -o run -- python3 scripts/bench_sharded_encoder.py --model local_aware --steps 10 > $OUT/sharded_trace.log 2>&1 || { tail -20 $OUT/sharded_trace.log; exit 1; }
timeout -k 10 300 python scripts/bench_hccf.py --variants hgd_device_mask,hgd_cpu_mask > $OUT/hccf.json 2> $OUT/hccf.err || { tail -20 $OUT/hccf.err; exit 1; }
cat $OUT/hccf.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/hccf_trace -o run -- python3 scripts/bench_hccf.py --variants hgd_device_mask --reps 10 > $OUT/hccf_trace.log 2>&1 || { tail -20 $OUT/hccf_trace.log; exit 1; }
timeout -k 10 600 python bench.py --workload zipf --pmc on --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_zipf.json 2> $OUT/bench_zipf.err || { tail -30 $OUT/bench_zipf.err; exit 1; }
timeout -k 10 600 python bench.py --dim 256 --pmc on --no-cpu-baseline --steps 10 --warmup 3 > $OUT/bench_d256.json 2> $OUT/bench_d256.err || { tail -30 $OUT/bench_d256.err; exit 1; }
echo ALL_OK
