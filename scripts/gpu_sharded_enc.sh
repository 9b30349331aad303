# sharded encoder bench: N=1 (sharded vs single-GPU encoder) + a 2-rank gloo rehearsal on one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-shenc}
mkdir -p $OUT
for m in local_aware hccf; do
  timeout -k 10 300 python scripts/bench_sharded_encoder.py --model $m > $OUT/n1_$m.json 2> $OUT/n1_$m.err || { tail -20 $OUT/n1_$m.err; exit 1; }
  cat $OUT/n1_$m.json
done
HGD_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 scripts/bench_sharded_encoder.py --model local_aware --steps 5 --warmup 1 > $OUT/n2_gloo.json 2> $OUT/n2_gloo.err || { tail -20 $OUT/n2_gloo.err; exit 1; }
cat $OUT/n2_gloo.json
