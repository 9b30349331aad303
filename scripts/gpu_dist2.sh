# rehearse the N=2 bench path on one GPU (gloo over the same device) + sharded parity check
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/${1:-dist2}
mkdir -p $OUT
HGD_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 3 --warmup 1 --users 1000000 --items 100000 --edges 10000000 > $OUT/bench2.json 2> $OUT/bench2.err || { tail -30 $OUT/bench2.err; exit 1; }
cat $OUT/bench2.json
HGD_DIST_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29518 scripts/check_sharded_gpu.py > $OUT/check.log 2>&1 || { tail -30 $OUT/check.log; exit 1; }
cat $OUT/check.log
