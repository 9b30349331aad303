#!/usr/bin/env python3
"""Encoder fwd+bwd on user-row shards (BASELINE configs[3]: Amazon-Book-shaped hypergraph
diffusion, d = 128, user-row sharded). One process per GPU:

    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P scripts/bench_sharded_encoder.py [--model local_aware|hccf]

A step is the encoder's forward over the whole graph plus the backward of a fixed random
upstream gradient (the loss terms are the harness's) and, for HCCF, the summed replicated
gradients. The graph is FIXED as N grows (strong scaling: each rank owns U/N users). At N = 1
the single-GPU encoder (encoders.py) is timed beside the sharded one. Backend "nccl" (= RCCL)
unless HGD_DIST_BACKEND says otherwise (gloo rehearsal of N ranks on one GPU: correctness
only). Rank 0 prints one JSON line (max over ranks of the timed loop)."""
import argparse
import json
import os
import sys
import time
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="local_aware", choices=["local_aware", "hccf"])
    ap.add_argument("--users", type=int, default=52_643)
    ap.add_argument("--items", type=int, default=91_599)
    ap.add_argument("--edges", type=int, default=2_240_000)
    ap.add_argument("--dim", type=int, default=128)
    ap.add_argument("--layers", type=int, default=2)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--chunks", type=int, default=4)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd import sharded_encoders as SE
    from hypergraph_diffusion_for_recommendation_amd.encoders import (HCCFEncoder,
                                                                      LocalAwareEncoder)
    from hypergraph_diffusion_for_recommendation_amd.sharded import (allreduce_replicated_grads,
                                                                       init_process_group)

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev = torch.device(f"cuda:{local % max(1, torch.cuda.device_count())}")
    torch.cuda.set_device(dev)
    backend = os.environ.get("HGD_DIST_BACKEND", "nccl")
    if world > 1:
        init_process_group(dev, backend)

    U, I, d = args.users, args.items, args.dim
    u, i = R.synthetic_incidence(U, I, args.edges, seed=0)  # same graph on every rank
    ui = R.bipartite_adjacency(u, i, U, I).tocsr()
    data = types.SimpleNamespace(n_users=U, n_items=I, ui_adj=ui,
                                 norm_adj=R.normalize_graph_mat(ui).tocsr())
    u0, u1 = SE.shard_bounds(U, world, rank)
    n = u1 - u0
    conf = dict(lrate=0.001, lr_decay=0.9, max_epoch=1, batch_size=4096, reg=0.01,
                embedding_size=d, hyper_dim=32, drop_rate=0.2, p=0.3, n_layers=args.layers)
    g = torch.Generator(device=dev).manual_seed(100 + rank)
    gu = torch.randn(n, d, device=dev, generator=g)
    gi = torch.randn(I, d, device=dev, generator=g)

    def build(sharded):
        if args.model == "local_aware":
            if sharded:
                enc = SE.ShardedLocalAwareEncoder(data, d, d, args.layers, 0.3, 0.2, u0, u1,
                                                  device=dev, n_chunks=args.chunks)
                ego = torch.randn(n + I, d, device=dev, generator=g).requires_grad_(True)

                def step():
                    ue, ie = enc(ego)
                    torch.autograd.backward([ue, ie], [gu, gi])
                    allreduce_replicated_grads(enc.replicated_parameters())
            else:
                enc = LocalAwareEncoder(data, d, d, args.layers, 0.3, 0.2, device=dev)
                ego = torch.randn(U + I, d, device=dev, generator=g).requires_grad_(True)
                gfull = torch.randn(U + I, d, device=dev, generator=g)

                def step():
                    ue, ie = enc(ego, enc.sparse_norm_adj)
                    torch.autograd.backward([ue, ie], [gfull[:U], gfull[U:]])
        else:
            if sharded:
                enc = SE.ShardedHCCFEncoder(conf, data, u0, u1, device=dev,
                                            n_chunks=args.chunks, device_rng=True)

                def step():
                    ue, ie, _, _ = enc(keep_rate=0.5)
                    torch.autograd.backward([ue, ie], [gu, gi])
                    allreduce_replicated_grads(enc.replicated_parameters())
            else:
                enc = HCCFEncoder(conf, data, device=dev)
                enc.edgeDropper.device_rng = True
                gfull = torch.randn(U + I, d, device=dev, generator=g)

                def step():
                    ue, ie, _, _ = enc(keep_rate=0.5)
                    torch.autograd.backward([ue, ie], [gfull[:U], gfull[U:]])
        enc.train()
        return step

    def timed(step):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([el], dtype=torch.float64, device=dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            el = float(t.item())
        return el / args.steps * 1e3

    ms = timed(build(True))
    single = timed(build(False)) if world == 1 else None
    if rank == 0:
        nnz_a = int(data.norm_adj.nnz)
        print(json.dumps({
            "bench": f"sharded {args.model} encoder fwd+bwd", "n_ranks": world,
            "backend": backend if world > 1 else None, "scaling": "strong",
            "ms_per_step": round(ms, 3),
            "single_gpu_encoder_ms": None if single is None else round(single, 3),
            "graph": {"users": U, "items": I, "interactions": len(u), "nnz_norm_adj": nnz_a},
            "d": d, "layers": args.layers, "chunks": args.chunks,
            "users_per_rank": n}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
