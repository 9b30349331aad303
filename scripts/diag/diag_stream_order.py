"""Is a copy or kernel queued on a SECOND stream behind an event really ordered after the kernel
that produced its input? A torch-only reproducer of the one-device gloo rehearsal's first-step
fault ("What's weak" 1; profiles/r05_scale/p2p_first/).

gloo's all-reduce of a CUDA tensor (ProcessGroupGloo AsyncAllreduceCUDAWork) records an event on
the caller's current stream, makes a pool stream wait for it, and stages the tensor to pinned host
memory with a non-blocking D2H copy on that pool stream; its worker thread then synchronises the
pool stream, sums on the host and copies back. This script replays exactly that ordering with no
libhgd code at all:

  producer  (current stream A): a long kernel, then ``M.fill_(v)`` with a value new to this trial
            (or, with --producer hop, libhgd's hgd_spmm writing M, for comparison)
  consumer  (stream B, after B.wait_event(event recorded on A)):
            d2h     pinned.copy_(M, non_blocking=True)       (gloo's staging copy)
            d2d     M2.copy_(M, non_blocking=True)
            kernel  torch.add(M, 0, out=M2)                  (what RCCL / hgd_p2p consume with)
  check     B.synchronize(), then every element of the consumer's result must equal v.

``--idle`` drains the device (synchronize + a short sleep) before each trial, as the rehearsal's
``torch.cuda.synchronize(); dist.barrier()`` did before its first step. ``--mode gloo`` runs the
same producer under a real gloo all_reduce on N ranks sharing the device.

    python scripts/diag/diag_stream_order.py --mode single --trials 200
    python scripts/diag/diag_stream_order.py --mode gloo --world 8 --cycles 40
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def make_producer(kind, M, dev, mm=4096):
    """Returns produce(v): queues work on the current stream that ends with every element of M
    equal to v (float). 'torch': an mm x mm fp32 matmul (a few ms) then M.fill_(v). 'hop':
    hgd_spmm of a synthetic [R, R] incidence with one nonzero per row into M, from an X whose
    rows are all v (so M == v exactly)."""
    import torch
    if kind == "torch":
        a = torch.randn(mm, mm, device=dev)
        b = torch.randn(mm, mm, device=dev)
        c = torch.empty(mm, mm, device=dev)

        def produce(v):
            torch.mm(a, b, out=c)
            M.fill_(v)
        return produce
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
    R, w = M.shape
    g = torch.Generator(device=dev).manual_seed(0)
    perm = torch.randperm(R, device=dev, generator=g)
    idx = torch.stack([torch.arange(R, device=dev), perm])
    inc = Incidence.from_coo(idx, None, (R, R), device=dev, validate=False, rows_sorted=True)
    X = torch.empty(R, w, device=dev)

    def produce(v):
        X.fill_(v)
        spmm_csr(inc.csr, X, val=inc.val, out=M)
    return produce


def single(args):
    import torch
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    rows, w = args.rows, args.width
    M = torch.zeros(rows, w, device=dev)
    M2 = torch.empty_like(M)
    pinned = torch.empty(rows, w, pin_memory=True)
    A = torch.cuda.current_stream(dev)
    B = torch.cuda.Stream(dev, priority=-1)  # gloo takes a high-priority pool stream
    out = {"mode": "single", "rows": rows, "width": w, "producer": args.producer,
           "HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA"), "results": {}}
    for producer in args.producer.split(","):
        produce = make_producer(producer, M, dev)
        for consumer in args.consumers.split(","):
            for idle in (True, False):
                bad, stale_vals = 0, {}
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for t in range(args.trials):
                    v = float(1 + (t % 1000) + 1000 * (hash((producer, consumer, idle)) % 7))
                    if idle:
                        torch.cuda.synchronize()
                        time.sleep(args.sleep_ms * 1e-3)
                    produce(v)
                    ev = torch.cuda.Event()
                    ev.record(A)
                    B.wait_event(ev)
                    with torch.cuda.stream(B):
                        if consumer == "d2h":
                            pinned.copy_(M, non_blocking=True)
                            res = pinned
                        elif consumer == "d2d":
                            M2.copy_(M, non_blocking=True)
                            res = M2
                        else:
                            torch.add(M, 0.0, out=M2)
                            res = M2
                    B.synchronize()
                    if consumer == "d2h":
                        wrong = res != v
                    else:
                        wrong = (res != v).cpu()
                    n = int(wrong.sum())
                    if n:
                        bad += 1
                        vals = res.cpu()[wrong] if consumer != "d2h" else res[wrong]
                        u = torch.unique(vals)[:4].tolist()
                        stale_vals[t] = {"elements_wrong": n, "frac": n / wrong.numel(),
                                         "values": u, "want": v}
                    if not idle:  # keep stream A busy: the next producer queues behind this one
                        A.wait_stream(B)
                torch.cuda.synchronize()
                key = f"{producer}/{consumer}/{'idle' if idle else 'busy'}"
                out["results"][key] = {"trials": args.trials, "trials_wrong": bad,
                                       "s": round(time.perf_counter() - t0, 2),
                                       "first_wrong": dict(list(stale_vals.items())[:3])}
                print(json.dumps({key: out["results"][key]}), flush=True)
    print(json.dumps(out), flush=True)


def gloo_worker(rank, world, port, args):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rows, w = args.rows, args.width
    M = torch.zeros(rows, w, device=dev)
    results = {}
    for producer in args.producer.split(","):
        produce = make_producer(producer, M, dev)
        for sync_first in (False, True):
            bad = 0
            worst = 0.0
            for c in range(args.cycles):
                torch.cuda.synchronize()
                dist.barrier()
                v = float(rank + 1 + world * (c % 64))
                produce(v)
                if sync_first:
                    torch.cuda.current_stream(dev).synchronize()
                work = dist.all_reduce(M, async_op=True)
                work.wait()
                want = sum(float(q + 1 + world * (c % 64)) for q in range(world))
                err = float((M - want).abs().max()) / want
                worst = max(worst, err)
                wrong = torch.tensor([1.0 if err > 0 else 0.0])
                dist.all_reduce(wrong, op=dist.ReduceOp.MAX)
                bad += int(wrong.item() > 0)
            results[f"{producer}/{'sync_then_allreduce' if sync_first else 'allreduce'}"] = {
                "cycles": args.cycles, "cycles_wrong_any_rank": bad, "worst_rel_rank0": worst}
            if rank == 0:
                print(json.dumps({"world": world, "rows": rows, "width": w,
                                  **{k: v for k, v in results.items()
                                     if k.startswith(producer + "/")}}), flush=True)
    dist.barrier()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="single", choices=["single", "gloo"])
    ap.add_argument("--producer", default="torch,hop",
                    help="comma list of torch (matmul + fill) and hop (hgd_spmm)")
    ap.add_argument("--consumers", default="d2h,d2d,kernel")
    ap.add_argument("--trials", type=int, default=200)
    ap.add_argument("--sleep-ms", type=float, default=2.0)
    ap.add_argument("--rows", type=int, default=250_000, help="rows of M (one item chunk)")
    ap.add_argument("--width", type=int, default=32, help="columns of M (one column slice)")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--cycles", type=int, default=40)
    args = ap.parse_args()
    if args.mode == "single":
        single(args)
        return
    import torch.multiprocessing as mp
    with socket.socket() as sck:
        sck.bind(("127.0.0.1", 0))
        port = sck.getsockname()[1]
    mp.spawn(gloo_worker, args=(args.world, port, args), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
