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

``--mode chunks`` replays the chunked staging order of ShardedIncidence.two_hop (4 item-row chunks
per 32-column slice, each staged D2H on its own stream right behind its producer); with
``--roundtrip`` the whole cycle (D2H, a host op, H2D back, a consumer kernel), and with
``--procs N`` in N processes sharing the device. Findings (profiles/r06_first_step/): no wrong
chunk in one process; with 8 processes, the first chunk after an idle device came back wrong now
and then — with libhgd's hop AND with a plain torch matmul as the producer (``--producer mm``,
no libhgd call at all) — in stripes of whole 64-row groups, holding neither the producer's
output nor zeros; draining the producing stream on the host first (``--drain``) removed it.

    python scripts/diag/diag_stream_order.py --mode single --trials 200
    python scripts/diag/diag_stream_order.py --mode gloo --world 8 --cycles 40
    python scripts/diag/diag_stream_order.py --mode chunks --roundtrip --producer mm \
        --rt-consumers clone --procs 8 --trials 100
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


def chunks(args):
    """gloo's staging order for the chunked exchange of ShardedIncidence.two_hop, in ONE process
    (no gloo, no other ranks): per column slice, hop 1 writes item-row chunk k of Ms on the
    current stream (libhgd's hgd_spmm over a rank-sized CSC, or a torch gather of the same rows),
    an event is recorded, a high-priority side stream k waits for it and copies the chunk to
    pinned host memory (d2h) or to another device buffer (d2d), and the next chunk's hop is
    launched at once. After the step everything is synchronised and every copied chunk is
    compared bitwise with the same hop recomputed. ``--idle`` state before every step."""
    import torch
    import bench
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    U, I, E, d, w = args.users, args.items, args.edges, args.dim, args.width
    X = torch.randn(U, d, device=dev)
    # libhgd is touched only when its hop is a producer or a consumer: with --producer mm|gather
    # and --rt-consumers clone the whole test is torch calls
    uses_hgd = "hgd" in args.producer.split(",") or (
        args.roundtrip and "hgd" in args.rt_consumers.split(",")) or not args.roundtrip
    inc = q = val_t = None
    if uses_hgd:
        from hypergraph_diffusion_for_recommendation_amd import Incidence
        idx = bench.make_graph(U, I, E, seed=0, zipf=None, device=dev)
        inc = Incidence.from_coo(idx, None, (U, I), device=dev, validate=False,
                                 rows_sorted=True)
        del idx
        q = inc.scale("col", "mean")
        val_t = inc.edge_values("csc", "sym")
    n_chunks = args.n_chunks
    step_ = (I + n_chunks - 1) // n_chunks
    bounds = [(k * step_, min((k + 1) * step_, I)) for k in range(n_chunks)]
    slices = [(c, min(c + w, d)) for c in range(0, d, w)]
    g = torch.Generator(device=dev).manual_seed(5)
    perm = torch.randperm(I, device=dev, generator=g)
    Xi = torch.randn(I, d, device=dev, generator=g)
    streams = [torch.cuda.Stream(dev, priority=-1) for _ in range(len(slices) * n_chunks)]
    cur = torch.cuda.current_stream(dev)
    out = {"mode": "chunks", "users": U, "items": I, "edges": E, "chunks": n_chunks,
           "libhgd_used": uses_hgd,
           "HSA_ENABLE_SDMA": os.environ.get("HSA_ENABLE_SDMA"), "results": {}}

    A_mm = W_mm = None
    if "mm" in args.producer.split(","):  # [items, K] x [K, w]: a writer as long as the hop
        A_mm = torch.randn(I, args.mm_k, device=dev, generator=g).div_(args.mm_k ** 0.5)
        W_mm = [torch.randn(args.mm_k, c1 - c0, device=dev, generator=g) for c0, c1 in slices]

    def hop(kind, c0, c1, Ms, a, b):
        if kind == "hgd":
            from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
            spmm_csr(inc.csc, X[:, c0:c1], val=val_t, row_scale=q, out=Ms, row_begin=a,
                     row_end=b)
        elif kind == "mm":
            torch.mm(A_mm[a:b], W_mm[c0 // w], out=Ms[a:b])
        else:
            torch.index_select(Xi[:, c0:c1], 0, perm[a:b], out=Ms[a:b])

    if args.roundtrip:
        return roundtrip(args, inc, X, q, val_t, bounds, slices, perm, Xi, streams, cur, out,
                         hop)
    for kind in args.producer.split(","):
        for consumer in args.consumers.split(","):
            bad_steps, bad_chunks = 0, 0
            t0 = time.perf_counter()
            for t in range(args.trials):
                torch.cuda.synchronize()
                time.sleep(args.sleep_ms * 1e-3)
                copies = []
                for s, (c0, c1) in enumerate(slices):
                    Ms = torch.empty((I, c1 - c0), device=dev)
                    for k, (a, b) in enumerate(bounds):
                        hop(kind, c0, c1, Ms, a, b)
                        ev = torch.cuda.Event()
                        ev.record(cur)
                        st = streams[s * n_chunks + k]
                        st.wait_event(ev)
                        with torch.cuda.stream(st):
                            if consumer == "d2h":
                                dst = torch.empty((b - a, c1 - c0), pin_memory=True)
                            else:
                                dst = torch.empty((b - a, c1 - c0), device=dev)
                            dst.copy_(Ms[a:b], non_blocking=True)
                        copies.append((c0, c1, a, b, dst, Ms))
                torch.cuda.synchronize()
                wrong = 0
                for c0, c1, a, b, dst, Ms in copies:
                    ref = torch.empty((I, c1 - c0), device=dev)
                    hop(kind, c0, c1, ref, a, b)
                    if not torch.equal(dst.to(dev), ref[a:b]):
                        wrong += 1
                bad_steps += wrong > 0
                bad_chunks += wrong
                del copies
            key = f"{kind}/{consumer}"
            out["results"][key] = {"steps": args.trials, "steps_wrong": bad_steps,
                                   "chunks_wrong": bad_chunks,
                                   "s": round(time.perf_counter() - t0, 2)}
            print(json.dumps({key: out["results"][key]}), flush=True)
    print(json.dumps(out), flush=True)


def roundtrip(args, inc, X, q, val_t, bounds, slices, perm, Xi, streams, cur, out, hop):
    """--roundtrip: gloo's whole staging cycle per chunk, in one process — the D2H copy to pinned
    memory on a side stream behind an event (issued right after the chunk's hop), then, once all
    chunks of all slices are issued, per chunk: the side stream synchronised on the host, the host
    copy multiplied by 8 (an exact stand-in for the sum of 8 equal partials), copied back H2D on
    the side stream, the current stream made to wait; then a consumer kernel on the current
    stream reads the whole Ms (torch clone, or libhgd's hop into users) and is compared with 8×
    the hop recomputed. Stale data anywhere on the way back shows as a mismatch."""
    import torch
    dev = X.device
    n_chunks = len(bounds)
    n_items = bounds[-1][1]
    for kind in args.producer.split(","):
        for consumer in args.rt_consumers.split(","):
            bad_steps, bad_rows = 0, 0
            details = []
            t0 = time.perf_counter()
            for t in range(args.trials):
                torch.cuda.synchronize()
                time.sleep(args.sleep_ms * 1e-3)
                staged = []
                prior = {}
                for s, (c0, c1) in enumerate(slices):
                    Ms = torch.empty((n_items, c1 - c0), device=dev)
                    prior[s] = Ms.clone() if args.prior else None  # what the block held before
                    for k, (a, b) in enumerate(bounds):
                        hop(kind, c0, c1, Ms, a, b)
                        if args.drain:  # the library's gloo ordering: drain on the host first
                            cur.synchronize()
                        ev = torch.cuda.Event()
                        ev.record(cur)
                        st = streams[s * n_chunks + k]
                        st.wait_event(ev)
                        with torch.cuda.stream(st):
                            host = torch.empty((b - a, c1 - c0), pin_memory=True)
                            host.copy_(Ms[a:b], non_blocking=True)
                        staged.append((s, c0, c1, a, b, Ms, st, host))
                results = []
                for s, (c0, c1) in enumerate(slices):
                    Ms = None
                    for s2, _, _, a, b, M2, st, host in staged:
                        if s2 != s:
                            continue
                        Ms = M2
                        st.synchronize()
                        host.mul_(args.host_factor)
                        with torch.cuda.stream(st):
                            Ms[a:b].copy_(host, non_blocking=True)
                        cur.wait_stream(st)
                    if consumer == "clone":
                        results.append((c0, c1, Ms.clone()))
                    else:
                        from hypergraph_diffusion_for_recommendation_amd.incidence import \
                            spmm_csr
                        results.append((c0, c1, spmm_csr(inc.csr, Ms, val=inc.val)))
                torch.cuda.synchronize()
                wrong = 0
                for si, (c0, c1, got) in enumerate(results):
                    ref = torch.empty((n_items, c1 - c0), device=dev)
                    for a, b in bounds:
                        hop(kind, c0, c1, ref, a, b)
                    part = ref.clone()
                    ref.mul_(args.host_factor)
                    if consumer == "hgd":
                        from hypergraph_diffusion_for_recommendation_amd.incidence import \
                            spmm_csr
                        ref = spmm_csr(inc.csr, ref, val=inc.val)
                    bad = (got != ref).any(1)
                    nb = int(bad.sum())
                    wrong += nb
                    if nb and consumer == "clone" and len(details) < 6:
                        rows = bad.nonzero().flatten()
                        g_b, p_b = got[rows], part[rows]
                        details.append({
                            "trial": t, "cols": [c0, c1], "rows_wrong": nb,
                            "first_row": int(rows[0]), "last_row": int(rows[-1]),
                            "chunks": sorted({int(r) // ((n_items + n_chunks - 1) // n_chunks)
                                              for r in rows.tolist()[::997]}),
                            "contiguous": int(rows[-1] - rows[0] + 1) == nb,
                            "got_equals_unscaled_partial": float((g_b == p_b).all(1).float()
                                                                 .mean()),
                            "got_is_zero": float((g_b == 0).all(1).float().mean())})
                        pr = prior.get(si)
                        if pr is not None:
                            p_r = pr[rows]
                            details[-1]["got_equals_prior_times_factor"] = float(
                                (g_b == p_r * args.host_factor).all(1).float().mean())
                            details[-1]["got_equals_prior"] = float((g_b == p_r).all(1).float()
                                                                    .mean())
                bad_steps += wrong > 0
                bad_rows += wrong
                del staged, results
            key = f"roundtrip/{kind}/{consumer}" + ("/drained" if args.drain else "")
            out["results"][key] = {"steps": args.trials, "steps_wrong": bad_steps,
                                   "rows_wrong": bad_rows, "host_factor": args.host_factor,
                                   "s": round(time.perf_counter() - t0, 2),
                                   "details": details}
            print(json.dumps({key: out["results"][key]}), flush=True)
    print(json.dumps(out), flush=True)


def _chunks_proc(rank, args):
    """--procs N: N processes run :func:`chunks` at once on the shared device (the rehearsal's
    contention without gloo); each prints its own lines, tagged with its index."""
    import builtins
    plain = builtins.print

    def tagged(*a, **k):
        plain(f"[proc {rank}]", *a, **k)
    builtins.print = tagged
    chunks(args)


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
    ap.add_argument("--mode", default="single", choices=["single", "gloo", "chunks"])
    ap.add_argument("--producer", default="torch,hop",
                    help="comma list of torch (matmul + fill) and hop (hgd_spmm)")
    ap.add_argument("--consumers", default="d2h,d2d,kernel")
    ap.add_argument("--trials", type=int, default=200)
    ap.add_argument("--sleep-ms", type=float, default=2.0)
    ap.add_argument("--rows", type=int, default=250_000, help="rows of M (one item chunk)")
    ap.add_argument("--width", type=int, default=32, help="columns of M (one column slice)")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--cycles", type=int, default=40)
    ap.add_argument("--users", type=int, default=1_250_000, help="--mode chunks: one rank's shard")
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=12_500_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--n-chunks", type=int, default=4)
    ap.add_argument("--roundtrip", action="store_true",
                    help="--mode chunks: the whole staging cycle (D2H, host op, H2D back, a "
                         "consumer kernel) instead of the D2H copies alone")
    ap.add_argument("--host-factor", type=float, default=8.0,
                    help="--roundtrip: what the host multiplies the staged chunk by (8: an exact "
                         "stand-in for a sum of 8 equal partials; 1: identity)")
    ap.add_argument("--rt-consumers", default="clone,hgd")
    ap.add_argument("--prior", action="store_true",
                    help="--roundtrip: snapshot each Ms block before its producer runs, to tell "
                         "whether a wrong chunk holds the block's earlier content")
    ap.add_argument("--drain", action="store_true",
                    help="--roundtrip: synchronise the current stream on the host after each "
                         "chunk's producer, before its event (what sharded.ordered_all_reduce "
                         "does for gloo)")
    ap.add_argument("--mm-k", type=int, default=512, help="inner size of the 'mm' producer")
    ap.add_argument("--procs", type=int, default=1,
                    help="--mode chunks: processes running it at once on the shared device")
    args = ap.parse_args()
    if args.mode == "single":
        single(args)
        return
    if args.mode == "chunks":
        if args.procs <= 1:
            chunks(args)
            return
        import torch.multiprocessing as mp
        mp.spawn(_chunks_proc, args=(args,), nprocs=args.procs, join=True)
        return
    import torch.multiprocessing as mp
    with socket.socket() as sck:
        sck.bind(("127.0.0.1", 0))
        port = sck.getsockname()[1]
    mp.spawn(gloo_worker, args=(args.world, port, args), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
