"""The first-step fault of the one-device gloo rehearsal, replayed with the EXACT call sequence of
ShardedIncidence.two_hop (sharded.py) — column slices x item chunks, one async all_reduce of each
chunk queued right behind the kernel that produced it, hop 2 of a slice after waiting for its
chunks — forward then backward, with each hop either libhgd's (``hgd``) or a torch kernel writing
an output of the same shape (``torch``). Bisects VERDICT r05 'Next' 2: if the fault shows with
both hops in torch, it belongs to the gloo/HIP stack, not to libhgd.

Per rank (N ranks share one device, gloo, as the rehearsal): a local incidence of
``edges / N`` uniform entries over [users / N, items]; the torch hops are

    hop 1   Ms[a:b] = (rank + 1) * B[a:b, c0:c1]         (torch.mul into the chunk view; a
            matmul of --mm first gives it the hop's duration)
    hop 2   Y[:, c0:c1] = Ms[g]                          (index_select of one item per user)

with small-integer B, so every value is exact and the right answer is known in closed form.

Cycle (as diag_p2p_first.py's all-reduce part): synchronize + barrier, then 4 steps
(fwd + bwd each); the first is compared with the last (bitwise) and, for torch hops, with the
closed form. ``--sync`` drains the current stream before every all_reduce (the candidate fix).

    python scripts/diag/diag_first_step_seq.py --world 8 --cycles 12 --hop1 torch --hop2 torch
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def worker(rank, world, port, args):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hypergraph_diffusion_for_recommendation_amd import Incidence
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
    U, I, d, w, n_chunks = args.users // world, args.items, args.dim, args.width, args.chunks
    E = args.edges // world
    import bench
    idx = bench.make_graph(U, I, E, seed=rank, zipf=None, device=dev)
    inc = Incidence.from_coo(idx, None, (U, I), device=dev, validate=False, rows_sorted=True)
    del idx
    g = torch.Generator(device=dev).manual_seed(7)
    B = torch.randint(-8, 9, (I, d), device=dev, generator=g).float()
    gather = torch.randint(0, I, (U,), device=dev, generator=g)
    X = torch.randint(-8, 9, (U, d), device=dev, generator=g).float() * 0.125
    dY = torch.randint(-8, 9, (U, d), device=dev, generator=g).float() * 0.25
    mm_a = torch.randn(args.mm, args.mm, device=dev, generator=g)
    mm_c = torch.empty_like(mm_a)
    tail_buf = torch.ones(64, device=dev)
    perm = torch.randperm(I, device=dev, generator=g)
    Bs = [B[:, c:c + w].contiguous() for c in range(0, d, w)]
    step_ = (I + n_chunks - 1) // n_chunks
    bounds = [(k * step_, min((k + 1) * step_, I)) for k in range(n_chunks)]
    slices = [(c, min(c + w, d)) for c in range(0, d, w)]
    q = inc.scale("col", "mean")
    val_t = inc.edge_values("csc", "sym")
    row_scale = inc.scale("row", "sym")
    tri = world * (world + 1) // 2

    pool = [torch.cuda.Stream(dev, priority=-1) for _ in range(32)]
    pool_next = [0]

    class _Staged:
        """--reduce emul: gloo's CUDA all-reduce restated with torch calls (ProcessGroupGloo's
        AsyncAllreduceCUDAWork): an event on the current stream, a high-priority pool stream
        waiting for it and copying the tensor to pinned host memory at once; at wait() the pool
        stream is synchronised, the host copy summed over the ranks (gloo on CPU tensors) and
        copied back on the pool stream, which the current stream then waits for."""

        def __init__(self, t):
            self.t = t
            cur = torch.cuda.current_stream(dev)
            ev = torch.cuda.Event()
            ev.record(cur)
            self.st = pool[pool_next[0] % len(pool)]
            pool_next[0] += 1
            self.st.wait_event(ev)
            with torch.cuda.stream(self.st):
                self.host = torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                self.host.copy_(t, non_blocking=True)

        def wait(self):
            self.st.synchronize()
            dist.all_reduce(self.host)
            with torch.cuda.stream(self.st):
                self.t.copy_(self.host, non_blocking=True)
            torch.cuda.current_stream(dev).wait_stream(self.st)

    def all_reduce(t):
        if args.sync:
            torch.cuda.current_stream(dev).synchronize()
        if args.reduce == "emul":
            return _Staged(t)
        return dist.all_reduce(t, async_op=True)

    def two_hop(Xin, mult):
        Y = torch.empty((U, d), dtype=torch.float32, device=dev)
        pieces = []
        for c0, c1 in slices:
            Xs = Xin[:, c0:c1]
            Ms = torch.empty((I, c1 - c0), dtype=torch.float32, device=dev)
            works = []
            for a, b in bounds:
                if args.hop1 == "hgd":
                    spmm_csr(inc.csc, Xs, val=val_t, row_scale=q, out=Ms, row_begin=a,
                             row_end=b)
                elif args.hop1 == "gather":  # a memory-bound torch gather of the same rows
                    torch.index_select(Bs[c0 // w], 0, perm[a:b], out=Ms[a:b])
                    Ms[a:b].mul_(float((rank + 1) * mult))
                else:
                    if args.mm:
                        torch.mm(mm_a, mm_a, out=mm_c)
                    torch.mul(B[a:b, c0:c1], float((rank + 1) * mult), out=Ms[a:b])
                if args.tail:  # one tiny torch kernel (on unrelated memory) after the producer
                    torch.mul(tail_buf, 1.0, out=tail_buf)
                works.append(all_reduce(Ms[a:b]))
            pieces.append((c0, c1, Ms, works))
        for c0, c1, Ms, works in pieces:
            for wk in works:
                wk.wait()
            if args.hop2 == "hgd":
                spmm_csr(inc.csr, Ms, val=inc.val, row_scale=row_scale, out=Y[:, c0:c1])
            else:
                Y[:, c0:c1].copy_(torch.index_select(Ms, 0, gather))
        return Y

    def step():
        return two_hop(X, 1), two_hop(dY, 2)

    closed = None
    if args.hop1 == "torch" and args.hop2 == "torch":
        closed = (B[gather] * tri, B[gather] * 2 * tri)
    elif args.hop1 == "gather" and args.hop2 == "torch":
        closed = (B[perm][gather] * tri, B[perm][gather] * 2 * tri)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    dist.barrier()
    bad_first = bad_other = 0
    t0 = time.perf_counter()
    for c in range(args.cycles):
        runs = [step() for _ in range(4)]
        last = runs[-1]
        diffs = []
        for r in runs[:-1]:
            diffs.append(max(float((r[0] - last[0]).abs().max() /
                                   last[0].abs().max().clamp_min(1e-30)),
                             float((r[1] - last[1]).abs().max() /
                                   last[1].abs().max().clamp_min(1e-30))))
        closed_bad = []
        if closed is not None:
            for r in runs:
                closed_bad.append(int(not (torch.equal(r[0], closed[0])
                                           and torch.equal(r[1], closed[1]))))
        res = torch.tensor(diffs + closed_bad, dtype=torch.float64)
        allres = [torch.zeros_like(res) for _ in range(world)]
        dist.all_gather(allres, res)
        first_off = any(float(r[0]) > 0 for r in allres) or (
            closed is not None and any(float(r[3]) > 0 for r in allres))
        other_off = any(float(v) > 0 for r in allres for v in r[1:3]) or (
            closed is not None and any(float(v) > 0 for r in allres for v in r[4:]))
        bad_first += first_off
        bad_other += other_off
        if rank == 0:
            print(json.dumps({"cycle": c, "first_step_off": first_off,
                              "later_step_off": other_off,
                              "first_vs_last_rel": [round(float(r[0]), 6) for r in allres],
                              "closed_form_wrong": ([[int(v) for v in r[3:]] for r in allres]
                                                    if closed is not None else None)}),
                  flush=True)
        del runs, last
        torch.cuda.synchronize()
        dist.barrier()
    if rank == 0:
        print(json.dumps({"summary": True, "world": world, "hop1": args.hop1,
                          "hop2": args.hop2, "sync": args.sync, "mm": args.mm, "tail": args.tail, "reduce": args.reduce,
                          "cycles": args.cycles, "cycles_first_step_off": bad_first,
                          "cycles_later_step_off": bad_other,
                          "seconds": round(time.perf_counter() - t0, 1)}), flush=True)
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--cycles", type=int, default=12)
    ap.add_argument("--users", type=int, default=10_000_000)
    ap.add_argument("--items", type=int, default=1_000_000)
    ap.add_argument("--edges", type=int, default=100_000_000)
    ap.add_argument("--dim", type=int, default=64)
    ap.add_argument("--width", type=int, default=32)
    ap.add_argument("--chunks", type=int, default=4)
    ap.add_argument("--hop1", default="torch", choices=["torch", "hgd", "gather"])
    ap.add_argument("--hop2", default="torch", choices=["torch", "hgd"])
    ap.add_argument("--mm", type=int, default=1024,
                    help="side of the matmul before each torch hop-1 chunk (0: none)")
    ap.add_argument("--tail", action="store_true",
                    help="launch one tiny torch kernel between each hop-1 chunk and its "
                         "all_reduce (the event gloo records then follows a torch kernel)")
    ap.add_argument("--reduce", default="gloo", choices=["gloo", "emul"],
                    help="gloo: dist.all_reduce of the device tensor; emul: its staging restated "
                         "with torch calls (pool stream, pinned copy, CPU all-reduce, copy back)")
    ap.add_argument("--sync", action="store_true",
                    help="drain the current stream before every all_reduce")
    args = ap.parse_args()
    import torch.multiprocessing as mp
    with socket.socket() as sck:
        sck.bind(("127.0.0.1", 0))
        port = sck.getsockname()[1]
    mp.spawn(worker, args=(args.world, port, args), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
