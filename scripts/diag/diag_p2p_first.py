"""Is the FIRST peer exchange after its set-up ever wrong? (round 5: one N = 8 rehearsal of
bench.py on one device saw the transport probe's first p2p step differ from RCCL by max |Y| on
every rank; reruns, and diag_p2p_stress.py's 720 exchanges per rank on a standing exchange, did
not.)

Replays bench.py's probe sequence ``--cycles`` times on the headline graph sharded over N ranks
(gloo stands in for RCCL, as in the rehearsal): one step over the all-reduce (the reference
result), three more, a barrier, then ONE step over a freshly created peer exchange compared with
the reference, and the exchange closed so the next cycle creates a new one. Prints one JSON line
per cycle from rank 0 (max over ranks of the relative difference, and which ranks failed) and a
summary.

Finding (profiles/r05_scale/p2p_first/): the peer step was right every time — bitwise equal to
the last all-reduce step, its send slots equal to the hop recomputed, a second exchange of them
equal to gloo's sum — and the FIRST gloo step after the barrier was the one that was off, in
about a third of the cycles. bench.py's probe now takes its reference from the last step.

    python scripts/diag/diag_p2p_first.py --world 8 --cycles 12
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
    import bench
    from hypergraph_diffusion_for_recommendation_amd.incidence import spmm_csr
    from hypergraph_diffusion_for_recommendation_amd.sharded import (ShardedIncidence,
                                                                       sharded_two_hop)
    U, I, E, d = args.users, args.items, args.edges, args.dim
    if args.sync_before_allreduce:
        # every all-reduce issued only once the current stream has drained: the producing hop is
        # complete before gloo records its event and stages the tensor to the host
        plain = dist.all_reduce

        def synced(t, *a, **k):
            if t.is_cuda:
                torch.cuda.current_stream(t.device).synchronize()
            return plain(t, *a, **k)
        dist.all_reduce = synced
    for turn in range(world):  # one graph build at a time on the shared device
        if turn == rank:
            idx = bench.make_graph(U, I, E, seed=0, zipf=None, device=dev)
            torch.cuda.synchronize()
        dist.barrier()
    sh, u0, u1 = ShardedIncidence.from_global(idx, U, I, device=dev, n_chunks=4, P="sym",
                                              Q="mean", R="sym", slice_width=None,
                                              transport="rccl")
    del idx
    X = bench.table_rows(u0, u1, d, 1000, dev, (6.0 / (U + d)) ** 0.5)
    dY = bench.table_rows(u0, u1, d, 1001, dev)
    X.requires_grad_(True)

    def step():
        Y = sharded_two_hop(sh, X)
        (dX,) = torch.autograd.grad(Y, X, dY)
        return Y.detach(), dX

    for _ in range(3):  # the bench's warm-up
        step()
    torch.cuda.synchronize()
    dist.barrier()
    bad = 0
    t0 = time.perf_counter()
    for c in range(args.cycles):
        sh.transport = "rccl"
        Y_r, dX_r = step()
        runs = [(Y_r, dX_r)] + [step() for _ in range(3)]

        def rel_of(a, b):
            return max(float((a[0] - b[0]).abs().max() / b[0].abs().max().clamp_min(1e-30)),
                       float((a[1] - b[1]).abs().max() / b[1].abs().max().clamp_min(1e-30)))
        # the all-reduce steps among themselves: each against the last one
        rccl_rel = [rel_of(r, runs[-1]) for r in runs[:-1]]
        torch.cuda.synchronize()
        dist.barrier()
        err = None
        rel = float("nan")
        precreate = args.precreate == "all" or (args.precreate == "odd" and c % 2 == 1)
        warm_bad = []
        if precreate:  # the exchange set up (collective) and the device idle before the step
            ex = sh.p2p(d)
            torch.cuda.synchronize()
            dist.barrier()
            # --warm: known-pattern exchanges through every send slot before the step (rank q
            # fills its slot with q + 1 + i/2^20 for element i); rows off per round and slot
            cur = torch.cuda.current_stream(dev)
            n = ex.max_count
            ramp = torch.arange(n, device=dev, dtype=torch.float32) * 2.0 ** -20
            want = ramp * world + world * (world + 1) / 2
            for r in range(args.warm):
                for k in range(ex.n_slots):
                    ex.slot(k, 1, n).view(-1).copy_(ramp + (rank + 1))
                    out = torch.empty(n, device=dev)
                    ex.allreduce(k, n, out, cur.cuda_stream)
                    ex.wait()
                    ex.check()
                    warm_bad.append(float(((out - want).abs() > 1e-3).float().mean()))
            torch.cuda.synchronize()
            dist.barrier()
        try:
            sh.transport = "p2p"
            Y_p, dX_p = step()
            sh._p2p.wait()
            sh._p2p.check()
            rel = max(float((Y_p - Y_r).abs().max() / Y_r.abs().max().clamp_min(1e-30)),
                      float((dX_p - dX_r).abs().max() / dX_r.abs().max().clamp_min(1e-30)))
            # where a wrong Y sits: the fraction of rows off, and of them the share that is 0
            off = (Y_p - Y_r).abs().amax(1) > 1e-5 * Y_r.abs().max()
            frac_off = float(off.float().mean())
            zero_rows = float((Y_p[off].abs().amax(1) == 0).float().mean()) if bool(off.any()) \
                else 0.0
        except Exception as e:  # noqa: BLE001 — reported
            err = repr(e)[:300]
            frac_off = zero_rows = float("nan")
        # where it went wrong: each rank's forward send slots against the same hop recomputed
        # (the slots of parity 0 still hold the forward's partial messages), and one more
        # exchange of those slots against gloo's sum of the recomputed partials
        extra = []
        ex = sh._p2p
        with torch.no_grad():
            val_t = sh.inc.edge_values("csc", sh.R)
            n_cols = sh.inc.n_cols
            cur = torch.cuda.current_stream(dev)
            for s, (c0, c1) in enumerate(sh.slices(d)):
                w = c1 - c0
                part = torch.empty((n_cols, w), device=dev)
                spmm_csr(sh.inc.csc, X.detach()[:, c0:c1], val=val_t, row_scale=sh.q, out=part)
                slot = ex.slot(s, n_cols, w)
                tol = 1e-6 * float(part.abs().max())
                extra.append(float(((slot - part).abs().amax(1) > tol).float().mean()))
                m_ref = part.clone()
                dist.all_reduce(m_ref)
                torch.cuda.synchronize()
                out2 = torch.empty((n_cols, w), device=dev)
                ex.allreduce(s, n_cols * w, out2, cur.cuda_stream)
                ex.wait()
                ex.check()
                tol = 1e-5 * float(m_ref.abs().max())
                extra.append(float(((out2 - m_ref).abs().amax(1) > tol).float().mean()))
        extra.append(float(Y_p.abs().max() / Y_r.abs().max()) if err is None else -1.0)
        extra += rccl_rel
        extra.append(rel_of((Y_p, dX_p), runs[-1]) if err is None else -1.0)
        res = torch.tensor(extra + [rel if rel == rel else 1e30, frac_off if frac_off == frac_off else 1.0,
                            zero_rows if zero_rows == zero_rows else 0.0,
                            1.0 if (err is not None or not rel <= 1e-5) else 0.0],
                           dtype=torch.float64)
        allres = [torch.zeros_like(res) for _ in range(world)]
        dist.all_gather(allres, res)
        ne = len(extra)
        failed = [q for q in range(world) if allres[q][ne + 3] > 0]
        bad += bool(failed)
        if rank == 0:
            print(json.dumps({"cycle": c, "precreated": precreate,
                              "max_rel_diff": max(float(r[ne]) for r in allres),
                              "failed_ranks": failed,
                              "frac_rows_off": [round(float(r[ne + 1]), 6) for r in allres],
                              "zero_share_of_off_rows": [round(float(r[ne + 2]), 4)
                                                         for r in allres],
                              # per rank: [send slot s0 rows off, re-exchange s0 rows off, s1 ..,
                              #            max|Y_p| / max|Y_r|, all-reduce steps 0-2 vs step 3
                              #            (rel. diff), the p2p step vs all-reduce step 3]
                              "slot_checks": [[round(float(v), 6) for v in r[:ne]]
                                              for r in allres],
                              "warm_rows_off_rank0": warm_bad,
                              "error_rank0": err}), flush=True)
        sh.close()  # collective; the next cycle's first p2p step creates a new exchange
        torch.cuda.synchronize()
        dist.barrier()
    if rank == 0:
        print(json.dumps({"summary": True, "world": world, "cycles": args.cycles,
                          "cycles_with_a_wrong_first_exchange": bad,
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
    ap.add_argument("--sync-before-allreduce", action="store_true",
                    help="drain the current stream before every all-reduce call")
    ap.add_argument("--warm", type=int, default=0,
                    help="with --precreate: rounds of known-pattern exchanges through every slot")
    ap.add_argument("--precreate", default="none", choices=["none", "odd", "all"],
                    help="set the exchange up before the p2p step (none: inside it, as bench.py)")
    args = ap.parse_args()
    import torch.multiprocessing as mp
    with socket.socket() as sck:
        sck.bind(("127.0.0.1", 0))
        port = sck.getsockname()[1]
    mp.spawn(worker, args=(args.world, port, args), nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
