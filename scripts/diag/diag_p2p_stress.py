"""Does the hgd_p2p exchange ever return a wrong sum? (round 5: one N = 8 rehearsal's probe step
differed from RCCL by max |Y| on every rank, the rerun agreed to 2.7e-7.)

N ranks on one device (gloo for the set-up), the access pattern of ShardedIncidence.two_hop:
per call the compute stream writes the send slot of the call's parity (slot = parity·S + s for
S slices), an event orders the side stream after it, the exchange runs on the side stream into
a fresh output, and the compute stream waits for it before reading the output. Every call's
data depend on (call, rank, slice), so a stale read shows up as the value of another call. Each
rank checks every output against the rank-ordered fp32 sum and prints one JSON line per mismatch
(which rank blocks are wrong and whose data they hold) and a summary.

    python scripts/diag/diag_p2p_stress.py --world 8 --calls 200
"""
import argparse
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def value(call, rank, s):
    return float(((call * 31 + rank * 7 + s * 3) % 997) + 1)


def worker(rank, world, port, count, slices, calls):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda:0")
    torch.cuda.set_device(dev)
    from hypergraph_diffusion_for_recommendation_amd.sharded import P2PExchange
    ex = P2PExchange(count, 2 * slices, dev, timeout_s=20.0)
    side = torch.cuda.Stream(dev, priority=-1)
    cur = torch.cuda.current_stream(dev)
    ramp = (torch.arange(count, device=dev, dtype=torch.float32) % 64.0) * 2.0 ** -8
    bad = 0
    t0 = time.perf_counter()
    for c in range(calls):
        parity = c % 2
        outs = []
        for s in range(slices):
            k = parity * slices + s
            send = ex.slot(k, 1, count).view(-1)
            torch.add(ramp, value(c, rank, s), out=send)  # the "hop" into the send slot
            out = torch.empty(count, device=dev)
            ready = torch.cuda.Event()
            ready.record(cur)
            side.wait_event(ready)
            ex.allreduce(k, count, out, side.cuda_stream)
            done = torch.cuda.Event()
            done.record(side)
            outs.append((s, out, done))
        for s, out, done in outs:
            cur.wait_event(done)
            want = sum(value(c, q, s) for q in range(world))
            ref = ramp * world + want
            err = (out - ref).abs()
            if bool((err > 1e-3).any()):
                bad += 1
                # which rank blocks are wrong, and the constant part of their value
                b4 = (count // 4 + world - 1) // world * 4
                blocks = []
                for q in range(world):
                    lo, hi = q * b4, min(count, (q + 1) * b4)
                    if lo < hi and bool((err[lo:hi] > 1e-3).any()):
                        got = float((out[lo:hi] - ramp[lo:hi] * world).median())
                        blocks.append({"block": q, "got_const": got, "want_const": want})
                print(json.dumps({"rank": rank, "call": c, "slice": s, "blocks": blocks}),
                      flush=True)
    ex.wait(side, timeout_s=60.0)
    ex.check()
    torch.cuda.synchronize()
    flag = torch.tensor([bad], dtype=torch.int64)
    dist.all_reduce(flag)
    if rank == 0:
        print(json.dumps({"summary": True, "world": world, "calls": calls, "slices": slices,
                          "count": count, "wrong_outputs_all_ranks": int(flag.item()),
                          "seconds": round(time.perf_counter() - t0, 2)}), flush=True)
    ex.close()
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--count", type=int, default=1 << 22)
    ap.add_argument("--slices", type=int, default=2)
    ap.add_argument("--calls", type=int, default=200)
    args = ap.parse_args()
    import torch.multiprocessing as mp
    with socket.socket() as sck:
        sck.bind(("127.0.0.1", 0))
        port = sck.getsockname()[1]
    mp.spawn(worker, args=(args.world, port, args.count, args.slices, args.calls),
             nprocs=args.world, join=True)


if __name__ == "__main__":
    main()
