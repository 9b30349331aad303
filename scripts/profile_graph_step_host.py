#!/usr/bin/env python3
"""Where the host time of the HCCF plugin's replayed step goes (HCCF.graph_step, the default):
per step, wall time of the before-replay work (SpAdjDropEdge.refill: the reference's CPU mask
stream; ReferenceAdam.prepare: step counters), of the replay call, and of the whole step with a
device sync (as the plugin's loop syncs on batch_loss.item()), beside the replay's device time
(HIP events); then the same steps back to back with no host read between them
(step_pipelined: wall time per step; host_issue_per_step: the host's time to issue one).
Yelp2018-shaped synthetic graph (SURVEY.md §8d generator), batch 4096, 3 layers, d = 64.
Prints one JSON line of medians (µs)."""
import argparse
import json
import os
import statistics
import sys
import time
import types

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(ROOT))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--switch-interval", type=float, default=None,
                    help="sys.setswitchinterval for the run (seconds; the interpreter's GIL "
                         "hand-off period, 0.005 by default)")
    args = ap.parse_args()
    if args.switch_interval:
        sys.setswitchinterval(args.switch_interval)
    import torch

    import refops as R
    from hypergraph_diffusion_for_recommendation_amd.encoders import HCCFEncoder
    from hypergraph_diffusion_for_recommendation_amd.functional import (bpr_loss_rows,
                                                                         contrast_loss_layers,
                                                                         unique_long_n_group)
    from hypergraph_diffusion_for_recommendation_amd.graphs import CapturedStep
    from hypergraph_diffusion_for_recommendation_amd.optim import ReferenceAdam
    dev = torch.device("cuda")
    nu, ni = 31_668, 38_048
    u, i = R.synthetic_incidence(nu, ni, 1_237_259, seed=0)
    A = R.normalize_graph_mat(R.bipartite_adjacency(u, i, nu, ni))
    data = types.SimpleNamespace(n_users=nu, n_items=ni, norm_adj=A)
    conf = dict(lrate=0.001, lr_decay=0.7, max_epoch=1, batch_size=4096, reg=0.1,
                embedding_size=64, hyper_dim=32, drop_rate=0.5, p=0.1, n_layers=3)
    torch.manual_seed(0)
    model = HCCFEncoder(conf, data, dev)
    model.edgeDropper.capture_safe = True
    opt = ReferenceAdam(model.parameters(), lr=1e-3)
    g = torch.Generator(device=dev).manual_seed(0)
    batches = [tuple(torch.randint(0, n, (4096,), device=dev, generator=g) for n in (nu, ni, ni))
               for _ in range(8)]
    capturing = [False]

    def body(uid, pid, nid):
        ue, ie, gcn, hyp = model(keep_rate=0.5)
        bpr, anc, pos = bpr_loss_rows(ue, ie, uid, pid, nid)
        (un, uc), (pn, pc) = unique_long_n_group([anc, pos], [nu, ni])
        ssl = contrast_loss_layers([t.detach() for t in gcn], hyp, nu, un, pn, 0.2, uc, pc)
        loss = bpr + 1e-4 * ssl
        opt.zero_grad()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 4)
        loss.backward()
        if capturing[0]:
            opt.launch()
        else:
            opt.step()
        return loss

    body(*batches[0])
    dropper = model.edgeDropper
    dropper.host_fed(True)
    capturing[0] = True
    cap = CapturedStep(body, batches[1], before_replay=None)
    capturing[0] = False
    # the draw the worker makes per step (one split draw of the step's three masks), alone
    from hypergraph_diffusion_for_recommendation_amd import layers as LY
    spec = tuple((n, keep) for n, keep, _ in dropper._slots)
    draws = []
    for _ in range(12):
        t0 = time.perf_counter()
        LY._draw_step_masks(torch.get_rng_state(), spec)
        draws.append((time.perf_counter() - t0) * 1e6)
    # how long refill waits for the worker's job
    waits = []
    orig_result = None

    def timed_result(fut):
        t0 = time.perf_counter()
        out = orig_result(fut)
        waits.append((time.perf_counter() - t0) * 1e6)
        return out
    import concurrent.futures as cf
    orig_result = cf.Future.result
    cf.Future.result = timed_result
    rec = {"refill": [], "prepare": [], "copy_inputs": [], "replay_call": [], "step_synced": [],
           "device_replay": []}
    for k in range(args.steps):
        b = batches[k % len(batches)]
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        dropper.refill()
        t1 = time.perf_counter()
        opt.prepare()
        t2 = time.perf_counter()
        for dst, src in zip(cap.static, b):
            dst.copy_(src)
        t3 = time.perf_counter()
        e0.record()
        cap.graph.replay()
        e1.record()
        t4 = time.perf_counter()
        float(cap.out.sum()) if hasattr(cap.out, "sum") else None
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        if k >= 5:
            for name, v in (("refill", t1 - t0), ("prepare", t2 - t1), ("copy_inputs", t3 - t2),
                            ("replay_call", t4 - t3), ("step_synced", t5 - t0),
                            ("device_replay", e0.elapsed_time(e1) * 1e-3)):
                rec[name].append(v * 1e6)
    cf.Future.result = orig_result
    # the same steps with no host read between them (the plugin's loop reads the losses once
    # per epoch): the host prepares step k+1 while the device runs step k
    stager = dropper._stager()
    stager.trace = []
    losses = []
    pipe = {"refill": [], "prepare": [], "copy_inputs": [], "replay_call": [], "loss_clone": []}
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        b = batches[k % len(batches)]
        ta = time.perf_counter()
        dropper.refill()
        tb = time.perf_counter()
        opt.prepare()
        tc = time.perf_counter()
        for dst, src in zip(cap.static, b):
            dst.copy_(src)
        td = time.perf_counter()
        cap.graph.replay()
        te = time.perf_counter()
        losses.append(cap.out.detach().clone())
        tf = time.perf_counter()
        for name, v in (("refill", tb - ta), ("prepare", tc - tb), ("copy_inputs", td - tc),
                        ("replay_call", te - td), ("loss_clone", tf - te)):
            pipe[name].append(v * 1e6)
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    out_pipe = {"step_pipelined": round((time.perf_counter() - t0) / args.steps * 1e6, 1),
                "host_issue_per_step": round(t_host / args.steps * 1e6, 1),
                "pipelined_host_us": {k: round(statistics.median(v[5:]), 1)
                                      for k, v in pipe.items()},
                "pipelined_host_max_us": {k: round(max(v[5:]), 1) for k, v in pipe.items()}}
    # two slot banks and one captured step per bank (the plugins' default): the worker copies
    # the next step's masks straight into the bank the running replay does not read
    dropper.host_fed(True, banks=2)
    caps = []
    for bank in range(2):
        dropper.use_bank(bank)
        capturing[0] = True
        caps.append(CapturedStep(body, batches[1], before_replay=None))
        capturing[0] = False
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(args.steps):
        b = batches[k % len(batches)]
        c = caps[dropper.upcoming_bank()]
        dropper.refill()
        opt.prepare()
        for dst, src in zip(c.static, b):
            dst.copy_(src)
        c.graph.replay()
        losses.append(c.out.detach().clone())
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    out_pipe["step_pipelined_banked"] = round((time.perf_counter() - t0) / args.steps * 1e6, 1)
    out_pipe["host_issue_per_step_banked"] = round(t_host / args.steps * 1e6, 1)
    out = {k: round(statistics.median(v), 1) for k, v in rec.items()}
    out.update(out_pipe)
    out["draw_step_masks_alone"] = round(statistics.median(draws[2:]), 1)
    out["refill_wait_for_worker"] = round(statistics.median(waits[5:]), 1) if waits else None
    out["spec"] = spec
    out["switch_interval"] = sys.getswitchinterval()
    jobs = stager.trace[5:]
    if jobs:
        out["pipelined_worker_job_us"] = {
            name: round(statistics.median(j[i] for j in jobs), 1)
            for i, name in enumerate(("wait_host_buffer", "draw", "stage_h2d_issue"))}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
