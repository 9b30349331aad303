#!/usr/bin/env python3
"""Where the wall time of one HCCF plugin epoch goes (bench_plugin_epoch.py's Yelp2018-shaped
set and default step, HCCF.graph_step): the sampler alone over an epoch
(next_batch_pairwise(device=cuda), no step), the steps alone over pre-sampled batches (no host
read between them), the full epoch, and a cProfile of the full epoch (top host functions by own
time). Prints one JSON line."""
import cProfile
import io
import json
import os
import pstats
import random
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    import torch

    import bench_plugin_epoch as B
    from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                     default_args)
    tmp = tempfile.mkdtemp(prefix="hgd_epoch_prof_")
    os.chdir(tmp)
    d = os.path.join(tmp, "dataset", "yelp_synth")
    B.write_files(d, 31_668, 38_048, 1_170_000, 390_000)
    with open("HCCF.conf", "w") as f:
        f.write(B.CONF)
    conf = ModelConf("HCCF.conf")
    kw = default_args(model="HCCF", dataset="yelp_synth", max_epoch=1, batch_size=4096,
                      embedding_size=64, hyper_dim=32, n_layers=3, lrate=0.001, drop_rate=0.5,
                      p=0.1, cl_rate=1e-4, temp=0.2, reg=0.1, item_ranking="10,20")
    train = FileIO.load_data_set(d + "/train.txt")
    test = FileIO.load_data_set(d + "/test.txt")
    torch.manual_seed(0)
    rec = HCCF(conf, train, test, None, **kw)
    dev = rec.device
    out = {}
    random.seed(1)
    for k, b in enumerate(next_batch_pairwise(rec.data, rec.batchSize, device=dev)):
        rec.graph_step(*b)  # warm-up: eager steps, capture, replays
        if k >= 4:
            break
    torch.cuda.synchronize()
    # the sampler alone (the first batch includes the epoch's in-place shuffle)
    t = time.perf_counter()
    first = None
    batches = []
    for b in next_batch_pairwise(rec.data, rec.batchSize, device=dev):
        if first is None:
            first = time.perf_counter() - t
        batches.append(b)
    torch.cuda.synchronize()
    out["sampler_epoch_s"] = round(time.perf_counter() - t, 4)
    out["sampler_first_batch_s"] = round(first, 4)
    out["batches"] = len(batches)
    # the steps alone over the pre-sampled batches
    t = time.perf_counter()
    for b in batches:
        rec.graph_step(*b)
    torch.cuda.synchronize()
    out["steps_only_s"] = round(time.perf_counter() - t, 4)
    del batches
    # the full epoch under cProfile
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    for b in next_batch_pairwise(rec.data, rec.batchSize, device=dev):
        rec.graph_step(*b)
    torch.cuda.synchronize()
    pr.disable()
    out["epoch_profiled_s"] = round(time.perf_counter() - t, 4)
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    out["top_tottime"] = [ln.strip() for ln in s.getvalue().splitlines() if ln.strip()][-20:]
    t = time.perf_counter()
    for b in next_batch_pairwise(rec.data, rec.batchSize, device=dev):
        rec.graph_step(*b)
    torch.cuda.synchronize()
    out["epoch_s"] = round(time.perf_counter() - t, 4)
    # the epoch with fewer host threads for the drop-edge draw (HGD_TUNE_CPU_RNG_THREADS = 12):
    # the draw's threads and the loop's own thread share the box's cores
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    by_threads = {}
    try:
        for th in (16, 12, 8, 4):
            nat.check(lib.hgd_set_tuning(12, th), "hgd_set_tuning")
            t = time.perf_counter()
            for b in next_batch_pairwise(rec.data, rec.batchSize, device=dev):
                rec.graph_step(*b)
            torch.cuda.synchronize()
            by_threads[str(th)] = round(time.perf_counter() - t, 4)
    finally:
        nat.check(lib.hgd_set_tuning(12, 0), "hgd_set_tuning")
    out["epoch_s_by_rng_threads"] = by_threads
    out["cpu_count"] = os.cpu_count()
    out["affinity"] = len(os.sched_getaffinity(0))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
