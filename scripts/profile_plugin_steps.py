#!/usr/bin/env python3
"""Per-step cost of the HCCF plugin on bench_plugin_epoch.py's data (Yelp shape, Zipf-1.2 items):
the sampler alone, then train_step in each drop-edge mode, wall clock per step with a sync after
each, so a kernel trace of this script (rocprofv3 --kernel-trace --stats) attributes the time.

    python scripts/profile_plugin_steps.py [--steps 20]
"""
import argparse
import json
import os
import random
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--modes", default="eager,capture_safe,device_rng")
    ap.add_argument("--uniform", action="store_true", help="uniform items instead of Zipf-1.2")
    args = ap.parse_args()
    import numpy as np
    import torch

    import bench_plugin_epoch as E
    from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                     default_args)
    tmp = tempfile.mkdtemp(prefix="hgd_steps_")
    os.chdir(tmp)
    d = os.path.join(tmp, "dataset", "yelp_synth")
    if args.uniform:
        rng = np.random.default_rng(0)
        os.makedirs(d, exist_ok=True)
        for name, n in (("train.txt", 1_170_000), ("test.txt", 390_000)):
            u, i = rng.integers(0, 31_668, n), rng.integers(0, 38_048, n)
            with open(os.path.join(d, name), "w") as f:
                f.write("user,item,rating\n")
                f.write("".join(f"{a},{b},1\n" for a, b in zip(u.tolist(), i.tolist())))
    else:
        E.write_files(d, 31_668, 38_048, 1_170_000, 390_000)
    with open("HCCF.conf", "w") as f:
        f.write(E.CONF)
    conf = ModelConf("HCCF.conf")
    kw = default_args(model="HCCF", dataset="yelp_synth", max_epoch=1, batch_size=4096,
                      embedding_size=64, hyper_dim=32, n_layers=3, lrate=0.001, drop_rate=0.5,
                      p=0.1, cl_rate=1e-4, temp=0.2, reg=0.1, item_ranking="10,20")
    train = FileIO.load_data_set(d + "/train.txt")
    test = FileIO.load_data_set(d + "/test.txt")
    out = {"data": "uniform" if args.uniform else "zipf-1.2"}
    for mode in args.modes.split(","):
        torch.manual_seed(0)
        rec = HCCF(conf, train, test, None, **dict(kw, hgd_device_rng=mode == "device_rng"))
        rec.model.edgeDropper.capture_safe = mode != "eager"
        dev = rec.device
        random.seed(1)
        batches = []
        t = time.perf_counter()
        for k, b in enumerate(next_batch_pairwise(rec.data, rec.batchSize, device=dev)):
            batches.append(b)
            if len(batches) == args.steps + 2:
                break
        torch.cuda.synchronize()
        out.setdefault("sampler_ms_per_batch", round((time.perf_counter() - t) * 1e3
                                                     / len(batches), 3))
        ts = []
        for k, b in enumerate(batches):
            torch.cuda.synchronize()
            t = time.perf_counter()
            rec.train_step(*b)
            torch.cuda.synchronize()
            if k >= 2:
                ts.append((time.perf_counter() - t) * 1e3)
        out[f"{mode}_ms_per_step"] = round(sorted(ts)[len(ts) // 2], 3)
        print(json.dumps(out), flush=True)
        del rec


if __name__ == "__main__":
    main()
