#!/usr/bin/env python3
"""Where does the plugin epoch (scripts/bench_plugin_epoch.py) go non-finite? That bench stopped
in its device-mask epoch with contrast_loss's "node index out of range" — the node list is
torch.unique(pos_emb.long()) (HCCF.py:65-66), so an embedding row had gone NaN / inf. This runs
the same set-up and epochs with a check after every step: the loss, the encoder's outputs and
every parameter and gradient, and prints the first step (epoch, batch, batch size, mode) at
which anything is non-finite, with the names of the tensors.

    python scripts/diag/diag_epoch_nan.py [--modes cpu,device,cs_cpu]
"""
import argparse
import os
import random
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--modes", default="cpu,device,cs_cpu")
    ap.add_argument("--users", type=int, default=31_668)
    ap.add_argument("--items", type=int, default=38_048)
    ap.add_argument("--train", type=int, default=1_170_000)
    ap.add_argument("--test", type=int, default=390_000)
    ap.add_argument("--warm", action="store_true",
                    help="one train_step on the first batch first, as bench_plugin_epoch.py")
    ap.add_argument("--nosync", action="store_true",
                    help="no per-step checks (the bench's timing): report the batch that raises "
                         "and check the parameters at each epoch's end")
    args = ap.parse_args()
    import torch

    import bench_plugin_epoch as E
    from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                     default_args)
    tmp = tempfile.mkdtemp(prefix="hgd_nan_")
    os.chdir(tmp)
    d = os.path.join(tmp, "dataset", "yelp_synth")
    E.write_files(d, args.users, args.items, args.train, args.test)
    with open("HCCF.conf", "w") as f:
        f.write(E.CONF)
    conf = ModelConf("HCCF.conf")
    kw = default_args(model="HCCF", dataset="yelp_synth", max_epoch=1, batch_size=4096,
                      embedding_size=64, hyper_dim=32, n_layers=3, lrate=0.001, drop_rate=0.5,
                      p=0.1, cl_rate=1e-4, temp=0.2, reg=0.1, item_ranking="10,20")
    train = FileIO.load_data_set(d + "/train.txt")
    test = FileIO.load_data_set(d + "/test.txt")
    torch.manual_seed(0)
    rec = HCCF(conf, train, test, None, **kw)
    dev = rec.device
    drop = rec.model.edgeDropper
    print(f"n_users {rec.data.n_users} n_items {rec.data.n_items}", flush=True)

    def bad_tensors(outs):
        names = []
        for k, t in outs.items():
            if t is not None and not bool(torch.isfinite(t).all()):
                names.append(k)
        for k, p in rec.model.named_parameters():
            if not bool(torch.isfinite(p).all()):
                names.append("param:" + k)
            if p.grad is not None and not bool(torch.isfinite(p.grad).all()):
                names.append("grad:" + k)
        return names

    random.seed(1)
    if args.warm:
        b0 = next(iter(next_batch_pairwise(rec.data, rec.batchSize, device=dev)))
        rec.train_step(*b0)
    for ep, mode in enumerate(args.modes.split(",")):
        if args.nosync:
            drop.device_rng = mode == "device"
            drop.capture_safe = mode.startswith("cs")
            b = -1
            try:
                for b, (u, i, j) in enumerate(next_batch_pairwise(rec.data, rec.batchSize,
                                                                  device=dev)):
                    rec.train_step(u, i, j)
            except Exception as e:  # noqa: BLE001
                print(f"mode {mode} epoch {ep}: batch {b} raised {e!r:.300}; non-finite now: "
                      f"{bad_tensors({})}", flush=True)
                return 1
            torch.cuda.synchronize()
            print(f"mode {mode}: epoch done ({b + 1} batches), non-finite: {bad_tensors({})}",
                  flush=True)
            continue
        drop.device_rng = mode == "device"
        drop.capture_safe = mode.startswith("cs")
        for b, (u, i, j) in enumerate(next_batch_pairwise(rec.data, rec.batchSize, device=dev)):
            # the encoder's outputs of this step's forward (same RNG draws as train_step makes)
            st_cpu, st_dev = torch.get_rng_state(), torch.cuda.get_rng_state(dev)
            with torch.no_grad():
                ue, ie, gcn, hyp = rec.model(keep_rate=1 - rec.dropRate)
            torch.set_rng_state(st_cpu)
            torch.cuda.set_rng_state(st_dev, dev)
            outs = {"user_emb": ue, "item_emb": ie}
            outs.update({f"gcn{k}": t for k, t in enumerate(gcn)})
            outs.update({f"hyp{k}": t for k, t in enumerate(hyp)})
            pre = bad_tensors(outs)
            try:
                loss = rec.train_step(u, i, j)
                err = None
            except Exception as e:  # noqa: BLE001
                loss, err = None, repr(e)[:300]
            post = bad_tensors({"loss": loss})
            if pre or post or err:
                print(f"mode {mode} epoch {ep} batch {b} size {u.numel()}: before step {pre}, "
                      f"after {post}, error {err}", flush=True)
                return 1
            if b % 25 == 0 or b >= 270:
                mags = " ".join(f"{k} {float(t.abs().max()):.3g}" for k, t in outs.items())
                print(f"mode {mode} batch {b} loss {float(loss):.6f} max|.|: {mags}",
                      flush=True)
        print(f"mode {mode}: epoch finite ({b + 1} batches, last size {u.numel()})", flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
