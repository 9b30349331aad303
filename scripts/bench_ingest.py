#!/usr/bin/env python3
"""Ingest + graph build on a synthetic "user\\titem\\t1" training file:
the native path (hgd_ingest_read with N host threads → device id remap, coalesce, normalisation,
CSR/CSC incidences) against the reference's Python path (FileIO.load_data_set's line loop, the
Interaction dict loop, scipy csr_matrix + normalize_graph_mat; restated in scripts/refops) on a
bounded sample. Prints one JSON line per measurement."""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lines", type=int, default=20_000_000)
    ap.add_argument("--users", type=int, default=1_000_000)
    ap.add_argument("--items", type=int, default=100_000)
    ap.add_argument("--threads", type=int, default=16)
    ap.add_argument("--cpu-sample", type=int, default=1_000_000)
    args = ap.parse_args()
    import numpy as np
    import pandas as pd
    import torch

    from hypergraph_diffusion_for_recommendation_amd.ingest import InteractionGraph, load_data_set
    import refops as O

    rng = np.random.default_rng(0)
    users = rng.integers(0, args.users, size=args.lines) * 7 + 3  # sparse raw id space
    items = rng.integers(0, args.items, size=args.lines) * 11 + 5
    tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
    path = os.path.join(tmp, "train.txt")
    t0 = time.perf_counter()
    pd.DataFrame({"user": users, "item": items, "rating": 1}).to_csv(path, sep="\t", index=False)
    size = os.path.getsize(path)
    print(json.dumps({"step": "write_file", "lines": args.lines, "bytes": size,
                      "s": round(time.perf_counter() - t0, 2)}), flush=True)

    dev = torch.device("cuda")
    torch.zeros(1, device=dev)
    for rep in range(2):  # second run: page cache warm
        t0 = time.perf_counter()
        u, i = load_data_set(path, n_threads=args.threads)
        t1 = time.perf_counter()
        g = InteractionGraph(u, i, dev)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(json.dumps({"step": "native", "rep": rep, "lines": args.lines,
                          "parse_s": round(t1 - t0, 3), "parse_MBps": round(size / (t1 - t0) / 1e6),
                          "device_build_s": round(t2 - t1, 3), "total_s": round(t2 - t0, 3),
                          "n_users": g.n_users, "n_items": g.n_items,
                          "nnz_ui_adj": g.ui_adj.csr.nnz}), flush=True)
    del g

    # the reference's Python path on a bounded sample (first cpu_sample lines)
    spath = os.path.join(tmp, "sample.txt")
    with open(path) as f, open(spath, "w") as o:
        for k, line in enumerate(f):
            if k > args.cpu_sample:
                break
            o.write(line)
    import scipy.sparse as sp
    t0 = time.perf_counter()
    data = O.load_data_set(spath)
    t1 = time.perf_counter()
    user, item = O.remap_ids((r[0], r[1]) for r in data)
    ui = np.array([user[r[0]] for r in data])
    ii = np.array([item[r[1]] for r in data])
    adj = O.bipartite_adjacency(ui, ii, len(user), len(item))
    O.normalize_graph_mat(adj)
    R = sp.csr_matrix((np.ones(len(ui), np.float32), (ui, ii)), shape=(len(user), len(item)))
    O.normalize_graph_mat(R)
    t2 = time.perf_counter()
    print(json.dumps({"step": "reference_python", "lines": args.cpu_sample,
                      "parse_s": round(t1 - t0, 3), "build_s": round(t2 - t1, 3),
                      "total_s": round(t2 - t0, 3),
                      "extrapolated_total_s_full": round((t2 - t0) * args.lines / args.cpu_sample,
                                                         1)}), flush=True)
    os.remove(path)
    os.remove(spath)
    os.rmdir(tmp)


if __name__ == "__main__":
    main()
