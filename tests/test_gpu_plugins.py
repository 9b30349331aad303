"""GPU: the SELFRec plugin surface (selfrec.py + plugins.py) end to end on a small dataset
written in the reference's file formats, and HCCF's training steps against the reference's
own torch calls (oracle/ref_cpu.py) with the same initial weights, batches and RNG draws."""
import copy
import os
import random

import numpy as np
import pytest
import torch

from oracle import hgd_oracle as O
from tests import _ref64 as R

pytestmark = pytest.mark.gpu

HCCF_CONF = """training.set=train.txt
test.set=test.txt
dataset=toy
model.name={model}
model.type=graph
item.ranking=-topN 10,20
embedding.size=32
num.max.epoch=2
batch_size=256
num_layers=2
learnRate=0.001
learnRateDecay=0.7
reg.lambda=0.01
use.knowledge=false
hyper.size=32
ss_rate=1
dropout=0.3
leaky=0.5
temp=1
"""


def _write_dataset(root, n_users=300, n_items=500, n_train=6000, seed=0, zipf=1.3):
    """train.txt / test.txt with a header line, comma separated (data/loader.py:24-38); raw ids
    are not dense; the test file holds unseen users (dropped) and unseen items (kept)."""
    rng = np.random.default_rng(seed)
    d = os.path.join(root, "toy")
    os.makedirs(d, exist_ok=True)
    u = rng.integers(0, n_users, n_train) * 3 + 1
    i = rng.zipf(zipf, n_train) % n_items * 7 + 2
    with open(os.path.join(d, "train.txt"), "w") as f:
        f.write("user,item,rating\n")
        f.writelines(f"{a},{b},1\n" for a, b in zip(u, i))
    tu = rng.integers(0, n_users + 20, 900) * 3 + 1
    ti = rng.integers(0, n_items + 10, 900) * 7 + 2
    with open(os.path.join(d, "test.txt"), "w") as f:
        f.write("user\titem\trating\n")
        f.writelines(f"{a}\t{b}\t1\n" for a, b in zip(tu, ti))
    return d


def _setup(tmp_path, monkeypatch, model="HCCF", **over):
    from hypergraph_diffusion_for_recommendation_amd.selfrec import ModelConf, default_args
    monkeypatch.chdir(tmp_path)
    _write_dataset(str(tmp_path / "dataset"))
    conf_path = tmp_path / f"{model}.conf"
    conf_path.write_text(HCCF_CONF.format(model=model))
    conf = ModelConf(str(conf_path))
    conf.config['dataset'] = 'toy'
    args = dict(dataset='toy', max_epoch=2, batch_size=256, embedding_size=32, hyper_dim=32,
                input_dim=32, n_layers=2, item_ranking='10,20', drop_rate=0.3, p=0.5, temp=0.2,
                cl_rate=1e-3, reg=0.01, early_stopping_steps=5, seed=7)
    extra = {k: over.pop(k) for k in list(over) if k.startswith("hgd_")}
    args.update(over)
    kwargs = default_args(**args)
    kwargs.update(extra)
    kwargs['dataset_root'] = str(tmp_path / "dataset")
    return conf, kwargs


@pytest.mark.parametrize("model,extra", [("HCCF", {}), ("HGNN_HD4", {"mode": "local_only"}),
                                         ("HGNN_HD3", {"mode": "local_only"}),
                                         ("HGCN", {}), ("HCCF_diffusion", {}), ("DHCF", {}),
                                         ("HCCF", {"hgd_device_rng": True}),
                                         ("HCCF", {"hgd_graph": True}),
                                         ("HCCF_diffusion", {"hgd_graph": True}),
                                         ("HCCF", {"hgd_graph": False}),
                                         ("HCCF_diffusion", {"hgd_graph": False})])
def test_selfrec_execute_end_to_end(dev, tmp_path, monkeypatch, model, extra):
    from hypergraph_diffusion_for_recommendation_amd.selfrec import SELFRec
    conf, kwargs = _setup(tmp_path, monkeypatch, model, **extra)
    random.seed(3)
    torch.manual_seed(3)
    rec = SELFRec(conf, kwargs).execute()
    # the lifecycle's files (graph_recommender.py:94-119, 201-239)
    out = rec.output + "/"
    assert os.path.exists(out + f"{model}-top-20items.txt")
    assert os.path.exists(out + f"{model}-performance.txt")
    assert os.path.exists(rec.output + "/performance.csv")
    # the device metrics are the reference's ranking_evaluation of the same lists
    rec_list = rec.test()
    assert list(rec_list) == list(rec.data.test_set)
    assert rec.result == O.ranking_evaluation(rec.data.test_set, rec_list, rec.topN)
    # users absent from training are dropped from the test set, unseen items are kept
    assert all(u in rec.data.user for u in rec.data.test_set)
    assert any(i not in rec.data.item for t in rec.data.test_set.values() for i in t)
    assert len(rec.bestPerformance) == 2 and rec.bestPerformance[1]['Recall'] >= 0.0


def _teacher_forced_hccf_steps(dev, tmp_path, monkeypatch, n_steps, zipf=None, fp32=False):
    """``n_steps`` HCCF training steps through the plugin (HCCF.py:79-97: libhgd hops, fused
    InfoNCE, MFMA E·W) on the plugin's own batches. At every step, from the parameters the plugin
    holds before it and with the same drop-edge and dropout draws, the float64 reference
    (tests/_ref64.py, the reference's torch calls) gives the batch loss and the gradient of every
    parameter that the plugin's optimizer then applies; held to 1e-5 (relative loss, every
    gradient row against its scale); with ``fp32`` the same torch calls' own deviation in float32
    is recorded beside. Returns the worst row ratio."""
    from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import FileIO
    conf, kwargs = _setup(tmp_path, monkeypatch, "HCCF")
    kwargs.pop('dataset_root')
    if zipf is not None:  # a more skewed catalogue than the toy set's Zipf(1.3) over 500 items
        _write_dataset(str(tmp_path / "dataset"), n_items=300, zipf=zipf)
    d = str(tmp_path / "dataset" / "toy") + "/"
    torch.manual_seed(0)
    rec = HCCF(conf, FileIO.load_data_set(d + "train.txt"), FileIO.load_data_set(d + "test.txt"),
               None, **kwargs)
    enc = rec.model
    nu, ni = rec.data.n_users, rec.data.n_items
    N, L = nu + ni, rec.nLayers
    enc.drop_out = R.FixedDropout(enc.drop_rate, 5)
    enc.edgeDropper = R.DropRecorder(enc.edgeDropper)
    idx, vals = enc.sparse_norm_adj._indices().cpu(), enc.sparse_norm_adj._values().cpu()
    keep_e, keep_h = 1 - rec.dropRate, 1 - enc.drop_rate
    random.seed(11)
    batches = list(next_batch_pairwise(rec.data, 256, device=dev))
    batches = (batches * (1 + n_steps // len(batches)))[:n_steps]
    worst = worst32 = 0.0

    def reference(before, dtype, adjs, masks, u, i, j):
        P = {n: v.to(dtype).clone().requires_grad_(True) for n, v in before.items()}
        ueR, ieR, gR, hR = R.hccf_encoder(P, [a.to(dtype) for a in adjs],
                                          [m.to(dtype) for m in masks], keep_h, nu, L)
        anc, pos, neg = ueR[u], ieR[i], ieR[j]
        u_nodes, p_nodes = torch.unique(anc.long()), torch.unique(pos.long())
        ssl = 0
        for layer in range(L):
            e1, e2 = gR[layer].detach(), hR[layer]
            ssl = ssl + R.contrast_loss(e1[:nu], e2[:nu], u_nodes, rec.temp) \
                + R.contrast_loss(e1[nu:], e2[nu:], p_nodes, rec.temp)
        loss = R.bpr_loss(anc, pos, neg) + ssl * rec.ss_rate
        names = list(P)
        return float(loss), dict(zip(names, torch.autograd.grad(loss, [P[n] for n in names])))

    for k, (u, i, j) in enumerate(batches):
        before = {n: p.detach().cpu().double() for n, p in enc.named_parameters()}
        n_masks, n_drops = len(enc.drop_out.masks), len(enc.edgeDropper.outputs)
        torch.manual_seed(100 + k)
        got = float(rec.train_step(u, i, j).detach())
        torch.manual_seed(100 + k)
        adjs = []
        for layer in range(L):
            di, dv = R.drop_edge_reference(idx, vals, keep_e)
            gi, gv = enc.edgeDropper.outputs[n_drops + layer]
            assert torch.equal(di, gi) and torch.equal(dv, gv), (k, layer)
            adjs.append(R.sparse(di, dv, (N, N)))
        masks = enc.drop_out.masks[n_masks:]
        uc, ic, jc = u.cpu(), i.cpu(), j.cpu()
        l64, g64 = reference(before, torch.float64, adjs, masks, uc, ic, jc)
        l32, g32 = reference(before, torch.float32, adjs, masks, uc, ic, jc) if fp32 else (l64, None)
        assert abs(got - l64) <= R.TOL * abs(l64), (k, got, l64)
        params = dict(enc.named_parameters())
        for n, g in g64.items():
            own = R.check_rows(g32[n], g, f"step {k} ref32 d {n}", tol=1e-2) if fp32 else 0.0
            worst = max(worst, R.check_rows(params[n].grad, g, f"step {k} d {n}"))
            worst32 = max(worst32, own)
    if fp32:  # the reference's own float32 deviation, recorded beside ours
        print(f"skewed-catalogue record: worst gradient row {worst:.3e} of its scale over "
              f"{n_steps} steps x {len(g64)} tensors (1e-5 outright); the reference's torch "
              f"calls in float32: {worst32:.3e}")
    return worst


def test_hccf_steps_match_reference_ops(dev, tmp_path, monkeypatch):
    """Six teacher-forced HCCF plugin steps at 1e-5 (:func:`_teacher_forced_hccf_steps`).
    Teacher-forced per step, because Adam's normalised update turns ULP-level gradient
    differences on near-zero entries into parameter differences of order lr: free-running
    trajectories are not comparable at 1e-5, the steps' arithmetic is."""
    worst = _teacher_forced_hccf_steps(dev, tmp_path, monkeypatch, 6)
    print(f"HCCF plugin steps: worst gradient row ratio {worst:.2e}")


def test_hccf_skewed_catalogue_steps_match_reference_ops(dev, tmp_path, monkeypatch):
    """A skewed catalogue (Zipf(1.1) over 300 items: the head item is the positive of a large
    share of every batch — the fused BPR backward's list-scan path, heavy split rows in the
    item orientation) for one and a half epochs of teacher-forced plugin steps, every tensor
    held to 1e-5 outright (round 5 allowed max(1e-5, the reference's own fp32 deviation); the
    round-6 record, worst 2.8e-6, never needed it), the reference's own fp32 deviation printed
    beside (the Yelp-shaped Zipf record is scripts/diag/diag_zipf_teacher_forced.py)."""
    worst = _teacher_forced_hccf_steps(dev, tmp_path, monkeypatch, 36, zipf=1.1, fp32=True)
    print(f"HCCF plugin steps, skewed catalogue: worst gradient row ratio {worst:.2e}")


@pytest.mark.parametrize("model", ["HCCF", "HCCF_diffusion"])
def test_graph_mode_steps_equal_eager_default_steps(dev, tmp_path, monkeypatch, model):
    """hgd_graph=True — the forward + backward replayed from one HIP graph, the reference's
    torch.optim.Adam(lr=float) (HCCF.py:33) stepping eagerly after each replay — takes bit for
    bit the steps of the eager default: same batches, the same CPU drop-edge stream (drawn before
    each replay), a short last batch run eagerly in between, and parameters and losses equal
    after two epochs' worth of steps."""
    from hypergraph_diffusion_for_recommendation_amd import plugins
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    from hypergraph_diffusion_for_recommendation_amd.selfrec import FileIO
    conf, kwargs = _setup(tmp_path, monkeypatch, model)
    kwargs.pop('dataset_root')
    d = str(tmp_path / "dataset" / "toy") + "/"
    runs = []
    for graph in (False, True):
        torch.manual_seed(0)
        rec = getattr(plugins, model)(conf, FileIO.load_data_set(d + "train.txt"),
                                      FileIO.load_data_set(d + "test.txt"), None,
                                      **dict(kwargs, hgd_graph=graph))
        random.seed(4)
        losses = []
        for _ep in range(2):
            for b in next_batch_pairwise(rec.data, rec.batchSize, device=dev):
                losses.append(float(rec.graph_step(*b)))
        assert (rec._captured is not None) == graph
        runs.append((losses, [p.detach().clone() for p in rec.model.parameters()],
                     torch.get_rng_state()))
    (l0, p0, s0), (l1, p1, s1) = runs
    assert l0 == l1
    assert all(torch.equal(a, b) for a, b in zip(p0, p1))
    assert torch.equal(s0, s1)  # the CPU generator ends where the eager draws leave it


def test_hgnn_hd4_rejects_broken_modes(dev, tmp_path, monkeypatch):
    from hypergraph_diffusion_for_recommendation_amd.selfrec import SELFRec
    conf, kwargs = _setup(tmp_path, monkeypatch, "HGNN_HD4", mode="full")
    with pytest.raises(NotImplementedError):
        SELFRec(conf, kwargs).execute()


def test_dhcf_encoder_matches_dense_reference(dev, tmp_path, monkeypatch):
    """DHCF_Encoder (DHCF.py:146-185) on the sparse interaction matrix against the reference's
    dense form: per layer leaky(A·(Aᵀ·E_u)) / leaky(Aᵀ·(A·E_i)) with A = interaction_mat
    densified, concatenated; values and gradients within 1e-5 of max |ref|."""
    from hypergraph_diffusion_for_recommendation_amd.plugins import DHCF
    from hypergraph_diffusion_for_recommendation_amd.selfrec import FileIO
    conf, kwargs = _setup(tmp_path, monkeypatch, "DHCF", n_layers=3, p=0.1)
    kwargs.pop('dataset_root')
    d = str(tmp_path / "dataset" / "toy") + "/"
    rec = DHCF(conf, FileIO.load_data_set(d + "train.txt"), FileIO.load_data_set(d + "test.txt"),
               None, **kwargs)
    m = rec.model.to(dev)
    A = torch.tensor(rec.data.interaction_mat.toarray(), dtype=torch.float64)
    eu = m.embedding_dict['user_emb'].detach().cpu().double().requires_grad_(True)
    ei = m.embedding_dict['item_emb'].detach().cpu().double().requires_grad_(True)
    act = torch.nn.LeakyReLU(0.1)
    ref_u = torch.cat([eu] + [act(A @ (A.t() @ eu)) for _ in range(3)], 1)
    ref_i = torch.cat([ei] + [act(A.t() @ (A @ ei)) for _ in range(3)], 1)
    got_u, got_i = m()
    g = torch.randn(ref_u.shape, dtype=torch.float64), torch.randn(ref_i.shape, dtype=torch.float64)
    R.check_rows(got_u, ref_u, "user")
    R.check_rows(got_i, ref_i, "item")
    (ref_u * g[0]).sum().add((ref_i * g[1]).sum()).backward()
    (got_u * g[0].to(dev).float()).sum().add((got_i * g[1].to(dev).float()).sum()).backward()
    R.check_rows(m.embedding_dict['user_emb'].grad, eu.grad, "d user_emb")
    R.check_rows(m.embedding_dict['item_emb'].grad, ei.grad, "d item_emb")


def test_hd3_local_encoder_matches_reference_ops(dev, tmp_path, monkeypatch):
    """encoders.LocalAwareEncoderHD3 (fused two-hop stores) against HGNN_HD3.py:410-427 /
    :596-720 composed from torch.sparse.mm, torch LayerNorm and the module's own Linear / MLP
    weights, eval mode (dropout off), edge-dropped adjacency for the ED-HNN layers, in float64
    on the host: outputs and the embedding gradient, every row within 1e-5 of its scale."""
    import torch.nn.functional as F
    from hypergraph_diffusion_for_recommendation_amd.encoders import (LocalAwareEncoderHD3,
                                                                      sparse_tensor_of)
    from hypergraph_diffusion_for_recommendation_amd.layers import SpAdjDropEdge
    from hypergraph_diffusion_for_recommendation_amd.selfrec import FileIO, Interaction
    _setup(tmp_path, monkeypatch, "HGNN_HD3")
    d = str(tmp_path / "dataset" / "toy") + "/"
    data = Interaction(None, FileIO.load_data_set(d + "train.txt"),
                       FileIO.load_data_set(d + "test.txt"), dev)
    torch.manual_seed(4)
    enc = LocalAwareEncoderHD3(data, 32, 32, 3, 0.3, 0.2, dev).eval()
    ego = torch.randn(data.n_users + data.n_items, 32, device=dev, requires_grad=True)
    full = sparse_tensor_of(data.norm_adj, dev)
    torch.manual_seed(9)
    dropped = SpAdjDropEdge()(full, 0.8)
    A_d = dropped.detach().coalesce()
    A_f = full.detach().coalesce()

    def hgcn(A, X, slope=None):
        Y = torch.sparse.mm(A, torch.sparse.mm(A.t(), X))
        return F.leaky_relu(Y, slope) if slope is not None else Y

    def ln(m, X):
        return F.layer_norm(X, (X.shape[-1],), m.weight, m.bias, m.eps)

    def ref_forward(x):
        res = x
        for k in range(3):
            if k < 2:
                blk = enc.edhnn_layers[k]
                h = F.relu(F.linear(x, blk.lin_in.weight, blk.lin_in.bias))
                conv = blk.conv
                xe = ln(conv.lns[0], hgcn(A_d, h, 0.5)) + h
                xv = ln(conv.lns[1], hgcn(A_d, xe, 0.5)) + xe
                x = F.relu(conv.W(xv)) + res
            else:
                x = ln(enc.lns[k], hgcn(A_f, x)) + res
        return x

    got_u, got_i = enc(ego, dropped)
    got = torch.cat([got_u, got_i], 0)
    # the reference formula in float64 on the host, same parameters and adjacencies
    enc_host = copy.deepcopy(enc).cpu().double()
    A_d, A_f = A_d.cpu().double(), A_f.cpu().double()
    enc_dev, enc = enc, enc_host
    ego_r = ego.detach().cpu().double().requires_grad_(True)
    ref = ref_forward(ego_r)
    R.check_rows(got, ref, "LocalAwareEncoderHD3")
    g = torch.randn(ref.shape, dtype=torch.float64)
    (gx,) = torch.autograd.grad(got, ego, g.to(dev).float())
    (rx,) = torch.autograd.grad(ref, ego_r, g)
    R.check_rows(gx, rx, "d ego")
    del enc_dev


def _sharded_worker(rank, world, port, root, out_q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hypergraph_diffusion_for_recommendation_amd.plugins import HCCF, HCCF_sharded
        from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
        from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                         default_args)
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        os.chdir(root)
        conf = ModelConf(os.path.join(root, "HCCF.conf"))
        kw = default_args(dataset='toy', max_epoch=1, batch_size=256, embedding_size=32,
                          hyper_dim=16, n_layers=2, item_ranking='10,20', drop_rate=0.0,
                          p=0.5, temp=0.2, cl_rate=1e-2, reg=0.01, seed=7)
        d = os.path.join(root, "dataset", "toy") + "/"
        train, test = FileIO.load_data_set(d + "train.txt"), FileIO.load_data_set(d + "test.txt")
        torch.manual_seed(0)
        single = HCCF(conf, [list(r) for r in train], test, None, **kw)
        sh = HCCF_sharded(conf, train, test, None, **kw)
        sh.model.load_global(single.model.embedding_dict)
        random.seed(11)
        batches = list(next_batch_pairwise(single.data, 256, device=dev))[:3]
        worst = 0.0
        for k, (u, i, j) in enumerate(batches):
            torch.manual_seed(100 + k)
            ref = float(single.train_step(u, i, j).detach())
            torch.manual_seed(100 + k)
            got = float(sh.train_step(u, i, j).detach())
            worst = max(worst, abs(got - ref) / abs(ref))
        e_s, e_r = sh.model.embedding_dict, single.model.embedding_dict
        perr = max((e_s['user_emb'] - e_r['user_emb'][sh.u0:sh.u1]).abs().max().item(),
                   *[(e_s[n] - e_r[n]).abs().max().item() for n in ('item_emb', 'user_w',
                                                                    'item_w')])
        torch.cuda.synchronize()
        dist.barrier()
        out_q.put((rank, worst, perr))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_hccf_sharded_steps_match_single_gpu(dev, tmp_path, world):
    """HCCF_sharded (user-row shards, gloo between processes sharing cuda:0 — RCCL cannot put
    two ranks on one device) takes the same three steps as HCCF on one GPU from the same
    weights, batches and CPU drop-edge masks (nn dropout 0): batch losses within 1e-5
    relative, parameters within 1e-5 (sharded item sums are added in another order)."""
    import socket

    import torch.multiprocessing as mp
    _write_dataset(str(tmp_path / "dataset"))
    (tmp_path / "HCCF.conf").write_text(HCCF_CONF.format(model="HCCF"))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_sharded_worker, args=(world, port, str(tmp_path), q), nprocs=world,
                       join=True, start_method="spawn")
    res = sorted(q.get() for _ in range(world))
    for rank, worst, perr in res:
        assert worst <= 1e-5, (rank, worst)
        assert perr <= 1e-5, (rank, perr)


def _sharded_hd4_worker(rank, world, port, root, out_q, base="HGNN_HD4"):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hypergraph_diffusion_for_recommendation_amd.plugins import PLUGINS
        from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
        from hypergraph_diffusion_for_recommendation_amd.selfrec import (FileIO, ModelConf,
                                                                         default_args)
        dev = torch.device("cuda:0")
        torch.cuda.set_device(dev)
        os.chdir(root)
        conf = ModelConf(os.path.join(root, "HGNN_HD4.conf"))
        kw = default_args(dataset='toy', max_epoch=1, batch_size=256, embedding_size=32,
                          hyper_dim=32, input_dim=32, n_layers=3, item_ranking='10,20',
                          drop_rate=0.2, p=0.3, reg=0.1, seed=7, mode='local_only',
                          lrate=0.001, weight_decay=5e-6)
        d = os.path.join(root, "dataset", "toy") + "/"
        train, test = FileIO.load_data_set(d + "train.txt"), FileIO.load_data_set(d + "test.txt")
        single = PLUGINS[base](conf, [list(r) for r in train], test, None, **kw)
        sh = PLUGINS[base + "_sharded"](conf, train, test, None, **kw)
        with torch.no_grad():
            es, er = sh.model.embedding_dict, single.model.embedding_dict
            es['user_emb'].copy_(er['user_emb'][sh.u0:sh.u1])
            es['item_emb'].copy_(er['item_emb'])
        missing, _ = sh.model.hgnn_layer_local.load_state_dict(
            single.model.hgnn_layer_local.state_dict(), strict=False)
        assert not missing, missing
        single.model.eval()
        sh.model.eval()
        # SGD instead of the plugins' Adam for the comparison: Adam's normalised update turns
        # ULP-level differences of near-zero gradients into parameter differences of up to ~lr,
        # while SGD keeps parameter differences proportional to gradient differences (Adam is
        # elementwise, so the shards change nothing about it)
        single.optimizer = torch.optim.SGD(single.model.parameters(), lr=0.05)
        sh.optimizer = torch.optim.SGD(sh.model.parameters(), lr=0.05)
        random.seed(11)
        batches = list(next_batch_pairwise(single.data, 256, device=dev))[:3]
        worst = 0.0
        for k, (u, i, j) in enumerate(batches):
            torch.manual_seed(100 + k)
            ue, ie = single.model(mode='local', keep_rate=1 - single.drop_rate)
            loss = single.model.calculate_cf_loss(ue[u], ie[i], ie[j], single.reg)
            single.optimizer.zero_grad()
            loss.backward()
            single.optimizer.step()
            torch.manual_seed(100 + k)
            got = float(sh.train_step(u, i, j).detach())
            worst = max(worst, abs(got - float(loss)) / abs(float(loss)))
        es, er = sh.model.embedding_dict, single.model.embedding_dict
        perr = max((es['user_emb'] - er['user_emb'][sh.u0:sh.u1]).abs().max().item(),
                   (es['item_emb'] - er['item_emb']).abs().max().item())
        rp = dict(single.model.hgnn_layer_local.named_parameters())
        for name, p in sh.model.hgnn_layer_local.named_parameters():
            perr = max(perr, (p - rp[name]).abs().max().item())
        torch.cuda.synchronize()
        dist.barrier()
        out_q.put((rank, worst, perr))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,base", [(2, "HGNN_HD4"), (3, "HGNN_HD4"), (2, "HGNN_HD3")])
def test_hgnn_hd4_sharded_steps_match_single_gpu(dev, tmp_path, world, base):
    """HGNN_HD4_sharded / HGNN_HD3_sharded (the ED-HNN models on user-row shards; gloo between
    processes sharing cuda:0) take the same three steps as HGNN_HD4 / HGNN_HD3 on one GPU from
    the same weights and batches with the same CPU drop-edge masks, eval mode (dropout off):
    batch losses within 1e-5 relative, embeddings and every encoder weight within 1e-5 after
    three SGD steps (see the worker for why SGD)."""
    import socket

    import torch.multiprocessing as mp
    _write_dataset(str(tmp_path / "dataset"))
    (tmp_path / "HGNN_HD4.conf").write_text(HCCF_CONF.format(model="HGNN_HD4"))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_sharded_hd4_worker, args=(world, port, str(tmp_path), q, base),
                       nprocs=world,
                       join=True, start_method="spawn")
    for rank, worst, perr in sorted(q.get() for _ in range(world)):
        assert worst <= 1e-5, (rank, worst)
        assert perr <= 1e-5, (rank, perr)


def _sharded_execute_worker(rank, world, port, root, model, out_q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from hypergraph_diffusion_for_recommendation_amd.selfrec import (ModelConf, SELFRec,
                                                                         default_args)
        torch.cuda.set_device(0)
        os.chdir(root)
        conf = ModelConf(os.path.join(root, f"{model}.conf"))
        kw = default_args(dataset='toy', max_epoch=2, batch_size=512, embedding_size=32,
                          hyper_dim=32, input_dim=32, n_layers=2, item_ranking='10,20',
                          drop_rate=0.2, p=0.3, temp=0.2, cl_rate=1e-3, reg=0.01, seed=7,
                          mode='local_only')
        kw['dataset_root'] = os.path.join(root, "dataset")
        # different host seeds per rank: the plugin itself must give every rank the same
        # batches (rank 0's random state is broadcast; _check_batch raises otherwise)
        random.seed(3 + rank)
        torch.manual_seed(3 + rank)
        rec = SELFRec(conf, kw).execute()
        out_q.put((rank, rec.result, os.path.exists(rec.output + f"/{model}-performance.txt")))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("model", ["HCCF_sharded", "HGNN_HD4_sharded",
                                   "HGNN_HD3_sharded"])
def test_sharded_plugins_execute(dev, tmp_path, model):
    """SELFRec(conf, kwargs).execute() of a sharded plugin at 2 ranks: both ranks end with the
    same measures (their evaluation all-reduces the user table), rank 0 writes the files."""
    import socket

    import torch.multiprocessing as mp
    _write_dataset(str(tmp_path / "dataset"))
    (tmp_path / f"{model}.conf").write_text(HCCF_CONF.format(model=model))
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    q = mp.get_context("spawn").Queue()
    mp.start_processes(_sharded_execute_worker, args=(2, port, str(tmp_path), model, q),
                       nprocs=2, join=True, start_method="spawn")
    res = sorted(q.get() for _ in range(2))
    assert res[0][1] == res[1][1] and len(res[0][1]) == 10
    assert res[0][2]
