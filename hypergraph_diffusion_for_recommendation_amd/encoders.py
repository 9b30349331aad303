"""Encoders of the hot-path carriers, rebuilt on the drop-in layers (the callers of the path).

They keep the reference's constructor arguments (the argparse ``kwargs`` dict and the
``Interaction`` data object with ``n_users``, ``n_items``, ``norm_adj``, ``ui_adj``), parameter
names (so ``state_dict``s load either way) and forward outputs, so a plugin can swap the whole
encoder (paths relative to /root/reference/HD_SELFRec):

* :class:`HCCFEncoder`       model/graph/HCCF.py:136-191
* :class:`LocalAwareEncoder` model/graph/HGNN_HD4.py:336-405 (``--mode=local_only``)
* :class:`LocalAwareEncoderHD3` model/graph/HGNN_HD3.py:352-427 (the SpMM-form ED-HNN blocks)
* :class:`HCCFDiffusionEncoder` model/graph/HCCF_diffusion.py:131-215
* :class:`SelfAwareEncoder`  model/graph/HGNN_cp.py:368-411, KHGRec.py:374-417 (the KG
  carriers' CF side)
* :class:`RelationalAwareEncoder` model/graph/HGNN_cp.py:413-446 (their KG side)
* :class:`SelfAwareEncoderHD` model/graph/HD.py:398-487 (ED-HNN blocks on the norm_adj pattern)

Everything sparse runs on libhgd, with the LayerNorm / residual after a hop fused into its store;
HCCF's dense ``E·W`` and learned-hypergraph products run on the skinny MFMA kernels; dropout
stays torch.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn

from .functional import (dense_two_hop_pair, fan, hccf_layers, hccf_layers_supported,
                         hyper_dropouts, split_rows, sum_n, table_projections,
                         two_hop_fused)
from .incidence import Incidence, incidence_of
from .layers import EquivSetGNN, GCNLayer, HGCNConv, HGNNLayer, LayerNorm, SpAdjDropEdge


def sparse_tensor_of(mat, device) -> torch.Tensor:
    """TorchGraphInterface.convert_sparse_mat_to_tensor (base/torch_interface.py:8-12) on the
    device, with its Incidence built once and cached on the tensor."""
    coo = mat.tocoo()
    i = torch.from_numpy(np.stack([coo.row, coo.col]).astype(np.int64))
    v = torch.from_numpy(coo.data.astype(np.float32))
    t = torch.sparse_coo_tensor(i, v, coo.shape).to(device)
    t._hgd_incidence = Incidence.from_coo(t._indices(), t._values(), coo.shape, device=device)
    return t


def _begin_step(dropper) -> None:
    """A step boundary for SpAdjDropEdge's per-call mask slots (a wrapped or foreign dropper
    without them is left alone)."""
    begin = getattr(dropper, "begin_step", None)
    if begin is not None:
        begin()


class HCCFEncoder(nn.Module):
    """HCCF propagation: per layer a GCN hop on the (edge-dropped) normalised bipartite graph plus
    the dense learned-hypergraph hop for users and items; outputs the layer sum and the per-layer
    GCN / hypergraph embeddings for the InfoNCE terms (HCCF.py:173-191)."""

    def __init__(self, conf, data, device=None):
        super().__init__()
        self.data = data
        self._parse_config(conf)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.gcnlayer = GCNLayer(self.leaky)
        self.hgnnlayer = HGNNLayer(self.leaky)
        self.norm_adj = data.norm_adj
        self.sparse_norm_adj = sparse_tensor_of(self.norm_adj, self.device)
        self.embedding_dict = self._init_model()
        self.drop_out = nn.Dropout(self.drop_rate)
        self.edgeDropper = SpAdjDropEdge()
        # False: the per-layer module graph below (GCNLayer / dense_two_hop_pair and torch adds)
        self.fused_layers = True
        # False: one nn.Dropout node per layer and table (bitwise the same results)
        self.fused_dropouts = True

    def _parse_config(self, config):
        self.lRate = float(config['lrate'])
        self.lr_decay = float(config['lr_decay'])
        self.maxEpoch = int(config['max_epoch'])
        self.batchSize = int(config['batch_size'])
        self.reg = float(config['reg'])
        self.latent_size = int(config['embedding_size'])
        self.hyperDim = int(config['hyper_dim'])
        self.drop_rate = float(config['drop_rate'])
        self.leaky = float(config['p'])
        self.n_layers = int(config['n_layers'])
        self.n_edges = int(config['hyper_dim'])

    def _init_model(self):
        init = nn.init.xavier_uniform_
        dev = self.device
        return nn.ParameterDict({
            'user_emb': nn.Parameter(init(torch.empty(self.data.n_users, self.latent_size)).to(dev)),
            'item_emb': nn.Parameter(init(torch.empty(self.data.n_items, self.latent_size)).to(dev)),
            'user_w': nn.Parameter(init(torch.empty(self.latent_size, self.n_edges)).to(dev)),
            'item_w': nn.Parameter(init(torch.empty(self.latent_size, self.n_edges)).to(dev)),
        })

    def forward(self, keep_rate=0.5):
        nu = self.data.n_users
        _begin_step(self.edgeDropper)
        # E·W [n, d]·[d, K] for both tables as one grouped op (functional.table_projections:
        # W read in its own layout, the gradients in grouped launches)
        hyper_uu, hyper_ii = table_projections(
            [self.embedding_dict['user_emb'], self.embedding_dict['item_emb']],
            [self.embedding_dict['user_w'], self.embedding_dict['item_w']])
        if self.fused_layers and hccf_layers_supported(self.embedding_dict['user_emb'],
                                                       self.embedding_dict['item_emb'], hyper_uu):
            # the whole loop as one op (functional.hccf_layers): the layer sum, the layer adds
            # and autograd's accumulations ride in the hop / product stores. Same draws in the
            # same order as the loop below (drop-edge, then the two dropouts, per layer).
            # (the drop-edge draws use the CPU generator, the dropouts the device's: drawing
            # the layers' drop-edges first leaves both streams as the reference's loop does)
            adjs = [incidence_of(self.edgeDropper(self.sparse_norm_adj, keep_rate))
                    for _ in range(self.n_layers)]
            if (self.fused_dropouts and type(self.drop_out) is nn.Dropout
                    and self.drop_out.training and not self.drop_out.inplace):
                # the 2L dropouts as one autograd node (functional.hyper_dropouts: the same
                # masks, the backward summed in one launch in autograd's order); a module put in
                # drop_out's place is called as it is
                drops = hyper_dropouts([hyper_uu, hyper_ii], self.drop_out.p, self.n_layers)
                hus, his = [d[0] for d in drops], [d[1] for d in drops]
            else:
                hus, his = [], []
                for _ in range(self.n_layers):
                    hus.append(self.drop_out(hyper_uu))
                    his.append(self.drop_out(hyper_ii))
            embeddings, gcn_hidden, hgnn_hidden = hccf_layers(
                adjs, self.embedding_dict['user_emb'], self.embedding_dict['item_emb'], hus, his)
            user_emb, item_emb = torch.split(embeddings, [nu, embeddings.shape[0] - nu])
            return user_emb, item_emb, gcn_hidden, hgnn_hidden
        embeddings = torch.cat([self.embedding_dict['user_emb'], self.embedding_dict['item_emb']], 0)
        hidden = [embeddings]
        gcn_hidden, hgnn_hidden = [], []
        for _ in range(self.n_layers):
            gcn_emb = self.gcnlayer(self.edgeDropper(self.sparse_norm_adj, keep_rate), hidden[-1])
            # the user and item HGNNLayer calls (hgnnlayer(·, hidden[-1][:nu]) and [nu:]) and
            # their cat as one pair op: grouped launches over both halves, the output and the
            # table gradient written in place (no split / cat forward or backward)
            gcn_hidden += [gcn_emb]
            hgnn_hidden += [dense_two_hop_pair(self.drop_out(hyper_uu), self.drop_out(hyper_ii),
                                               hidden[-1], nu)]
            hidden += [gcn_emb + hgnn_hidden[-1]]
        embeddings = sum(hidden)
        user_emb, item_emb = torch.split(embeddings, [nu, embeddings.shape[0] - nu])
        return user_emb, item_emb, gcn_hidden, hgnn_hidden


def edhnn_config(hyper_size):
    """LocalAwareEncoder.init_edhnn_config (HGNN_HD4.py:371-388)."""
    return {
        'MLP_hidden': hyper_size, 'MLP1_num_layers': 0, 'MLP2_num_layers': 0,
        'MLP3_num_layers': 1, 'MLP_num_layers': 0, 'restart_alpha': 0.0, 'aggregate': 'mean',
        'dropout': 0.5, 'normalization': 'ln', 'input_norm': True, 'All_num_layers': 1,
        'activation': 'relu', 'input_dropout': 0.6, 'AllSet_input_norm': True,
    }


class LocalAwareEncoder(nn.Module):
    """HGNN_HD4's local encoder: layers 0..L-2 are ED-HNN blocks on V/E = nonzero(ui_adj > 0),
    the last is LayerNorm(HGCNConv(Â, ·, act=False)); every layer adds the layer-0 residual
    (HGNN_HD4.py:390-405).

    The reference densifies ``ui_adj`` on the CPU (``torch.tensor(ui_adj.todense())``,
    HGNN_HD4.py:367-369: 83 GB at Amazon-Book) and scans it twice per block per step; here the
    same V/E (row-major nonzero order) come from the sparse matrix, once.
    """

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, device=None,
                 use_self_att=False):
        super().__init__()
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.norm_adj = data.norm_adj
        self.ui_adj = data.ui_adj
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.relu = nn.ReLU()
        self.act = nn.LeakyReLU(leaky)
        self.dropout = nn.Dropout(drop_rate)
        self.edgeDropper = SpAdjDropEdge()
        self.sparse_norm_adj = sparse_tensor_of(data.norm_adj, self.device)
        self.edhnn_args = edhnn_config(self.hyper_size)
        self.hgcn_layers = nn.ModuleList([HGCNConv(leaky=0.5) for _ in range(self.layers)])
        self.edhnn_layers = nn.ModuleList(
            [EquivSetGNN(hyper_size, self.edhnn_args, None, data) for _ in range(self.layers)])
        self.lns = nn.ModuleList([LayerNorm(hyper_size) for _ in range(self.layers)])
        self.edhnn_ui_n = data.n_items + data.n_users
        ui = data.ui_adj.tocsr().copy()
        ui.sort_indices()  # nonzero(dense > 0) order: rows, then ascending columns
        ui.eliminate_zeros()
        self.hypergraph = sparse_tensor_of(ui, self.device)
        self.to(self.device)  # the reference moves it with HGNNModel.to(device)

    def forward(self, ego_embeddings, sparse_norm_adj):
        # res is read by every layer (and is layer 0's input): its gradients meet in one n-ary
        # sum (functional.fan) instead of a chain of full-table accumulations
        uses = fan(ego_embeddings, self.layers + 1)
        res = uses[1:]
        ego_embeddings = uses[0]
        all_embeddings = []
        for k in range(self.layers):
            if k != self.layers - 1:
                # the "+ res" rides in the block's last Linear store when its fused path runs
                ego_embeddings = self.edhnn_layers[k](ego_embeddings, self.hypergraph,
                                                      self.edhnn_ui_n, residual=res[k])
            else:
                # LN0(HGCNConv(Â, x, act=False)) + res in one fused hop store
                ego_embeddings = two_hop_fused(incidence_of(sparse_norm_adj), ego_embeddings,
                                               norm=self.lns[0], res1=res[k], res1_scale=1.0)
            all_embeddings += [ego_embeddings]
        nu = self.data.n_users
        return split_rows(all_embeddings[-1], nu)


class HCCFDiffusionEncoder(HCCFEncoder):
    """HCCF_diffusion's encoder (model/graph/HCCF_diffusion.py:131-215): HCCF with the learned
    hypergraph hop replaced by one shared ED-HNN block (EquivSetGNN, mean aggregation) run on the
    dense learned hypergraph dropout(E·W) [n, K] of users and of items — the repo's "hypergraph
    diffusion". The V/E of that hypergraph (nonzero(H > 0)) change every call; they are taken on
    the device (hgd_dense_threshold_*) and the two scatter-means run as one fused two-hop.
    ``edhnn_user_n`` / ``edhnn_item_n`` (n + K) are the reference's E offsets, which do not
    change the result (the extra hyperedge slots are empty)."""

    def __init__(self, conf, data, device=None):
        super().__init__(conf, data, device)
        self.edhnn_user_n = self.data.n_users + self.n_edges
        self.edhnn_item_n = self.data.n_items + self.n_edges
        self.edhnn_args = dict(edhnn_config(self.latent_size))
        self.edhnnlayer = EquivSetGNN(self.latent_size, self.edhnn_args).to(self.device)
        del self.hgnnlayer

    def forward(self, keep_rate=0.5):
        nu = self.data.n_users
        _begin_step(self.edgeDropper)
        e = self.embedding_dict
        hidden = [torch.cat([e['user_emb'], e['item_emb']], 0)]
        gcn_hidden, hgnn_hidden = [], []
        hyper_uu, hyper_ii = table_projections([e['user_emb'], e['item_emb']],
                                               [e['user_w'], e['item_w']])
        blk = self.edhnnlayer
        terms = []  # the sum(hidden) operands
        for _ in range(self.n_layers):
            # hidden[-1] feeds the GCN hop, the block and the layer sum: its three gradients
            # meet in one n-ary pass (functional.fan)
            h_gcn, h_blk, h_sum = fan(hidden[-1], 3)
            terms.append(h_sum)
            gcn_emb = self.gcnlayer(self.edgeDropper(self.sparse_norm_adj, keep_rate), h_gcn)
            hu = self.drop_out(hyper_uu)
            if blk.dense_pair_ok(h_blk, hu, hyper_ii):
                # the user and the item call of the block as one pass over all rows
                # (EquivSetGNN.forward_dense_pair: grouped mean two-hops, no cat)
                hyp = blk.forward_dense_pair(h_blk, hu, self.drop_out(hyper_ii))
            else:
                hyper_uemb = blk(h_blk[:nu], hu, self.edhnn_user_n)
                hyper_iemb = blk(h_blk[nu:], self.drop_out(hyper_ii), self.edhnn_item_n)
                hyp = torch.cat([hyper_uemb, hyper_iemb], 0)
            gcn_hidden += [gcn_emb]
            hgnn_hidden += [hyp]
            hidden += [gcn_emb + hyp]
        emb = sum_n(terms + [hidden[-1]])  # sum(hidden), same order, one pass
        return (*split_rows(emb, nu), gcn_hidden, hgnn_hidden)


class LocalAwareEncoderHD3(nn.Module):
    """HGNN_HD3's local encoder (HGNN_HD3.py:352-427): layers 0..L-2 are the SpMM form of the
    ED-HNN block (``edhnn_spmm.EquivSetGNN``, both aggregations HGCNConv(0.5) two-hops over the
    edge-dropped ``norm_adj``, HGNN_HD3.py:555-720) plus the layer-0 residual; the last layer is
    ``lns[L-1](HGCNConv(Â, ·, act=False)) + res`` on the UN-dropped ``norm_adj`` (the reference
    uses ``self.sparse_norm_adj`` there), fused into one hop store. The dense ``ui_adj`` copies
    the reference builds for its group encoder (``hyper_uu`` / ``hyper_ii``, :386-387) are
    unused by this encoder and not built."""

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, device=None):
        super().__init__()
        from .edhnn_spmm import EquivSetGNN as EquivSetGNNSpMM
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.relu = nn.ReLU()
        self.act = nn.LeakyReLU(leaky)
        self.dropout = nn.Dropout(drop_rate)
        self.edgeDropper = SpAdjDropEdge()
        self.sparse_norm_adj = sparse_tensor_of(data.norm_adj, self.device)
        self.edhnn_args = edhnn_config(self.hyper_size)
        self.hgcn_layer = HGCNConv(leaky=0.3)
        self.hgnn_layers = nn.ModuleList([HGCNConv(leaky=0.3) for _ in range(self.layers)])
        self.edhnn_layers = nn.ModuleList([
            EquivSetGNNSpMM(hyper_size, self.edhnn_args, None, data, data.n_users, data.n_items,
                            leaky=0.5) for _ in range(self.layers)])
        self.lns = nn.ModuleList([LayerNorm(hyper_size) for _ in range(self.layers)])
        self.edhnn_ui_n = data.n_users + data.n_items
        self.to(self.device)

    def forward(self, ego_embeddings, sparse_norm_adj):
        uses = fan(ego_embeddings, self.layers + 1)  # one n-ary gradient sum of the residual
        ego_embeddings, res = uses[0], uses[1:]
        for k in range(self.layers):
            if k != self.layers - 1:
                ego_embeddings = self.edhnn_layers[k](ego_embeddings, sparse_norm_adj,
                                                      self.edhnn_ui_n) + res[k]
            else:
                ego_embeddings = two_hop_fused(incidence_of(self.sparse_norm_adj), ego_embeddings,
                                               norm=self.lns[k], res1=res[k], res1_scale=1.0)
        nu = self.data.n_users
        return split_rows(ego_embeddings, nu)


def ugformer_layers(hyper_size, n_layers, drop_rate, device=None) -> nn.ModuleList:
    """The per-layer UGformer blocks of the KG carriers' SelfAwareEncoder (HGNN_cp.py:387-392,
    HD.py:453-459): ``TransformerEncoder(TransformerEncoderLayer(d, nhead=1, ff=32), 1,
    norm=LayerNorm(d))`` over all nodes as one sequence. Self-attention over n nodes is the
    library's dense O(n²) attention, not a hop of the path; it runs only with ``use_self_att``."""
    return nn.ModuleList([
        nn.TransformerEncoder(nn.TransformerEncoderLayer(d_model=hyper_size, nhead=1,
                                                         dim_feedforward=32, dropout=drop_rate),
                              1, norm=nn.LayerNorm(hyper_size), enable_nested_tensor=False)
        .to(device) for _ in range(n_layers)])


def _self_attend(block, x):
    # [seq = n nodes, batch = 1, d], the reference's unsqueeze / squeeze (HGNN_cp.py:400-402)
    return block(x.unsqueeze(1)).squeeze(1)


def _hgcn_ln_res_stack(inc, x, lns, slope, res, attend=None):
    """``lns[k](HGCNConv(A, x)) + res`` per layer, no activation on the last (HGNN_cp.py:403-406,
    :428-433): one fused two-hop per layer whose store applies the LeakyReLU, the LayerNorm
    and the residual; ``attend[k]`` (the UGformer blocks) first when given."""
    L = len(lns)
    # every layer reads res (and layer 0 reads x, the same table at the call sites): one n-ary
    # gradient pass instead of a chain of full-table accumulations (functional.fan)
    if res is x:
        uses = fan(x, L + 1)
        x, ress = uses[0], uses[1:]
    else:
        ress = fan(res, L)
    for k in range(L):
        if attend is not None:
            x = _self_attend(attend[k], x)
        x = two_hop_fused(inc, x, epilogue=None if k == L - 1 else "leaky_relu", slope=slope,
                          norm=lns[k], res1=ress[k], res1_scale=1.0)
    return x


class SelfAwareEncoder(nn.Module):
    """The CF encoder of the KG carriers HGNN_cp / KHGRec (HGNN_cp.py:368-411, KHGRec.py:374-
    417): per layer ``lns[k](HGCNConv(Â, x)) + res`` with HGCNConv = LeakyReLU(Â·Âᵀ·x) (no
    activation on the last layer) over the edge-dropped ``norm_adj`` the model passes in.
    ``use_self_att`` (HGNN_cp's default True; KHGRec forces False) runs the UGformer block
    before each layer's hop."""

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, device=None,
                 use_self_att=True):
        super().__init__()
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.norm_adj = data.norm_adj
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.relu = nn.ReLU()
        self.leaky = float(leaky)
        self.act = nn.LeakyReLU(leaky)
        self.dropout = nn.Dropout(drop_rate)
        self.edgeDropper = SpAdjDropEdge()
        self.use_self_att = use_self_att
        self.hgnn_layers = nn.ModuleList()
        self.ugformer_layers = nn.ModuleList()
        self.lns = nn.ModuleList()
        for _ in range(n_layers):  # the reference's construction (and init) order
            self.ugformer_layers.extend(ugformer_layers(hyper_size, 1, drop_rate))
            self.hgnn_layers.append(HGCNConv(leaky=leaky))
            self.lns.append(LayerNorm(hyper_size))
        self.to(self.device)

    def forward(self, ego_embeddings, sparse_norm_adj):
        inc = incidence_of(sparse_norm_adj)
        attend = self.ugformer_layers if self.use_self_att else None
        ego_embeddings = _hgcn_ln_res_stack(inc, ego_embeddings, list(self.lns), self.leaky,
                                            ego_embeddings, attend)
        nu = self.data.n_users
        return split_rows(ego_embeddings, nu)


class RelationalAwareEncoder(nn.Module):
    """HGNN_cp's KG encoder (HGNN_cp.py:413-446): the same ``lns[i](HGCNConv(A, x)) + res``
    stack over the (edge-dropped) KG adjacency; its AttHGCNConv ignores ``att_adj`` (``adj =
    inp_adj``, :440-446), as here. (KHGRec's variant multiplies ``att_adj·inp_adj`` first,
    KHGRec.py:445-449 — a KG-attention SpGEMM outside the path.)"""

    def __init__(self, leaky, dropout, n_layers, hyper_dim):
        super().__init__()
        self.leaky = leaky
        self.dropout = dropout
        self.n_layers = n_layers
        self.act = nn.LeakyReLU(self.leaky)
        self.convs = nn.ModuleList()
        self.lns = nn.ModuleList()
        for _ in range(n_layers):
            self.convs.append(HGCNConv(leaky=leaky))
            self.lns.append(LayerNorm(hyper_dim))

    def forward(self, embs, sparse_adj, att_adj=None):
        return _hgcn_ln_res_stack(incidence_of(sparse_adj), embs, list(self.lns),
                                  float(self.leaky), embs)


class SelfAwareEncoderHD(nn.Module):
    """HD's CF encoder (HD.py:398-487): two ED-HNN blocks (layers2 EquivSetGNN, mean
    aggregation, edhnn_config) on V/E = nonzero(norm_adj > 0) of the UN-dropped ``norm_adj`` —
    ``edhnn_layers[0]`` for layers 0..L-2, ``edhnn_layers[1]`` for the last, each plus the layer-0
    residual; the ``sparse_norm_adj`` argument of ``forward`` is ignored, as in the reference.
    Each block's aggregation is one fused mean two-hop over the adjacency pattern.
    ``use_self_att`` (default False) runs the UGformer block first. The dense ``ui_adj`` copies
    the reference builds (``hyper_uu`` / ``hyper_ii`` / ``dense_hypergraph``, :447-450) are never
    read by its forward and are not built."""

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, device=None,
                 use_self_att=False):
        super().__init__()
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.norm_adj = data.norm_adj
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.relu = nn.ReLU()
        self.act = nn.LeakyReLU(leaky)
        self.dropout = nn.Dropout(drop_rate)
        self.edgeDropper = SpAdjDropEdge()
        self.drop_out = nn.Dropout(drop_rate)
        self.sparse_norm_adj = sparse_tensor_of(data.norm_adj, self.device)
        self.use_self_att = use_self_att
        self.edhnn_args = edhnn_config(hyper_size)
        self.edhnn_layers = nn.ModuleList([
            EquivSetGNN(hyper_size, self.edhnn_args, None, data) for _ in range(2)])
        self.ugformer_layers = nn.ModuleList()
        self.lns = nn.ModuleList()
        for _ in range(n_layers):
            self.ugformer_layers.extend(ugformer_layers(hyper_size, 1, drop_rate))
            self.lns.append(nn.LayerNorm(hyper_size))
        self.edhnn_user_n = data.n_users
        self.edhnn_item_n = data.n_items
        self.edhnn_ui_n = data.n_items + data.n_users
        self.to(self.device)

    def forward(self, ego_embeddings, sparse_norm_adj=None):
        uses = fan(ego_embeddings, self.layers + 1)  # one n-ary gradient sum of the residual
        ego_embeddings, res = uses[0], uses[1:]
        for k in range(self.layers):
            if self.use_self_att:
                ego_embeddings = _self_attend(self.ugformer_layers[k], ego_embeddings)
            blk = self.edhnn_layers[0 if k != self.layers - 1 else 1]
            ego_embeddings = blk(ego_embeddings, self.sparse_norm_adj, self.edhnn_ui_n) + res[k]
        nu = self.data.n_users
        return split_rows(ego_embeddings, nu)
