"""The hot-path carriers on user-row shards (BASELINE configs[3]: hypergraph
diffusion, user-row sharded on the GPUs of one node). Paths relative to
/root/reference/HD_SELFRec.

Rank g owns users [u0, u1): their embedding rows, their rows of the bipartite graphs (and the
item rows' entries in their columns, :class:`~.sharded.ShardedBipartite`) and their rows of the
learned user hypergraph. Items, the item hypergraph and every weight matrix are replicated.
The local node layout is ``[users u0..u1-1; all items]`` — the reference's ``[users; items]``
restricted to this rank's users. Exchanges (RCCL over xGMI with backend "nccl"):

* every bipartite hop: one all-reduce of the item rows forward, one backward (chunked, overlapped
  with the local user hop / the item partial);
* HCCF's learned user hypergraph: one [K, d] all-reduce forward and one backward.

Replicated tensors follow :mod:`.sharded`'s convention (same value on every rank, per-rank
partial gradients): call :func:`~.sharded.allreduce_replicated_grads` on the replicated
parameters (:meth:`replicated_parameters`) before the optimizer step. Dropout on replicated rows
draws from a generator seeded identically on every rank (``seed``), so the replicas stay equal;
dropout on a rank's own user rows draws from a per-rank generator, so the users of different ranks
get independent masks (:class:`_SplitDropout`).
"""
from __future__ import annotations

from typing import Iterator, Optional

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .encoders import edhnn_config
from .functional import dense_two_hop, fan, hccf_layers_supported, linear, sum_n
from .layers import EquivSetGNN, LayerNorm, input_norm_linear
from .sharded import (ShardedBipartite, bipartite_hop, bipartite_hop_fused,  # noqa: F401
                      shard_bounds, sharded_dense_two_hop, sharded_hccf_layers,
                      sharded_mean_two_hop)


def _coo_tensor(mat, binary: bool = False):
    """(indices int64 [2, nnz], values fp32 or None) of a scipy matrix. Weighted: ``tocoo()``
    order, exactly as ``convert_sparse_mat_to_tensor`` (base/torch_interface.py:8-12) — the
    order the reference's drop-edge mask indexes. Binary: the V/E order of
    ``nonzero(ui_adj > 0)`` (sorted rows, ascending columns, zeros dropped; HGNN_HD4.py:367-369)."""
    if binary:
        csr = mat.tocsr().copy()
        csr.sort_indices()
        csr.eliminate_zeros()
        coo = csr.tocoo()
    else:
        coo = mat.tocoo()
    idx = torch.from_numpy(np.stack([coo.row, coo.col]).astype(np.int64))
    val = None if binary else torch.from_numpy(coo.data.astype(np.float32))
    return idx, val


class _SplitDropout(nn.Module):
    """nn.Dropout over the local layout: rows before ``start`` are this rank's own (local users),
    rows from ``start`` on are replicated (items). Local rows draw from ``local_gen``, seeded per
    rank, so users on different ranks get independent masks (one i.i.d. mask over all users, as
    the reference's single nn.Dropout); replicated rows draw from ``gen``, identical on every rank,
    so the replicas stay equal. ``start`` = rows.shape[0] drops every row as local."""

    def __init__(self, p: float, gen: torch.Generator, local_gen: torch.Generator):
        super().__init__()
        self.p, self.gen, self.local_gen = float(p), gen, local_gen

    def forward(self, x: torch.Tensor, start: int) -> torch.Tensor:
        if not self.training or self.p == 0.0:
            return x
        if self.p == 1.0:
            return torch.zeros_like(x)
        if not torch.distributed.is_initialized() or torch.distributed.get_world_size() == 1:
            return F.dropout(x, self.p, True)  # one rank: no replicas to keep equal
        q = 1.0 - self.p
        # one mask tensor drawn in two parts, pre-scaled by 1/q: a single product with x (and
        # one in the backward), no per-part products and concatenation
        mask = torch.empty_like(x)
        mask[:start].bernoulli_(q, generator=self.local_gen)
        mask[start:].bernoulli_(q, generator=self.gen)
        return x * mask.mul_(1.0 / q)


def _rank_generators(device, seed: int, group):
    """(replicated, local) dropout generators: the first seeded identically on every rank, the
    second per rank."""
    rank = torch.distributed.get_rank(group) if torch.distributed.is_initialized() else 0
    rep = torch.Generator(device=device).manual_seed(int(seed))
    loc = torch.Generator(device=device).manual_seed(int(seed) * 65537 + 1 + rank)
    return rep, loc


class ShardedHCCFEncoder(nn.Module):
    """HCCFEncoder (HCCF.py:136-191) on user-row shards, same parameter names: ``user_emb``
    holds this rank's rows. Per layer: the edge-dropped GCN hop (:func:`bipartite_hop` on the
    dropped shard), the user hypergraph hop over the split users (:func:`sharded_dense_two_hop`)
    and the replicated item hypergraph hop (:func:`dense_two_hop`).

    ``device_rng=False`` draws the reference's global CPU ``torch.rand(nnz)`` mask per layer (the
    same bits as the single-GPU encoder for a seed; every rank draws it); ``True`` draws each
    rank's blocks on the device (independent Bernoulli per nonzero, as the reference's)."""

    def __init__(self, conf, data, u0: int, u1: int, group=None, device=None, n_chunks: int = 4,
                 device_rng: bool = True, seed: int = 0):
        super().__init__()
        from .encoders import HCCFEncoder
        HCCFEncoder._parse_config(self, conf)
        self.data = data
        self.u0, self.u1, self.n_local = int(u0), int(u1), int(u1) - int(u0)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.group = group
        self.device_rng = device_rng
        U, I = data.n_users, data.n_items
        self.adj = ShardedBipartite.from_global(_coo_tensor(data.norm_adj), U, I, u0, u1,
                                                device=self.device, group=group,
                                                n_chunks=n_chunks)
        self.nnz_global = int(data.norm_adj.nnz)
        d, K = self.latent_size, self.n_edges
        bu = (6.0 / (U + d)) ** 0.5  # xavier_uniform_ bound of the GLOBAL [U, d] table
        self.embedding_dict = nn.ParameterDict({
            'user_emb': nn.Parameter(torch.empty(self.n_local, d, device=self.device)
                                     .uniform_(-bu, bu)),
            'item_emb': nn.Parameter(nn.init.xavier_uniform_(torch.empty(I, d)).to(self.device)),
            'user_w': nn.Parameter(nn.init.xavier_uniform_(torch.empty(d, K)).to(self.device)),
            'item_w': nn.Parameter(nn.init.xavier_uniform_(torch.empty(d, K)).to(self.device)),
        })
        self.rep_gen, self.loc_gen = _rank_generators(self.device, seed, group)
        self.rep_drop = _SplitDropout(self.drop_rate, self.rep_gen, self.loc_gen)
        # False: the per-layer module graph (bipartite hops, dense two-hops, torch adds)
        self.fused_layers = True

    @torch.no_grad()
    def load_global(self, embedding_dict) -> None:
        """Takes this rank's slice of a single-GPU HCCFEncoder's parameters."""
        e = self.embedding_dict
        e['user_emb'].copy_(embedding_dict['user_emb'][self.u0:self.u1])
        for k in ('item_emb', 'user_w', 'item_w'):
            e[k].copy_(embedding_dict[k])

    def replicated_parameters(self) -> Iterator[nn.Parameter]:
        e = self.embedding_dict
        return iter([e['item_emb'], e['user_w'], e['item_w']])

    def _dropped(self, keep_rate: float) -> ShardedBipartite:
        if keep_rate == 1.0:
            return self.adj
        if self.device_rng:
            seed = int(torch.randint(0, 2 ** 40, (1,)).item())  # same draw on every rank
            rank = torch.distributed.get_rank(self.group) if self.adj.world > 1 else 0
            return self.adj.drop_device(keep_rate, seed * 4096 + rank)
        from .layers import torch_cpu_keep_mask  # the reference's torch.rand stream, natively
        mask, _ = torch_cpu_keep_mask(self.nnz_global, keep_rate)
        return self.adj.drop_global(keep_rate, mask.bool())

    def forward(self, keep_rate=0.5):
        nl = self.n_local
        e = self.embedding_dict
        hyper_uu = linear(e['user_emb'], e['user_w'].t())
        hyper_ii = linear(e['item_emb'], e['item_w'].t())
        if self.fused_layers and hccf_layers_supported(e['user_emb'], e['item_emb'], hyper_ii):
            # the whole loop as one op (sharded.sharded_hccf_layers, the counterpart of the
            # single-GPU encoder's hccf_layers); same draws in the same order as the loop below
            shs, hus, his = [], [], []
            for _ in range(self.n_layers):
                shs.append(self._dropped(keep_rate))
                hus.append(self.rep_drop(hyper_uu, nl))
                his.append(self.rep_drop(hyper_ii, 0))
            embeddings, gcn_hidden, hgnn_hidden = sharded_hccf_layers(
                shs, e['user_emb'], e['item_emb'], hus, his, self.group)
            return embeddings[:nl], embeddings[nl:], gcn_hidden, hgnn_hidden
        embeddings = torch.cat([e['user_emb'], e['item_emb']], 0)
        hidden = [embeddings]
        gcn_hidden, hgnn_hidden = [], []
        terms = []  # the sum(hidden) operands
        for _ in range(self.n_layers):
            # hidden[-1] feeds the hop, the learned-hypergraph pair and the layer sum: one n-ary
            # gradient pass (functional.fan)
            h_hop, h_hyp, h_sum = fan(hidden[-1], 3)
            terms.append(h_sum)
            gcn_emb = bipartite_hop(self._dropped(keep_rate), h_hop)
            hyper_u = sharded_dense_two_hop(self.rep_drop(hyper_uu, nl), h_hyp[:nl], self.group)
            hyper_i = dense_two_hop(self.rep_drop(hyper_ii, 0), h_hyp[nl:])
            gcn_hidden += [gcn_emb]
            hgnn_hidden += [torch.cat([hyper_u, hyper_i], 0)]
            hidden += [gcn_emb + hgnn_hidden[-1]]
        embeddings = sum_n(terms + [hidden[-1]])  # sum(hidden), same order, one pass
        return embeddings[:nl], embeddings[nl:], gcn_hidden, hgnn_hidden


class ShardedLocalAwareEncoder(nn.Module):
    """LocalAwareEncoder (HGNN_HD4.py:336-405, ``--mode=local_only``) on user-row shards, same
    submodules and parameter names (``state_dict``s load either way): layers 0..L-2 are ED-HNN
    blocks whose vertex/edge mean pair over V/E = nonzero(ui_adj) runs as
    :func:`sharded_mean_two_hop`; the last layer is LN0(HGCNConv(Â, ·, act=False)) + res with
    the two hops as :func:`~.sharded.bipartite_hop` and :func:`~.sharded.bipartite_hop_fused`
    (LayerNorm and residual in the second hop's store); every layer adds the layer-0 residual.
    All other ops are row-wise, so they run on the local layout unchanged."""

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, u0: int, u1: int,
                 group=None, device=None, n_chunks: int = 4, seed: int = 0):
        super().__init__()
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.u0, self.u1, self.n_local = int(u0), int(u1), int(u1) - int(u0)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.group = group
        U, I = data.n_users, data.n_items
        self.edhnn_args = edhnn_config(hyper_size)
        self.edhnn_layers = nn.ModuleList(
            [EquivSetGNN(hyper_size, self.edhnn_args, None, data) for _ in range(n_layers)])
        self.lns = nn.ModuleList([LayerNorm(hyper_size) for _ in range(n_layers)])
        self.ui = ShardedBipartite.from_global(_coo_tensor(data.ui_adj, binary=True), U, I, u0,
                                               u1, device=self.device, group=group,
                                               n_chunks=n_chunks)
        self.norm = ShardedBipartite.from_global(_coo_tensor(data.norm_adj), U, I, u0, u1,
                                                 device=self.device, group=group,
                                                 n_chunks=n_chunks)
        self.rep_gen, self.loc_gen = _rank_generators(self.device, seed, group)
        self._drops = {}
        self.to(self.device)

    def replicated_parameters(self) -> Iterator[nn.Parameter]:
        return self.parameters()  # every weight is replicated; embeddings come from the caller

    def _drop(self, module: nn.Dropout, x: torch.Tensor) -> torch.Tensor:
        d = self._drops.get(id(module))
        if d is None:
            d = self._drops[id(module)] = _SplitDropout(module.p, self.rep_gen, self.loc_gen)
        d.training = self.training
        return d(x, self.n_local)

    def _edhnn(self, blk: EquivSetGNN, x: torch.Tensor) -> torch.Tensor:
        """EquivSetGNN.forward (EquivSetGNN2.py:83-103) with the sharded aggregation."""
        x = self._drop(blk.dropout, x)
        x = blk.lin_in(x, relu=True)
        x0 = x
        conv = blk.conv
        ln_lin = input_norm_linear(conv.W) if not conv.alpha else None
        for _ in range(blk.nlayer):
            x = self._drop(blk.dropout, x)
            if ln_lin is not None:  # W's InputNorm LayerNorm in the second hop's store
                xv = bipartite_hop_fused(self.ui, bipartite_hop(self.ui, conv.W1(x), "mean"),
                                         "mean", norm=ln_lin[0])
                if isinstance(blk.act, nn.ReLU):
                    x = ln_lin[1](xv, relu=True)  # the block's ReLU fused into the Linear
                else:
                    x = blk.act(ln_lin[1](xv))
                continue
            xv = sharded_mean_two_hop(self.ui, conv.W1(x))
            if conv.alpha:
                xv = (1 - conv.alpha) * xv + conv.alpha * x0
            x = blk.act(conv.W(xv))
        return self._drop(blk.dropout, x)

    def dropped(self, keep_rate: float, device_rng: bool = False) -> ShardedBipartite:
        """The edge-dropped ``norm_adj`` shard (HGNN_HD4.py:304, SpAdjDropEdge): the reference's
        global CPU ``torch.rand(nnz)`` mask (same draw on every rank, same bits as one GPU) or,
        with ``device_rng``, per-rank device masks."""
        if keep_rate == 1.0:
            return self.norm
        if device_rng:
            seed = int(torch.randint(0, 2 ** 40, (1,)).item())  # same draw on every rank
            rank = torch.distributed.get_rank(self.group) if self.norm.world > 1 else 0
            return self.norm.drop_device(keep_rate, seed * 4096 + rank)
        from .layers import torch_cpu_keep_mask
        mask, _ = torch_cpu_keep_mask(int(self.data.norm_adj.nnz), keep_rate)
        return self.norm.drop_global(keep_rate, mask.bool())

    def forward(self, ego_embeddings, sparse_norm_adj=None):
        """``sparse_norm_adj``: None (the full ``norm_adj``) or a :meth:`dropped` shard, which the
        last layer's HGCNConv uses as the reference's does (HGNN_HD4.py:399)."""
        norm = sparse_norm_adj if isinstance(sparse_norm_adj, ShardedBipartite) else self.norm
        # layer 0's input and every layer's residual: one n-ary gradient sum (functional.fan)
        uses = fan(ego_embeddings, self.layers + 1)
        ego_embeddings, res = uses[0], uses[1:]
        for k in range(self.layers):
            if k != self.layers - 1:
                ego_embeddings = self._edhnn(self.edhnn_layers[k], ego_embeddings) + res[k]
            else:
                # LN0(A·(Aᵀ·x)) + res, the LayerNorm and residual in the second hop's store
                ego_embeddings = bipartite_hop_fused(
                    norm, bipartite_hop(norm.transpose(), ego_embeddings), norm=self.lns[0],
                    res1=res[k])
        nl = self.n_local
        return ego_embeddings[:nl], ego_embeddings[nl:]


class ShardedLocalAwareEncoderHD3(ShardedLocalAwareEncoder):
    """LocalAwareEncoderHD3 (HGNN_HD3.py:352-427) on user-row shards, same submodules and
    parameter names: layers 0..L-2 are the SpMM-form ED-HNN blocks (HGNN_HD3.py:555-720), whose
    two aggregations are HGCNConv two-hops over the edge-dropped ``norm_adj`` shard
    (:func:`~.sharded.bipartite_hop_fused`: the LeakyReLU / LayerNorm / residual / restart
    blend in the second hop's store for user rows, one row pass after the exchange for item
    rows); the last layer is ``lns[L-1](HGCNConv(Â, ·,
    act=False)) + res`` on the un-dropped shard. Every layer adds the layer-0 residual."""

    def __init__(self, data, emb_size, hyper_size, n_layers, leaky, drop_rate, u0: int, u1: int,
                 group=None, device=None, n_chunks: int = 4, seed: int = 0):
        nn.Module.__init__(self)
        from .edhnn_spmm import EquivSetGNN as EquivSetGNNSpMM
        from .layers import HGCNConv
        self.data = data
        self.latent_size = emb_size
        self.hyper_size = hyper_size
        self.layers = n_layers
        self.u0, self.u1, self.n_local = int(u0), int(u1), int(u1) - int(u0)
        self.device = torch.device(device) if device is not None else torch.device("cuda")
        self.group = group
        U, I = data.n_users, data.n_items
        self.edhnn_args = edhnn_config(hyper_size)
        self.hgcn_layer = HGCNConv(leaky=0.3)
        self.hgnn_layers = nn.ModuleList([HGCNConv(leaky=0.3) for _ in range(n_layers)])
        self.edhnn_layers = nn.ModuleList([
            EquivSetGNNSpMM(hyper_size, self.edhnn_args, None, data, U, I, leaky=0.5)
            for _ in range(n_layers)])
        self.lns = nn.ModuleList([LayerNorm(hyper_size) for _ in range(n_layers)])
        self.norm = ShardedBipartite.from_global(_coo_tensor(data.norm_adj), U, I, u0, u1,
                                                 device=self.device, group=group,
                                                 n_chunks=n_chunks)
        self.rep_gen, self.loc_gen = _rank_generators(self.device, seed, group)
        self._drops = {}
        self.to(self.device)

    def _edhnn_spmm(self, blk, x: torch.Tensor, sh: ShardedBipartite) -> torch.Tensor:
        """edhnn_spmm.EquivSetGNN.forward (HGNN_HD3.py:680-720) with sharded hops."""
        x = self._drop(blk.dropout, x)
        x = blk.lin_in(x, relu=True)
        x0 = x
        conv = blk.conv
        s0 = conv.hgcn_layers[0].act.negative_slope
        s1 = conv.hgcn_layers[1].act.negative_slope
        for _ in range(blk.nlayer):
            x = self._drop(blk.dropout, x)
            xve = conv.W1(x)
            # Xe = LN0(leaky(A·(Aᵀ·Xve))) + Xve, the epilogue in the second hop's store
            xe = bipartite_hop_fused(sh, bipartite_hop(sh.transpose(), xve),
                                     epilogue="leaky_relu", slope=s0, norm=conv.lns[0], res1=xve)
            xev = xe if conv.W2 is None else conv.W2(torch.cat([x, xe], -1))
            if xev.shape[-1] != conv.out_features:
                xev = conv.mean_pooling(xev)
            # (1-α)·(LN1(leaky(A·(Aᵀ·Xev))) + Xev) + α·X0
            a = conv.alpha
            xv = bipartite_hop_fused(sh, bipartite_hop(sh.transpose(), xev),
                                     epilogue="leaky_relu", slope=s1, norm=conv.lns[1],
                                     out_scale=1 - a, res1=xev, res1_scale=1 - a,
                                     res2=x0 if a != 0 else None, res2_scale=a)
            x = blk.act(conv.W(xv))
        return self._drop(blk.dropout, x)

    def forward(self, ego_embeddings, sparse_norm_adj=None):
        """``sparse_norm_adj``: None (the full ``norm_adj``) or a :meth:`dropped` shard, which
        the ED-HNN blocks use (HGNN_HD3.py:416-418); the last layer uses the full one (:420)."""
        dropped = sparse_norm_adj if isinstance(sparse_norm_adj, ShardedBipartite) else self.norm
        uses = fan(ego_embeddings, self.layers + 1)  # one n-ary gradient sum of the residual
        ego_embeddings, res = uses[0], uses[1:]
        for k in range(self.layers):
            if k != self.layers - 1:
                ego_embeddings = self._edhnn_spmm(self.edhnn_layers[k], ego_embeddings,
                                                  dropped) + res[k]
            else:
                ego_embeddings = bipartite_hop_fused(
                    self.norm, bipartite_hop(self.norm.transpose(), ego_embeddings),
                    norm=self.lns[k], res1=res[k])
        nl = self.n_local
        return ego_embeddings[:nl], ego_embeddings[nl:]
