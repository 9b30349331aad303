"""The SpMM form of the ED-HNN block — the variant in which both
aggregation steps are HGCNConv two-hops over ``norm_adj`` instead of scatter-means over V/E
(paths relative to /root/reference/HD_SELFRec):

* :class:`EquivSetConv` — model/layers/EquivSetConv.py:36-107 (HGCNConv slope 0.2) and
  model/graph/HGNN_HD3.py:652-720 (slope 0.5, extra ``ui_adj`` argument, accepted and unused
  as there): ``Xe = LN(leaky(A·(Aᵀ·W1(X)))) + W1(X)``, ``Xev = W2([X, Xe])`` (the Xe slice when
  mlp2_layers = 0), ``AdaptiveAvgPool1d``, ``Xv = LN(leaky(A·(Aᵀ·Xev))) + Xev``,
  ``W((1-α)·Xv + α·X0)``.
* :class:`EquivSetGNN` — model/layers/EquivSetGNN.py:32-101: dropout → ReLU(lin_in) → x0 →
  [dropout → conv → act] × All_num_layers → dropout.

Both two-hops run as hgd_spmm pairs whose second store also applies the LeakyReLU, the LayerNorm,
the residual and the restart blend (hgd_spmm_fused, functional.two_hop_fused; SURVEY.md §8f
rank 1); only the Linear layers stay torch (rocBLAS). The wavelet (HWNN) layers
the reference constructs but never calls are not built.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from .functional import two_hop_fused
from .incidence import incidence_of
from .layers import MLP, HGCNConv, LayerNorm, Linear


class EquivSetConv(nn.Module):
    def __init__(self, in_features, out_features, ncount=None, mcount=None, mlp1_layers=1,
                 mlp2_layers=1, mlp3_layers=1, aggr='add', alpha=0.5, dropout=0.,
                 normalization='None', input_norm=False, hypergraph=None, data=None,
                 leaky=0.2):
        super().__init__()
        self.W1 = (MLP(in_features, out_features, out_features, mlp1_layers, dropout=dropout,
                       Normalization=normalization, InputNorm=input_norm)
                   if mlp1_layers > 0 else nn.Identity())
        self.in_features = in_features
        self.out_features = out_features
        self.W2 = (MLP(in_features + out_features, out_features, out_features, mlp2_layers,
                       dropout=dropout, Normalization=normalization, InputNorm=input_norm)
                   if mlp2_layers > 0 else None)
        self.W = (MLP(out_features, out_features, out_features, mlp3_layers, dropout=dropout,
                      Normalization=normalization, InputNorm=input_norm)
                  if mlp3_layers > 0 else nn.Identity())
        self.aggr = aggr
        self.alpha = alpha
        self.dropout = dropout
        self.data = data
        self.hgcn_layers = nn.ModuleList([HGCNConv(leaky) for _ in range(2)])
        self.mean_pooling = nn.AdaptiveAvgPool1d(out_features)
        self.lns = nn.ModuleList([LayerNorm(out_features) for _ in range(2)])
        self.fused_epilogue = True  # False: the reference's separate LN / add / blend ops

    def reset_parameters(self):
        for m in (self.W1, self.W2, self.W):
            if isinstance(m, MLP):
                m.reset_parameters()

    def forward(self, X, sparse_norm_adj, X0, *ui_adj, act=True):
        Xve = self.W1(X)
        fused = self.fused_epilogue and torch.is_tensor(X0) and tuple(X0.shape) == tuple(Xve.shape)
        if fused:
            inc = incidence_of(sparse_norm_adj)
            slope0 = self.hgcn_layers[0].act.negative_slope
            # Xe = LN0(leaky(A·(Aᵀ·Xve))) + Xve in one store
            Xe = two_hop_fused(inc, Xve, epilogue="leaky_relu", slope=slope0, norm=self.lns[0],
                               res1=Xve, res1_scale=1.0)
        else:
            Xe = self.lns[0](self.hgcn_layers[0](sparse_norm_adj, Xve, act=True)) + Xve
        if self.W2 is None:
            Xev = Xe  # W2 = X[..., in_features:] of cat([X, Xe])
        else:
            Xev = self.W2(torch.cat([X, Xe], -1))
        if Xev.shape[-1] != self.out_features:  # AdaptiveAvgPool1d is the identity otherwise
            Xev = self.mean_pooling(Xev)
        if fused and tuple(Xev.shape) == tuple(X0.shape):
            slope1 = self.hgcn_layers[1].act.negative_slope
            # (1-α)·(LN1(leaky(A·(Aᵀ·Xev))) + Xev) + α·X0 in one store
            # (α = 0, the configs' restart_alpha: X0 drops out exactly, so it is not read)
            X = two_hop_fused(inc, Xev, epilogue="leaky_relu", slope=slope1, norm=self.lns[1],
                              out_scale=1 - self.alpha, res1=Xev, res1_scale=1 - self.alpha,
                              res2=X0 if self.alpha != 0 else None, res2_scale=self.alpha)
        else:
            X_v = self.lns[1](self.hgcn_layers[1](sparse_norm_adj, Xev, act=True)) + Xev
            X = (1 - self.alpha) * X_v + self.alpha * X0
        return self.W(X)


class EquivSetGNN(nn.Module):
    def __init__(self, num_features, args, dense_hypergraph=None, data=None, ncount=None,
                 mcount=None, leaky=0.2):
        super().__init__()
        act = {'Id': nn.Identity(), 'relu': nn.ReLU(), 'prelu': nn.PReLU()}
        self.act = act[args['activation']]
        self.input_drop = nn.Dropout(args['input_dropout'])
        self.dropout = nn.Dropout(args['dropout'])
        self.data = data
        self.in_channels = num_features
        self.hidden_channels = args['MLP_hidden']
        self.mlp1_layers = args['MLP_num_layers']
        self.mlp2_layers = (args['MLP_num_layers'] if args['MLP2_num_layers'] < 0
                            else args['MLP2_num_layers'])
        self.mlp3_layers = (args['MLP_num_layers'] if args['MLP3_num_layers'] < 0
                            else args['MLP3_num_layers'])
        self.nlayer = args['All_num_layers']
        self.lin_in = Linear(num_features, args['MLP_hidden'])
        self.conv = EquivSetConv(args['MLP_hidden'], args['MLP_hidden'], ncount, mcount,
                                 mlp1_layers=self.mlp1_layers, mlp2_layers=self.mlp2_layers,
                                 mlp3_layers=self.mlp3_layers, alpha=args['restart_alpha'],
                                 aggr=args['aggregate'], dropout=args['dropout'],
                                 normalization=args['normalization'],
                                 input_norm=args['AllSet_input_norm'],
                                 hypergraph=dense_hypergraph, data=data, leaky=leaky)

    def reset_parameters(self):
        self.lin_in.reset_parameters()
        self.conv.reset_parameters()

    def forward(self, x, sparse_norm_adj, n_nodes, act=True):
        x = self.dropout(x)
        x = self.lin_in(x, relu=True)  # F.relu(lin_in(x)) fused
        x0 = x
        for _ in range(self.nlayer):
            x = self.dropout(x)
            x = self.conv(x, sparse_norm_adj, x0, act=act)
            x = self.act(x)
        return self.dropout(x)
