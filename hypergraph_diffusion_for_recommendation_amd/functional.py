"""Autograd operators over :class:`~.incidence.Incidence` — the propagation hot path.

Every forward and backward hop is one ``hgd_spmm`` launch (plus, for the LeakyReLU variant, one
elementwise backward). The backward of a hop over ``A`` is a hop over ``Aᵀ``, served by the
incidence's CSC, so no transpose is materialised per call (the reference rebuilds ``adj.t()``
and re-coalesces the COO inside every ``torch.sparse.mm``).

Operators (reference call sites, relative to /root/reference/HD_SELFRec):

* :func:`spmm`      ``Y = A·X``                — GCNLayer.forward, model/graph/HCCF.py:198-199
* :func:`two_hop`   ``Y = epi(P·A·Q·Aᵀ·R·X)``  — HGCNConv.forward (P=Q=R=I, A = norm_adj,
                                                  model/graph/HGNN_HD4.py:455-462, HGCN.py:171-175);
                                                  the ED-HNN scatter-mean pair (A = binary V/E
                                                  incidence, P = D_v^-1, Q = D_e^-1, R = I,
                                                  layers2/EquivSetConv2.py:88-93);
                                                  the HGNN normalisation D_v^-1/2 H D_e^-1 Hᵀ D_v^-1/2
                                                  (data/graph.py:28-42) — the benchmarked op.

Scales are named: None, 'mean' (1/deg), 'sym' (deg^-1/2), or the weighted 'wmean'/'wsym'.
The math of the backward: with Z = P·A·Q·Aᵀ·R·X, dX = R·A·Q·Aᵀ·P·dZ (the diagonals commute
through the transposes), so forward and backward are the same pair of hops with the outer
diagonals swapped.
"""
from __future__ import annotations

from typing import Optional

import torch

from . import _native as nat
from .incidence import Incidence, spmm_csr

_EPI = {None: nat.EPI_NONE, "none": nat.EPI_NONE, "leaky_relu": nat.EPI_LEAKY_RELU,
        "relu": nat.EPI_RELU}


def _epilogue_backward(ref: torch.Tensor, dy: torch.Tensor, epi: int, slope: float):
    ref = ref.contiguous()
    dy = dy.contiguous()
    dz = torch.empty_like(dy)
    nat.check(nat.load().hgd_epilogue_backward(ref.data_ptr(), dy.data_ptr(), dy.numel(), epi,
                                               float(slope), dz.data_ptr(),
                                               torch.cuda.current_stream(dy.device).cuda_stream),
              "hgd_epilogue_backward")
    return dz


def _epilogue_apply(z: torch.Tensor, epi: int, slope: float):
    y = torch.empty_like(z)
    nat.check(nat.load().hgd_epilogue_apply(z.data_ptr(), z.numel(), epi, float(slope),
                                            y.data_ptr(),
                                            torch.cuda.current_stream(z.device).cuda_stream),
              "hgd_epilogue_apply")
    return y


class _SpMM(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, inc: Incidence, transpose: bool):
        ctx.inc = inc
        ctx.transpose = transpose
        X = X.contiguous()
        if transpose:
            return spmm_csr(inc.csc, X, val=inc.val_t)
        return spmm_csr(inc.csr, X, val=inc.val)

    @staticmethod
    def backward(ctx, dY):
        inc = ctx.inc
        dY = dY.contiguous()
        if ctx.transpose:
            dX = spmm_csr(inc.csr, dY, val=inc.val)
        else:
            dX = spmm_csr(inc.csc, dY, val=inc.val_t)
        return dX, None, None


def spmm(inc: Incidence, X: torch.Tensor, transpose: bool = False) -> torch.Tensor:
    """``A·X`` (or ``Aᵀ·X``) with autograd; ``torch.sparse.mm(adj, X)`` drop-in."""
    return _SpMM.apply(X, inc, transpose)


class _TwoHop(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, inc: Incidence, P, Q, R, epi: int, slope: float):
        X = X.contiguous()
        q = inc.scale("col", Q)
        # hop 1 into the columns (hyperedges) of A: M = Q·Aᵀ·(R·X)
        M = spmm_csr(inc.csc, X, val=inc.edge_values("csc", R), row_scale=q)
        # hop 2 back into the rows (vertices): Z = P·A·M, epilogue fused when the sign test on
        # the output is equivalent to the one on the pre-activation (slope >= 0)
        p = inc.scale("row", P)
        fuse = epi != nat.EPI_NONE and slope >= 0.0
        Y = spmm_csr(inc.csr, M, val=inc.val, row_scale=p, epilogue=epi if fuse else 0,
                     slope=slope)
        ref = Y
        if epi != nat.EPI_NONE and not fuse:
            ref = Y
            Y = _epilogue_apply(Y, epi, slope)
        ctx.inc = inc
        ctx.scales = (P, Q, R)
        ctx.epi = epi
        ctx.slope = slope
        if epi != nat.EPI_NONE:
            ctx.save_for_backward(ref)
        return Y

    @staticmethod
    def backward(ctx, dY):
        inc = ctx.inc
        P, Q, R = ctx.scales
        dZ = dY.contiguous()
        if ctx.epi != nat.EPI_NONE:
            (ref,) = ctx.saved_tensors
            dZ = _epilogue_backward(ref, dZ, ctx.epi, ctx.slope)
        q = inc.scale("col", Q)
        dM = spmm_csr(inc.csc, dZ, val=inc.edge_values("csc", P), row_scale=q)
        r = inc.scale("row", R)
        dX = spmm_csr(inc.csr, dM, val=inc.val, row_scale=r)
        return dX, None, None, None, None, None, None


def two_hop(inc: Incidence, X: torch.Tensor, P: Optional[str] = None, Q: Optional[str] = None,
            R: Optional[str] = None, epilogue: Optional[str] = None,
            slope: float = 0.0) -> torch.Tensor:
    """``epi(P·A·Q·Aᵀ·R·X)`` with autograd (see module docstring for the scale names)."""
    return _TwoHop.apply(X, inc, P, Q, R, _EPI[epilogue], float(slope))


def hgconv2(inc: Incidence, X: torch.Tensor) -> torch.Tensor:
    """HGNN normalised 2-hop ``D_v^-1/2·H·D_e^-1·Hᵀ·D_v^-1/2·X`` (data/graph.py:28-42)."""
    return two_hop(inc, X, P="sym", Q="mean", R="sym")


def mean2hop(inc: Incidence, X: torch.Tensor) -> torch.Tensor:
    """ED-HNN edge-mean then vertex-mean ``D_v^-1·B·D_e^-1·Bᵀ·X`` (EquivSetConv2.py:88-93)."""
    return two_hop(inc, X, P="mean", Q="mean", R=None)
