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

import ctypes
from typing import List, Optional, Tuple

import torch
import torch.nn.functional as F

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
                                               nat.stream_handle(dy.device)),
              "hgd_epilogue_backward")
    return dz


def _epilogue_apply(z: torch.Tensor, epi: int, slope: float):
    y = torch.empty_like(z)
    nat.check(nat.load().hgd_epilogue_apply(z.data_ptr(), z.numel(), epi, float(slope),
                                            y.data_ptr(),
                                            nat.stream_handle(z.device)),
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


def _ln_supported(d: int) -> bool:
    # hgd_spmm_fused / hgd_row_epilogue_backward keep a whole row in one lane group
    return d <= 256 if d % 4 == 0 else d <= 64


class _FusedTwoHop(torch.autograd.Function):
    """``Y = out_scale·LN(epi(P·A·Q·Aᵀ·R·X)) + s1·res1 + s2·res2`` — the second hop's store runs
    the activation, LayerNorm and residual blend (hgd_spmm_fused); the backward runs their
    gradient in one pass (hgd_row_epilogue_backward) before the two backward hops."""

    @staticmethod
    def forward(ctx, X, gamma, beta, res1, res2, inc: Incidence, cfg):
        P, Q, R, epi, slope, ln, eps, out_scale, s1, s2 = cfg
        X = X.contiguous()
        dev = X.device
        n, d = inc.n_rows, X.shape[1]
        q = inc.scale("col", Q)
        M = spmm_csr(inc.csc, X, val=inc.edge_values("csc", R), row_scale=q)
        p = inc.scale("row", P)
        need_a = ln or epi != nat.EPI_NONE
        A = torch.empty((n, d), dtype=torch.float32, device=dev) if need_a else None
        stats = torch.empty((n, 2), dtype=torch.float32, device=dev) if ln else None
        res1 = None if res1 is None else res1.contiguous()
        res2 = None if res2 is None else res2.contiguous()
        ex = nat.RowEpilogue(
            act=epi, slope=slope, layer_norm=int(ln), ln_eps=eps,
            ln_gamma=nat.ptr(gamma) if ln else None, ln_beta=nat.ptr(beta) if ln else None,
            out_scale=out_scale,
            res1=nat.ptr(res1), ld_res1=0 if res1 is None else res1.stride(0), res1_scale=s1,
            res2=nat.ptr(res2), ld_res2=0 if res2 is None else res2.stride(0), res2_scale=s2,
            act_out=nat.ptr(A), ld_act=0 if A is None else A.stride(0), stats=nat.ptr(stats))
        Y = spmm_csr(inc.csr, M, val=inc.val, row_scale=p, ex=ex)
        ctx.inc = inc
        ctx.cfg = cfg
        ctx.has_res = (res1 is not None, res2 is not None)
        ctx.save_for_backward(A, stats, gamma if ln else None)
        return Y

    @staticmethod
    def backward(ctx, dY):
        inc = ctx.inc
        P, Q, R, epi, slope, ln, eps, out_scale, s1, s2 = ctx.cfg
        A, stats, gamma = ctx.saved_tensors
        dY = dY.contiguous()
        n, d = dY.shape
        dev = dY.device
        want_g = ln and ctx.needs_input_grad[1]
        want_b = ln and ctx.needs_input_grad[2]
        if not ln and epi == nat.EPI_NONE:
            # a pure blend: dZ = out_scale·dY, folded into the item-side row scale of the first
            # backward hop (n_cols multiplies instead of an [n, d] pass)
            dX = None
            if ctx.needs_input_grad[0]:
                q = inc.scale("col", Q)
                if out_scale != 1.0:
                    q = (torch.full((inc.n_cols,), out_scale, dtype=torch.float32, device=dev)
                         if q is None else q * out_scale)
                dM = spmm_csr(inc.csc, dY, val=inc.edge_values("csc", P), row_scale=q)
                dX = spmm_csr(inc.csr, dM, val=inc.val, row_scale=inc.scale("row", R))
            return (dX, None, None, _res_grad(ctx, dY, 0, s1), _res_grad(ctx, dY, 1, s2), None,
                    None)
        dgamma = torch.empty(d, dtype=torch.float32, device=dev) if want_g else None
        dbeta = torch.empty(d, dtype=torch.float32, device=dev) if want_b else None
        lib = nat.load()
        wsb = lib.hgd_row_epilogue_backward_workspace_size(n, d) if (want_g or want_b) else 0
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev) if wsb else None
        dZ = torch.empty_like(dY)
        nat.check(lib.hgd_row_epilogue_backward(
            dY.data_ptr(), dY.stride(0), nat.ptr(A), 0 if A is None else A.stride(0),
            nat.ptr(stats), nat.ptr(gamma), n, d, epi, float(slope), int(ln), float(out_scale),
            dZ.data_ptr(), dZ.stride(0), nat.ptr(dgamma), nat.ptr(dbeta), nat.ptr(ws), wsb,
            nat.stream_handle(dev)), "hgd_row_epilogue_backward")
        dX = None
        if ctx.needs_input_grad[0]:
            q = inc.scale("col", Q)
            dM = spmm_csr(inc.csc, dZ, val=inc.edge_values("csc", P), row_scale=q)
            dX = spmm_csr(inc.csr, dM, val=inc.val, row_scale=inc.scale("row", R))
        return (dX, dgamma, dbeta, _res_grad(ctx, dY, 0, s1), _res_grad(ctx, dY, 1, s2), None,
                None)


def _res_grad(ctx, dY, k, s):
    if not ctx.has_res[k] or not ctx.needs_input_grad[3 + k]:
        return None
    return dY if s == 1.0 else dY * s


def two_hop_fused(inc: Incidence, X: torch.Tensor, P: Optional[str] = None,
                  Q: Optional[str] = None, R: Optional[str] = None,
                  epilogue: Optional[str] = None, slope: float = 0.0,
                  norm: Optional[torch.nn.LayerNorm] = None, out_scale: float = 1.0,
                  res1: Optional[torch.Tensor] = None, res1_scale: float = 1.0,
                  res2: Optional[torch.Tensor] = None, res2_scale: float = 1.0) -> torch.Tensor:
    """``out_scale·norm(epi(P·A·Q·Aᵀ·R·X)) + res1_scale·res1 + res2_scale·res2`` with autograd.

    One fused hgd_spmm_fused store replaces the reference's separate LayerNorm, residual add and
    restart blend kernels. ``norm`` is an ``nn.LayerNorm`` over the last
    dim (its weight/bias get gradients). Shapes the fused store cannot hold (LayerNorm with
    d > 256, or a negative slope) run the same math as separate device ops."""
    epi = _EPI[epilogue]
    d = X.shape[1]
    ln = norm is not None
    if ln and (tuple(norm.normalized_shape) != (d,)):
        raise ValueError(f"two_hop_fused: LayerNorm over {tuple(norm.normalized_shape)}, d={d}")
    for r in (res1, res2):
        if r is not None and tuple(r.shape) != (inc.n_rows, d):
            raise ValueError(f"two_hop_fused: residual {tuple(r.shape)} != {(inc.n_rows, d)}")
    if (ln and not _ln_supported(d)) or (epi != nat.EPI_NONE and slope < 0):
        y = two_hop(inc, X, P=P, Q=Q, R=R, epilogue=epilogue, slope=slope)
        if ln:
            y = norm(y)
        y = out_scale * y
        if res1 is not None:
            y = y + res1_scale * res1
        if res2 is not None:
            y = y + res2_scale * res2
        return y
    gamma = norm.weight if ln and norm.weight is not None else None
    beta = norm.bias if ln and norm.bias is not None else None
    cfg = (P, Q, R, epi, float(slope), ln, float(norm.eps) if ln else 0.0, float(out_scale),
           float(res1_scale), float(res2_scale))
    return _FusedTwoHop.apply(X, gamma, beta, res1, res2, inc, cfg)


def _linear_native_ok(X: torch.Tensor, weight: torch.Tensor) -> bool:
    out_f, in_f = weight.shape
    return (X.is_cuda and X.dtype == torch.float32 and weight.dtype == torch.float32
            and in_f % 16 == 0 and out_f % 16 == 0 and 16 <= in_f <= 128 and 16 <= out_f <= 128)


class _Linear(torch.autograd.Function):
    """``relu?(X·Wᵀ + b)`` on hgd_linear_* (f32 MFMA; forward, backward-data, split-K
    backward-weight with the bias gradient folded in)."""

    @staticmethod
    def forward(ctx, X, weight, bias, relu: bool):
        lib = nat.load()
        X = X.contiguous()
        W = weight.contiguous()
        n, in_f = X.shape
        out_f = W.shape[0]
        Y = torch.empty((n, out_f), dtype=torch.float32, device=X.device)
        st = nat.stream_handle(X.device)
        nat.check(lib.hgd_linear_forward(X.data_ptr(), X.stride(0), n, in_f, W.data_ptr(),
                                         W.stride(0), out_f, nat.ptr(bias), int(relu),
                                         Y.data_ptr(), Y.stride(0), st), "hgd_linear_forward")
        ctx.relu = relu
        ctx.has_bias = bias is not None
        ctx.save_for_backward(X, W, Y if relu else None)
        return Y

    @staticmethod
    def backward(ctx, dY):
        lib = nat.load()
        X, W, Y = ctx.saved_tensors
        dY = dY.contiguous()
        n, in_f = X.shape
        out_f = W.shape[0]
        st = nat.stream_handle(dY.device)
        dX = dW = db = None
        if ctx.needs_input_grad[0]:
            dX = torch.empty_like(X)
            nat.check(lib.hgd_linear_backward_data(
                dY.data_ptr(), dY.stride(0), nat.ptr(Y), 0 if Y is None else Y.stride(0), n,
                out_f, W.data_ptr(), W.stride(0), in_f, dX.data_ptr(), dX.stride(0), st),
                "hgd_linear_backward_data")
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            dW = torch.empty((out_f, in_f), dtype=torch.float32, device=dY.device)
            db = torch.empty(out_f, dtype=torch.float32, device=dY.device) if want_b else None
            wsb = lib.hgd_linear_backward_weight_workspace_size(n, out_f, in_f)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dY.device)
            nat.check(lib.hgd_linear_backward_weight(
                dY.data_ptr(), dY.stride(0), nat.ptr(Y), 0 if Y is None else Y.stride(0),
                X.data_ptr(), X.stride(0), n, out_f, in_f, dW.data_ptr(), nat.ptr(db),
                ws.data_ptr(), wsb, st), "hgd_linear_backward_weight")
            if not ctx.needs_input_grad[1]:
                dW = None
        return dX, dW, db, None


def linear(X: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor] = None,
           relu: bool = False) -> torch.Tensor:
    """``F.linear`` (optionally followed by ``F.relu``) for the skinny ED-HNN shapes: features
    multiples of 16 up to 128 run on hgd_linear_*; other shapes use the library GEMM."""
    if not _linear_native_ok(X, weight):
        Y = torch.nn.functional.linear(X, weight, bias)
        return torch.relu(Y) if relu else Y
    lead = X.shape[:-1]
    Y = _Linear.apply(X.reshape(-1, X.shape[-1]), weight, bias, bool(relu))
    return Y.reshape(*lead, weight.shape[0])


def dropout_seed(device) -> torch.Tensor:
    """A fresh seed for the library's device dropout, drawn from torch's generator of ``device``
    (so ``torch.manual_seed`` fixes the stream, and a captured step draws it inside the graph)."""
    return torch.randint(0, 2 ** 62, (1,), device=device, dtype=torch.int64)


def _drop_consts(p: float):
    keep = 1.0 - float(p)
    return keep, float(torch.tensor(1.0 / keep, dtype=torch.float32))  # nn.Dropout's 1/(1-p)


def _dropout_call(x: torch.Tensor, p: float, seed: torch.Tensor) -> torch.Tensor:
    keep, scale = _drop_consts(p)
    y = torch.empty_like(x)
    nat.check(nat.load().hgd_dropout_apply(x.data_ptr(), x.numel(), seed.data_ptr(), keep, scale,
                                           y.data_ptr(),
                                           nat.stream_handle(x.device)),
              "hgd_dropout_apply")
    return y


class _Dropout(torch.autograd.Function):
    """nn.Dropout(p) on the library's counter-based RNG (hgd_dropout_apply): the backward
    regenerates the mask from the seed instead of storing it."""

    @staticmethod
    def forward(ctx, x, p: float, seed):
        ctx.p = p
        ctx.save_for_backward(seed)
        return _dropout_call(x.contiguous(), p, seed)

    @staticmethod
    def backward(ctx, g):
        (seed,) = ctx.saved_tensors
        return _dropout_call(g.contiguous(), ctx.p, seed), None, None


def dropout(x: torch.Tensor, p: float, seed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.dropout(x, p, training=True)`` for device fp32 tensors on the library RNG (same
    distribution, its own stream: oracle.hgd_oracle.dropout_keep_mask restates the mask)."""
    if p == 0.0:
        return x
    if not (0.0 < p < 1.0):
        raise ValueError(f"dropout: p = {p} outside (0, 1)")
    if x.numel() > 0xFFFFFFFF or not x.is_cuda or x.dtype != torch.float32:
        return torch.nn.functional.dropout(x, p, training=True)  # beyond the 32-bit counter
    if seed is None:
        seed = dropout_seed(x.device)
    return _Dropout.apply(x, float(p), seed)


class _Fan(torch.autograd.Function):
    """``n`` aliases of one table whose gradients meet in ONE n-ary sum (hgd_sum_arrays) instead
    of autograd's chain of n − 1 binary accumulations (each a full read-read-write of the table)."""

    @staticmethod
    def forward(ctx, x, n: int):
        # an alias whose output gets no gradient arrives as None (no zero table to read)
        ctx.set_materialize_grads(False)
        return tuple(x.view_as(x) for _ in range(n))

    @staticmethod
    def backward(ctx, *grads):
        gs = [g.contiguous() for g in grads if g is not None]
        if not gs:
            return None, None
        if len(gs) == 1:
            return gs[0], None
        # hgd_sum_arrays reads 16-byte pieces: a contiguous view at an odd offset is copied
        gs = [g if g.data_ptr() % 16 == 0 else g.clone() for g in gs]
        out = torch.empty_like(gs[0])
        ptrs = (ctypes.c_void_p * len(gs))(*[g.data_ptr() for g in gs])
        nat.check(nat.load().hgd_sum_arrays(ptrs, len(gs), out.numel(), out.data_ptr(),
                                            nat.stream_handle(out.device)), "hgd_sum_arrays")
        return out, None


def split_rows(x: torch.Tensor, nu: int):
    """``(x[:nu], x[nu:])`` (the encoders' user / item halves of the node table) as one split:
    its backward is ONE cat of the two gradients, where two slicing views each materialise a
    zero-filled full table, copy their half into it and add the two (≈ 90 µs per LocalAware step
    at 144 k × 128: two fills, two copies and a full-table add)."""
    return torch.split(x, [nu, x.shape[0] - nu], dim=0)


def fan(x: torch.Tensor, n: int):
    """``n`` uses of ``x`` (e.g. HGNN_HD4's layer-0 residual ``res``, read by every layer,
    HGNN_HD4.py:390-405) whose gradients are summed in one pass. Off the device path (or for
    more than 8 uses) the plain tensor is returned n times."""
    if (n < 2 or n > 8 or not x.is_cuda or x.dtype != torch.float32 or not x.requires_grad
            or not torch.is_grad_enabled()):
        return (x,) * n
    return _Fan.apply(x, int(n))


class _SumN(torch.autograd.Function):
    """``((t_0 + t_1) + t_2) + …`` of equal-shape tables in one pass (hgd_sum_arrays); the
    backward hands the output gradient to every input (no kernels)."""

    @staticmethod
    def forward(ctx, *ts):
        ts = [t.contiguous() for t in ts]
        out = torch.empty_like(ts[0])
        ptrs = (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])
        nat.check(nat.load().hgd_sum_arrays(ptrs, len(ts), out.numel(), out.data_ptr(),
                                            nat.stream_handle(out.device)), "hgd_sum_arrays")
        ctx.n = len(ts)
        return out

    @staticmethod
    def backward(ctx, g):
        return (g,) * ctx.n


def sum_n(ts):
    """``sum(ts)`` (e.g. HCCF's ``sum(hidden)``, HCCF.py:188 / HCCF_diffusion.py:221) as one
    n-ary pass on the device, in list order; Python's ``sum`` elsewhere."""
    ts = list(ts)
    if (2 <= len(ts) <= 8 and all(t.is_cuda and t.dtype == torch.float32 for t in ts)
            and all(t.shape == ts[0].shape for t in ts)):
        return _SumN.apply(*ts)
    return sum(ts)


class _LinearReluDrop(torch.autograd.Function):
    """``dropout(relu(dropout(X, in_p)·Wᵀ + b), p) (+ res)`` in the row GEMM (hgd_gemm_rows: the
    input dropout as X is loaded, the ReLU, the dropout mask of the library RNG and its 1/(1-p)
    in the store, the residual as a second output). Backward: a row GEMM (dX, with the input
    dropout's mask and scale in its store) and a split-K product (dW, db; the input dropout
    re-applied as X is loaded) with the stored dropped activation as the mask (it is > 0 exactly
    where the ReLU passed and the element was kept) and 1/(1-p) folded into W as it is staged
    and into the dW / db reduction's store. The dropped input is never materialised."""

    @staticmethod
    def forward(ctx, X, weight, bias, res, p: float, seed, in_p: float, in_seed):
        X = X.contiguous()
        W = weight.contiguous()
        n, in_f = X.shape
        out_f = W.shape[0]
        dev = X.device
        Y = torch.empty((n, out_f), dtype=torch.float32, device=dev)
        d = _rows_desc(X, W, 1, W.stride(0), in_f, out_f, Y)
        d.bias, d.relu = nat.ptr(bias), 1
        in_keep = in_scale = 1.0
        if in_p > 0.0:
            in_keep, in_scale = _drop_consts(in_p)
            d.a_drop_seed, d.a_drop_keep, d.a_drop_scale = in_seed.data_ptr(), in_keep, in_scale
        scale = 1.0
        if p > 0.0:
            keep, scale = _drop_consts(p)
            d.drop_seed, d.drop_keep, d.drop_scale = seed.data_ptr(), keep, scale
        out = Y
        if res is not None:
            res = res.contiguous()
            out = torch.empty_like(Y)
            d.res, d.ldres, d.Y2, d.ldy2 = res.data_ptr(), res.stride(0), out.data_ptr(), \
                out.stride(0)
        _gemm_rows([d], dev)
        ctx.scale = scale
        ctx.in_drop = (in_keep, in_scale) if in_p > 0.0 else None
        ctx.has_bias, ctx.has_res = bias is not None, res is not None
        ctx.save_for_backward(X, W, Y, in_seed if in_p > 0.0 else None)
        return out

    @staticmethod
    def backward(ctx, dout):
        lib = nat.load()
        X, W, Y, in_seed = ctx.saved_tensors
        dY = dout.contiguous()
        n, in_f = X.shape
        out_f = W.shape[0]
        dev = dY.device
        s = ctx.scale
        dX = dW = db = None
        if ctx.needs_input_grad[0]:
            # dX = (dY ⊙ [Y > 0])·(W·s): the 1/(1-p) scales W as the row GEMM stages it; the
            # input dropout's backward (its keep-bits × 1/(1-in_p)) in the store
            dX = torch.empty_like(X)
            d = _rows_desc(dY, W, W.stride(0), 1, out_f, in_f, dX)
            d.relu_mask, d.ldm = Y.data_ptr(), Y.stride(0)
            d.b_scale = s if s != 1.0 else 0.0
            if ctx.in_drop is not None:
                d.drop_seed, d.drop_keep, d.drop_scale = (in_seed.data_ptr(),) + ctx.in_drop
            _gemm_rows([d], dev)
        want_b = ctx.has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_b:
            # dW = s·(dY ⊙ [Y > 0])ᵀ·X, db = s·Σ_rows (dY ⊙ [Y > 0]): s applied in the reduction
            dW = torch.empty((out_f, in_f), dtype=torch.float32, device=dev)
            db = torch.empty(out_f, dtype=torch.float32, device=dev) if want_b else None
            t = nat.GemmTnDesc()
            t.A, t.lda, t.relu_mask, t.ldm = dY.data_ptr(), dY.stride(0), Y.data_ptr(), Y.stride(0)
            t.B, t.ldb, t.rows, t.M, t.N = X.data_ptr(), X.stride(0), n, out_f, in_f
            t.C, t.colsum_A = dW.data_ptr(), nat.ptr(db)
            t.c_scale = s if s != 1.0 else 0.0
            if ctx.in_drop is not None:  # dropout(X) re-drawn as X is loaded
                t.b_drop_seed, t.b_drop_keep, t.b_drop_scale = (in_seed.data_ptr(),) + ctx.in_drop
            arr = (nat.GemmTnDesc * 1)(t)
            wsb = lib.hgd_gemm_tn_workspace_size(arr, 1)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            nat.check(lib.hgd_gemm_tn(arr, 1, ws.data_ptr(), wsb,
                                      nat.stream_handle(dev)), "hgd_gemm_tn")
            if not ctx.needs_input_grad[1]:
                dW = None
        dres = dY if ctx.has_res and ctx.needs_input_grad[3] else None
        return dX, dW, db, dres, None, None, None, None


def linear_relu_dropout(X: torch.Tensor, weight: torch.Tensor, bias: Optional[torch.Tensor],
                        p: float, res: Optional[torch.Tensor] = None,
                        seed: Optional[torch.Tensor] = None, in_p: float = 0.0,
                        in_seed: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``F.dropout(F.relu(F.linear(F.dropout(X, in_p), weight, bias)), p) + res`` (the ED-HNN
    block's dropout → lin_in → ReLU and W → ReLU → dropout → + residual,
    layers2/EquivSetGNN2.py:91-101 and HGNN_HD4.py:399) with the input dropout in the row GEMM's
    operand load and everything after the product in its store. ``p`` / ``in_p = 0``: no
    dropout; ``res`` None: no residual. Bitwise ``linear_relu_dropout(dropout(X, in_p, in_seed),
    …)``. Shapes outside the kernels run the torch ops (with the library dropout)."""
    if res is not None and tuple(res.shape) != (X.shape[0], weight.shape[0]):
        raise ValueError("linear_relu_dropout: residual shape mismatch")
    if in_p > 0.0 and in_seed is None:
        in_seed = dropout_seed(X.device)
    if not (_linear_native_ok(X, weight) and X.dim() == 2
            and X.shape[0] * max(weight.shape[0], weight.shape[1]) <= 0xFFFFFFFF):
        if in_p > 0.0:
            X = dropout(X, in_p, in_seed)
        y = dropout(linear(X, weight, bias, relu=True), p, seed)
        return y if res is None else y + res
    if p > 0.0 and seed is None:
        seed = dropout_seed(X.device)
    return _LinearReluDrop.apply(X, weight, bias, res, float(p), seed, float(in_p), in_seed)


class _RowEpilogue(torch.autograd.Function):
    """``out_scale·LN(act(Z)) + s1·res1 + s2·res2`` on an existing matrix
    (hgd_row_epilogue_forward / hgd_row_epilogue_backward)."""

    @staticmethod
    def forward(ctx, Z, gamma, beta, res1, res2, cfg):
        epi, slope, ln, eps, out_scale, s1, s2 = cfg
        Z = Z.contiguous()
        n, d = Z.shape
        dev = Z.device
        need_a = ln or epi != nat.EPI_NONE
        A = (Z if epi == nat.EPI_NONE else torch.empty_like(Z)) if need_a else None
        stats = torch.empty((n, 2), dtype=torch.float32, device=dev) if ln else None
        res1 = None if res1 is None else res1.contiguous()
        res2 = None if res2 is None else res2.contiguous()
        ex = nat.RowEpilogue(
            act=epi, slope=slope, layer_norm=int(ln), ln_eps=eps,
            ln_gamma=nat.ptr(gamma) if ln else None, ln_beta=nat.ptr(beta) if ln else None,
            out_scale=out_scale,
            res1=nat.ptr(res1), ld_res1=0 if res1 is None else res1.stride(0), res1_scale=s1,
            res2=nat.ptr(res2), ld_res2=0 if res2 is None else res2.stride(0), res2_scale=s2,
            act_out=nat.ptr(A) if (A is not None and A is not Z) else None,
            ld_act=0 if A is None else A.stride(0), stats=nat.ptr(stats))
        Y = torch.empty_like(Z)
        nat.check(nat.load().hgd_row_epilogue_forward(
            Z.data_ptr(), Z.stride(0), n, d, ctypes.byref(ex), Y.data_ptr(), Y.stride(0),
            nat.stream_handle(dev)), "hgd_row_epilogue_forward")
        ctx.cfg = cfg
        ctx.has_res = (res1 is not None, res2 is not None)
        ctx.save_for_backward(A, stats, gamma if ln else None)
        return Y

    @staticmethod
    def backward(ctx, dY):
        epi, slope, ln, eps, out_scale, s1, s2 = ctx.cfg
        A, stats, gamma = ctx.saved_tensors
        dY = dY.contiguous()
        n, d = dY.shape
        dev = dY.device
        lib = nat.load()
        want_g = ln and ctx.needs_input_grad[1]
        want_b = ln and ctx.needs_input_grad[2]
        dgamma = torch.empty(d, dtype=torch.float32, device=dev) if want_g else None
        dbeta = torch.empty(d, dtype=torch.float32, device=dev) if want_b else None
        wsb = lib.hgd_row_epilogue_backward_workspace_size(n, d) if (want_g or want_b) else 0
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev) if wsb else None
        dZ = None
        if ctx.needs_input_grad[0] or want_g or want_b:
            dZ = torch.empty_like(dY)
            nat.check(lib.hgd_row_epilogue_backward(
                dY.data_ptr(), dY.stride(0), nat.ptr(A), 0 if A is None else A.stride(0),
                nat.ptr(stats), nat.ptr(gamma), n, d, epi, float(slope), int(ln),
                float(out_scale), dZ.data_ptr(), dZ.stride(0), nat.ptr(dgamma), nat.ptr(dbeta),
                nat.ptr(ws), wsb, nat.stream_handle(dev)),
                "hgd_row_epilogue_backward")

        def res_grad(k, s):
            if not ctx.has_res[k] or not ctx.needs_input_grad[3 + k]:
                return None
            return dY if s == 1.0 else dY * s

        return (dZ if ctx.needs_input_grad[0] else None, dgamma, dbeta, res_grad(0, s1),
                res_grad(1, s2), None)


def row_epilogue(Z: torch.Tensor, epilogue: Optional[str] = None, slope: float = 0.0,
                 norm: Optional[torch.nn.LayerNorm] = None, out_scale: float = 1.0,
                 res1: Optional[torch.Tensor] = None, res1_scale: float = 1.0,
                 res2: Optional[torch.Tensor] = None, res2_scale: float = 1.0) -> torch.Tensor:
    """The fused store of :func:`two_hop_fused` applied to an existing [n, d] matrix."""
    epi = _EPI[epilogue]
    d = Z.shape[-1]
    ln = norm is not None
    if (Z.dim() != 2 or not Z.is_cuda or Z.dtype != torch.float32 or not _ln_supported(d)
            or (epi != nat.EPI_NONE and slope < 0)):
        raise ValueError("row_epilogue: needs a 2-D float32 device matrix with d <= 256 "
                         "(d <= 64 when d % 4 != 0) and slope >= 0")
    gamma = norm.weight if ln and norm.weight is not None else None
    beta = norm.bias if ln and norm.bias is not None else None
    cfg = (epi, float(slope), ln, float(norm.eps) if ln else 0.0, float(out_scale),
           float(res1_scale), float(res2_scale))
    return _RowEpilogue.apply(Z, gamma, beta, res1, res2, cfg)


def layer_norm(x: torch.Tensor, norm: torch.nn.LayerNorm) -> torch.Tensor:
    """``norm(x)`` for a LayerNorm over the last dim: hgd_row_epilogue_* on device float32 rows
    that fit one lane group, the library op otherwise."""
    d = x.shape[-1]
    if (x.is_cuda and x.dtype == torch.float32 and tuple(norm.normalized_shape) == (d,)
            and _ln_supported(d) and x.numel() > 0):
        lead = x.shape[:-1]
        return row_epilogue(x.reshape(-1, d), norm=norm).reshape(*lead, d)
    return torch.nn.functional.layer_norm(x, norm.normalized_shape, norm.weight, norm.bias,
                                          norm.eps)


class _ContrastLoss(torch.autograd.Function):
    """hgd_infonce_forward / hgd_infonce_backward (see contrast_loss)."""

    @staticmethod
    def forward(ctx, E1, E2, nodes, temp: float, count=None):
        lib = nat.load()
        dev = E1.device
        E1c = E1 if E1.stride(1) == 1 else E1.contiguous()
        E2c = E2 if E2.stride(1) == 1 else E2.contiguous()
        nodes = nodes.to(device=dev, dtype=torch.int64).contiguous()
        B, d = nodes.numel(), E1.shape[1]
        f = dict(dtype=torch.float32, device=dev)
        P1, P2 = torch.empty((B, d), **f), torch.empty((B, d), **f)
        inv1, inv2, pos = (torch.empty(B, **f) for _ in range(3))
        deno = torch.empty(2 * B, **f)  # [deno; off-diagonal part] (include/hgd.h)
        loss = torch.empty((), **f)
        wsb = lib.hgd_infonce_workspace_size(B, d)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        st = nat.stream_handle(dev)
        if count is None:
            nat.check(lib.hgd_infonce_forward(
                E1c.data_ptr(), E1c.stride(0), E2c.data_ptr(), E2c.stride(0), E1.shape[0],
                nodes.data_ptr(), B, d, float(temp), P1.data_ptr(), P2.data_ptr(),
                inv1.data_ptr(), inv2.data_ptr(), pos.data_ptr(), deno.data_ptr(),
                loss.data_ptr(), ws.data_ptr(), wsb, st), "hgd_infonce_forward")
        else:  # B is the capacity, the live count stays on the device
            nat.check(lib.hgd_infonce_forward_n(
                E1c.data_ptr(), E1c.stride(0), E2c.data_ptr(), E2c.stride(0), E1.shape[0],
                nodes.data_ptr(), B, count.data_ptr(), d, float(temp), P1.data_ptr(),
                P2.data_ptr(), inv1.data_ptr(), inv2.data_ptr(), pos.data_ptr(), deno.data_ptr(),
                loss.data_ptr(), ws.data_ptr(), wsb, st), "hgd_infonce_forward_n")
        ctx.temp = float(temp)
        ctx.shapes = (E1.shape, E2.shape)
        ctx.has_count = count is not None
        ctx.save_for_backward(P1, P2, inv1, inv2, deno, nodes, count)
        return loss

    @staticmethod
    def backward(ctx, g):
        lib = nat.load()
        P1, P2, inv1, inv2, deno, nodes, count = ctx.saved_tensors
        B, d = P1.shape
        dev = P1.device
        g = g.to(dtype=torch.float32).reshape(1).contiguous()
        wsb = lib.hgd_infonce_workspace_size(B, d)
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        st = nat.stream_handle(dev)
        dE1 = dE2 = None
        if ctx.has_count:
            # the scatter into the table gradients runs inside the backward kernel (live rows
            # only); the capacity rows past the count add nothing
            f = dict(dtype=torch.float32, device=dev)
            dE1 = torch.zeros(ctx.shapes[0], **f) if ctx.needs_input_grad[0] else None
            dE2 = torch.zeros(ctx.shapes[1], **f) if ctx.needs_input_grad[1] else None
            if dE1 is None and dE2 is None:
                return None, None, None, None, None
            nat.check(lib.hgd_infonce_backward_n(
                P1.data_ptr(), P2.data_ptr(), inv1.data_ptr(), inv2.data_ptr(), deno.data_ptr(),
                B, count.data_ptr(), d, ctx.temp, g.data_ptr(), nodes.data_ptr(),
                ctx.shapes[0][0], nat.ptr(dE1), d, nat.ptr(dE2), d, ws.data_ptr(), wsb, st),
                "hgd_infonce_backward_n")
            return dE1, dE2, None, None, None
        dX1, dX2 = torch.empty_like(P1), torch.empty_like(P2)
        nat.check(lib.hgd_infonce_backward(
            P1.data_ptr(), P2.data_ptr(), inv1.data_ptr(), inv2.data_ptr(), deno.data_ptr(),
            B, d, ctx.temp, g.data_ptr(), dX1.data_ptr(), dX2.data_ptr(), ws.data_ptr(), wsb,
            st), "hgd_infonce_backward")
        if ctx.needs_input_grad[0]:
            dE1 = torch.zeros(ctx.shapes[0], dtype=torch.float32, device=dev)
            dE1.index_add_(0, nodes, dX1)
        if ctx.needs_input_grad[1]:
            dE2 = torch.zeros(ctx.shapes[1], dtype=torch.float32, device=dev)
            dE2.index_add_(0, nodes, dX2)
        return dE1, dE2, None, None, None


class _ContrastLossLayers(torch.autograd.Function):
    """The user and item contrastLoss terms of every HCCF layer on the halves of the [U + I, d]
    tables (HCCF.py:62-67), with device counts: all 2·L InfoNCE terms as ONE launch per kernel
    (hgd_infonce_forward_group / _backward_group, each term on its row offset of its layer's
    tables), and in the backward ONE zeroed [U + I, d] gradient per table that both of its
    terms' scatters write into — instead of per-term launches, per-half zeroed gradients, the
    slice backward's zeroed full table plus copy, and the adds joining halves and layers.
    Inputs after the scalars: E1 of layer 0, E2 of layer 0, E1 of layer 1, …; the output is
    the sum of the 2·L term losses."""

    @staticmethod
    def forward(ctx, nu, nodes_u, count_u, nodes_i, count_i, temp: float, *tables):
        lib = nat.load()
        L = len(tables) // 2
        dev = tables[0].device
        d = tables[0].shape[1]
        N = tables[0].shape[0]
        halves = []
        for r0, rows, nodes, count in ((0, nu, nodes_u, count_u), (nu, N - nu, nodes_i, count_i)):
            halves.append((r0, rows, nodes.to(device=dev, dtype=torch.int64).contiguous(), count))
        # every term's operands in ONE float buffer and every workspace in ONE byte buffer (an
        # eager step otherwise made ~40 allocator calls here): the term losses first, then per
        # term P1, P2 [B, d], inv1, inv2, pos_logit [B] and deno [2, B], each at a 256-byte
        # boundary
        offs, cur = [], _al64(2 * L)
        for layer in range(L):
            for _r0, _rows, nodes, _c in halves:
                B = nodes.numel()
                o = {}
                for name, size in (("P1", B * d), ("P2", B * d), ("inv1", B), ("inv2", B),
                                   ("pos", B), ("deno", 2 * B)):
                    o[name] = cur
                    cur += _al64(size)
                offs.append(o)
        buf = torch.empty(cur, dtype=torch.float32, device=dev)
        wsbs = [lib.hgd_infonce_workspace_size(h[2].numel(), d) for h in halves]
        wsbuf = torch.empty(max(1, L * sum(_al256(w) for w in wsbs)), dtype=torch.uint8,
                            device=dev)
        fp, wp = buf.data_ptr(), wsbuf.data_ptr()
        terms = (nat.InfonceTerm * (2 * L))()
        keep = []
        for layer in range(L):
            E1c, E2c = tables[2 * layer].contiguous(), tables[2 * layer + 1].contiguous()
            keep += [E1c, E2c]
            for k, (r0, rows, nodes, count) in enumerate(halves):
                o = offs[2 * layer + k]
                t = terms[2 * layer + k]
                off = r0 * d * 4
                t.E1, t.ld1, t.E2, t.ld2 = E1c.data_ptr() + off, d, E2c.data_ptr() + off, d
                t.n_rows, t.nodes, t.capacity, t.batch_count = rows, nodes.data_ptr(), \
                    nodes.numel(), count.data_ptr()
                t.P1, t.P2 = fp + 4 * o["P1"], fp + 4 * o["P2"]
                t.inv_norm1, t.inv_norm2 = fp + 4 * o["inv1"], fp + 4 * o["inv2"]
                t.pos_logit, t.deno = fp + 4 * o["pos"], fp + 4 * o["deno"]
                t.loss = fp + 4 * (2 * layer + k)
                t.workspace, t.workspace_bytes = wp, wsbs[k]
                wp += _al256(wsbs[k])
        nat.check(lib.hgd_infonce_forward_group(terms, 2 * L, d, float(temp),
                                                nat.stream_handle(dev)),
                  "hgd_infonce_forward_group")
        ctx.temp = float(temp)
        ctx.nu, ctx.N, ctx.d, ctx.L, ctx.offs, ctx.wsbs = nu, N, d, L, offs, wsbs
        ctx.save_for_backward(halves[0][2], count_u, halves[1][2], count_i, buf)
        losses = buf[:2 * L]
        return losses.sum() if L > 1 else losses[0] + losses[1]

    @staticmethod
    def backward(ctx, g):
        lib = nat.load()
        nodes_u, count_u, nodes_i, count_i, buf = ctx.saved_tensors
        dev = buf.device
        nu, N, d, L = ctx.nu, ctx.N, ctx.d, ctx.L
        g = g.to(dtype=torch.float32).reshape(1).contiguous()
        f = dict(dtype=torch.float32, device=dev)
        need = ctx.needs_input_grad[6:]
        # the needed gradients as slices of ONE zeroed block (one fill launch, not one per layer)
        n_need = sum(1 for j in range(2 * L) if need[j])
        block = torch.zeros((max(n_need, 1), N, d), **f) if n_need else None
        grads, taken = [], 0
        for j in range(2 * L):
            if need[j]:
                grads.append(block[taken])
                taken += 1
            else:
                grads.append(None)
        none = (None,) * 6
        if all(x is None for x in grads):
            return none + tuple(grads)
        wsbuf = torch.empty(max(1, L * sum(_al256(w) for w in ctx.wsbs)), dtype=torch.uint8,
                            device=dev)
        fp, wp = buf.data_ptr(), wsbuf.data_ptr()
        terms = (nat.InfonceTerm * (2 * L))()
        for layer in range(L):
            dE1, dE2 = grads[2 * layer], grads[2 * layer + 1]
            for k, (r0, rows, nodes, count) in enumerate(((0, nu, nodes_u, count_u),
                                                          (nu, N - nu, nodes_i, count_i))):
                o = ctx.offs[2 * layer + k]
                t = terms[2 * layer + k]
                off = r0 * d * 4
                t.n_rows, t.nodes, t.capacity, t.batch_count = rows, nodes.data_ptr(), \
                    nodes.numel(), count.data_ptr()
                t.P1, t.P2 = fp + 4 * o["P1"], fp + 4 * o["P2"]
                t.inv_norm1, t.inv_norm2 = fp + 4 * o["inv1"], fp + 4 * o["inv2"]
                t.deno = fp + 4 * o["deno"]
                if dE1 is not None:
                    t.dE1, t.ldE1 = dE1.data_ptr() + off, d
                if dE2 is not None:
                    t.dE2, t.ldE2 = dE2.data_ptr() + off, d
                t.workspace, t.workspace_bytes = wp, ctx.wsbs[k]
                wp += _al256(ctx.wsbs[k])
        nat.check(lib.hgd_infonce_backward_group(terms, 2 * L, d, ctx.temp, g.data_ptr(),
                                                 nat.stream_handle(dev)),
                  "hgd_infonce_backward_group")
        return none + tuple(grads)


def _al64(n: int) -> int:
    return -(-int(n) // 64) * 64


def _al256(n: int) -> int:
    return -(-int(n) // 256) * 256


_NCE_MAX_LAYERS = 4  # 2 terms per layer, hgd_infonce_*_group takes up to 8


def _nce_group_ok(embeds1, embeds2, nu, nodes_u, nodes_i, count_u, count_i) -> bool:
    d = embeds1.shape[-1]
    return (count_u is not None and count_i is not None and embeds1.dim() == 2
            and embeds2.shape == embeds1.shape and embeds1.is_cuda
            and embeds1.dtype == torch.float32 and embeds2.dtype == torch.float32
            and d % 16 == 0 and 16 <= d <= 256 and 0 < nu < embeds1.shape[0]
            and nodes_u.numel() > 0 and nodes_i.numel() > 0)


def contrast_loss_layers(embeds1s, embeds2s, nu: int, nodes_u: torch.Tensor,
                         nodes_i: torch.Tensor, temp: float,
                         count_u: Optional[torch.Tensor] = None,
                         count_i: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``Σ_layers contrastLoss(e1[:nu], e2[:nu], nodes_u, temp) + contrastLoss(e1[nu:], e2[nu:],
    nodes_i, temp)`` — HCCF.calcLosses' InfoNCE loop (HCCF.py:62-67) before ``ss_rate`` — as ONE
    op over all layers when the node lists carry device counts (:func:`unique_long_n`), up to
    four layers per launch; otherwise per-layer :func:`contrast_loss_pair` calls."""
    e1s, e2s = list(embeds1s), list(embeds2s)
    if len(e1s) != len(e2s) or not e1s:
        raise ValueError("contrast_loss_layers: one embeds2 per embeds1, at least one layer")
    ok = all(_nce_group_ok(a, b, nu, nodes_u, nodes_i, count_u, count_i) and
             a.shape == e1s[0].shape for a, b in zip(e1s, e2s))
    if not ok:
        total = 0
        for a, b in zip(e1s, e2s):
            total = total + contrast_loss_pair(a, b, nu, nodes_u, nodes_i, temp, count_u, count_i)
        return total
    total = 0
    for c0 in range(0, len(e1s), _NCE_MAX_LAYERS):
        tables = [t for ab in zip(e1s[c0:c0 + _NCE_MAX_LAYERS], e2s[c0:c0 + _NCE_MAX_LAYERS])
                  for t in ab]
        total = total + _ContrastLossLayers.apply(int(nu), nodes_u, count_u, nodes_i, count_i,
                                                  float(temp), *tables)
    return total


def contrast_loss_pair(embeds1: torch.Tensor, embeds2: torch.Tensor, nu: int,
                       nodes_u: torch.Tensor, nodes_i: torch.Tensor, temp: float,
                       count_u: Optional[torch.Tensor] = None,
                       count_i: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``contrastLoss(e1[:nu], e2[:nu], nodes_u, temp) + contrastLoss(e1[nu:], e2[nu:], nodes_i,
    temp)`` (HCCF.py:65-66, util/loss_torch.py:103-110) as one op when both node lists carry
    device counts (:func:`unique_long_n`); otherwise the two :func:`contrast_loss` calls."""
    if not _nce_group_ok(embeds1, embeds2, nu, nodes_u, nodes_i, count_u, count_i):
        return (contrast_loss(embeds1[:nu], embeds2[:nu], nodes_u, temp, count_u)
                + contrast_loss(embeds1[nu:], embeds2[nu:], nodes_i, temp, count_i))
    return _ContrastLossLayers.apply(int(nu), nodes_u, count_u, nodes_i, count_i, float(temp),
                                     embeds1, embeds2)


def contrast_loss(embeds1: torch.Tensor, embeds2: torch.Tensor, nodes: torch.Tensor,
                  temp: float, count: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``contrastLoss(embeds1, embeds2, nodes, temp)`` of util/loss_torch.py:103-110 (InfoNCE over
    the batch rows ``nodes``), fused: only the B batch rows are normalised and the [B, B]
    logits are never materialised. Device float32 tables with d a multiple of 16 up to 256;
    other inputs are rejected (the reference formula is three lines of torch for those)."""
    d = embeds1.shape[-1]
    if (embeds1.dim() != 2 or embeds2.shape != embeds1.shape or not embeds1.is_cuda
            or embeds1.dtype != torch.float32 or embeds2.dtype != torch.float32
            or d % 16 != 0 or not 16 <= d <= 256):
        raise ValueError("contrast_loss: needs two float32 device tables [N, d] with d a "
                         "multiple of 16 in [16, 256]")
    if nodes.numel() == 0:
        raise ValueError("contrast_loss: empty batch")
    n = embeds1.shape[0]
    if count is not None:
        # capacity-sized node list with its live count on the device (unique_long_n): no bounds
        # read to the host — the kernels wrap live ids like torch indexing (and clamp them),
        # skip the rows past the count and scatter the gradient rows themselves
        return _ContrastLoss.apply(embeds1, embeds2, nodes, float(temp), count)
    # torch indexing semantics (negative ids wrap; HCCF passes torch.unique(emb.long()), which
    # holds -1 / 0 / 1); out of range raises like embeds[nodes] would
    rng = getattr(nodes, "_hgd_range", None)  # set by unique_long: no device read needed
    if rng is not None and rng[2] != nodes._version:
        rng = None  # modified in place since
    bad = (rng[0] < -n or rng[1] >= n) if rng is not None else bool(
        ((nodes < -n) | (nodes >= n)).any())
    if bad:
        raise IndexError(f"contrast_loss: node index out of range for a table of {n} rows")
    nodes = torch.where(nodes < 0, nodes + n, nodes)  # the gradient scatter needs [0, n)
    return _ContrastLoss.apply(embeds1, embeds2, nodes, float(temp))


def unique_long(x: torch.Tensor) -> torch.Tensor:
    """``torch.unique(x.long())`` (sorted, int64) of a device float32 or int64 tensor — the node
    list HCCF's loss builds every step, ``torch.unique(ancs.long())`` (model/graph/HCCF.py:65-66).
    Floats truncate toward zero like ``Tensor.long()``. Range-bitmap kernels (hgd_unique_*);
    a key range beyond 2^24 takes the device radix-sort path. One device→host read, as
    torch.unique: the count together with the key range, which is attached to the result
    (``_hgd_range``) so that :func:`contrast_loss` checks its bounds without another read."""
    if not x.is_cuda or x.dtype not in (torch.float32, torch.int64):
        raise ValueError("unique_long: needs a float32 or int64 device tensor")
    x = x.detach().contiguous().view(-1)
    n = x.numel()
    lib = nat.load()
    dev = x.device
    out = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    wsb = lib.hgd_unique_workspace_size(n)
    # [count | pad | workspace]: the workspace starts with the kernels' (min, max) state, so one
    # 272-byte copy returns the count and the range
    buf = torch.empty(_UQ_HEAD + max(wsb, 1), dtype=torch.uint8, device=dev)
    st = nat.stream_handle(dev)
    f = x.dtype == torch.float32
    fast = lib.hgd_unique_trunc_f32 if f else lib.hgd_unique_i64
    base = buf.data_ptr()
    nat.check(fast(x.data_ptr(), n, out.data_ptr(), base, base + _UQ_HEAD, wsb, st),
              "hgd_unique")
    head = buf[:_UQ_HEAD + 16].cpu().view(torch.int64)
    k = int(head[0])
    if k < 0:  # key range beyond the bitmap
        slow = lib.hgd_unique_sort_trunc_f32 if f else lib.hgd_unique_sort_i64
        nat.check(slow(x.data_ptr(), n, out.data_ptr(), base, base + _UQ_HEAD, wsb, st),
                  "hgd_unique_sort")
        k = int(buf[:8].cpu().view(torch.int64)[0])
        return out[:k]
    res = out[:k]
    if k:
        res._hgd_range = (int(head[_UQ_HEAD // 8]), int(head[_UQ_HEAD // 8 + 1]), res._version)
    return res


_UQ_HEAD = 256  # bytes before the unique workspace (count at 0; 256-byte aligned workspace)


def unique_long_n(x: torch.Tensor, n_rows: Optional[int] = None
                  ) -> Tuple[torch.Tensor, torch.Tensor]:
    """:func:`unique_long` without the device→host read, for a captured training step:
    ``(nodes, count)`` with ``nodes`` int64 capacity-sized, its first ``count[0]`` entries the
    sorted unique values of ``x.long()`` and the rest 0, ``count`` an int64 [1] device tensor
    (hgd_unique_dev_group: the range bitmap with the far keys merged on the device, so no host
    decision). Feed both to :func:`contrast_loss`. The capacity is x.numel(), or at most
    2·n_rows when the ids index a table of ``n_rows`` rows: valid torch indices lie in
    [-n_rows, n_rows), so no valid list is longer (HCCF's ``torch.unique(anchor_emb.long())``,
    HCCF.py:65-66, reads a [B, d] table of a handful of distinct ints — B·d capacity made every
    InfoNCE buffer and grid that size); a list of out-of-range ids is cut to the capacity, and
    such ids are the caller's error either way (the reference's gather raises)."""
    return unique_long_n_group([x], [n_rows])[0]


def unique_long_n_group(xs, n_rows=None) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """:func:`unique_long_n` of several tensors in one launch per kernel (up to four per group;
    HCCF's anchor and positive lists, HCCF.py:65-66): ``[(nodes, count)]`` in order, each
    exactly as :func:`unique_long_n` gives it; ``n_rows`` a list of table sizes (or None)."""
    xs = list(xs)
    n_rows = list(n_rows) if n_rows is not None else [None] * len(xs)
    if len(n_rows) != len(xs) or not xs:
        raise ValueError("unique_long_n_group: one n_rows entry per tensor, at least one tensor")
    lib = nat.load()
    res = []
    for c0 in range(0, len(xs), 4):
        chunk = list(zip(xs[c0:c0 + 4], n_rows[c0:c0 + 4]))
        jobs = (nat.UniqueJob * len(chunk))()
        keep = []
        dev = None
        for q, (x, nr) in enumerate(chunk):
            if not x.is_cuda or x.dtype not in (torch.float32, torch.int64):
                raise ValueError("unique_long_n: needs a float32 or int64 device tensor")
            x = x.detach().contiguous().view(-1)
            n = x.numel()
            if n == 0:
                raise ValueError("unique_long_n: empty input")
            dev = x.device
            out = torch.empty(n, dtype=torch.int64, device=dev)
            count = torch.empty(1, dtype=torch.int64, device=dev)
            wsb = lib.hgd_unique_workspace_size(n)
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            cap = n if nr is None else max(1, min(n, 2 * int(nr)))
            j = jobs[q]
            if x.dtype == torch.float32:
                j.x_f32 = x.data_ptr()
            else:
                j.x_i64 = x.data_ptr()
            j.n, j.capacity = n, cap
            j.out, j.n_out = out.data_ptr(), count.data_ptr()
            j.workspace, j.workspace_bytes = ws.data_ptr(), wsb
            keep += [x, ws]
            res.append((out[:cap] if cap < n else out, count))
        nat.check(lib.hgd_unique_dev_group(jobs, len(chunk), nat.stream_handle(dev)),
                  "hgd_unique_dev_group")
    return res


def _mm_ok(H: torch.Tensor, X: torch.Tensor) -> bool:
    n, K = H.shape
    d = X.shape[1]
    return (H.is_cuda and X.is_cuda and H.dtype == torch.float32 and X.dtype == torch.float32
            and K % 16 == 0 and d % 16 == 0 and 16 <= K <= 128 and 16 <= d <= 128
            and X.shape[0] == n)


def _tn(A: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """Aᵀ·B for tall A [n, m], B [n, k] (split-K hgd_linear_backward_weight)."""
    lib = nat.load()
    n, m = A.shape
    k = B.shape[1]
    C = torch.empty((m, k), dtype=torch.float32, device=A.device)
    wsb = lib.hgd_linear_backward_weight_workspace_size(n, m, k)
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=A.device)
    nat.check(lib.hgd_linear_backward_weight(
        A.data_ptr(), A.stride(0), None, 0, B.data_ptr(), B.stride(0), n, m, k, C.data_ptr(),
        None, ws.data_ptr(), wsb, nat.stream_handle(A.device)),
        "hgd_linear_backward_weight")
    return C


def _nn(A: torch.Tensor, M: torch.Tensor) -> torch.Tensor:
    """A·M for tall A [n, m] and small M [m, k] (hgd_linear_backward_data)."""
    lib = nat.load()
    n, m = A.shape
    k = M.shape[1]
    Y = torch.empty((n, k), dtype=torch.float32, device=A.device)
    nat.check(lib.hgd_linear_backward_data(
        A.data_ptr(), A.stride(0), None, 0, n, m, M.data_ptr(), M.stride(0), k, Y.data_ptr(),
        Y.stride(0), nat.stream_handle(A.device)), "hgd_linear_backward_data")
    return Y


def _nt(A: torch.Tensor, M: torch.Tensor) -> torch.Tensor:
    """A·Mᵀ for tall A [n, k] and small M [m, k] (hgd_linear_forward without bias)."""
    lib = nat.load()
    n, k = A.shape
    m = M.shape[0]
    Y = torch.empty((n, m), dtype=torch.float32, device=A.device)
    nat.check(lib.hgd_linear_forward(A.data_ptr(), A.stride(0), n, k, M.data_ptr(), M.stride(0),
                                     m, None, 0, Y.data_ptr(), Y.stride(0),
                                     nat.stream_handle(A.device)),
              "hgd_linear_forward")
    return Y


class _DenseTwoHop(torch.autograd.Function):
    """``H·(Hᵀ·X)`` with H [n, K] dense (HGNNLayer, HCCF.py:201-211) on the skinny MFMA kernels:
    Hᵀ·X is a split-K product, H·M a row GEMM; the backward reuses the same three kernels."""

    @staticmethod
    def forward(ctx, H, X):
        H = H.contiguous()
        X = X.contiguous()
        M = _tn(H, X)             # [K, d] = Hᵀ·X
        Y = _nn(H, M)             # [n, d] = H·M
        ctx.save_for_backward(H, X, M)
        return Y

    @staticmethod
    def backward(ctx, dY):
        H, X, M = ctx.saved_tensors
        dY = dY.contiguous()
        dM = _tn(H, dY)           # Hᵀ·dY
        dH = dX = None
        if ctx.needs_input_grad[1]:
            dX = _nn(H, dM)       # H·dM
        if ctx.needs_input_grad[0]:
            dH = _nt(dY, M)       # dY·Mᵀ
            dH += _nt(X, dM)      # + X·dMᵀ
        return dH, dX


def dense_two_hop(H: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """``torch.mm(H, torch.mm(H.T, X))`` for the learned dense hypergraph; features (K, d)
    multiples of 16 up to 128 run on hgd_linear_*, others on the library GEMM."""
    if not _mm_ok(H, X):
        return torch.mm(H, torch.mm(H.T, X))
    return _DenseTwoHop.apply(H, X)


def _rows_desc(A, B, bsk, bsn, K, N, Y, accumulate=False):
    d = nat.GemmRowsDesc()
    d.A, d.lda = A.data_ptr(), A.stride(0)
    d.B, d.bsk, d.bsn = B.data_ptr(), bsk, bsn
    d.accumulate = 1 if accumulate else 0
    d.Y, d.ldy = Y.data_ptr(), Y.stride(0)
    d.rows, d.K, d.N = A.shape[0], K, N
    return d


def _gemm_rows(descs, device):
    arr = (nat.GemmRowsDesc * len(descs))(*descs)
    nat.check(nat.load().hgd_gemm_rows(arr, len(descs),
                                       nat.stream_handle(device)),
              "hgd_gemm_rows")


def _gemm_tn_pair(pairs, device):
    """[Aᵢᵀ·Bᵢ] for (A [n_i, m], B [n_i, k]) pairs in one grouped split-K launch."""
    lib = nat.load()
    descs, outs = [], []
    for A, B in pairs:
        C = torch.empty((A.shape[1], B.shape[1]), dtype=torch.float32, device=device)
        d = nat.GemmTnDesc()
        d.A, d.lda = A.data_ptr(), A.stride(0)
        d.B, d.ldb = B.data_ptr(), B.stride(0)
        d.rows, d.M, d.N = A.shape[0], A.shape[1], B.shape[1]
        d.C = C.data_ptr()
        descs.append(d)
        outs.append(C)
    arr = (nat.GemmTnDesc * len(descs))(*descs)
    wsb = lib.hgd_gemm_tn_workspace_size(arr, len(descs))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=device)
    nat.check(lib.hgd_gemm_tn(arr, len(descs), ws.data_ptr(), wsb,
                              nat.stream_handle(device)), "hgd_gemm_tn")
    return outs


class _DenseTwoHopPair(torch.autograd.Function):
    """HCCF's two HGNNLayer calls of a layer (HCCF.py:184-186, 201-211) on the halves of one
    [U + I, d] table: ``cat([H_u·(H_uᵀ·X_u), H_i·(H_iᵀ·X_i)])`` with every product a grouped
    launch over both halves (hgd_gemm_tn / hgd_gemm_rows) and the output written in place — no
    split / cat of the table forward or backward."""

    @staticmethod
    def forward(ctx, H_u, H_i, X, nu):
        H_u, H_i, X = H_u.contiguous(), H_i.contiguous(), X.contiguous()
        dev = X.device
        K, d = H_u.shape[1], X.shape[1]
        X_u, X_i = X[:nu], X[nu:]
        M_u, M_i = _gemm_tn_pair([(H_u, X_u), (H_i, X_i)], dev)
        Y = torch.empty_like(X)
        _gemm_rows([_rows_desc(H_u, M_u, d, 1, K, d, Y[:nu]),
                    _rows_desc(H_i, M_i, d, 1, K, d, Y[nu:])], dev)
        ctx.save_for_backward(H_u, H_i, X, M_u, M_i)
        ctx.nu = nu
        return Y

    @staticmethod
    def backward(ctx, dY):
        H_u, H_i, X, M_u, M_i = ctx.saved_tensors
        nu = ctx.nu
        dev = X.device
        K, d = H_u.shape[1], X.shape[1]
        dY = dY.contiguous()
        dY_u, dY_i = dY[:nu], dY[nu:]
        dM_u, dM_i = _gemm_tn_pair([(H_u, dY_u), (H_i, dY_i)], dev)
        dX = None
        if ctx.needs_input_grad[2]:
            dX = torch.empty_like(X)
            _gemm_rows([_rows_desc(H_u, dM_u, d, 1, K, d, dX[:nu]),
                        _rows_desc(H_i, dM_i, d, 1, K, d, dX[nu:])], dev)
        dH_u = dH_i = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            # dH = dY·Mᵀ + X·dMᵀ: Bm[k][n] = M[n][k] (bsk 1, bsn d), the second accumulated
            dH_u = torch.empty_like(H_u)
            dH_i = torch.empty_like(H_i)
            _gemm_rows([_rows_desc(dY_u, M_u, 1, d, d, K, dH_u),
                        _rows_desc(dY_i, M_i, 1, d, d, K, dH_i)], dev)
            _gemm_rows([_rows_desc(X[:nu], dM_u, 1, d, d, K, dH_u, accumulate=True),
                        _rows_desc(X[nu:], dM_i, 1, d, d, K, dH_i, accumulate=True)], dev)
        return dH_u, dH_i, dX, None


def dense_two_hop_pair(H_u: torch.Tensor, H_i: torch.Tensor, X: torch.Tensor,
                       nu: int) -> torch.Tensor:
    """``torch.cat([H_u·(H_uᵀ·X[:nu]), H_i·(H_iᵀ·X[nu:])])`` (HCCF's user and item HGNNLayer of
    one layer); falls back to two :func:`dense_two_hop` calls outside the kernels' shapes."""
    if not (_mm_ok(H_u, X[:nu]) and _mm_ok(H_i, X[nu:]) and H_u.shape[1] == H_i.shape[1]):
        return torch.cat([dense_two_hop(H_u, X[:nu]), dense_two_hop(H_i, X[nu:])], 0)
    return _DenseTwoHopPair.apply(H_u, H_i, X, int(nu))


def _res_epilogue(res: Optional[torch.Tensor], act_out: Optional[torch.Tensor] = None,
                  res2: Optional[torch.Tensor] = None, sum_res: Optional[torch.Tensor] = None,
                  sum_out: Optional[torch.Tensor] = None):
    """hgd_row_epilogue of a plain hop whose store adds ``res`` and ``res2`` (either may be the
    output itself), keeps the bare hop in ``act_out`` and writes ``sum_out = Y + sum_res``."""
    def ld(t):
        return 0 if t is None else t.stride(0)
    return nat.RowEpilogue(
        act=nat.EPI_NONE, slope=0.0, layer_norm=0, ln_eps=0.0, ln_gamma=None, ln_beta=None,
        out_scale=1.0, res1=nat.ptr(res), ld_res1=ld(res), res1_scale=1.0,
        res2=nat.ptr(res2), ld_res2=ld(res2), res2_scale=1.0, act_out=nat.ptr(act_out),
        ld_act=ld(act_out), stats=None, sum_res=nat.ptr(sum_res), ld_sum_res=ld(sum_res),
        sum_out=nat.ptr(sum_out), ld_sum_out=ld(sum_out))


class _HCCFLayers(torch.autograd.Function):
    """HCCF's layer loop (model/graph/HCCF.py:173-191) as one op, so that none of its sums is a
    separate kernel:

    * forward, layer k: the learned-hypergraph pair ``hgnn_k = [H_u·(H_uᵀ·h_u); H_i·(H_iᵀ·h_i)]``
      (grouped skinny MFMA products), then ONE GCN hop over the (edge-dropped) adjacency whose
      store writes ``gcn_k = A·h_k`` (act_out) and ``h_{k+1} = gcn_k + hgnn_k`` (res1) — the
      reference's ``hidden += [gcn_emb + hgnn_hidden[-1]]``; the hidden tables are slices of one
      [L+1, N, d] buffer and ``sum(hidden)`` is one slice-sum pass (hgd_sum_slices, same order);
    * backward, layer k: the grouped row product H·dM, then ``dh_k = dE + Aᵀ·dgcn_k + H·dM``
      as one backward hop whose store adds both, and writes, in the same pass, the next layer's
      ``dhgnn_{k-1} = dh_k + dInfoNCE_{k-1}`` (the row epilogue's sum_out). Autograd's
      accumulation adds (≈ 2 per layer), the layer adds and the L sum adds of the per-layer
      graph disappear.

    Inputs: the per-layer adjacency incidences (plain, compacted-dropped or masked views),
    user / item embedding tables, and the per-layer dropped hypergraphs H_u [nu, K], H_i
    [ni, K]. Outputs: E = sum(hidden) [N, d], gcn_0..gcn_{L-1}, hgnn_0..hgnn_{L-1}."""

    @staticmethod
    def forward(ctx, adjs, nu, user_emb, item_emb, *Hs):
        L = len(adjs)
        dev = user_emb.device
        N = user_emb.shape[0] + item_emb.shape[0]
        d = user_emb.shape[1]
        K = Hs[0].shape[1]
        f = dict(dtype=torch.float32, device=dev)
        hid = torch.empty((L + 1, N, d), **f)
        torch.cat([user_emb, item_emb], 0, out=hid[0])
        Hs = [H.contiguous() for H in Hs]
        gcn, hgnn, Ms = [], [], []
        for k in range(L):
            H_u, H_i = Hs[2 * k], Hs[2 * k + 1]
            h = hid[k]
            M_u, M_i = _gemm_tn_pair([(H_u, h[:nu]), (H_i, h[nu:])], dev)
            Hh = torch.empty((N, d), **f)
            _gemm_rows([_rows_desc(H_u, M_u, d, 1, K, d, Hh[:nu]),
                        _rows_desc(H_i, M_i, d, 1, K, d, Hh[nu:])], dev)
            G = torch.empty((N, d), **f)
            inc = adjs[k]
            spmm_csr(inc.csr, h, val=inc.val, ex=_res_epilogue(Hh, act_out=G), out=hid[k + 1])
            gcn.append(G)
            hgnn.append(Hh)
            Ms += [M_u, M_i]
        E = torch.empty((N, d), **f)
        nat.check(nat.load().hgd_sum_slices(hid.data_ptr(), L + 1, N * d, N * d, E.data_ptr(),
                                            nat.stream_handle(dev)),
                  "hgd_sum_slices")
        ctx.adjs, ctx.nu, ctx.L, ctx.K = adjs, nu, L, K
        ctx.save_for_backward(hid, *Hs, *Ms)
        ctx.set_materialize_grads(False)
        return (E, *gcn, *hgnn)

    @staticmethod
    def backward(ctx, dE, *grads):
        L, nu, K = ctx.L, ctx.nu, ctx.K
        saved = ctx.saved_tensors
        hid = saved[0]
        Hs = saved[1:1 + 2 * L]
        Ms = saved[1 + 2 * L:]
        dgcn, dhgnn = grads[:L], grads[L:]
        _, N, d = hid.shape
        dev = hid.device
        f = dict(dtype=torch.float32, device=dev)
        if dE is not None:
            dE = dE.contiguous()
        dh = dE if dE is not None else torch.zeros((N, d), **f)
        dHh = dh if dhgnn[L - 1] is None else dh + dhgnn[L - 1].contiguous()
        want_emb = ctx.needs_input_grad[2] or ctx.needs_input_grad[3]
        dHs = [None] * (2 * L)
        for k in reversed(range(L)):
            H_u, H_i = Hs[2 * k], Hs[2 * k + 1]
            M_u, M_i = Ms[2 * k], Ms[2 * k + 1]
            h = hid[k]
            dG = dh if dgcn[k] is None else dh + dgcn[k]
            dM_u, dM_i = _gemm_tn_pair([(H_u, dHh[:nu]), (H_i, dHh[nu:])], dev)
            if ctx.needs_input_grad[4 + 2 * k] or ctx.needs_input_grad[5 + 2 * k]:
                # dH = dhgnn·Mᵀ + h·dMᵀ (Bm[k][n] = M[n][k]: bsk 1, bsn d), the second accumulated
                dH_u, dH_i = torch.empty_like(H_u), torch.empty_like(H_i)
                _gemm_rows([_rows_desc(dHh[:nu], M_u, 1, d, d, K, dH_u),
                            _rows_desc(dHh[nu:], M_i, 1, d, d, K, dH_i)], dev)
                _gemm_rows([_rows_desc(h[:nu], dM_u, 1, d, d, K, dH_u, accumulate=True),
                            _rows_desc(h[nu:], dM_i, 1, d, d, K, dH_i, accumulate=True)], dev)
                dHs[2 * k], dHs[2 * k + 1] = dH_u, dH_i
            if k == 0 and not want_emb:
                break
            inc = ctx.adjs[k]
            # H·dM first (plain grouped store), then the backward hop adds it and dE in its
            # store (res2 = its own output row, read before written) and writes the next
            # layer's dhgnn = dh + dInfoNCE as a second output
            dh_new = torch.empty((N, d), **f)
            _gemm_rows([_rows_desc(H_u, dM_u, d, 1, K, d, dh_new[:nu]),
                        _rows_desc(H_i, dM_i, d, 1, K, d, dh_new[nu:])], dev)
            nxt = dhgnn[k - 1].contiguous() if k > 0 and dhgnn[k - 1] is not None else None
            dHh_new = torch.empty((N, d), **f) if nxt is not None else None
            spmm_csr(inc.csc, dG.contiguous(), val=inc.val_t,
                     ex=_res_epilogue(dE, res2=dh_new, sum_res=nxt, sum_out=dHh_new),
                     out=dh_new)
            dh = dh_new
            dHh = dHh_new if nxt is not None else dh_new
        d_u = dh[:nu] if ctx.needs_input_grad[2] else None
        d_i = dh[nu:] if ctx.needs_input_grad[3] else None
        return (None, None, d_u, d_i, *dHs)


def hccf_layers_supported(user_emb: torch.Tensor, item_emb: torch.Tensor,
                          H: torch.Tensor) -> bool:
    """Shapes :func:`hccf_layers` runs (the skinny MFMA products and float4 slice sums)."""
    d = user_emb.shape[1]
    return (user_emb.is_cuda and item_emb.is_cuda and H.is_cuda
            and user_emb.dtype == item_emb.dtype == H.dtype == torch.float32
            and item_emb.shape[1] == d and d % 16 == 0 and 16 <= d <= 128
            and H.shape[1] % 16 == 0 and 16 <= H.shape[1] <= 128
            and user_emb.shape[0] > 0 and item_emb.shape[0] > 0)


def hccf_layers(adjs, user_emb: torch.Tensor, item_emb: torch.Tensor, hypers_u, hypers_i):
    """HCCF's propagation (model/graph/HCCF.py:173-191) over per-layer adjacencies ``adjs``
    (Incidences of ``edgeDropper(sparse_norm_adj)``) and per-layer dropped hypergraphs:
    returns ``(sum(hidden), gcn_hidden, hgnn_hidden)`` (see :class:`_HCCFLayers`)."""
    L = len(adjs)
    nu, N = user_emb.shape[0], user_emb.shape[0] + item_emb.shape[0]
    for inc in adjs:
        if inc.n_rows != N or inc.n_cols != N:
            raise ValueError(f"hccf_layers: adjacency {inc.n_rows}x{inc.n_cols}, tables have {N} rows")
    Hs = []
    for Hu, Hi in zip(hypers_u, hypers_i):
        Hs += [Hu, Hi]
    out = _HCCFLayers.apply(list(adjs), int(nu), user_emb, item_emb, *Hs)
    return out[0], list(out[1:1 + L]), list(out[1 + L:])


class _TableProjections(torch.autograd.Function):
    """HCCF's learned hypergraphs ``[E_u·W_u, E_i·W_i]`` (HCCF.py:178-179; E [n, d], W [d, K]
    as the parameters are stored) in grouped launches: the forward one row-GEMM launch for both
    tables (W read in place — no transposed copy), the backward one row-GEMM launch for both
    dE = dH·Wᵀ and one split-K launch for both dW = Eᵀ·dH, written in W's own layout. The
    ``F.linear(E, W.t())`` form cost a contiguous copy of each Wᵀ, two launches per table each
    way and a transposing copy of each weight gradient."""

    @staticmethod
    def forward(ctx, *EW):
        T = len(EW) // 2
        Es, Ws = [e.contiguous() for e in EW[:T]], [w.contiguous() for w in EW[T:]]
        dev = Es[0].device
        outs, descs = [], []
        for E, W in zip(Es, Ws):
            Y = torch.empty((E.shape[0], W.shape[1]), dtype=torch.float32, device=dev)
            descs.append(_rows_desc(E, W, W.stride(0), 1, E.shape[1], W.shape[1], Y))
            outs.append(Y)
        _gemm_rows(descs, dev)
        ctx.save_for_backward(*Es, *Ws)
        ctx.T = T
        return tuple(outs)

    @staticmethod
    def backward(ctx, *dHs):
        T = ctx.T
        saved = ctx.saved_tensors
        Es, Ws = saved[:T], saved[T:]
        dev = Es[0].device
        dHs = [torch.zeros((E.shape[0], W.shape[1]), dtype=torch.float32, device=dev)
               if g is None else g.contiguous() for g, E, W in zip(dHs, Es, Ws)]
        dEs = [None] * T
        if any(ctx.needs_input_grad[:T]):
            descs = []
            for t in range(T):
                dE = torch.empty_like(Es[t])
                W = Ws[t]
                descs.append(_rows_desc(dHs[t], W, 1, W.stride(0), W.shape[1], W.shape[0], dE))
                dEs[t] = dE
            _gemm_rows(descs, dev)
        dWs = [None] * T
        if any(ctx.needs_input_grad[T:]):
            dWs = _gemm_tn_pair(list(zip(Es, dHs)), dev)
        return (*dEs, *dWs)


def table_projections(tables, weights):
    """``[E @ W for E, W in zip(tables, weights)]`` (HCCF's E_u·W_u, E_i·W_i) as one grouped op
    (:class:`_TableProjections`) for device fp32 operands whose feature sizes are multiples of 16
    up to 128 (the row GEMM's K and N); ``torch.mm`` otherwise."""
    ok = all(E.is_cuda and W.is_cuda and E.dtype == W.dtype == torch.float32 and E.dim() == 2
             and W.dim() == 2 and E.shape[1] == W.shape[0] and E.shape[0] > 0
             and all(x % 16 == 0 and 16 <= x <= 128 for x in W.shape)
             for E, W in zip(tables, weights))
    if not ok or len(tables) != len(weights) or not 1 <= len(tables) <= 4:
        return [torch.mm(E, W) for E, W in zip(tables, weights)]
    return list(_TableProjections.apply(*tables, *weights))


class _HyperDropouts(torch.autograd.Function):
    """``nn.Dropout(p)`` applied to each of ``tables`` once per layer, in the reference's call
    order (HCCF.py:182-186: layer 0's user then item table, then layer 1's, …: the device
    generator's stream), as ONE autograd node: the forward is torch's own ``native_dropout`` per
    call (the same masks and outputs as the module), the backward one ``hgd_masked_scale_sum``
    launch for all tables — per table the L masked gradients summed as autograd sums L separate
    dropout nodes (the last call's first, each ((float)mask · dy) · scale), where the separate
    nodes cost 2L masked-scale kernels and 2(L − 1) accumulation adds per step."""

    @staticmethod
    def forward(ctx, p, L, *tables):
        outs, masks = [], []
        for _ in range(L):
            for t in tables:
                o, m = torch.native_dropout(t, p, True)
                outs.append(o)
                masks.append(m)
        ctx.save_for_backward(*masks)
        ctx.p, ctx.L, ctx.T = p, L, len(tables)
        ctx.shapes = [t.shape for t in tables]
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        masks = ctx.saved_tensors
        L, T = ctx.L, ctx.T
        dev = masks[0].device
        scale = float(torch.tensor(1.0 / (1.0 - ctx.p), dtype=torch.float32))
        outs, jobs, keep = [], [], []
        for t in range(T):
            out = torch.empty(ctx.shapes[t], dtype=torch.float32, device=dev)
            job = nat.MaskedSum()
            live = 0
            for k in range(L):
                g = grads[k * T + t]
                if g is None:
                    g = torch.zeros(ctx.shapes[t], dtype=torch.float32, device=dev)
                g = g.contiguous()
                keep.append(g)
                job.dy[k] = g.data_ptr()
                job.mask[k] = masks[k * T + t].data_ptr()
                live += 1
            job.out, job.n, job.count, job.scale = out.data_ptr(), out.numel(), live, scale
            jobs.append(job)
            outs.append(out)
        arr = (nat.MaskedSum * len(jobs))(*jobs)
        nat.check(nat.load().hgd_masked_scale_sum(arr, len(jobs), nat.stream_handle(dev)),
                  "hgd_masked_scale_sum")
        return (None, None, *outs)


def hyper_dropouts(tables, p: float, L: int):
    """``[[dropout(t) for t in tables] for _ in range(L)]`` with HCCF's module order and masks
    (see :class:`_HyperDropouts`); falls back to the plain calls outside 0 < p < 1, for tables
    that are not device fp32 with 16-byte-aligned rows, or for more than 8 layers / 4 tables."""
    ok = (0.0 < p < 1.0 and 1 <= L <= 8 and 1 <= len(tables) <= 4
          and all(t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()
                  and t.data_ptr() % 16 == 0 and t.numel() % 4 == 0 for t in tables))
    if not ok:
        return [[F.dropout(t, p, True) for t in tables] for _ in range(L)]
    outs = _HyperDropouts.apply(float(p), int(L), *tables)
    T = len(tables)
    return [list(outs[k * T:(k + 1) * T]) for k in range(L)]


_BPR_BAD = {}


def _bpr_bad_word(dev: torch.device) -> torch.Tensor:
    """The per-device int32 word every fused BPR forward adds its out-of-range id count to (a
    fixed address, so captured steps keep counting into it)."""
    key = (dev.type, dev.index if dev.index is not None else torch.cuda.current_device())
    w = _BPR_BAD.get(key)
    if w is None:
        w = _BPR_BAD[key] = torch.zeros(1, dtype=torch.int32, device=dev)
    return w


def bpr_index_errors(dev: torch.device, reset: bool = True) -> int:
    """Batch rows with an out-of-range uid / pid / nid seen by :func:`bpr_loss_rows` on ``dev``
    since the last reset (one device→host read). The kernels clamp such ids where the
    reference's ``E[idx]`` gather raises (HCCF.py:84-86); the training loops call this once per
    epoch and raise IndexError on a non-zero count."""
    w = _bpr_bad_word(dev)
    n = int(w.item())
    if reset and n:
        w.zero_()
    return n


class _BPRTable(torch.autograd.Function):
    """bpr_loss(E[uid], E[nu + pid], E[nu + nid]) (util/loss_torch.py:5-9) on one [N, d] table
    (hgd_bpr_forward / hgd_bpr_backward); also returns the gathered anchor and positive rows
    (non-differentiable: HCCF takes its InfoNCE node lists from them, HCCF.py:65-66)."""

    @staticmethod
    def forward(ctx, E, nu, uid, pid, nid):
        lib = nat.load()
        dev = E.device
        N, d = E.shape
        B = uid.numel()
        f = dict(dtype=torch.float32, device=dev)
        anc, pos = torch.empty((B, d), **f), torch.empty((B, d), **f)
        coef, loss = torch.empty(B, **f), torch.empty((), **f)
        wsb = lib.hgd_bpr_workspace_size(B, N)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        nat.check(lib.hgd_bpr_forward(
            E.data_ptr(), E.stride(0), nu, N - nu, d, uid.data_ptr(), pid.data_ptr(),
            nid.data_ptr(), B, anc.data_ptr(), pos.data_ptr(), coef.data_ptr(), loss.data_ptr(),
            _bpr_bad_word(dev).data_ptr(), ws.data_ptr(), wsb, nat.stream_handle(dev)),
            "hgd_bpr_forward")
        ctx.nu = nu
        ctx.save_for_backward(E, uid, pid, nid, coef)
        ctx.mark_non_differentiable(anc, pos)
        return loss, anc, pos

    @staticmethod
    def backward(ctx, g, _g_anc, _g_pos):
        E, uid, pid, nid, coef = ctx.saved_tensors
        lib = nat.load()
        dev = E.device
        N, d = E.shape
        B = uid.numel()
        g = g.to(dtype=torch.float32).reshape(1).contiguous()
        dE = torch.empty_like(E)
        wsb = lib.hgd_bpr_workspace_size(B, N)
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        nat.check(lib.hgd_bpr_backward(
            E.data_ptr(), E.stride(0), ctx.nu, N - ctx.nu, d, uid.data_ptr(), pid.data_ptr(),
            nid.data_ptr(), B, coef.data_ptr(), g.data_ptr(), dE.data_ptr(), dE.stride(0),
            ws.data_ptr(), wsb, nat.stream_handle(dev)), "hgd_bpr_backward")
        return dE, None, None, None, None


def _table_of(user_emb: torch.Tensor, item_emb: torch.Tensor) -> Optional[torch.Tensor]:
    """The [nu + ni, d] table whose row blocks ``user_emb`` / ``item_emb`` are (the split of an
    encoder's layer sum, HCCF.py:189-190), or None."""
    base = user_emb._base
    if base is None or item_emb._base is not base or base.dim() != 2 or not base.is_contiguous():
        return None
    nu, d = user_emb.shape
    if (base.shape != (nu + item_emb.shape[0], d) or user_emb.data_ptr() != base.data_ptr()
            or item_emb.data_ptr() != base.data_ptr() + nu * d * base.element_size()
            or user_emb.stride() != base.stride() or item_emb.stride() != base.stride()):
        return None
    return base


def bpr_loss_rows(user_emb: torch.Tensor, item_emb: torch.Tensor, uid: torch.Tensor,
                  pid: torch.Tensor, nid: torch.Tensor):
    """``bpr_loss(user_emb[uid], item_emb[pid], item_emb[nid])`` (util/loss_torch.py:5-9 on the
    gathers of HCCF.py:84-86) → ``(loss, anchor_rows, positive_rows)``. When both tables are the
    row blocks of one device table (an encoder's split layer sum) it is one fused op
    (:class:`_BPRTable`: two kernels forward, three backward, deterministic, the table gradient
    written whole — no index_put sorts, no split/cat); otherwise the reference's torch ops."""
    E = _table_of(user_emb, item_emb)
    d = user_emb.shape[1]
    if (E is not None and E.is_cuda and E.dtype == torch.float32 and d % 4 == 0 and d <= 256
            and uid.numel() > 0 and uid.numel() == pid.numel() == nid.numel()
            and E.data_ptr() % 16 == 0):
        idx = [t.to(device=E.device, dtype=torch.int64).contiguous() for t in (uid, pid, nid)]
        return _BPRTable.apply(E, int(user_emb.shape[0]), *idx)
    anc, pos, neg = user_emb[uid], item_emb[pid], item_emb[nid]
    pos_score = torch.mul(anc, pos).sum(dim=1)
    neg_score = torch.mul(anc, neg).sum(dim=1)
    loss = torch.mean(-torch.log(10e-6 + torch.sigmoid(pos_score - neg_score)))
    return loss, anc, pos


def _bin_tn(parts, K: int, d: int, dev, colsum: Optional[torch.Tensor],
            b_scale: Optional[torch.Tensor]) -> torch.Tensor:
    """(H_g > 0)ᵀ·B_g [K, d] for each (H_g, B_g, row offset) of ``parts`` (one or two products,
    one split-K launch + one reduction) → [G, K, d]; ``colsum`` [G, K] receives the column counts
    of (H_g > 0), ``b_scale`` scales B's rows as they are loaded (rows at the part's offset)."""
    lib = nat.load()
    C = torch.empty((len(parts), K, d), dtype=torch.float32, device=dev)
    arr = (nat.GemmTnDesc * len(parts))()
    for g, (H, B, off) in enumerate(parts):
        t = arr[g]
        t.A, t.lda, t.B, t.ldb = H.data_ptr(), H.stride(0), B.data_ptr(), B.stride(0)
        t.rows, t.M, t.N, t.C = H.shape[0], K, d, C[g].data_ptr()
        t.colsum_A = nat.ptr(colsum[g]) if colsum is not None else None
        t.binarize_a = 1
        t.b_row_scale = nat.ptr(b_scale[off:]) if b_scale is not None else None
    wsb = lib.hgd_gemm_tn_workspace_size(arr, len(parts))
    ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
    nat.check(lib.hgd_gemm_tn(arr, len(parts), ws.data_ptr(), wsb,
                              nat.stream_handle(dev)), "hgd_gemm_tn")
    return C


def _bin_rows(parts, M: torch.Tensor, count: torch.Tensor, Y: torch.Tensor,
              row_inv: Optional[torch.Tensor]) -> None:
    """Y[off : off + n_g] = (H_g > 0)·(D_g^-1·M[g]) for each (H_g, off) of ``parts`` (one row-GEMM
    launch), D_g = diag(max(count[g], 1)); with ``row_inv`` each row is divided by max(its
    nonzero count, 1), which is stored there."""
    K, d = M.shape[1], M.shape[2]
    descs = []
    for g, (H, off) in enumerate(parts):
        n = H.shape[0]
        desc = _rows_desc(H, M[g], d, 1, K, d, Y[off:off + n])
        desc.binarize_a = 1
        desc.b_row_count = count[g].data_ptr()
        desc.row_inv = nat.ptr(row_inv[off:off + n]) if row_inv is not None else None
        descs.append(desc)
    _gemm_rows(descs, Y.device)


class _DenseMeanTwoHop(torch.autograd.Function):
    """The ED-HNN scatter-mean pair over V/E = nonzero(H > 0) of a DENSE learned hypergraph
    H [n, K] (HCCF_diffusion.py:205-206 → EquivSetGNN.generate_V_E :382-402, EquivSetConv
    :291-308, torch_scatter means): Xv = D_v^-1·B·D_e^-1·Bᵀ·X with B = (H > 0), empty means 0.
    Bᵀ·X is a split-K product that counts B's columns as it goes, B·(D_e^-1·Xe) a row GEMM that
    scales Xe's rows by the counts as it stages them and divides each output row by its own count
    (both read H and binarize it on load): no nonzero list, no structure build, no host read —
    the same means as the sparse V/E path.

    Two hypergraphs over the row blocks [0, nu) and [nu, N) of one X (HCCF_diffusion's user and
    item calls of the block, :213-216) run as one grouped product per stage: 3 launches forward
    (split-K, reduction, rows) and 3 backward, whatever the pairing."""

    @staticmethod
    def forward(ctx, X, nu, H0, H1):
        X = X.contiguous()
        N, d = X.shape
        K = H0.shape[1]
        parts = [(H0.contiguous(), 0)] + ([(H1.contiguous(), nu)] if H1 is not None else [])
        f = dict(dtype=torch.float32, device=X.device)
        cnt = torch.empty((len(parts), K), **f)
        Xe = _bin_tn([(H, X[off:off + H.shape[0]], off) for H, off in parts], K, d, X.device,
                     cnt, None)
        row_inv = torch.empty(N, **f)
        Y = torch.empty((N, d), **f)
        _bin_rows(parts, Xe, cnt, Y, row_inv)
        ctx.parts = [off for _, off in parts]
        ctx.save_for_backward(cnt, row_inv, *[H for H, _ in parts])
        return Y

    @staticmethod
    def backward(ctx, dY):
        cnt, row_inv, *Hs = ctx.saved_tensors
        parts = list(zip(Hs, ctx.parts))
        dY = dY.contiguous()
        N, d = dY.shape
        K = cnt.shape[1]
        dM = _bin_tn([(H, dY[off:off + H.shape[0]], off) for H, off in parts], K, d, dY.device,
                     None, row_inv)
        dX = torch.empty_like(dY)
        _bin_rows(parts, dM, cnt, dX, None)
        # the structure carries no gradient (nonzero(H > 0) is integer)
        return dX, None, None, None


def dense_mean_two_hop_ok(H, X) -> bool:
    return (H.is_cuda and X.is_cuda and H.dim() == 2 and X.dim() == 2
            and H.dtype == X.dtype == torch.float32 and H.shape[0] == X.shape[0]
            and H.shape[1] % 16 == 0 and 16 <= H.shape[1] <= 128
            and X.shape[1] % 16 == 0 and X.shape[1] >= 16 and H.shape[0] > 0
            and X.stride(1) == 1 and X.stride(0) % 4 == 0 and X.data_ptr() % 16 == 0)


def dense_mean_two_hop(H: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """``scatter_mean(scatter_mean(X[V], E)[E], V, dim_size=n)`` for V/E = nonzero(H > 0) of a
    dense [n, K] hypergraph (see :class:`_DenseMeanTwoHop`); K a multiple of 16 up to 128."""
    if not dense_mean_two_hop_ok(H, X):
        raise ValueError("dense_mean_two_hop: needs device fp32 H [n, K] (K % 16 == 0, <= 128) "
                         "and X [n, d] (d % 16 == 0)")
    return _DenseMeanTwoHop.apply(X, X.shape[0], H.detach(), None)


def dense_mean_two_hop_pair(H_u: torch.Tensor, H_i: torch.Tensor, X: torch.Tensor) -> torch.Tensor:
    """``cat([dense_mean_two_hop(H_u, X[:nu]), dense_mean_two_hop(H_i, X[nu:])])`` with
    nu = H_u.shape[0] — both halves in the same launches, the output written whole."""
    nu = H_u.shape[0]
    if not (H_i.shape[1] == H_u.shape[1] and H_i.shape[0] == X.shape[0] - nu
            and dense_mean_two_hop_ok(H_u, X[:nu]) and dense_mean_two_hop_ok(H_i, X[nu:])):
        raise ValueError("dense_mean_two_hop_pair: needs H_u [nu, K], H_i [N - nu, K] and X [N, d] "
                         "(device fp32, K % 16 == 0, <= 128, d % 16 == 0)")
    return _DenseMeanTwoHop.apply(X, nu, H_u.detach(), H_i.detach())
