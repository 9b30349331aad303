"""User-row sharding of the 2-hop hypergraph conv across the GPUs of one node.

Each rank owns a contiguous block of users (vertex rows of H), their embedding rows and the
CSR/CSC of its slice of H; the item (hyperedge) dimension is replicated. The two hops are

    hop 1  M_g = Q·H_gᵀ·(R·X_g)         partial item sums on every rank      (CSC, hgd_spmm)
           M   = Σ_g M_g                RCCL all-reduce over xGMI             (torch.distributed)
    hop 2  Y_g = P·H_g·M                purely local                          (CSR, hgd_spmm)

and the backward is the same pair with P and R swapped. Q = D_e^-1 must use the GLOBAL item
degree, which is all-reduced once when the shard is built. To hide the exchange, hop 1 is
issued in item chunks and each chunk's all-reduce is queued (async_op) right behind the kernel
that produced it, so RCCL moves chunk k while the GPU computes chunk k+1; only the last chunk's
exchange is exposed before hop 2.

The reference has no distributed code at all; this is new design.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.distributed as dist

from .incidence import Incidence, spmm_csr


class ShardedIncidence:
    """One rank's slice of H (users [u0,u1) × all items) plus global item scales."""

    def __init__(self, inc: Incidence, group=None, n_chunks: int = 4,
                 P: Optional[str] = "sym", Q: Optional[str] = "mean", R: Optional[str] = "sym"):
        self.inc = inc
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.P, self.R = P, R
        self.n_chunks = max(1, int(n_chunks)) if self.world > 1 else 1
        self.q = self._global_col_scale(Q)
        # item-row chunk boundaries for the overlapped exchange
        n_items = inc.n_cols
        step = (n_items + self.n_chunks - 1) // self.n_chunks if n_items else 0
        self.bounds = [(min(k * step, n_items), min((k + 1) * step, n_items))
                       for k in range(self.n_chunks)]
        self.bounds = [(a, b) for a, b in self.bounds if b > a] or [(0, n_items)]

    def _global_col_scale(self, kind: Optional[str]) -> Optional[torch.Tensor]:
        if kind is None:
            return None
        if self.world == 1:
            return self.inc.scale("col", kind)
        if kind not in ("mean", "sym"):
            raise ValueError(f"sharded: unsupported item scale {kind!r}")
        deg = (self.inc.csc.rowptr[1:] - self.inc.csc.rowptr[:-1]).to(torch.float64)
        dist.all_reduce(deg, group=self.group)
        p = -1.0 if kind == "mean" else -0.5
        s = torch.where(deg > 0, deg.pow(p), torch.zeros_like(deg))
        return s.to(torch.float32)

    def _hop1_exchange(self, X: torch.Tensor, src_kind: Optional[str]) -> torch.Tensor:
        inc = self.inc
        M = torch.empty((inc.n_cols, X.shape[1]), dtype=torch.float32, device=X.device)
        val = inc.edge_values("csc", src_kind)
        works: List = []
        for a, b in self.bounds:
            spmm_csr(inc.csc, X, val=val, row_scale=self.q, out=M, row_begin=a, row_end=b)
            if self.world > 1:
                works.append(dist.all_reduce(M[a:b], group=self.group, async_op=True))
        for w in works:
            w.wait()
        return M


class _ShardedHGConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, sh: ShardedIncidence):
        ctx.sh = sh
        X = X.contiguous()
        M = sh._hop1_exchange(X, sh.R)
        return spmm_csr(sh.inc.csr, M, val=sh.inc.val, row_scale=sh.inc.scale("row", sh.P))

    @staticmethod
    def backward(ctx, dY):
        sh = ctx.sh
        dM = sh._hop1_exchange(dY.contiguous(), sh.P)
        dX = spmm_csr(sh.inc.csr, dM, val=sh.inc.val, row_scale=sh.inc.scale("row", sh.R))
        return dX, None


def sharded_two_hop(sh: ShardedIncidence, X_local: torch.Tensor) -> torch.Tensor:
    """P·H·Q·Hᵀ·R·X on user-row shards (X_local = this rank's user rows)."""
    return _ShardedHGConv.apply(X_local, sh)
