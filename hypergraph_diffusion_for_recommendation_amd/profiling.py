"""Per-hop timing with HIP events plus the algorithmic-byte model of SURVEY.md §8(d).

While a :class:`HopTimer` is active every :func:`incidence.spmm_csr` call records a start and
an end event on the stream the hop is launched on (the current torch stream, which is the
stream handed to ``hgd_spmm``) and remembers two byte counts for the hop:

* algorithmic (the figure ``roofline.achieved`` uses):
      B_hop = nnz·(4 [int32 col] + 4d [gathered row]) + R·(4d [Y row] + 4 [row scale])
              + (R+1)·4 [rowptr]
  — every index once, one d-wide fp32 row gathered per nonzero, every output row written once;
  the per-nonzero weights add 4·nnz only for an intrinsically weighted matrix (norm_adj);
* implementation: what hgd_spmm actually streams besides — the rowptr is int64 (8 B per row)
  and the source-side degree scale is folded into per-nonzero weights (4 B per nonzero), which
  the algorithmic model does not count for the binary incidence of the benchmark.
"""
from __future__ import annotations

from typing import List, Optional

import torch

_ACTIVE: Optional["HopTimer"] = None

MODEL_NOTE = ("SURVEY.md §8d B_hop = nnz*(4+4d) + R*(4d+4) + (R+1)*4 (binary H; the folded "
              "per-nonzero source scale and the int64 rowptr are counted only in "
              "implementation_bytes_per_launch)")


def hop_bytes(nnz: int, rows: int, d: int, weighted: bool = False) -> int:
    """SURVEY.md §8d algorithmic bytes of one hop (+4·nnz for an intrinsically weighted A)."""
    return nnz * (4 + (4 if weighted else 0) + 4 * d) + rows * (4 * d + 4) + (rows + 1) * 4


def impl_bytes(nnz: int, rows: int, d: int, has_val: bool, has_scale: bool,
               blocks: int = 0) -> int:
    """Bytes the hgd_spmm launch streams at minimum as implemented (int64 rowptr, weights).
    A source-blocked hop (hgd_spmm_blocked, ``blocks`` = P > 1) reads the [R × (P+1)] int64
    block starts instead of the rowptr, writes every Y row P times, reads it back P−1 times and
    applies the row scale in every pass."""
    if blocks > 1:
        return (nnz * (4 + (4 if has_val else 0) + 4 * d)
                + rows * (4 * d * (2 * blocks - 1) + (4 * blocks if has_scale else 0))
                + rows * (blocks + 1) * 8)
    return (nnz * (4 + (4 if has_val else 0) + 4 * d)
            + rows * (4 * d + (4 if has_scale else 0)) + (rows + 1) * 8)


class HopTimer:
    def __init__(self):
        self.records: List[tuple] = []

    def __enter__(self):
        global _ACTIVE
        self._prev = _ACTIVE
        _ACTIVE = self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = self._prev
        return False

    def begin(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def end(self, start, nbytes_fn):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        self.records.append((start, ev, nbytes_fn))

    def summary(self) -> dict:
        """Synchronises, then returns launches, total ms, total algorithmic bytes, GB/s."""
        torch.cuda.synchronize()
        ms = [s.elapsed_time(e) for s, e, _ in self.records]
        pairs = [f() for _, _, f in self.records]
        nbytes = [p[0] for p in pairs]
        impl = [p[1] for p in pairs]
        tot_ms = float(sum(ms))
        tot_b = int(sum(nbytes))
        n = len(ms)
        return {
            "launches": n,
            "total_ms": tot_ms,
            "avg_ms": tot_ms / n if n else 0.0,
            "bytes": tot_b,
            "avg_bytes": tot_b / n if n else 0.0,
            "avg_impl_bytes": sum(impl) / n if n else 0.0,
            "gbps": (tot_b / (tot_ms * 1e-3) / 1e9) if tot_ms > 0 else 0.0,
            "per_launch_ms": ms,
            "per_launch_bytes": nbytes,
        }


def active() -> Optional[HopTimer]:
    return _ACTIVE
