"""Device-resident incidence structures for the propagation hops.

An :class:`Incidence` holds one sparse matrix ``A`` of shape ``[n_rows, n_cols]`` twice:

* ``csr``  — rows of ``A`` (the hop ``Y = A·X``, ``torch.sparse.mm(adj, X)``), and
* ``csc``  — rows of ``Aᵀ`` (the hop ``M = Aᵀ·X``, ``torch.sparse.mm(adj.t(), X)``),

plus the per-nonzero weights in both orders and cached degree scales. Everything is built on
the GPU by libhgd (``include/hgd.h``); this module only allocates buffers with the PyTorch
caching allocator and sequences the C-ABI calls. It replaces the per-call COO handling of the
reference (``base/torch_interface.py:8-12`` builds the COO; ``torch.sparse.mm`` coalesces it and
``HGCNConv`` rebuilds ``adj.t()`` on every call, ``model/graph/HGNN_HD4.py:459-462``).

Layout in HBM (N rows, E nonzeros): rowptr int64[N+1], col int32[E], val fp32[E] (optional),
for each orientation; split plans for rows longer than ``split_threshold`` nonzeros.
"""
from __future__ import annotations

import copy
import ctypes
import os
import weakref
from typing import Dict, Optional, Tuple

import torch

from . import _native as nat
from . import profiling

DEFAULT_SPLIT_THRESHOLD = 2048
DEFAULT_SPLIT_CHUNK = 512
SPLIT_THRESHOLD_MIN = 128
SPLIT_NNZ_PER_THRESHOLD = 8192
SEGMENTED_MAX_AVG_DEGREE = 32
# lane-group tasks needed to fill MI355X: 256 CUs × 16 waves × 4 groups of 16 lanes (d = 64)
TARGET_GROUPS = 16384


def auto_split(n_rows: int, nnz: int) -> Tuple[int, int]:
    """(threshold, chunk) for the long-row split. A row walked by one lane group costs ~1.4 µs
    per 16 nonzeros (dependent index → gather round trips), so one unsplit row of T nonzeros
    ends the hop no sooner than ~T/11 µs: large structures split rows above
    pow2_floor(nnz / 8192) nonzeros, clamped to [128, 2048], into chunks of half that (at most
    512) — the longest walk stays a fraction of the hop's streaming time. (A skewed catalogue's hop,
    scripts/bench_skewed_hop.py: 180 µs at 2048 / 512, 43 µs at 128 / 64; uniform graphs keep
    their rows whole — their degrees stay far below the threshold.) A structure with fewer
    rows than TARGET_GROUPS (e.g. ML-1M's 3,706 items × ~200 nonzeros) would leave most CUs idle
    with one group per row, so its rows are cut into chunks of ≈ nnz / TARGET_GROUPS nonzeros
    (power of two in [32, 512])."""
    if n_rows >= TARGET_GROUPS or nnz == 0:
        t = SPLIT_THRESHOLD_MIN
        while 2 * t <= nnz // SPLIT_NNZ_PER_THRESHOLD and t < DEFAULT_SPLIT_THRESHOLD:
            t *= 2
        return t, min(t // 2, DEFAULT_SPLIT_CHUNK)
    want = max(1, nnz // TARGET_GROUPS)
    chunk = 32
    while chunk < want and chunk < DEFAULT_SPLIT_CHUNK:
        chunk *= 2
    return 2 * chunk, chunk


def _ws(nbytes: int, device) -> torch.Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def _stream(device) -> int:
    return nat.stream_handle(device)


class CSR:
    """One orientation: ``rowptr`` int64 [n_rows+1], ``col`` int32 [nnz] (device tensors),
    and the long-row split plan used by :func:`spmm_csr`."""

    def __init__(self, rowptr: torch.Tensor, col: torch.Tensor, n_rows: int, n_cols: int,
                 split_threshold: int = DEFAULT_SPLIT_THRESHOLD,
                 split_chunk: int = DEFAULT_SPLIT_CHUNK, plan_counts: Optional[Tuple] = None):
        self.rowptr = rowptr
        self.col = col
        self._ws_bytes: Dict[int, int] = {}  # hgd_spmm_workspace_size per width (spmm_csr)
        self.n_rows = int(n_rows)
        self.n_cols = int(n_cols)
        self.nnz = int(col.numel())
        self.device = rowptr.device
        self.split_threshold = int(split_threshold)
        self.split_chunk = int(split_chunk)
        # the columns of every row ascending (the CSC built by Incidence._from_sorted): required
        # by the source-blocked hop, whose block starts are binary searches inside each row
        self.cols_ascending = False
        self._col_blocks: Dict[int, Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = {}
        self._blk_vals: Dict[Tuple[int, int], tuple] = {}
        self._plan_arrays = ()
        self.plan = nat.SplitPlan()
        self.plan.threshold = 0
        if plan_counts is not None:
            self._build_plan(*plan_counts)

    # -- split plan ---------------------------------------------------------------------
    def plan_count_async(self) -> Optional[torch.Tensor]:
        """Queues the (n_heavy, n_chunks) count; returns the device tensor to read later."""
        if self.split_threshold <= 0 or self.n_rows == 0 or self.nnz <= self.split_threshold:
            return None
        counts = torch.empty(2, dtype=torch.int64, device=self.device)
        nat.check(nat.load().hgd_split_plan_count(
            self.rowptr.data_ptr(), self.n_rows, self.split_threshold, self.split_chunk,
            counts.data_ptr(), _stream(self.device)), "hgd_split_plan_count")
        return counts

    def _build_plan(self, n_heavy: int, n_chunks: int) -> None:
        self._ws_bytes = {}
        n_heavy, n_chunks = int(n_heavy), int(n_chunks)
        if n_heavy == 0:
            self.plan.threshold = 0
            return
        dev = self.device
        heavy_rows = torch.empty(n_heavy, dtype=torch.int32, device=dev)
        heavy_cptr = torch.empty(n_heavy + 1, dtype=torch.int64, device=dev)
        chunk_heavy = torch.empty(n_chunks, dtype=torch.int32, device=dev)
        lib = nat.load()
        ws = _ws(lib.hgd_split_plan_workspace_size(self.n_rows), dev)
        nat.check(lib.hgd_split_plan_build(
            self.rowptr.data_ptr(), self.n_rows, self.split_threshold, self.split_chunk,
            heavy_rows.data_ptr(), heavy_cptr.data_ptr(), chunk_heavy.data_ptr(), n_heavy,
            n_chunks, ws.data_ptr(), ws.numel(), _stream(dev)), "hgd_split_plan_build")
        self._plan_arrays = (heavy_rows, heavy_cptr, chunk_heavy)
        p = self.plan
        p.threshold = self.split_threshold
        p.chunk = self.split_chunk
        p.n_heavy = n_heavy
        p.n_chunks = n_chunks
        p.heavy_rows = heavy_rows.data_ptr()
        p.heavy_cptr = heavy_cptr.data_ptr()
        p.chunk_heavy = chunk_heavy.data_ptr()

    def configure_kernel(self, segmented: Optional[bool] = None) -> None:
        """Selects the hop kernel: one row per lane group (default), or the segmented short-row
        walk (HGD_PLAN_SEGMENTED; only without split rows and for average degree below
        SEGMENTED_MAX_AVG_DEGREE). Measured on MI355X the segmented walk is 6 %
        faster on a Zipf item graph's user hop and 6 % slower on a uniform one, so it is opt-in:
        ``segmented=True`` or ``HGD_SEGMENTED=1`` in the environment."""
        env = os.environ.get("HGD_SEGMENTED")
        if segmented is None and env is not None:
            segmented = env == "1"
        if segmented is None:
            segmented = False
        short = (self.n_rows > 0 and self.nnz < SEGMENTED_MAX_AVG_DEGREE * self.n_rows)
        self.plan.flags = 1 if (segmented and short and self.n_heavy == 0) else 0
        self._ws_bytes = {}

    @property
    def segmented(self) -> bool:
        return bool(self.plan.flags & 1)

    def __deepcopy__(self, memo):
        # immutable device structure: copies of a module share it (the ctypes plan struct
        # holding raw device pointers cannot be pickled or duplicated meaningfully)
        return self

    def col_blocks(self, n_blocks: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """The block-major copy of this structure for the source-blocked hop
        (hgd_spmm_col_blocks): ``(blk_start [n_blocks·n_rows+1] int64, blk_col [nnz] int32,
        blk_perm [nnz] int32)``, built once per block count on the current stream."""
        got = self._col_blocks.get(n_blocks)
        if got is None:
            if not self.cols_ascending:
                raise RuntimeError("col_blocks: the rows' columns are not known to be ascending")
            dev = self.device
            lib = nat.load()
            start = torch.empty(n_blocks * self.n_rows + 1, dtype=torch.int64, device=dev)
            bcol = torch.empty(self.nnz, dtype=torch.int32, device=dev)
            perm = torch.empty(self.nnz, dtype=torch.int32, device=dev)
            if self.n_rows:
                ws = _ws(lib.hgd_spmm_col_blocks_workspace_size(self.n_rows, n_blocks), dev)
                nat.check(lib.hgd_spmm_col_blocks(
                    self.rowptr.data_ptr(), self.col.data_ptr() if self.nnz else None,
                    self.n_rows, self.n_cols, n_blocks, start.data_ptr(),
                    bcol.data_ptr() if self.nnz else None, perm.data_ptr() if self.nnz else None,
                    ws.data_ptr(), ws.numel(), _stream(dev)), "hgd_spmm_col_blocks")
            else:
                start.zero_()
            got = self._col_blocks[n_blocks] = (start, bcol, perm)
        return got

    def blocked_values(self, n_blocks: int, val: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """``val`` (per-nonzero weights in this structure's order) gathered into the block-major
        order of :meth:`col_blocks`. Cached per tensor while it is alive and unmodified (its
        version counter), e.g. the cached ``Incidence.edge_values`` a training step passes to
        every hop; the last 8 are kept."""
        if val is None:
            return None
        try:
            version = val._version
        except RuntimeError:  # an inference tensor tracks no version: gathered every call
            return _gather32(val, self.col_blocks(n_blocks)[2])
        key = (n_blocks, id(val))
        hit = self._blk_vals.get(key)
        if hit is not None and hit[0]() is val and hit[1] == version:
            return hit[2]
        bval = _gather32(val, self.col_blocks(n_blocks)[2])
        if len(self._blk_vals) >= 8:
            self._blk_vals.pop(next(iter(self._blk_vals)))
        self._blk_vals[key] = (weakref.ref(val), version, bval)
        return bval

    @property
    def n_heavy(self) -> int:
        return int(self.plan.n_heavy) if self.plan.threshold > 0 else 0

    def degrees(self) -> torch.Tensor:
        return self.rowptr[1:] - self.rowptr[:-1]


def spmm_blocks(csr: CSR, d: int) -> int:
    """How many source blocks the hop over ``csr`` at width ``d`` runs in (0 = one pass).

    The hop gathers one d-wide row of X per nonzero at random. When X is small enough for the
    256 MB Infinity Cache (the item table a hop into users reads: 256 MB at d = 64) the gathers
    run at ~7.5 TB/s; a larger table (the 2.56 GB user table the hop into items reads) runs at the
    random-gather rate of HBM, ~5.9 TB/s. hgd_spmm_blocked cuts the source rows into P ranges
    and sums a row's nonzeros of one range per pass, so each pass gathers from a slice 1/P as
    large, for P−1 extra read+write passes over Y. Measured on MI355X at 10 M users × 1 M items
    × 100 M edges (scripts/bench_mall_blocked.py): d = 64 −13 % at P = 4,
    d = 128 −7 % at P = 8, d = 32 −4 % at P = 4 (−1 % at P = 2); hence about one block per
    640 MiB of the table a pass gathers from, at least 4, from 1 GiB. Between 512 MiB and 1 GiB
    two blocks: the 32-column slices of a 5 M-user shard (the sharded hop at N = 2, 640 MB)
    −4 % at P = 2; a 320 MB table (N = 4) is 3 % slower blocked. A blocked hop runs rows wider
    than 128 as 128-column passes (d = 256: −6 % at P = 8; in the plain hop's 64-column passes
    blocking gained nothing, 256 B gathered from every 1 KB row).

    Only for a structure whose rows' columns ascend (the CSC of an Incidence), without split
    rows or the segmented walk. ``HGD_SPMM_BLOCKS``: ``0`` turns it off, an integer P forces P
    blocks (1 = off) wherever it applies, unset = the size rule."""
    if not csr.cols_ascending or csr.n_heavy or csr.segmented or csr.nnz == 0:
        return 0
    env = os.environ.get("HGD_SPMM_BLOCKS", "")
    if env not in ("", "auto"):
        p = int(env)
        if p < 0 or p > 64:
            raise ValueError(f"HGD_SPMM_BLOCKS must be 0..64, got {env!r}")
        return p if p > 1 else 0
    # the library's size rule (hgd_spmm_blocks_for), shared with the native incidence objects
    return int(nat.load().hgd_spmm_blocks_for(csr.n_cols, int(d)))


def spmm_csr(csr: CSR, X: torch.Tensor, val: Optional[torch.Tensor] = None,
             row_scale: Optional[torch.Tensor] = None, epilogue: int = nat.EPI_NONE,
             slope: float = 0.0, out: Optional[torch.Tensor] = None,
             row_begin: int = 0, row_end: Optional[int] = None,
             ex: Optional[nat.RowEpilogue] = None, blocks: Optional[int] = None) -> torch.Tensor:
    """``Y[r] = epi(row_scale[r] * Σ_e val[e] * X[col[e]])`` for r in [row_begin, row_end).

    With ``ex`` (an ``hgd_row_epilogue``) the call is ``hgd_spmm_fused``: ``ex.act``/``ex.slope``
    replace ``epilogue``/``slope`` and the LayerNorm / residual epilogue runs in the store.
    ``blocks``: None = :func:`spmm_blocks` decides whether the hop runs source-blocked
    (hgd_spmm_blocked); 0 = never (e.g. into uncached exchange memory, which the blocked hop
    would read back P−1 times)."""
    if X.dim() != 2:
        raise ValueError(f"spmm: X must be 2-D, got {tuple(X.shape)}")
    if X.dtype != torch.float32:
        raise TypeError(f"spmm: X must be float32, got {X.dtype}")
    if X.device.type != "cuda":
        raise RuntimeError("spmm: X must be a device (cuda/hip) tensor; there is no CPU path")
    if X.shape[0] != csr.n_cols:
        raise ValueError(f"spmm: X has {X.shape[0]} rows, structure expects {csr.n_cols}")
    if X.stride(1) != 1:
        X = X.contiguous()
    d = X.shape[1]
    if out is None:
        out = torch.empty((csr.n_rows, d), dtype=torch.float32, device=X.device)
    if row_end is None:
        row_end = csr.n_rows
    if d == 0 or row_end <= row_begin:
        return out
    if val is not None and val.numel() != csr.nnz:
        raise ValueError("spmm: val size mismatch")
    if row_scale is not None and row_scale.numel() != csr.n_rows:
        raise ValueError("spmm: row_scale size mismatch")
    lib = nat.load()
    plan_ptr = ctypes.byref(csr.plan)
    # the plan is immutable once built: its workspace size per width is asked for once
    wsb = csr._ws_bytes.get(d)
    if wsb is None:
        wsb = csr._ws_bytes[d] = lib.hgd_spmm_workspace_size(plan_ptr, d)
    ws = _ws(wsb, X.device) if wsb else None
    timer = profiling.active()
    if timer is not None:
        t0 = timer.begin()
    mask = getattr(csr, "mask", None)
    if mask is not None or ex is not None or blocks == 0:
        blocks = 0
    else:
        blocks = spmm_blocks(csr, d)
    if mask is not None and ex is not None:
        nat.check(lib.hgd_spmm_masked_fused(
            csr.rowptr.data_ptr(), csr.col.data_ptr() if csr.nnz else None, nat.ptr(val),
            mask.data_ptr() if csr.nnz else None, float(csr.keep), nat.ptr(row_scale),
            csr.n_rows, csr.n_cols, int(row_begin), int(row_end), X.data_ptr(), X.stride(0),
            out.data_ptr(), out.stride(0), d, ctypes.byref(ex), plan_ptr, nat.ptr(ws), wsb,
            _stream(X.device)), "hgd_spmm_masked_fused")
    elif mask is not None:
        nat.check(lib.hgd_spmm_masked(
            csr.rowptr.data_ptr(), csr.col.data_ptr() if csr.nnz else None, nat.ptr(val),
            mask.data_ptr() if csr.nnz else None, float(csr.keep), nat.ptr(row_scale),
            csr.n_rows, csr.n_cols, int(row_begin), int(row_end), X.data_ptr(), X.stride(0),
            out.data_ptr(), out.stride(0), d, int(epilogue), float(slope), plan_ptr, nat.ptr(ws),
            wsb, _stream(X.device)), "hgd_spmm_masked")
    elif ex is None and blocks:
        start, bcol, _ = csr.col_blocks(blocks)
        bval = csr.blocked_values(blocks, val)
        nat.check(lib.hgd_spmm_blocked(
            start.data_ptr(), bcol.data_ptr(), nat.ptr(bval), nat.ptr(row_scale), csr.n_rows,
            csr.n_cols, int(row_begin), int(row_end), X.data_ptr(), X.stride(0), out.data_ptr(),
            out.stride(0), d, int(epilogue), float(slope), blocks, _stream(X.device)),
            "hgd_spmm_blocked")
    elif ex is None:
        nat.check(lib.hgd_spmm(
            csr.rowptr.data_ptr(), csr.col.data_ptr() if csr.nnz else None, nat.ptr(val),
            nat.ptr(row_scale), csr.n_rows, csr.n_cols, int(row_begin), int(row_end),
            X.data_ptr(), X.stride(0), out.data_ptr(), out.stride(0), d, int(epilogue),
            float(slope), plan_ptr, nat.ptr(ws), wsb, _stream(X.device)), "hgd_spmm")
    else:
        nat.check(lib.hgd_spmm_fused(
            csr.rowptr.data_ptr(), csr.col.data_ptr() if csr.nnz else None, nat.ptr(val),
            nat.ptr(row_scale), csr.n_rows, csr.n_cols, int(row_begin), int(row_end),
            X.data_ptr(), X.stride(0), out.data_ptr(), out.stride(0), d, ctypes.byref(ex),
            plan_ptr, nat.ptr(ws), wsb, _stream(X.device)), "hgd_spmm_fused")
    if timer is not None:
        rb, re_ = int(row_begin), int(row_end)
        full = rb == 0 and re_ == csr.n_rows

        def nbytes(csr=csr, rb=rb, re_=re_, full=full, d=d, hv=val is not None,
                   hs=row_scale is not None, blocks=blocks):
            nnz = csr.nnz if full else int(csr.rowptr[re_].item() - csr.rowptr[rb].item())
            return (profiling.hop_bytes(nnz, re_ - rb, d),
                    profiling.impl_bytes(nnz, re_ - rb, d, hv, hs, blocks))

        timer.end(t0, nbytes)
    return out


class Incidence:
    """Sparse ``A [n_rows, n_cols]`` as CSR + CSC on the device (see module docstring)."""

    def __init__(self, csr: CSR, csc: CSR, val: Optional[torch.Tensor],
                 val_t: Optional[torch.Tensor]):
        self.csr = csr
        self.csc = csc
        self.val = val          # per-nonzero weights in CSR order (None = binary)
        self.val_t = val_t      # the same weights in CSC order
        self.n_rows = csr.n_rows
        self.n_cols = csr.n_cols
        self.nnz = csr.nnz
        self.device = csr.device
        self._scales: Dict[Tuple[str, str], torch.Tensor] = {}
        self._edge_vals: Dict[Tuple[str, str, str], Optional[torch.Tensor]] = {}
        self.perm_t: Optional[torch.Tensor] = None  # CSC position → CSR position
        self.coo_sorted = False  # True when built from a row-sorted COO (COO order = CSR order)

    @property
    def shape(self):
        return (self.n_rows, self.n_cols)

    def __deepcopy__(self, memo):
        return self  # immutable once built (scale / edge-value caches are derived data)

    # -- construction ------------------------------------------------------------------
    @classmethod
    def from_coo(cls, indices: torch.Tensor, values: Optional[torch.Tensor], shape,
                 device=None, validate: bool = True, rows_sorted: Optional[bool] = None,
                 split_threshold: Optional[int] = None,
                 split_chunk: Optional[int] = None) -> "Incidence":
        """Builds from COO ``indices`` int64 [2, nnz] (+ fp32 ``values`` or None = ones).

        ``split_threshold`` / ``split_chunk`` default to :func:`auto_split` per orientation.

        Entries keep their order within a row (duplicates stay separate nonzeros, which is the
        same linear map as torch's coalesced sum). Raises ValueError on out-of-range indices.
        """
        n_rows, n_cols = int(shape[0]), int(shape[1])
        if n_rows >= 2 ** 31 or n_cols >= 2 ** 31:
            raise ValueError("Incidence: dimensions must be < 2^31")
        device = torch.device(device) if device is not None else indices.device
        if device.type != "cuda":
            raise RuntimeError("Incidence: needs a device (cuda/hip) target; there is no CPU path")
        lib = nat.load()
        st = _stream(device)
        indices = indices.to(device=device, dtype=torch.int64)
        nnz = int(indices.shape[1])
        if values is not None:
            values = values.to(device=device, dtype=torch.float32).contiguous()
            if values.numel() != nnz:
                raise ValueError("Incidence: values/indices size mismatch")
        rows64 = indices[0].contiguous()
        cols64 = indices[1].contiguous()
        rows = torch.empty(nnz, dtype=torch.int32, device=device)
        cols = torch.empty(nnz, dtype=torch.int32, device=device)
        flags = torch.zeros(3, dtype=torch.int64, device=device)
        if nnz:
            nat.check(lib.hgd_index_narrow(rows64.data_ptr(), nnz, n_rows, rows.data_ptr(),
                                           flags[0:1].data_ptr(), st), "hgd_index_narrow(rows)")
            nat.check(lib.hgd_index_narrow(cols64.data_ptr(), nnz, n_cols, cols.data_ptr(),
                                           flags[1:2].data_ptr(), st), "hgd_index_narrow(cols)")
            if rows_sorted is None:
                nat.check(lib.hgd_check_sorted(rows.data_ptr(), nnz, n_rows,
                                               flags[2:3].data_ptr(), st), "hgd_check_sorted")
        if validate or rows_sorted is None:
            f = flags.tolist()
            if f[0] or f[1]:
                raise ValueError(f"Incidence: {f[0]} row / {f[1]} col indices out of range "
                                 f"for shape {(n_rows, n_cols)}")
            if rows_sorted is None:
                rows_sorted = f[2] == 0
        if nnz and not rows_sorted:
            perm = torch.empty(nnz, dtype=torch.int32, device=device)
            rows_s = torch.empty_like(rows)
            ws = _ws(lib.hgd_sort_perm_workspace_size(nnz), device)
            nat.check(lib.hgd_sort_perm(rows.data_ptr(), nnz, n_rows, rows_s.data_ptr(),
                                        perm.data_ptr(), ws.data_ptr(), ws.numel(), st),
                      "hgd_sort_perm(rows)")
            rows = rows_s
            cols = _gather32(cols, perm)
            if values is not None:
                values = _gather32(values, perm)
        inc = cls._from_sorted(rows, cols, values, n_rows, n_cols, split_threshold, split_chunk)
        inc.coo_sorted = bool(rows_sorted) or nnz == 0
        return inc

    @classmethod
    def _from_sorted(cls, rows: torch.Tensor, cols: torch.Tensor, values: Optional[torch.Tensor],
                     n_rows: int, n_cols: int, split_threshold: Optional[int] = None,
                     split_chunk: Optional[int] = None) -> "Incidence":
        device = rows.device
        lib = nat.load()
        st = _stream(device)
        nnz = int(rows.numel())
        rowptr = torch.empty(n_rows + 1, dtype=torch.int64, device=device)
        nat.check(lib.hgd_rowptr_from_sorted(rows.data_ptr() if nnz else None, nnz, n_rows,
                                             rowptr.data_ptr(), st), "hgd_rowptr_from_sorted")
        # CSC: stable sort of the column ids keeps rows ascending inside each column.
        colptr = torch.empty(n_cols + 1, dtype=torch.int64, device=device)
        csc_col = torch.empty(nnz, dtype=torch.int32, device=device)
        val_t = None
        if nnz:
            keys = torch.empty(nnz, dtype=torch.int32, device=device)
            perm = torch.empty(nnz, dtype=torch.int32, device=device)
            ws = _ws(lib.hgd_sort_perm_workspace_size(nnz), device)
            nat.check(lib.hgd_sort_perm(cols.data_ptr(), nnz, n_cols, keys.data_ptr(),
                                        perm.data_ptr(), ws.data_ptr(), ws.numel(), st),
                      "hgd_sort_perm(cols)")
            del ws
            nat.check(lib.hgd_rowptr_from_sorted(keys.data_ptr(), nnz, n_cols,
                                                 colptr.data_ptr(), st),
                      "hgd_rowptr_from_sorted(csc)")
            del keys
            csc_col = _gather32(rows, perm)
            if values is not None:
                val_t = _gather32(values, perm)
        else:
            colptr.zero_()
            perm = torch.empty(0, dtype=torch.int32, device=device)

        def split(n):
            if split_threshold is None:
                return auto_split(n, nnz)
            return split_threshold, split_chunk or DEFAULT_SPLIT_CHUNK

        csr = CSR(rowptr, cols, n_rows, n_cols, *split(n_rows))
        csc = CSR(colptr, csc_col, n_cols, n_rows, *split(n_cols))
        csc.cols_ascending = True
        c1, c2 = csr.plan_count_async(), csc.plan_count_async()
        if c1 is not None:
            csr._build_plan(*c1.tolist())
        if c2 is not None:
            csc._build_plan(*c2.tolist())
        csr.configure_kernel()
        csc.configure_kernel()
        inc = cls(csr, csc, values, val_t)
        inc.perm_t = perm  # CSC position → CSR position (sort-free drop-edge rebuilds)
        return inc

    def drop(self, mask: torch.Tensor, keep: float, kept: Optional[int] = None,
             capacity: bool = False) -> "Incidence":
        """The incidence of SpAdjDropEdge's output (HCCF.py:217-226) built from this one without
        any sort: ``mask`` (uint8/bool, CSR order) keeps nonzeros in order and values are divided
        by ``keep``; the CSC comes from compacting this CSC through ``perm_t``
        (hgd_dropedge_structure). One device→host read (the kept count) unless the caller passes
        ``kept`` (e.g. counted with a host-drawn mask) or asks for ``capacity``: then the kept
        count stays on the device (the row pointers end at it), the arrays keep the parent's
        length with a zeroed tail (hgd_dropedge_fill_tail), and rows longer than the split
        threshold are walked by one lane group (no split plan: it would need the count) — no
        host read, so a training step can be captured in a HIP graph."""
        lib = nat.load()
        dev = self.device
        st = _stream(dev)
        nnz, R, C = self.nnz, self.n_rows, self.n_cols
        m = mask.to(device=dev, dtype=torch.uint8).contiguous()
        if m.numel() != nnz:
            raise ValueError("Incidence.drop: mask size mismatch")
        rowptr = torch.empty(R + 1, dtype=torch.int64, device=dev)
        colptr = torch.empty(C + 1, dtype=torch.int64, device=dev)
        col = torch.empty(nnz, dtype=torch.int32, device=dev)
        row_t = torch.empty(nnz, dtype=torch.int32, device=dev)
        weighted = self.val is not None
        val = torch.empty(nnz, dtype=torch.float32, device=dev) if weighted else None
        val_t = torch.empty(nnz, dtype=torch.float32, device=dev) if weighted else None
        ws = _ws(lib.hgd_dropedge_structure_workspace_size(nnz), dev)
        nat.check(lib.hgd_dropedge_structure(
            self.csr.rowptr.data_ptr(), nat.ptr(self.csr.col) if nnz else None, nat.ptr(self.val),
            self.csc.rowptr.data_ptr(), nat.ptr(self.csc.col) if nnz else None,
            nat.ptr(self.val_t), nat.ptr(self.perm_t) if nnz else None, R, C, nnz,
            m.data_ptr() if nnz else None, float(keep), rowptr.data_ptr(),
            col.data_ptr() if nnz else None, nat.ptr(val), colptr.data_ptr(),
            row_t.data_ptr() if nnz else None, nat.ptr(val_t), ws.data_ptr(), ws.numel(), st),
            "hgd_dropedge_structure")
        if capacity:
            if nnz:
                nat.check(lib.hgd_dropedge_fill_tail(
                    rowptr.data_ptr() + 8 * R, nnz, col.data_ptr(), nat.ptr(val),
                    row_t.data_ptr(), nat.ptr(val_t), st), "hgd_dropedge_fill_tail")
            csr = CSR(rowptr, col, R, C, 0, self.csr.split_chunk)
            csc = CSR(colptr, row_t, C, R, 0, self.csc.split_chunk)
            for child, parent in ((csr, self.csr), (csc, self.csc)):
                child.plan.flags = parent.plan.flags if parent.n_heavy == 0 else 0
            out = Incidence(csr, csc, val, val_t)
            out.perm_t = None
            return out
        if kept is None:
            kept = int(rowptr[R].item()) if R else 0
        col, row_t = col[:kept], row_t[:kept]
        if weighted:
            val, val_t = val[:kept], val_t[:kept]
        csr = CSR(rowptr, col, R, C, self.csr.split_threshold, self.csr.split_chunk)
        csc = CSR(colptr, row_t, C, R, self.csc.split_threshold, self.csc.split_chunk)
        # degrees only shrink: a parent without split rows has none after dropping (no count)
        for child, parent in ((csr, self.csr), (csc, self.csc)):
            if parent.n_heavy:
                cnt = child.plan_count_async()
                if cnt is not None:
                    child._build_plan(*cnt.tolist())
            child.plan.flags = parent.plan.flags if child.n_heavy == 0 else 0
        out = Incidence(csr, csc, val, val_t)
        out.perm_t = None  # a dropped structure is not dropped again (the reference drops the base)
        return out

    def masked(self, mask: torch.Tensor, keep: float,
               mask_t: Optional[torch.Tensor] = None) -> "MaskedIncidence":
        """SpAdjDropEdge's output (HCCF.py:217-226) as a VIEW of this incidence: no compaction
        at all. The hops run over this structure and skip the dropped edges
        (hgd_spmm_masked: weight val[e] / keep, kept edges in edge order — the sums of the
        compacted matrix of :meth:`drop`, bitwise when no row is split). The CSC-order mask is
        one byte gather through ``perm_t``; nothing is read back to the host, so a step using
        it can be captured in a HIP graph. For the plain hops (GCNLayer, HGCNConv without
        degree scales); degree scales of the dropped matrix need :meth:`drop`. ``mask_t``: the
        same mask already in CSC order (hgd_bernoulli_mask_dev_pair draws both)."""
        if self.perm_t is None:
            raise RuntimeError("Incidence.masked: needs the CSC→CSR permutation (a structure "
                               "built from a COO)")
        dev = self.device
        m = mask.to(device=dev, dtype=torch.uint8).contiguous()
        if m.numel() != self.nnz:
            raise ValueError("Incidence.masked: mask size mismatch")
        if not keep > 0.0:
            raise ValueError("Incidence.masked: keep must be > 0")
        if mask_t is not None:
            m_t = mask_t.to(device=dev, dtype=torch.uint8).contiguous()
            if m_t.numel() != self.nnz:
                raise ValueError("Incidence.masked: mask_t size mismatch")
        else:
            m_t = torch.empty_like(m)
            if self.nnz:
                nat.check(nat.load().hgd_gather_u8(m.data_ptr(), self.perm_t.data_ptr(),
                                                   self.nnz, m_t.data_ptr(), _stream(dev)),
                          "hgd_gather_u8")
        csr = copy.copy(self.csr)
        csc = copy.copy(self.csc)
        csr.mask, csr.keep = m, float(keep)
        csc.mask, csc.keep = m_t, float(keep)
        out = MaskedIncidence(csr, csc, self.val, self.val_t)
        out.parent = self
        return out

    @classmethod
    def from_dense(cls, A: torch.Tensor, device=None, **kw) -> "Incidence":
        """The nonzero pattern and values of a dense matrix (``torch.nonzero(A)`` order), e.g.
        DHCF's dense interaction matrix fed to HGCNConv (DHCF.py:140, :131-133)."""
        device = torch.device(device) if device is not None else (
            A.device if A.device.type == "cuda" else torch.device("cuda"))
        A = A.to(device=device, dtype=torch.float32)
        rowptr, cols, vals = dense_threshold(A, 0.0, nonzero=True, values=True)
        rows = expand_rows(rowptr, cols.numel())
        inc = cls._from_sorted(rows, cols, vals, A.shape[0], A.shape[1], **kw)
        inc.coo_sorted = True
        return inc

    @classmethod
    def from_torch_sparse(cls, adj: torch.Tensor, device=None, **kw) -> "Incidence":
        """From a torch sparse COO tensor as built by ``convert_sparse_mat_to_tensor``."""
        if adj.layout != torch.sparse_coo:
            raise TypeError("Incidence.from_torch_sparse expects a sparse COO tensor")
        if device is None:
            device = adj.device if adj.device.type == "cuda" else torch.device("cuda")
        return cls.from_coo(adj._indices(), adj._values(), adj.shape, device=device, **kw)

    @classmethod
    def from_scipy(cls, mat, device="cuda", binary: bool = False, **kw) -> "Incidence":
        """From a scipy sparse matrix (row-major COO order of ``tocoo()``, like the reference)."""
        coo = mat.tocoo()
        idx = torch.stack([torch.from_numpy(coo.row.astype("int64")),
                           torch.from_numpy(coo.col.astype("int64"))])
        vals = None if binary else torch.from_numpy(coo.data.astype("float32"))
        return cls.from_coo(idx, vals, coo.shape, device=device, **kw)

    @classmethod
    def from_index_lists(cls, vertex: torch.Tensor, edges: torch.Tensor, n_vertices: int,
                         n_edges: Optional[int] = None, device=None, **kw) -> "Incidence":
        """Binary incidence B[vertex[k], edges[k]] (ED-HNN's V/E lists, EquivSetConv2.py:85-93).

        ``n_edges`` defaults to max(edges)+1, the row count torch_scatter gives the edge means.
        """
        device = torch.device(device) if device is not None else vertex.device
        if device.type != "cuda":
            device = torch.device("cuda")
        if n_edges is None:
            n_edges = int(edges.max().item()) + 1 if edges.numel() else 0
        idx = torch.stack([vertex.to(device=device, dtype=torch.int64),
                           edges.to(device=device, dtype=torch.int64)])
        return cls.from_coo(idx, None, (int(n_vertices), int(n_edges)), device=device, **kw)

    # -- derived per-row / per-nonzero quantities --------------------------------------
    def scale(self, side: str, kind: Optional[str]) -> Optional[torch.Tensor]:
        """Degree scale over rows ('row') or columns ('col') of A.

        kind: None → no scale; 'mean' → 1/deg (torch_scatter mean; 0 for empty);
        'sym' → deg^-1/2 (data/graph.py:15-16, inf→0); 'wmean'/'wsym' use the weighted
        degree Σ val (normalize_graph_mat's rowsum of a weighted matrix).
        """
        if kind is None:
            return None
        key = (side, kind)
        s = self._scales.get(key)
        if s is not None:
            return s
        o = self.csr if side == "row" else self.csc
        weighted = kind.startswith("w")
        power = {"mean": -1.0, "sym": -0.5}[kind[1:] if weighted else kind]
        w = None
        if weighted:
            w = self.val if side == "row" else self.val_t
        s = torch.empty(o.n_rows, dtype=torch.float32, device=self.device)
        nat.check(nat.load().hgd_degree_scale(o.rowptr.data_ptr(), nat.ptr(w), o.n_rows, power,
                                              s.data_ptr(), _stream(self.device)),
                  "hgd_degree_scale")
        self._scales[key] = s
        return s

    def edge_values(self, orient: str, src_kind: Optional[str]) -> Optional[torch.Tensor]:
        """Per-nonzero weights for a hop over ``orient`` ('csr' or 'csc') with the SOURCE-side
        diagonal folded in: w[e] = a[e] * S[src(e)], S = scale over the gathered side."""
        key = (orient, src_kind or "")
        if key in self._edge_vals:
            return self._edge_vals[key]
        o = self.csr if orient == "csr" else self.csc
        base = self.val if orient == "csr" else self.val_t
        src_side = "col" if orient == "csr" else "row"
        s = self.scale(src_side, src_kind)
        if s is None:
            out = base
        else:
            out = torch.empty(o.nnz, dtype=torch.float32, device=self.device)
            nat.check(nat.load().hgd_edge_values(
                nat.ptr(base), None, s.data_ptr(), o.col.data_ptr() if o.nnz else None, o.nnz,
                out.data_ptr(), _stream(self.device)), "hgd_edge_values")
        self._edge_vals[key] = out
        return out

    def to_dense_cpu(self) -> torch.Tensor:
        """Debug helper: the matrix as a dense CPU tensor (test use)."""
        rp = self.csr.rowptr.cpu()
        rows = torch.repeat_interleave(torch.arange(self.n_rows), rp[1:] - rp[:-1])
        out = torch.zeros(self.n_rows, self.n_cols)
        v = self.val.cpu() if self.val is not None else torch.ones(self.nnz)
        out.index_put_((rows, self.csr.col.cpu().long()), v, accumulate=True)
        return out


class MaskedIncidence(Incidence):
    """An edge-dropped view of a parent incidence (:meth:`Incidence.masked`): both orientations
    share the parent's arrays and carry a keep-mask; hops skip the dropped edges. ``nnz`` is
    the parent's (the kept count stays on the device). Degree scales of the dropped matrix are
    not available on a view."""

    def scale(self, side: str, kind: Optional[str]) -> Optional[torch.Tensor]:
        if kind is None:
            return None
        raise NotImplementedError("MaskedIncidence: degree scales of an edge-dropped view; "
                                  "build the dropped structure with Incidence.drop")

    def materialize(self, capacity: bool = True) -> Incidence:
        """The compacted structure of the same drop (Incidence.drop)."""
        return self.parent.drop(self.csr.mask, self.csr.keep, capacity=capacity)


def drop_edges(indices: torch.Tensor, values: torch.Tensor, mask: torch.Tensor,
               keep_rate: float, count: Optional[int] = None):
    """Device compaction of SpAdjDropEdge (model/graph/HCCF.py:217-226): keeps the COO entries
    whose ``mask`` is set, in order, with ``values / keep_rate`` (IEEE fp32 division).
    Returns (indices int64 [2, kept], values fp32 [kept]). ``count`` (kept entries) avoids a
    device→host read when the caller already knows it (e.g. a host-drawn mask)."""
    device = values.device
    lib = nat.load()
    st = _stream(device)
    nnz = int(values.numel())
    indices = indices.to(device=device, dtype=torch.int64)
    rows = indices[0].contiguous()
    cols = indices[1].contiguous()
    m = mask.to(device=device, dtype=torch.uint8).contiguous()
    if m.numel() != nnz:
        raise ValueError("drop_edges: mask size mismatch")
    n_out = torch.empty(1, dtype=torch.int64, device=device)
    if count is None:
        count = int(m.sum().item()) if nnz else 0
    out_idx = torch.empty((2, count), dtype=torch.int64, device=device)
    out_val = torch.empty(count, dtype=torch.float32, device=device)
    ws = _ws(lib.hgd_dropedge_workspace_size(nnz), device)
    nat.check(lib.hgd_dropedge_compact(
        rows.data_ptr() if nnz else None, cols.data_ptr() if nnz else None,
        values.contiguous().data_ptr() if nnz else None, m.data_ptr() if nnz else None, nnz,
        float(keep_rate), out_idx[0].data_ptr() if count else None,
        out_idx[1].data_ptr() if count else None, out_val.data_ptr() if count else None,
        n_out.data_ptr(), ws.data_ptr(), ws.numel(), st), "hgd_dropedge_compact")
    return out_idx, out_val


def dense_threshold(H: torch.Tensor, thresh: float = 0.0, nonzero: bool = False,
                    values: bool = False):
    """``torch.nonzero(H > thresh)`` (or ``torch.nonzero(H)`` with ``nonzero=True``) of a dense
    2-D fp32 device matrix as CSR (rowptr int64 [n+1], cols int32 [nnz][, values fp32]) in
    row-major order (EquivSetGNN.generate_V_E, model/layers/layers2/EquivSetGNN2.py:105-133)."""
    if H.dim() != 2 or H.dtype != torch.float32:
        raise TypeError("dense_threshold: expects a 2-D float32 matrix")
    if H.stride(1) != 1:
        H = H.contiguous()
    device = H.device
    lib = nat.load()
    st = _stream(device)
    n, k = H.shape
    mode = 1 if nonzero else 0
    rowptr = torch.empty(n + 1, dtype=torch.int64, device=device)
    ws = _ws(lib.hgd_dense_threshold_workspace_size(n), device)
    nat.check(lib.hgd_dense_threshold_rowptr(H.data_ptr(), n, k, H.stride(0), float(thresh),
                                             mode, rowptr.data_ptr(), ws.data_ptr(), ws.numel(),
                                             st), "hgd_dense_threshold_rowptr")
    nnz = int(rowptr[n].item())
    cols = torch.empty(nnz, dtype=torch.int32, device=device)
    vals = torch.empty(nnz, dtype=torch.float32, device=device) if values else None
    if nnz:
        nat.check(lib.hgd_dense_threshold_fill(H.data_ptr(), n, k, H.stride(0), float(thresh),
                                               mode, rowptr.data_ptr(), cols.data_ptr(),
                                               nat.ptr(vals), st), "hgd_dense_threshold_fill")
    if values:
        return rowptr, cols, vals
    return rowptr, cols


def expand_rows(rowptr: torch.Tensor, nnz: int) -> torch.Tensor:
    """Row id of every CSR nonzero (int32)."""
    n_rows = rowptr.numel() - 1
    out = torch.empty(nnz, dtype=torch.int32, device=rowptr.device)
    if nnz:
        nat.check(nat.load().hgd_expand_rows(rowptr.data_ptr(), n_rows, nnz, out.data_ptr(),
                                             _stream(rowptr.device)), "hgd_expand_rows")
    return out


def _gather32(src: torch.Tensor, perm: torch.Tensor) -> torch.Tensor:
    out = torch.empty_like(src)
    n = perm.numel()
    if n:
        nat.check(nat.load().hgd_gather32(src.data_ptr(), perm.data_ptr(), n, out.data_ptr(),
                                          _stream(src.device)), "hgd_gather32")
    return out


def incidence_of(adj, cache: bool = True) -> Incidence:
    """The Incidence behind a torch sparse COO tensor (cached on the tensor object), or the
    argument itself when it already is one."""
    if isinstance(adj, Incidence):
        return adj
    inc = getattr(adj, "_hgd_incidence", None) if cache else None
    if (inc is not None and adj.layout == torch.strided
            and getattr(adj, "_hgd_incidence_version", None) != adj._version):
        inc = None  # a dense adjacency modified in place since its structure was taken
    if inc is None:
        if adj.layout == torch.sparse_coo:
            inc = Incidence.from_torch_sparse(adj)
        elif adj.layout == torch.strided and adj.dim() == 2:
            inc = Incidence.from_dense(adj)  # the pattern of a dense adjacency (DHCF)
        else:
            raise TypeError(f"incidence_of: unsupported adjacency layout {adj.layout}")
        if cache:
            try:
                adj._hgd_incidence = inc
                adj._hgd_incidence_version = adj._version
            except (AttributeError, RuntimeError):
                pass
    return inc
