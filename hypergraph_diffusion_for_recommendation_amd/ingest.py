"""Native ingest and device graph build — the data path that
produces the hot path's input matrices (paths relative to /root/reference/HD_SELFRec):

* :func:`load_data_set` — ``FileIO.load_data_set`` (data/loader.py:24-38): the multi-threaded
  host parser ``hgd_ingest_read`` (same line rules, same failures) returning the raw
  (user, item) ids in file order.
* :class:`InteractionGraph` — the matrices ``Interaction.__init__`` builds with dicts and scipy
  (data/ui_graph.py:12-41, :43-112) and ``Graph.normalize_graph_mat`` (data/graph.py:11-25),
  built on the device: first-appearance id maps (``hgd_remap_first_appearance``), the canonical
  bipartite ``ui_adj`` and ``interaction_mat`` with duplicates summed (``hgd_coo_coalesce``),
  their normalisations (``hgd_degree_scale`` + ``hgd_normalize_values``), as
  :class:`~.incidence.Incidence` objects ready for the hops, or torch sparse tensors / scipy
  matrices for the reference harness.

Parity: ids, structure, counts and the normalised values are bit-exact with the reference's
dict loop and scipy (the per-row scale is numpy's own float32 ``np.power``, see
:func:`normalize_graph_mat`).
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Tuple

import numpy as np
import torch

from . import _native as nat
from .incidence import Incidence, _stream, _ws, expand_rows


def load_data_set(path: str, n_threads: int = 0,
                  skip_header: bool = True) -> Tuple[np.ndarray, np.ndarray]:
    """(user_raw, item_raw) int64 arrays in file order, parsed like FileIO.load_data_set
    (the constant weight it appends is implied). Raises HGDNativeError on lines the reference
    would reject (with the line number)."""
    lib = nat.load()
    h = ctypes.c_void_p()
    nat.check(lib.hgd_ingest_read(os.fsencode(path), int(skip_header), int(n_threads),
                                  ctypes.byref(h)), "hgd_ingest_read")
    try:
        n = lib.hgd_ingest_count(h)
        users = np.empty(n, dtype=np.int64)
        items = np.empty(n, dtype=np.int64)
        if n:
            nat.check(lib.hgd_ingest_copy(h, users.ctypes.data, items.ctypes.data),
                      "hgd_ingest_copy")
    finally:
        lib.hgd_ingest_free(h)
    return users, items


def remap_first_appearance(keys: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """(ids int32 [n], uniq int64 [n_unique]): ids in order of first appearance
    (data/ui_graph.py:43-56), uniq[id] = the raw key."""
    lib = nat.load()
    keys = keys.to(torch.int64).contiguous()
    dev = keys.device
    n = keys.numel()
    ids = torch.empty(n, dtype=torch.int32, device=dev)
    uniq = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    n_u = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = _ws(lib.hgd_remap_workspace_size(n), dev)
    nat.check(lib.hgd_remap_first_appearance(keys.data_ptr() if n else None, n, ids.data_ptr(),
                                             uniq.data_ptr(), n_u.data_ptr(), ws.data_ptr(),
                                             ws.numel(), _stream(dev)),
              "hgd_remap_first_appearance")
    return ids, uniq[: int(n_u.item())]


def coalesce(rows: torch.Tensor, cols: torch.Tensor, n_rows: int,
             n_cols: int) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
    """Canonical CSR (rowptr, col, counts) of the COO, duplicates summed (scipy csr_matrix)."""
    lib = nat.load()
    dev = rows.device
    rows = rows.to(torch.int32).contiguous()
    cols = cols.to(torch.int32).contiguous()
    n = rows.numel()
    rowptr = torch.empty(n_rows + 1, dtype=torch.int64, device=dev)
    col = torch.empty(max(n, 1), dtype=torch.int32, device=dev)
    val = torch.empty(max(n, 1), dtype=torch.float32, device=dev)
    nnz = torch.zeros(1, dtype=torch.int64, device=dev)
    ws = _ws(lib.hgd_coo_coalesce_workspace_size(n), dev)
    nat.check(lib.hgd_coo_coalesce(rows.data_ptr() if n else None, cols.data_ptr() if n else None,
                                   n, n_rows, n_cols, rowptr.data_ptr(), col.data_ptr(),
                                   val.data_ptr(), nnz.data_ptr(), ws.data_ptr(), ws.numel(),
                                   _stream(dev)), "hgd_coo_coalesce")
    k = int(nnz.item())
    return rowptr, col[:k], val[:k]


def normalize_graph_mat(rowptr: torch.Tensor, col: torch.Tensor, val: torch.Tensor,
                        shape) -> torch.Tensor:
    """Values of Graph.normalize_graph_mat (data/graph.py:11-25) for a CSR with float32 values:
    D^-1/2·A·D^-1/2 when square, D^-1·A otherwise (rowsum 0 → scale 0), bit-identical to the
    reference's scipy path.

    The float32 row sums (scipy sums the float32 matrix in float32) come from the device
    (hgd_degree_scale with power 1); the N-element scale ``np.power(rowsum, -0.5)`` (or ``-1``)
    is then taken with numpy itself, exactly the reference's call: numpy's float32 power is not
    correctly rounded and its rounding depends on the host's SIMD dispatch, so only numpy on this
    host reproduces it (N floats through PCIe, once per graph). The per-nonzero products
    ``(a·d_r)·d_c`` run on the device in the reference's float32 order (hgd_normalize_values)."""
    lib = nat.load()
    dev = val.device
    n_rows, n_cols = shape
    square = n_rows == n_cols
    rowsum = torch.empty(n_rows, dtype=torch.float32, device=dev)
    st = _stream(dev)
    nat.check(lib.hgd_degree_scale(rowptr.data_ptr(), val.data_ptr() if val.numel() else None,
                                   n_rows, 1.0, rowsum.data_ptr(), st), "hgd_degree_scale")
    rs = rowsum.cpu().numpy().reshape(-1, 1)  # np.array(adj_mat.sum(1)): [n, 1] float32
    with np.errstate(divide="ignore"):
        d_inv = np.power(rs, -0.5 if square else -1).flatten()
    d_inv[np.isinf(d_inv)] = 0.
    d = torch.from_numpy(np.ascontiguousarray(d_inv, dtype=np.float32)).to(dev)
    out = torch.empty_like(val)
    if val.numel():
        nat.check(lib.hgd_normalize_values(rowptr.data_ptr(), col.data_ptr(), val.data_ptr(),
                                           n_rows, d.data_ptr(),
                                           d.data_ptr() if square else None, out.data_ptr(), st),
                  "hgd_normalize_values")
    return out


def _incidence(rowptr, col, val, n_rows, n_cols) -> Incidence:
    rows = expand_rows(rowptr, col.numel())
    inc = Incidence._from_sorted(rows, col, val, n_rows, n_cols)
    inc.coo_sorted = True
    inc._coo_rows = rows
    return inc


class InteractionGraph:
    """Interaction's training matrices (data/ui_graph.py:12-41) built on the device.

    Attributes: ``n_users``, ``n_items``, ``n_nodes``; ``user_raw`` / ``item_raw`` (int64 device:
    raw id of every dense id, i.e. ``id2user``/``id2item``); ``user_idx`` / ``item_idx`` (int32
    device, per training record); ``ui_adj`` / ``norm_adj`` ([N, N], N = users + items, counts /
    D^-1/2 A D^-1/2) and ``interaction_mat`` / ``norm_interaction_mat`` ([U, I], counts /
    D^-1 A) as :class:`Incidence` (values in CSR order).
    """

    def __init__(self, users_raw, items_raw, device=None):
        dev = torch.device(device) if device is not None else torch.device("cuda")
        u = torch.as_tensor(np.asarray(users_raw, dtype=np.int64)).to(dev)
        i = torch.as_tensor(np.asarray(items_raw, dtype=np.int64)).to(dev)
        if u.numel() != i.numel():
            raise ValueError("InteractionGraph: user and item arrays differ in length")
        self.device = dev
        self.n_records = int(u.numel())
        self.user_idx, self.user_raw = remap_first_appearance(u)
        self.item_idx, self.item_raw = remap_first_appearance(i)
        self.n_users = int(self.user_raw.numel())
        self.n_items = int(self.item_raw.numel())
        self.n_nodes = self.n_users + self.n_items
        nu = self.n_users
        # ui_adj = tmp + tmp.T with tmp = csr((1, (u, i + n_users))) (ui_graph.py:70-84)
        shifted = self.item_idx + nu
        rows = torch.cat([self.user_idx, shifted])
        cols = torch.cat([shifted, self.user_idx])
        n = max(self.n_nodes, 1)
        rp, c, v = coalesce(rows, cols, n, n)
        self.ui_adj = _incidence(rp, c, v, n, n)
        self.norm_adj = _incidence(rp, c, normalize_graph_mat(rp, c, v, (n, n)), n, n)
        # interaction_mat [U, I] (ui_graph.py:95-112) and its row normalisation
        rp, c, v = coalesce(self.user_idx, self.item_idx, max(nu, 1), max(self.n_items, 1))
        shape = (max(nu, 1), max(self.n_items, 1))
        self.interaction_mat = _incidence(rp, c, v, *shape)
        self.norm_interaction_mat = _incidence(rp, c, normalize_graph_mat(rp, c, v, shape),
                                               *shape)

    @classmethod
    def from_file(cls, path: str, device=None, n_threads: int = 0) -> "InteractionGraph":
        users, items = load_data_set(path, n_threads=n_threads)
        return cls(users, items, device)

    # ---- views for the reference harness -------------------------------------------------
    def sparse_tensor(self, name: str = "norm_adj") -> torch.Tensor:
        """torch sparse COO on the device (TorchGraphInterface.convert_sparse_mat_to_tensor,
        base/torch_interface.py:8-12), carrying its Incidence so the drop-in layers reuse it."""
        inc: Incidence = getattr(self, name)
        idx = torch.stack([inc._coo_rows.to(torch.int64), inc.csr.col.to(torch.int64)])
        t = torch.sparse_coo_tensor(idx, inc.val, inc.shape, device=self.device)
        t = t._coalesced_(True)
        t._hgd_incidence = inc
        return t

    def to_scipy(self, name: str = "norm_adj"):
        """Host scipy CSR of one of the matrices (what the reference keeps in ``data``)."""
        import scipy.sparse as sp
        inc: Incidence = getattr(self, name)
        return sp.csr_matrix((inc.val.cpu().numpy(), inc.csr.col.cpu().numpy(),
                              inc.csr.rowptr.cpu().numpy()), shape=inc.shape)

    @property
    def user(self) -> dict:
        """raw user id → dense id (Interaction.user)."""
        return {int(r): k for k, r in enumerate(self.user_raw.cpu().tolist())}

    @property
    def item(self) -> dict:
        """raw item id → dense id (Interaction.item)."""
        return {int(r): k for k, r in enumerate(self.item_raw.cpu().tolist())}
