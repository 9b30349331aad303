"""User-row sharding of the 2-hop hypergraph conv across the GPUs of one node.

Each rank owns a contiguous, degree-balanced block of users (vertex rows of H), their embedding
rows and the CSR/CSC of its slice of H; the item (hyperedge) dimension is replicated. The two
hops are

    hop 1  M_g = Q·H_gᵀ·(R·X_g)         partial item sums on every rank      (CSC, hgd_spmm)
           M   = Σ_g M_g                RCCL all-reduce over xGMI             (torch.distributed)
    hop 2  Y_g = P·H_g·M                purely local                          (CSR, hgd_spmm)

and the backward is the same pair with P and R swapped. Q = D_e^-1 must use the GLOBAL item
degree, which is all-reduced once when the shard is built.

The exchange is pipelined over COLUMN SLICES of the embedding (``slice_width`` columns, 32 at
d = 64): hop 1 of slice s writes its own contiguous [I, w] message block, whose all-reduce is
queued (async_op) right behind the kernel that produced it, and hop 2 of slice s only waits for
that block. So RCCL moves slice 0 while hop 1 computes slice 1, and hop 2 of slice 0 computes
while slice 1 is in flight: only the first slice's hop 1 and the last slice's hop 2 are exposed
around the exchange. Each slice is a full hop over a narrower row (w·4 bytes per gathered row,
128 B = one L2 line at w = 32), so it adds no accumulation traffic; the cost is re-reading the
index stream once per slice (4 B per nonzero). Item-row chunks (``n_chunks``) split each slice's
exchange further (hop 2 of a slice then waits for all of its chunks).

The reference has no distributed code at all; this is new design.
"""
from __future__ import annotations

import atexit
import ctypes
import os
import threading
import time
from typing import List, Optional, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .incidence import Incidence, spmm_csr


def init_process_group(device: torch.device, backend: str = "nccl", **kw) -> None:
    """One rank per GPU: ``torch.distributed`` over RCCL ("nccl" on ROCm) bound to ``device``,
    with the communicator's kernels on a HIGH-PRIORITY stream. The exchanges run beside hop
    kernels whose grids fill every CU; at high priority the dispatcher places RCCL's few
    workgroups as soon as a CU slot frees instead of behind the queued hop workgroups, so the
    all-reduce of slice s starts when its producer finishes, not when the next hop drains.
    Other backends (gloo, for CPU / one-device rehearsals) are initialised plainly."""
    if backend == "nccl":
        opts = dist.ProcessGroupNCCL.Options()
        opts.is_high_priority_stream = True
        dist.init_process_group("nccl", device_id=device, pg_options=opts, **kw)
    else:
        dist.init_process_group(backend, **kw)


def _host_staged(t: torch.Tensor, group) -> bool:
    """True when ``group``'s backend reduces a device tensor through host memory (gloo)."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def ordered_all_reduce(t: torch.Tensor, group=None, op=dist.ReduceOp.SUM,
                       async_op: bool = False):
    """``dist.all_reduce`` of a tensor the current stream is still producing, ordered after that
    work on every backend. RCCL ('nccl') enqueues on its own stream behind an event of the
    current stream. gloo stages a device tensor to pinned host memory on a pool stream behind such
    an event; in the one-device gloo rehearsals that copy sometimes read the tensor before the
    kernel producing it had written it (profiles/r05_scale/p2p_first/), so for gloo
    the current stream is drained on the host first. gloo's sum runs on the host anyway: the wait
    costs it nothing it would not pay."""
    if _host_staged(t, group):
        torch.cuda.current_stream(t.device).synchronize()
    return dist.all_reduce(t, op=op, group=group, async_op=async_op)


def ordered_broadcast(t: torch.Tensor, src: int, group=None, async_op: bool = False):
    """``dist.broadcast`` with :func:`ordered_all_reduce`'s ordering on gloo."""
    if _host_staged(t, group):
        torch.cuda.current_stream(t.device).synchronize()
    return dist.broadcast(t, src, group=group, async_op=async_op)


def shard_bounds(n_users: int, world: int, rank: int, degrees=None):
    """Contiguous user range of ``rank``. Without ``degrees``: sizes differ by at most one. With
    the users' interaction counts: degree-balanced ranges — cut ``r`` is the first
    user whose prefix count reaches r/world of the total (each hop's work and its
    nonzero bytes on a rank are its users' nonzeros plus their rows), so every rank gets the same
    share of nonzeros to within one user's degree. Cuts are non-decreasing; a rank may get no
    users when a few users hold most interactions."""
    if degrees is None:
        cuts = np.linspace(0, n_users, world + 1).astype(np.int64)
        return int(cuts[rank]), int(cuts[rank + 1])
    deg = np.asarray(degrees, dtype=np.int64).reshape(-1)
    if deg.shape[0] != n_users:
        raise ValueError(f"shard_bounds: {deg.shape[0]} degrees for {n_users} users")
    # weight = nonzeros + 1 (the row itself), so users without interactions still spread out
    prefix = np.concatenate([[0], np.cumsum(deg + 1)])
    total = int(prefix[-1])

    def cut(r):
        if r <= 0:
            return 0
        if r >= world:
            return n_users
        return int(np.searchsorted(prefix, (total * r + world - 1) // world, side="left"))

    return cut(rank), cut(rank + 1)


def shard_rows_of_sorted_coo(indices: torch.Tensor, n_users: int, world: int, rank: int,
                             degrees: Optional[torch.Tensor] = None):
    """This rank's share of a GLOBAL user×item COO whose rows are sorted (the row-major order of
    ``convert_sparse_mat_to_tensor``, base/torch_interface.py:8-12): the degree-balanced user
    range (:func:`shard_bounds`) and its entries re-indexed to local rows, in the input's order.
    Returns ``(u0, u1, local_indices)``; every global entry lies in exactly one rank's share."""
    rows = indices[0]
    if degrees is None:
        degrees = torch.bincount(rows, minlength=n_users)
    if rows.numel() > 1 and bool((rows[1:] < rows[:-1]).any()):
        raise ValueError("shard_rows_of_sorted_coo: rows must be sorted")
    u0, u1 = shard_bounds(n_users, world, rank, degrees.cpu().numpy())
    bounds = torch.tensor([u0, u1], dtype=rows.dtype, device=rows.device)
    lo, hi = torch.searchsorted(rows, bounds).tolist()
    loc = indices[:, lo:hi].clone()
    loc[0] -= u0
    return u0, u1, loc


TRANSPORTS = ("rccl", "p2p")


def _scale_of_degrees(deg: torch.Tensor, kind: str) -> torch.Tensor:
    """1/deg ('mean') or 1/sqrt(deg) ('sym') of float64 degrees, 0 where deg = 0, rounded to
    fp32: every step correctly rounded, so it is bitwise the library's hgd_degree_scale and the
    native communicator's global scales (handle.hip k_scale_from_f64)."""
    inv = deg if kind == "mean" else deg.sqrt()
    return torch.where(deg > 0, 1.0 / inv, torch.zeros_like(deg)).to(torch.float32)


# Deadline of each P2PExchange set-up call (HGD_P2P_SETUP_TIMEOUT_S, seconds), and the number of
# set-up calls that never returned in this process (p2p_setup_stuck).
_P2P_SETUP_TIMEOUT_S = float(os.environ.get("HGD_P2P_SETUP_TIMEOUT_S", "180"))
_P2P_STUCK = 0


def p2p_setup_stuck() -> int:
    """How many P2PExchange set-up calls of this process never returned. They are left running on
    daemon threads; a process with any should end with ``os._exit`` once its output is flushed,
    since the runtime's teardown may wait for them."""
    return _P2P_STUCK


# Lifetime of the exported peer segments. A segment may be freed only when (1) no peer can still
# be reading it — every rank has synchronised its device and passed the barrier of a COLLECTIVE
# close() — and (2) no slot view's storage is alive in this process. The destruction itself
# (hgd_p2p_destroy synchronises the device) never runs inside torch's storage release (a DLPack
# deleter can fire inside a graph capture or at interpreter teardown): a handle that becomes due
# there waits in _PENDING for the next safe point (P2PExchange set-up or close(),
# release_pending_p2p(), exit). An exchange dropped or released WITHOUT the collective close()
# goes to _ABANDONED and stays mapped — a peer's exchange kernel may still read it — until a
# collective close() in this process covers it too, or the process ends.
_PENDING: List["_P2PHandle"] = []
_ABANDONED: List["_P2PHandle"] = []
_PLOCK = threading.Lock()


class _P2PHandle:
    """Owns one ``hgd_p2p`` handle (its exported send / reduced slots); see the rules above."""

    def __init__(self, lib, h, group=None):
        self.lib, self.h = lib, h
        self.group = group   # the process group whose ranks map these segments
        self.live = 0
        self.closed = False  # a collective close() covered it: no peer reads it any more
        self.lock = threading.Lock()

    def view_born(self):
        with self.lock:
            self.live += 1

    def view_gone(self):
        """nat.float_view's deleter: bookkeeping only, never a HIP call."""
        with self.lock:
            self.live -= 1
            due = self.closed and self.live == 0 and self.h is not None
        if due:
            with _PLOCK:
                _PENDING.append(self)

    def close_collective(self):
        """After a collective close's barrier: destroy now, or when the last view goes."""
        with self.lock:
            self.closed = True
            due = self.live == 0
        if due:
            self.destroy()

    def abandon(self):
        """Dropped or released without the collective close: keep it mapped for now."""
        with self.lock:
            if self.closed or self.h is None:
                return
        with _PLOCK:
            _ABANDONED.append(self)

    def destroy(self):
        with self.lock:
            h, self.h = self.h, None
        if h is not None:
            self.lib.hgd_p2p_destroy(h)  # synchronises the device, closes the peers' mappings

    @property
    def alive(self) -> bool:
        return self.h is not None


def release_pending_p2p() -> int:
    """Destroys the peer-exchange handles whose last slot view went after their collective
    close() (a safe point: not inside a graph capture). Returns how many were destroyed."""
    with _PLOCK:
        due = list(_PENDING)
        _PENDING.clear()
    for hd in due:
        hd.destroy()
    return len(due)


def _close_abandoned(group):
    """Inside a collective close() over ``group``, after its barrier: every rank of the group has
    drained its device, so the segments of exchanges this process dropped earlier over the SAME
    group can go too (those of another group wait for a close over theirs)."""
    with _PLOCK:
        dropped = [hd for hd in _ABANDONED if hd.group is group]
        _ABANDONED[:] = [hd for hd in _ABANDONED if hd.group is not group]
    for hd in dropped:
        hd.close_collective()


def abandoned_p2p() -> int:
    """Handles of exchanges dropped without close() that are still mapped (tests)."""
    with _PLOCK:
        return sum(1 for hd in _ABANDONED if hd.alive)


@atexit.register
def _p2p_at_exit():
    try:
        release_pending_p2p()
    except Exception:  # noqa: BLE001 — the runtime may already be going down
        pass


class P2PExchange:
    """The direct xGMI peer transport (``hgd_p2p_*``, csrc/p2p.hip): every rank exposes one
    uncached buffer of ``n_slots`` send slots to its peers; an all-reduce of a slot is a two-shot
    reduce over the mesh (rank r sums block r of every rank's slot, reading the N-1 peers at once,
    then gathers the other blocks from the peers). Construction is collective over ``group``
    (the IPC handles travel by ``all_gather_object``)."""

    def __init__(self, max_count: int, n_slots: int, device: torch.device, group=None,
                 timeout_s: float = 30.0, trace=None, setup_timeout_s: Optional[float] = None):
        self.lib = nat.load()
        # the set-up calls (allocation, export, the peers' IPC opens) run on a helper thread with
        # a deadline: one that never returns — hipIpcOpenMemHandle of a ≥ 3.5 GiB uncached
        # allocation did that on ROCm 7.2 — becomes an error on every rank instead of a hang
        self.setup_timeout_s = float(setup_timeout_s if setup_timeout_s is not None else
                                     _P2P_SETUP_TIMEOUT_S)
        self._stuck = False
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        self.device = torch.device(device)
        self.max_count = int(-(-int(max_count) // 4) * 4)
        self.n_slots = int(n_slots)
        self.timeout_s = float(timeout_s)
        trace = trace or (lambda msg: None)
        self.h = None
        self._handle = None  # _P2PHandle: the handle's lifetime (slot views may outlive close)
        release_pending_p2p()  # a safe point: handles whose last view went since
        self._views = {}
        # every step that can fail locally is followed by an agreement among the ranks, so a
        # failure on one rank raises on all of them (none is left waiting in a collective)
        h = ctypes.c_void_p()
        mine = ctypes.create_string_buffer(nat.P2P_HANDLE_BYTES)
        err = self._try(lambda: self.lib.hgd_p2p_create(self.world, self.rank, self.max_count,
                                                        self.n_slots, ctypes.byref(h)),
                        "hgd_p2p_create")
        if err is None:
            self.h = h
            self._handle = _P2PHandle(self.lib, h, group)
            err = self._try(lambda: self.lib.hgd_p2p_set_timeout(h, self.timeout_s),
                            "hgd_p2p_set_timeout") or self._try(
                lambda: self.lib.hgd_p2p_export(h, mine), "hgd_p2p_export")
        trace("p2p: created and exported" if err is None else f"p2p: {err}")
        entries = [None] * self.world
        if self.world > 1:
            dist.all_gather_object(entries, (mine.raw if err is None else None, err),
                                   group=group)
        else:
            entries = [(mine.raw, err)]
        self._agree([e[1] for e in entries])
        trace("p2p: handles gathered")
        blob = ctypes.create_string_buffer(b"".join(e[0] for e in entries),
                                           nat.P2P_HANDLE_BYTES * self.world)
        err = self._try(lambda: self.lib.hgd_p2p_open(h, blob), "hgd_p2p_open")
        errs = [err]
        if self.world > 1:
            errs = [None] * self.world
            dist.all_gather_object(errs, err, group=group)
        self._agree(errs)
        trace("p2p: peers opened")

    def _try(self, call, what):
        """Runs one hgd_p2p_* set-up call on a helper thread (bound to this exchange's device)
        and waits at most ``setup_timeout_s`` for it: None, or the error text. A call that has
        not returned by then is left running; the exchange is marked stuck and its buffers are
        never released (the call may still be using them)."""
        if self._stuck:
            return f"{what}: skipped after an earlier set-up call did not return"
        box = {}

        def run():
            try:
                if self.device.type == "cuda":
                    torch.cuda.set_device(self.device)
                st = call()
                box["err"] = None if st == nat.HGD_OK else (
                    f"{what}: {self.lib.hgd_get_last_error_string().decode(errors='replace')}")
            except Exception as e:  # noqa: BLE001 — reported like a failed call
                box["err"] = f"{what}: {e!r}"
        th = threading.Thread(target=run, name=f"hgd-p2p-{what}", daemon=True)
        th.start()
        th.join(self.setup_timeout_s)
        if th.is_alive():
            global _P2P_STUCK
            _P2P_STUCK += 1
            self._stuck = True
            return f"{what}: did not return within {self.setup_timeout_s:.0f} s"
        return box["err"]

    def _agree(self, errs):
        bad = [(q, e) for q, e in enumerate(errs) if e is not None]
        if bad:
            if self._handle is not None and not self._stuck:
                self._handle.destroy()  # set-up failed on some rank: no exchange ever ran
            self._handle = None
            self.h = None
            raise nat.HGDNativeError("P2PExchange: " + "; ".join(f"rank {q}: {e}"
                                                                  for q, e in bad))

    def slot(self, k: int, rows: int, cols: int) -> torch.Tensor:
        """Send slot ``k`` as a [rows, cols] float32 view (the hop kernels write into it)."""
        if rows * cols > self.max_count:
            raise ValueError(f"P2PExchange: slot of {rows}x{cols} > {self.max_count} floats")
        if self.h is None:
            raise RuntimeError("P2PExchange: closed")
        key = (k, rows, cols)
        v = self._views.get(key)
        if v is None:
            addr = self.lib.hgd_p2p_slot(self.h, int(k))
            if not addr:
                raise ValueError(f"P2PExchange: no slot {k}")
            hd = self._handle
            hd.view_born()
            v = self._views[key] = nat.float_view(addr, (rows, cols), self.device,
                                                  on_release=hd.view_gone)
        return v

    def allreduce(self, k: int, count: int, out: torch.Tensor, stream_handle: int) -> None:
        """out[:count] = Σ_ranks slot k[:count], ordered on the given raw stream."""
        nat.check(self.lib.hgd_p2p_allreduce(self.h, int(k), int(count), out.data_ptr(),
                                             stream_handle), "hgd_p2p_allreduce")

    def check(self) -> None:
        nat.check(self.lib.hgd_p2p_check(self.h), "hgd_p2p")

    def poll(self) -> None:
        """Raises if a wait that has already run timed out (a host-visible flag: no sync)."""
        nat.check(self.lib.hgd_p2p_poll(self.h), "hgd_p2p")

    def wait(self, stream: Optional[torch.cuda.Stream] = None,
             timeout_s: Optional[float] = None) -> None:
        """Waits on the host until the work queued so far on ``stream`` (default: the current
        stream) has finished, for at most ``timeout_s`` (default: twice the device wait bound
        plus a minute); raises TimeoutError instead of blocking forever, so a stall anywhere in
        the device queue — not only in a wait kernel that is running — surfaces as an error."""
        stream = stream or torch.cuda.current_stream(self.device)
        ev = torch.cuda.Event()
        ev.record(stream)
        limit = timeout_s if timeout_s is not None else 2.0 * self.timeout_s + 60.0
        t0 = time.perf_counter()
        pause = 1e-4
        while not ev.query():
            if time.perf_counter() - t0 > limit:
                raise TimeoutError(f"hgd_p2p rank {self.rank}: device queue not drained after "
                                   f"{limit:.0f} s (device-side wait bound {self.timeout_s} s)")
            time.sleep(pause)
            pause = min(2 * pause, 0.05)

    def close(self) -> None:
        """Collective: every rank synchronises its device and passes a barrier, so no peer reads
        this exchange's segments (nor those of exchanges this process dropped earlier) any more.
        The exchange is unusable afterwards; its memory is freed now, or — if a slot view handed
        out is still alive — at the first safe point after the last one goes."""
        if self.h is None:
            return
        torch.cuda.synchronize(self.device)
        if self.world > 1:
            dist.barrier(group=self.group)
        self.h = None
        self._views.clear()
        if self._handle is not None and not self._stuck:
            self._handle.close_collective()
        self._handle = None
        _close_abandoned(self.group)
        release_pending_p2p()

    def release(self) -> None:
        """Non-collective close (no barrier): the exchange stops being usable, but its segments
        stay mapped — a peer's exchange kernel may still be reading them — until a collective
        close() in this process covers them, or the process ends. What a dropped exchange does."""
        self.h = None
        self._views.clear()
        if self._handle is not None and not self._stuck:
            self._handle.abandon()
        self._handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        try:
            if getattr(self, "h", None) is not None:
                self.release()
        except Exception:  # noqa: BLE001 — interpreter teardown
            pass


class ExchangeTimer:
    """Exposed exchange time of the sharded hops: while active, each hop 2 records an event on
    the compute stream just before it waits for its slice's exchange and one right after; the
    pair's interval is the time the compute stream sat idle waiting for the all-reduce (0 when
    the exchange was hidden behind the preceding hop-1 kernels)."""

    def __init__(self):
        self.pairs: List[Tuple] = []

    def __enter__(self):
        global _XTIMER
        self._prev, _XTIMER = _XTIMER, self
        return self

    def __exit__(self, *exc):
        global _XTIMER
        _XTIMER = self._prev
        return False

    def mark(self):
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        return ev

    def add(self, a, b):
        self.pairs.append((a, b))

    def total_ms(self) -> float:
        torch.cuda.synchronize()
        return float(sum(a.elapsed_time(b) for a, b in self.pairs))


_XTIMER: Optional[ExchangeTimer] = None


class ShardedIncidence:
    """One rank's slice of H (users [u0,u1) × all items) plus global item scales.

    ``slice_width``: embedding columns per pipelined exchange block (None: 32 for d ≤ 128, else
    64; a multiple of 4 keeps the float4 gathers). ``n_chunks``: item-row chunks per slice (RCCL
    transport). ``transport``: 'rccl' (torch.distributed all-reduce, backend "nccl" = RCCL) or
    'p2p' (:class:`P2PExchange`: hop 1 writes each slice straight into an exposed send slot and
    the slice's two-shot mesh reduce runs on a high-priority side stream)."""

    def __init__(self, inc: Incidence, group=None, n_chunks: int = 1,
                 P: Optional[str] = "sym", Q: Optional[str] = "mean", R: Optional[str] = "sym",
                 slice_width: Optional[int] = None, transport: str = "rccl",
                 p2p_timeout_s: float = 30.0, trace=None):
        if transport not in TRANSPORTS:
            raise ValueError(f"ShardedIncidence: transport must be one of {TRANSPORTS}")
        self.inc = inc
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.P, self.R = P, R
        self.transport = transport
        self.p2p_timeout_s = float(p2p_timeout_s)
        self.trace = trace
        self.n_chunks = max(1, int(n_chunks)) if self.world > 1 else 1
        self.slice_width = slice_width
        self._p2p = None
        self._side = None
        self._calls = 0
        self.q = self._global_col_scale(Q)
        # item-row chunk boundaries for the overlapped exchange
        n_items = inc.n_cols
        step = (n_items + self.n_chunks - 1) // self.n_chunks if n_items else 0
        self.bounds = [(min(k * step, n_items), min((k + 1) * step, n_items))
                       for k in range(self.n_chunks)]
        self.bounds = [(a, b) for a, b in self.bounds if b > a] or [(0, n_items)]

    @classmethod
    def from_global(cls, indices: torch.Tensor, n_users: int, n_items: int, group=None,
                    device=None, **kw) -> Tuple["ShardedIncidence", int, int]:
        """Shards a global row-sorted user×item COO (int64 [2, nnz]) over the ranks of ``group``
        by degree-balanced user ranges; returns ``(shard, u0, u1)``."""
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        u0, u1, loc = shard_rows_of_sorted_coo(indices, n_users, world, rank)
        inc = Incidence.from_coo(loc, None, (u1 - u0, n_items),
                                 device=device if device is not None else indices.device,
                                 validate=False, rows_sorted=True)
        return cls(inc, group=group, **kw), u0, u1

    def slices(self, d: int) -> List[Tuple[int, int]]:
        """Column ranges of the pipelined exchange (one range on a single rank unless
        ``slice_width`` is given explicitly, which measures the sliced hops alone)."""
        if self.world == 1 and self.slice_width is None:
            return [(0, d)]
        w = self.slice_width or (32 if d <= 128 else 64)
        w = max(4, (int(w) // 4) * 4)
        return [(c, min(c + w, d)) for c in range(0, d, w)]

    def exchange_bytes(self, d: int) -> int:
        """fp32 bytes all-reduced per hop pair (the [I, d] item messages)."""
        return 0 if self.world == 1 else 4 * self.inc.n_cols * d

    def _global_col_scale(self, kind: Optional[str]) -> Optional[torch.Tensor]:
        if kind is None:
            return None
        if self.world == 1:
            return self.inc.scale("col", kind)
        if kind not in ("mean", "sym"):
            raise ValueError(f"sharded: unsupported item scale {kind!r}")
        deg = (self.inc.csc.rowptr[1:] - self.inc.csc.rowptr[:-1]).to(torch.float64)
        ordered_all_reduce(deg, group=self.group)
        return _scale_of_degrees(deg, kind)

    def p2p(self, d: int) -> P2PExchange:
        """The peer transport for width ``d`` (created on first use: collective)."""
        sl = self.slices(d)
        need = self.inc.n_cols * max(c1 - c0 for c0, c1 in sl)
        if self._p2p is None or self._p2p.max_count < need or self._p2p.n_slots < 2 * len(sl):
            if self._p2p is not None:
                self._p2p.close()
            self._p2p = P2PExchange(need, 2 * len(sl), self.inc.device, group=self.group,
                                    timeout_s=self.p2p_timeout_s, trace=self.trace)
        if self._side is None:
            lo, _hi = torch.cuda.Stream.priority_range()
            self._side = torch.cuda.Stream(self.inc.device, priority=min(lo, _hi))
        return self._p2p

    def close(self) -> None:
        """Collective when the peer transport is up (its close is)."""
        if self._p2p is not None:
            self._p2p.close()
            self._p2p = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def __del__(self):
        # dropped without close(): the exchange is released without a collective, its segments
        # kept mapped until a collective close() (P2PExchange.release)
        try:
            if getattr(self, "_p2p", None) is not None:
                self._p2p.release()
                self._p2p = None
        except Exception:  # noqa: BLE001 — interpreter teardown
            pass

    def two_hop(self, X: torch.Tensor, src_kind: Optional[str],
                dst_kind: Optional[str]) -> torch.Tensor:
        """``S_dst·H_g·Σ_ranks(Q·H_gᵀ·S_src·X_g)`` with the slice pipeline described above."""
        inc = self.inc
        d = X.shape[1]
        Y = torch.empty((inc.n_rows, d), dtype=torch.float32, device=X.device)
        val_t = inc.edge_values("csc", src_kind)
        row_scale = inc.scale("row", dst_kind)
        use_p2p = self.transport == "p2p" and self.world > 1
        sl = self.slices(d)
        if use_p2p:
            ex = self.p2p(d)
            # an earlier exchange that timed out leaves NaN in its output; stop at the next call
            # instead of propagating it (the flag is host-visible, no synchronisation)
            ex.poll()
            parity = self._calls % 2
            self._calls += 1
            cur = torch.cuda.current_stream(X.device)
            side_h = self._side.cuda_stream
        pieces = []
        for s, (c0, c1) in enumerate(sl):
            w = c1 - c0
            Xs = X if w == d else X[:, c0:c1]
            works: List = []
            if use_p2p:
                k = parity * len(sl) + s
                send = ex.slot(k, inc.n_cols, w)
                # never source-blocked: the send slot is uncached exchange memory, which the
                # blocked hop would read back once per extra block
                spmm_csr(inc.csc, Xs, val=val_t, row_scale=self.q, out=send, blocks=0)
                Ms = torch.empty((inc.n_cols, w), dtype=torch.float32, device=X.device)
                ready = torch.cuda.Event()
                ready.record(cur)
                self._side.wait_event(ready)
                ex.allreduce(k, inc.n_cols * w, Ms, side_h)
                done = torch.cuda.Event()
                done.record(self._side)
                works.append(done)
            else:
                Ms = torch.empty((inc.n_cols, w), dtype=torch.float32, device=X.device)
                for a, b in self.bounds:
                    spmm_csr(inc.csc, Xs, val=val_t, row_scale=self.q, out=Ms, row_begin=a,
                             row_end=b)
                    if self.world > 1:
                        works.append(ordered_all_reduce(Ms[a:b], group=self.group,
                                                        async_op=True))
            pieces.append((c0, c1, Ms, works))
        xt = _XTIMER if self.world > 1 else None
        for c0, c1, Ms, works in pieces:
            before = xt.mark() if xt is not None else None
            for wk in works:
                if use_p2p:
                    torch.cuda.current_stream(X.device).wait_event(wk)
                else:
                    wk.wait()
            if xt is not None:
                xt.add(before, xt.mark())
            out = Y if c1 - c0 == d else Y[:, c0:c1]
            spmm_csr(inc.csr, Ms, val=inc.val, row_scale=row_scale, out=out)
        return Y


class _ShardedHGConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, sh: ShardedIncidence):
        ctx.sh = sh
        return sh.two_hop(X.contiguous(), sh.R, sh.P)

    @staticmethod
    def backward(ctx, dY):
        sh = ctx.sh
        return sh.two_hop(dY.contiguous(), sh.P, sh.R), None


def sharded_two_hop(sh: ShardedIncidence, X_local: torch.Tensor) -> torch.Tensor:
    """P·H·Q·Hᵀ·R·X on user-row shards (X_local = this rank's user rows)."""
    return _ShardedHGConv.apply(X_local, sh)


# ---------------------------------------------------------------------------------------------
# The model-side operators on user-row shards (SURVEY.md §8e "HCCF specifics"): the bipartite
# node graph of HCCF / HGCNConv / ED-HNN and HCCF's learned dense hypergraph.
#
# Convention for replicated tensors (item rows, the [K, d] hyperedge messages): every rank holds
# the same VALUE, and the gradient a rank computes for it is that rank's PARTIAL gradient (its own
# loss terms); the true gradient is the sum over ranks. So an all-reduce in the forward has an
# all-reduce as its backward, a replicated tensor consumed by a local op needs no exchange, and
# replicated parameters (item embeddings, W) get their partial gradients summed once before the
# optimizer step (:func:`allreduce_replicated_grads`, what DDP does for every parameter).
# ---------------------------------------------------------------------------------------------

from . import _native as nat  # noqa: E402
from .functional import _epilogue_apply, _epilogue_backward, _nn, _nt, _tn  # noqa: E402,F401


class _AllReduceSum(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, group):
        ctx.group = group
        y = x.contiguous().clone()
        ordered_all_reduce(y, group=group)
        return y

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous().clone()
        ordered_all_reduce(g, group=ctx.group)
        return g, None


def all_reduce_sum(x: torch.Tensor, group=None) -> torch.Tensor:
    """Σ over ranks of per-rank partials, differentiable (backward = the same sum)."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return x
    return _AllReduceSum.apply(x, group)


def allreduce_replicated_grads(params, group=None) -> None:
    """Sums the partial gradients of replicated parameters over ranks (call before step())."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        return
    for p in params:
        if p.grad is not None:
            ordered_all_reduce(p.grad, group=group)


def block_coo(indices: torch.Tensor, values: Optional[torch.Tensor], n_users: int, u0: int,
              u1: int):
    """The two blocks of a bipartite [N, N] COO (users first) that user rows [u0, u1) own:
    ``B = A[u0:u1, U:]`` (local users → items) and ``C = A[U:, u0:u1]`` (items → local users),
    re-indexed locally in CSR order (the input's order when it is row-sorted, else a stable row
    sort of it), with the positions of their entries in the input (to slice a global drop-edge
    mask the same way)."""
    r, c = indices[0], indices[1]
    sel_b = ((r >= u0) & (r < u1) & (c >= n_users)).nonzero().flatten()
    sel_c = ((r >= n_users) & (c >= u0) & (c < u1)).nonzero().flatten()
    # a row-unsorted (or uncoalesced) input: order each block by row, stably, so the block COO is
    # in CSR order and a global mask sliced by sel_b / sel_c lines up with Incidence.drop's
    for_sort = []
    for sel in (sel_b, sel_c):
        rs = r[sel]
        if rs.numel() > 1 and bool((rs[1:] < rs[:-1]).any()):
            sel = sel[torch.sort(rs, stable=True).indices]
        for_sort.append(sel)
    sel_b, sel_c = for_sort
    b_idx = torch.stack([r[sel_b] - u0, c[sel_b] - n_users])
    c_idx = torch.stack([r[sel_c] - n_users, c[sel_c] - u0])
    b_val = None if values is None else values[sel_b]
    c_val = None if values is None else values[sel_c]
    return b_idx, b_val, c_idx, c_val, sel_b, sel_c


def _transposed(inc):
    """Aᵀ of an Incidence as an Incidence sharing its arrays (CSR and CSC swap roles)."""
    t = Incidence(inc.csc, inc.csr, inc.val_t, inc.val)
    if inc.perm_t is not None:
        inv = torch.empty_like(inc.perm_t)
        inv[inc.perm_t.long()] = torch.arange(inc.nnz, dtype=inv.dtype, device=inv.device)
        t.perm_t = inv
    t.coo_sorted = True
    return t


def _fold(base: Optional[torch.Tensor], scale: torch.Tensor, col: torch.Tensor, nnz: int):
    """w[e] = base[e] · scale[col[e]] (hgd_edge_values): a source-side diagonal folded into the
    per-nonzero weights of a hop."""
    out = torch.empty(nnz, dtype=torch.float32, device=scale.device)
    if nnz:
        nat.check(nat.load().hgd_edge_values(
            nat.ptr(base), None, scale.data_ptr(), col.data_ptr(), nnz, out.data_ptr(),
            nat.stream_handle(scale.device)), "hgd_edge_values")
    return out


class ShardedBipartite:
    """One rank's share of a bipartite node operator ``A [N, N] = [[0, B], [C, 0]]`` (users
    first: ``Interaction.__create_sparse_bipartite_adjacency`` / ``normalize_graph_mat``,
    data/ui_graph.py:70-84, data/graph.py:11-25) under user-row sharding.

    The rank owns users [u0, u1) and holds ``B_g = A[u0:u1, U:]`` and ``C_g = A[U:, u0:u1]`` as
    incidences; for a symmetric A (norm_adj, ui_adj) ``C_g = B_gᵀ`` is B_g's own CSC. A hop
    ``Y = S·A·X`` on the local layout ``[X_u[u0:u1]; X_i]`` is

        Y_i = Σ_g S_i·C_g·X_u,g    CSR hop of C_g into the item rows, chunked, RCCL all-reduce
        Y_u = S_u·B_g·X_i          local CSR hop, issued while the item chunks are in flight

    and its backward (partial dY_i per rank) is dY_i ← Σ_g dY_i (all-reduce, overlapped with
    dX_i = B_gᵀ·S_u·dY_u, a partial), then dX_u = C_gᵀ·S_i·dY_i. S is an optional row scale of
    the GLOBAL degrees ('mean' 1/deg, the ED-HNN means; 'sym' deg^-1/2); item degrees are
    all-reduced once per kind."""

    def __init__(self, B, C=None, group=None, n_chunks: int = 4):
        self.B = B
        self.C = C if C is not None else _transposed(B)
        self.symmetric = C is None
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.n_local = B.n_rows
        self.n_items = B.n_cols
        if self.C.n_rows != self.n_items or self.C.n_cols != self.n_local:
            raise ValueError("ShardedBipartite: C must be [items, local users]")
        self.n_chunks = max(1, int(n_chunks)) if self.world > 1 else 1
        step = -(-self.n_items // self.n_chunks) if self.n_items else 0
        self.bounds = [(k * step, min((k + 1) * step, self.n_items))
                       for k in range(self.n_chunks) if k * step < self.n_items] or [(0, 0)]
        self.sel_b = self.sel_c = None
        self._scales = {}
        self._folded = {}

    @classmethod
    def from_global(cls, adj, n_users: int, n_items: int, u0: int, u1: int, device=None,
                    group=None, n_chunks: int = 4, symmetric: Optional[bool] = None):
        """Slices a global bipartite adjacency — a torch sparse COO as
        ``convert_sparse_mat_to_tensor`` builds it (base/torch_interface.py:8-12), or
        (indices, values) — into this rank's blocks. ``symmetric=None`` checks C_g == B_gᵀ on
        the device and then keeps only B_g."""
        if isinstance(adj, torch.Tensor):
            idx, val = adj._indices(), adj._values()
            if tuple(adj.shape) != (n_users + n_items, n_users + n_items):
                raise ValueError("ShardedBipartite: adjacency must be [U+I, U+I]")
        else:
            idx, val = adj
        device = torch.device(device) if device is not None else torch.device("cuda")
        idx = idx.to(device)
        val = None if val is None else val.to(device=device, dtype=torch.float32)
        b_idx, b_val, c_idx, c_val, sel_b, sel_c = block_coo(idx, val, n_users, u0, u1)
        n_loc = u1 - u0
        B = Incidence.from_coo(b_idx, b_val, (n_loc, n_items), device=device)
        C = None
        if symmetric is not True:
            C = Incidence.from_coo(c_idx, c_val, (n_items, n_loc), device=device)
            if symmetric is None and _same_transpose(B, C):
                C = None
        sh = cls(B, C, group=group, n_chunks=n_chunks)
        sh.sel_b, sh.sel_c = sel_b, sel_c
        return sh

    def transpose(self) -> "ShardedBipartite":
        """Aᵀ = [[0, Cᵀ], [Bᵀ, 0]] on the same partition (B' = C_gᵀ, C' = B_gᵀ, sharing their
        arrays); a symmetric A is its own transpose. Needed once A is edge-dropped: HGCNConv is
        A·(Aᵀ·X) (HGNN_HD4.py:459)."""
        if self.symmetric:
            return self
        t = getattr(self, "_t", None)
        if t is None:
            t = ShardedBipartite(_transposed(self.C), _transposed(self.B), group=self.group,
                                 n_chunks=self.n_chunks)
            t._t = self
            self._t = t
        return t

    # -- scales ------------------------------------------------------------------------------
    def scale(self, side: str, kind: Optional[str]) -> Optional[torch.Tensor]:
        """Global-degree row scale of the user ('user') or item ('item') rows of A."""
        if kind is None:
            return None
        key = (side, kind)
        if key in self._scales:
            return self._scales[key]
        if kind not in ("mean", "sym"):
            raise ValueError(f"ShardedBipartite: unsupported scale {kind!r}")
        o = self.B.csr if side == "user" else self.C.csr
        deg = (o.rowptr[1:] - o.rowptr[:-1]).to(torch.float64)
        if side == "item" and self.world > 1:
            ordered_all_reduce(deg, group=self.group)
        s = _scale_of_degrees(deg, kind)
        self._scales[key] = s
        return s

    def _src_folded(self, which: str, kind: Optional[str]):
        """Backward-hop weights with the forward's output scale folded in as a source scale:
        'c_t' = C_gᵀ·S_i (into users), 'b_t' = B_gᵀ·S_u (into items)."""
        inc = self.C if which == "c_t" else self.B
        if kind is None:
            return inc.val_t
        key = (which, kind)
        if key not in self._folded:
            s = self.scale("item" if which == "c_t" else "user", kind)
            self._folded[key] = _fold(inc.val_t, s, inc.csc.col, inc.nnz)
        return self._folded[key]

    # -- drop-edge (SpAdjDropEdge, HCCF.py:213-226) ------------------------------------------
    def drop(self, keep: float, mask_b: torch.Tensor, mask_c: torch.Tensor) -> "ShardedBipartite":
        """The shard of the edge-dropped adjacency: ``mask_b`` / ``mask_c`` select B_g's and C_g's
        nonzeros in CSR order (for parity with the reference's global ``torch.rand(nnz)`` mask,
        :meth:`drop_global`). The result is never symmetric (the blocks drop independently)."""
        B = self.B.drop(mask_b, keep)
        C = self.C.drop(mask_c, keep)
        return ShardedBipartite(B, C, group=self.group, n_chunks=self.n_chunks)

    def drop_global(self, keep: float, mask: torch.Tensor) -> "ShardedBipartite":
        """:meth:`drop` with the reference's mask over the GLOBAL COO (same draw on every rank)."""
        if self.sel_b is None:
            raise RuntimeError("drop_global needs a shard built by from_global")
        mask = mask.to(self.sel_b.device)
        return self.drop(keep, mask[self.sel_b], mask[self.sel_c])

    def drop_device(self, keep: float, seed: int) -> "ShardedBipartite":
        """:meth:`drop` with device keep-masks (hgd_bernoulli_mask): every global nonzero lies in
        exactly one rank's B_g or C_g, so per-rank draws are one independent Bernoulli per
        entry, as the reference's. ``seed`` should differ per rank."""
        lib = nat.load()
        masks = []
        for k, inc in enumerate((self.B, self.C)):
            m = torch.empty(inc.nnz, dtype=torch.uint8, device=inc.device)
            if inc.nnz:
                nat.check(lib.hgd_bernoulli_mask(
                    (int(seed) * 2 + k) & ((1 << 62) - 1), inc.nnz, float(keep), m.data_ptr(),
                    nat.stream_handle(inc.device)), "hgd_bernoulli_mask")
            masks.append(m)
        return self.drop(keep, masks[0], masks[1])


def _same_transpose(B, C) -> bool:
    """C == Bᵀ exactly (structure and values): C's CSR against B's CSC."""
    if B.nnz != C.nnz:
        return False
    if not torch.equal(B.csc.rowptr, C.csr.rowptr) or not torch.equal(B.csc.col, C.csr.col):
        return False
    if (B.val is None) != (C.val is None):
        return False
    return B.val is None or torch.equal(B.val_t, C.val)


class _BipartiteHop(torch.autograd.Function):
    @staticmethod
    def forward(ctx, X, sh: ShardedBipartite, kind):
        ctx.sh, ctx.kind = sh, kind
        n = sh.n_local
        X = X.contiguous()
        Y = torch.empty_like(X)
        Yi = Y[n:]
        works: List = []
        for a, b in sh.bounds:
            if b > a:
                spmm_csr(sh.C.csr, X[:n], val=sh.C.val, row_scale=sh.scale("item", kind),
                         out=Yi, row_begin=a, row_end=b)
            if sh.world > 1:
                works.append(ordered_all_reduce(Yi[a:b], group=sh.group, async_op=True))
        spmm_csr(sh.B.csr, X[n:], val=sh.B.val, row_scale=sh.scale("user", kind), out=Y[:n])
        for w in works:
            w.wait()
        return Y

    @staticmethod
    def backward(ctx, dY):
        return _bipartite_backward(ctx.sh, ctx.kind, dY.contiguous()), None, None


def _bipartite_backward(sh: "ShardedBipartite", kind, dY: torch.Tensor) -> torch.Tensor:
    """dX of ``S·A·X`` on the local layout: the item rows' partial gradients are summed over
    the ranks (all-reduce, overlapped with dX_i = B_gᵀ·S_u·dY_u, a partial), then
    dX_u = C_gᵀ·S_i·dY_i."""
    n = sh.n_local
    w_b, w_c = sh._src_folded("b_t", kind), sh._src_folded("c_t", kind)  # before the async
    dYi = dY[n:]
    work = None
    if sh.world > 1:
        dYi = dYi.clone()
        work = ordered_all_reduce(dYi, group=sh.group, async_op=True)
    dX = torch.empty_like(dY)
    # partial dX_i = B_gᵀ·S_u·dY_u while the item gradient is summed
    spmm_csr(sh.B.csc, dY[:n], val=w_b, out=dX[n:])
    if work is not None:
        work.wait()
    spmm_csr(sh.C.csc, dYi, val=w_c, out=dX[:n])
    return dX


class _BipartiteHopFused(torch.autograd.Function):
    """``out_scale·LN(act(S·A·X)) + s1·res1 + s2·res2`` on the local layout: the user rows'
    epilogue runs in the store of their (local, complete) hop (hgd_spmm_fused); the item rows are
    complete only after their exchange, so on N > 1 ranks their epilogue is one row pass after it
    (hgd_row_epilogue_forward) — on one rank it is fused too. The backward is one
    hgd_row_epilogue_backward over all local rows, then the hop's backward."""

    @staticmethod
    def forward(ctx, X, gamma, beta, res1, res2, sh: "ShardedBipartite", kind, cfg):
        epi, slope, ln, eps, out_scale, s1, s2 = cfg
        X = X.contiguous()
        n = sh.n_local
        N, d = X.shape
        dev = X.device
        Y = torch.empty_like(X)
        A = torch.empty_like(X) if (ln or epi != nat.EPI_NONE) else None
        stats = torch.empty((N, 2), dtype=torch.float32, device=dev) if ln else None
        res1 = None if res1 is None else res1.contiguous()
        res2 = None if res2 is None else res2.contiguous()

        def ex_rows(r0):  # the epilogue descriptor for local rows r0, r0+1, ...
            return nat.RowEpilogue(
                act=epi, slope=slope, layer_norm=int(ln), ln_eps=eps,
                ln_gamma=nat.ptr(gamma) if ln else None, ln_beta=nat.ptr(beta) if ln else None,
                out_scale=out_scale,
                res1=None if res1 is None else res1[r0:].data_ptr(),
                ld_res1=0 if res1 is None else res1.stride(0), res1_scale=s1,
                res2=None if res2 is None else res2[r0:].data_ptr(),
                ld_res2=0 if res2 is None else res2.stride(0), res2_scale=s2,
                act_out=None if A is None else A[r0:].data_ptr(),
                ld_act=0 if A is None else A.stride(0),
                stats=None if stats is None else stats[r0:].data_ptr())

        si, su = sh.scale("item", kind), sh.scale("user", kind)
        works: List = []
        Zi = None
        if sh.world > 1:
            Zi = torch.empty((sh.n_items, d), dtype=torch.float32, device=dev)
            for a, b in sh.bounds:
                if b > a:
                    spmm_csr(sh.C.csr, X[:n], val=sh.C.val, row_scale=si, out=Zi, row_begin=a,
                             row_end=b)
                works.append(ordered_all_reduce(Zi[a:b], group=sh.group, async_op=True))
        else:
            spmm_csr(sh.C.csr, X[:n], val=sh.C.val, row_scale=si, out=Y[n:], ex=ex_rows(n))
        spmm_csr(sh.B.csr, X[n:], val=sh.B.val, row_scale=su, out=Y[:n], ex=ex_rows(0))
        for w in works:
            w.wait()
        if Zi is not None and sh.n_items:
            ex = ex_rows(n)
            nat.check(nat.load().hgd_row_epilogue_forward(
                Zi.data_ptr(), Zi.stride(0), sh.n_items, d, ctypes.byref(ex), Y[n:].data_ptr(),
                Y.stride(0), nat.stream_handle(dev)),
                "hgd_row_epilogue_forward")
        ctx.sh, ctx.kind, ctx.cfg = sh, kind, cfg
        ctx.has_res = (res1 is not None, res2 is not None)
        ctx.save_for_backward(A, stats, gamma if ln else None)
        return Y

    @staticmethod
    def backward(ctx, dY):
        epi, slope, ln, eps, out_scale, s1, s2 = ctx.cfg
        A, stats, gamma = ctx.saved_tensors
        dY = dY.contiguous()
        N, d = dY.shape
        dev = dY.device
        want_g = ln and ctx.needs_input_grad[1]
        want_b = ln and ctx.needs_input_grad[2]
        dgamma = torch.empty(d, dtype=torch.float32, device=dev) if want_g else None
        dbeta = torch.empty(d, dtype=torch.float32, device=dev) if want_b else None
        if not ln and epi == nat.EPI_NONE:
            dZ = dY if out_scale == 1.0 else dY * out_scale
        else:
            lib = nat.load()
            wsb = lib.hgd_row_epilogue_backward_workspace_size(N, d) if (want_g or want_b) else 0
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev) if wsb else None
            dZ = torch.empty_like(dY)
            nat.check(lib.hgd_row_epilogue_backward(
                dY.data_ptr(), dY.stride(0), nat.ptr(A), 0 if A is None else A.stride(0),
                nat.ptr(stats), nat.ptr(gamma), N, d, epi, float(slope), int(ln),
                float(out_scale), dZ.data_ptr(), dZ.stride(0), nat.ptr(dgamma), nat.ptr(dbeta),
                nat.ptr(ws), wsb, nat.stream_handle(dev)),
                "hgd_row_epilogue_backward")
        dX = _bipartite_backward(ctx.sh, ctx.kind, dZ) if ctx.needs_input_grad[0] else None

        def res_grad(k, s):
            if not ctx.has_res[k] or not ctx.needs_input_grad[3 + k]:
                return None
            return dY if s == 1.0 else dY * s

        return dX, dgamma, dbeta, res_grad(0, s1), res_grad(1, s2), None, None, None


def bipartite_hop_fused(sh: "ShardedBipartite", X_local: torch.Tensor,
                        scale: Optional[str] = None, epilogue: Optional[str] = None,
                        slope: float = 0.0, norm: Optional[torch.nn.LayerNorm] = None,
                        out_scale: float = 1.0, res1: Optional[torch.Tensor] = None,
                        res1_scale: float = 1.0, res2: Optional[torch.Tensor] = None,
                        res2_scale: float = 1.0) -> torch.Tensor:
    """``out_scale·norm(epi(S·A·X)) + res1_scale·res1 + res2_scale·res2`` on this rank's
    layout (functional.two_hop_fused's store for the sharded hop); falls back to the separate
    row pass where the fused store cannot hold a row (LayerNorm with d > 256)."""
    from .functional import _EPI, _ln_supported, row_epilogue
    if X_local.shape[0] != sh.n_local + sh.n_items:
        raise ValueError(f"bipartite_hop_fused: X has {X_local.shape[0]} rows, shard expects "
                         f"{sh.n_local} users + {sh.n_items} items")
    d = X_local.shape[1]
    ln = norm is not None
    epi = _EPI[epilogue]
    if (ln and not _ln_supported(d)) or (epi != nat.EPI_NONE and slope < 0):
        return row_epilogue(bipartite_hop(sh, X_local, scale), epilogue=epilogue, slope=slope,
                            norm=norm, out_scale=out_scale, res1=res1, res1_scale=res1_scale,
                            res2=res2, res2_scale=res2_scale)
    gamma = norm.weight if ln and norm.weight is not None else None
    beta = norm.bias if ln and norm.bias is not None else None
    cfg = (epi, float(slope), ln, float(norm.eps) if ln else 0.0, float(out_scale),
           float(res1_scale), float(res2_scale))
    return _BipartiteHopFused.apply(X_local, gamma, beta, res1, res2, sh, scale, cfg)


def bipartite_hop(sh: ShardedBipartite, X_local: torch.Tensor,
                  scale: Optional[str] = None) -> torch.Tensor:
    """``S·A·X`` on this rank's layout ``[X_u[u0:u1]; X_i]`` (see :class:`ShardedBipartite`)."""
    if X_local.shape[0] != sh.n_local + sh.n_items:
        raise ValueError(f"bipartite_hop: X has {X_local.shape[0]} rows, shard expects "
                         f"{sh.n_local} users + {sh.n_items} items")
    return _BipartiteHop.apply(X_local, sh, scale)


class _Epilogue(torch.autograd.Function):
    @staticmethod
    def forward(ctx, Z, epi: int, slope: float):
        Y = _epilogue_apply(Z.contiguous(), epi, slope)
        ctx.save_for_backward(Y)
        ctx.epi, ctx.slope = epi, slope
        return Y

    @staticmethod
    def backward(ctx, dY):
        (Y,) = ctx.saved_tensors
        return _epilogue_backward(Y, dY, ctx.epi, ctx.slope), None, None


def sharded_gcn_hop(sh: ShardedBipartite, X_local: torch.Tensor) -> torch.Tensor:
    """GCNLayer (``torch.sparse.mm(adj, embeds)``, HCCF.py:193-199) on user-row shards."""
    return bipartite_hop(sh, X_local)


def sharded_hgcn_conv(sh: ShardedBipartite, X_local: torch.Tensor, act: bool = True,
                      slope: float = 0.5) -> torch.Tensor:
    """HGCNConv (``leaky(A·(Aᵀ·X))``, HGNN_HD4.py:450-462) on user-row shards: the Aᵀ hop, then
    the A hop (for the symmetric norm_adj both are A; an edge-dropped A is not symmetric), the
    LeakyReLU after the second exchange (it is not linear)."""
    Z = bipartite_hop(sh, bipartite_hop(sh.transpose(), X_local))
    if not act:
        return Z
    return _Epilogue.apply(Z, nat.EPI_LEAKY_RELU, float(slope))


def sharded_mean_two_hop(sh: ShardedBipartite, X_local: torch.Tensor) -> torch.Tensor:
    """The ED-HNN scatter-mean pair over V/E = nonzero(ui_adj) (EquivSetConv2.py:88-93:
    Xe = mean of X over each hyperedge's vertices, then Xv = mean of Xe over each vertex's
    hyperedges) on user-row shards. ui_adj is symmetric, so both means are D^-1·A with the
    global degrees."""
    return bipartite_hop(sh, bipartite_hop(sh, X_local, "mean"), "mean")


class _ShardedDenseTwoHop(torch.autograd.Function):
    @staticmethod
    def forward(ctx, H, X, group):
        H = H.contiguous()
        X = X.contiguous()
        M = _tn(H, X)                      # this rank's Hᵀ·X [K, d]
        ordered_all_reduce(M, group=group)    # K·d·4 bytes: 8 KB at K = 32, d = 64
        ctx.save_for_backward(H, X, M)
        ctx.group = group
        return _nn(H, M)

    @staticmethod
    def backward(ctx, dY):
        H, X, M = ctx.saved_tensors
        dY = dY.contiguous()
        dM = _tn(H, dY)
        ordered_all_reduce(dM, group=ctx.group)
        dH = dX = None
        if ctx.needs_input_grad[1]:
            dX = _nn(H, dM)
        if ctx.needs_input_grad[0]:
            dH = _nt(dY, M)
            dH += _nt(X, dM)
        return dH, dX, None


def sharded_dense_two_hop(H_local: torch.Tensor, X_local: torch.Tensor,
                          group=None) -> torch.Tensor:
    """HGNNLayer's ``H·(Hᵀ·X)`` (HCCF.py:201-211) over user rows split across ranks: the [K, d]
    hyperedge messages Hᵀ·X are all-reduced (forward and backward), the rest is local."""
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        from .functional import dense_two_hop
        return dense_two_hop(H_local, X_local)
    return _ShardedDenseTwoHop.apply(H_local, X_local, group)


class _ShardedHCCFLayers(torch.autograd.Function):
    """HCCF's layer loop (model/graph/HCCF.py:173-191) on user-row shards as ONE op — the sharded
    counterpart of functional._HCCFLayers, on the local layout ``[h_u (local users); h_i (items,
    replicated)]``. Per layer k, forward:

    * hypergraph pair: ``M_u = Σ_ranks H_uᵀ·h_u`` (grouped split-K with the replicated
      ``M_i = H_iᵀ·h_i``, then an all-reduce of the [K, d] user part), ``Hh = [H_u·M_u; H_i·M_i]``;
    * GCN hop over the edge-dropped shard: the user rows ``B_g·h_i`` are complete locally, so
      their store writes ``gcn_k`` (act_out) and ``h_{k+1} = gcn_k + Hh`` (res1) as on one GPU;
      the item rows ``Σ_g C_g·h_u`` are written straight into ``gcn_k`` in chunks, each chunk
      all-reduced behind its kernel, and ``h_{k+1}`` of the items is one add after the exchange
      (fused into the store too on a single rank);
    * ``sum(hidden)`` is one slice-sum pass.

    Backward, layer k (item-row gradients are per-rank partials, as everywhere in this module):
    ``dM_u`` all-reduced, the grouped ``H·dM`` store, then the two transposed block hops whose
    stores add it and dE and write the next layer's ``dhgnn`` (sum_out); the item part of
    ``dgcn`` is all-reduced while the into-items hop ``B_gᵀ·dgcn_u`` runs. Exchanges per layer:
    forward [K, d] + [I, d], backward [K, d] + [I, d] — the same as the per-layer module graph,
    with none of its adds and accumulations."""

    @staticmethod
    def forward(ctx, shs, group, user_local, item, *Hs):
        from .functional import _gemm_rows, _gemm_tn_pair, _res_epilogue, _rows_desc
        L = len(shs)
        dev = user_local.device
        nl, I = user_local.shape[0], item.shape[0]
        N, d = nl + I, user_local.shape[1]
        K = Hs[0].shape[1]
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        f = dict(dtype=torch.float32, device=dev)
        hid = torch.empty((L + 1, N, d), **f)
        torch.cat([user_local, item], 0, out=hid[0])
        Hs = [H.contiguous() for H in Hs]
        gcn, hgnn, Ms = [], [], []
        for k in range(L):
            sh = shs[k]
            H_u, H_i = Hs[2 * k], Hs[2 * k + 1]
            h = hid[k]
            M_u, M_i = _gemm_tn_pair([(H_u, h[:nl]), (H_i, h[nl:])], dev)
            if world > 1:
                ordered_all_reduce(M_u, group=group)
            Hh = torch.empty((N, d), **f)
            _gemm_rows([_rows_desc(H_u, M_u, d, 1, K, d, Hh[:nl]),
                        _rows_desc(H_i, M_i, d, 1, K, d, Hh[nl:])], dev)
            G = torch.empty((N, d), **f)
            out = hid[k + 1]
            works: List = []
            if world > 1:
                for a, b in sh.bounds:  # item rows: partial sums, chunk by chunk into G
                    if b > a:
                        spmm_csr(sh.C.csr, h[:nl], val=sh.C.val, out=G[nl:], row_begin=a,
                                 row_end=b)
                    works.append(ordered_all_reduce(G[nl:][a:b], group=group, async_op=True))
            else:
                spmm_csr(sh.C.csr, h[:nl], val=sh.C.val,
                         ex=_res_epilogue(Hh[nl:], act_out=G[nl:]), out=out[nl:])
            spmm_csr(sh.B.csr, h[nl:], val=sh.B.val, ex=_res_epilogue(Hh[:nl], act_out=G[:nl]),
                     out=out[:nl])
            for w in works:
                w.wait()
            if world > 1:
                torch.add(G[nl:], Hh[nl:], out=out[nl:])
            gcn.append(G)
            hgnn.append(Hh)
            Ms += [M_u, M_i]
        E = torch.empty((N, d), **f)
        nat.check(nat.load().hgd_sum_slices(hid.data_ptr(), L + 1, N * d, N * d, E.data_ptr(),
                                            nat.stream_handle(dev)), "hgd_sum_slices")
        ctx.shs, ctx.group, ctx.world, ctx.nl, ctx.L, ctx.K = shs, group, world, nl, L, K
        ctx.save_for_backward(hid, *Hs, *Ms)
        ctx.set_materialize_grads(False)
        return (E, *gcn, *hgnn)

    @staticmethod
    def backward(ctx, dE, *grads):
        from .functional import _gemm_rows, _gemm_tn_pair, _res_epilogue, _rows_desc
        L, nl, K, world, group = ctx.L, ctx.nl, ctx.K, ctx.world, ctx.group
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
            sh = ctx.shs[k]
            H_u, H_i = Hs[2 * k], Hs[2 * k + 1]
            M_u, M_i = Ms[2 * k], Ms[2 * k + 1]
            h = hid[k]
            dG = dh if dgcn[k] is None else dh + dgcn[k]
            dG = dG.contiguous()
            dM_u, dM_i = _gemm_tn_pair([(H_u, dHh[:nl]), (H_i, dHh[nl:])], dev)
            if world > 1:  # M_u was all-reduced: its gradient is summed too
                ordered_all_reduce(dM_u, group=group)
            if ctx.needs_input_grad[4 + 2 * k] or ctx.needs_input_grad[5 + 2 * k]:
                dH_u, dH_i = torch.empty_like(H_u), torch.empty_like(H_i)
                _gemm_rows([_rows_desc(dHh[:nl], M_u, 1, d, d, K, dH_u),
                            _rows_desc(dHh[nl:], M_i, 1, d, d, K, dH_i)], dev)
                _gemm_rows([_rows_desc(h[:nl], dM_u, 1, d, d, K, dH_u, accumulate=True),
                            _rows_desc(h[nl:], dM_i, 1, d, d, K, dH_i, accumulate=True)], dev)
                dHs[2 * k], dHs[2 * k + 1] = dH_u, dH_i
            if k == 0 and not want_emb:
                break
            dh_new = torch.empty((N, d), **f)
            _gemm_rows([_rows_desc(H_u, dM_u, d, 1, K, d, dh_new[:nl]),
                        _rows_desc(H_i, dM_i, d, 1, K, d, dh_new[nl:])], dev)
            nxt = dhgnn[k - 1].contiguous() if k > 0 and dhgnn[k - 1] is not None else None
            dHh_new = torch.empty((N, d), **f) if nxt is not None else None

            def ex(r0, r1):
                return _res_epilogue(None if dE is None else dE[r0:r1], res2=dh_new[r0:r1],
                                     sum_res=None if nxt is None else nxt[r0:r1],
                                     sum_out=None if dHh_new is None else dHh_new[r0:r1])

            dZi, work = dG[nl:], None
            if world > 1:  # the items' gradient summed while the into-items hop runs
                dZi = dZi.clone()
                work = ordered_all_reduce(dZi, group=group, async_op=True)
            spmm_csr(sh.B.csc, dG[:nl], val=sh.B.val_t, ex=ex(nl, N), out=dh_new[nl:])
            if work is not None:
                work.wait()
            spmm_csr(sh.C.csc, dZi, val=sh.C.val_t, ex=ex(0, nl), out=dh_new[:nl])
            dh = dh_new
            dHh = dHh_new if nxt is not None else dh_new
        d_u = dh[:nl] if ctx.needs_input_grad[2] else None
        d_i = dh[nl:] if ctx.needs_input_grad[3] else None
        return (None, None, d_u, d_i, *dHs)


def sharded_hccf_layers(shs, user_local: torch.Tensor, item: torch.Tensor, hypers_u, hypers_i,
                        group=None):
    """HCCF's propagation (HCCF.py:173-191) over per-layer edge-dropped shards ``shs``
    (:class:`ShardedBipartite`) and per-layer dropped hypergraphs (user rows local, item rows
    replicated): ``(sum(hidden), gcn_hidden, hgnn_hidden)`` on the local layout
    (:class:`_ShardedHCCFLayers`)."""
    L = len(shs)
    for sh in shs:
        if sh.n_local != user_local.shape[0] or sh.n_items != item.shape[0]:
            raise ValueError("sharded_hccf_layers: shard shape does not match the tables")
    Hs = []
    for Hu, Hi in zip(hypers_u, hypers_i):
        Hs += [Hu, Hi]
    out = _ShardedHCCFLayers.apply(list(shs), group, user_local, item, *Hs)
    return out[0], list(out[1:1 + L]), list(out[1 + L:])
