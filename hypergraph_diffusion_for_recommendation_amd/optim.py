"""The reference's optimizer, capturable: ``torch.optim.Adam(params, lr=…)`` (model/graph/HCCF.py:33)
with its step as ONE libhgd kernel (``hgd_adam_step``) that a HIP graph can hold.

torch's device Adam (the multi-tensor, non-capturable form) rounds its per-step bias corrections
on the host in double and hands them to six foreach kernels as float scalars; a capturable Adam
rounds them on the device instead, so its steps differ from the reference's from the first one
(``scripts/diag/diag_adam_bitwise.py``). Here the host computes the same doubles exactly as torch
does — for 512 steps at a time, into a device table whose row the kernel reads and advances
itself, so a replayed graph needs only the host's step counting (:meth:`ReferenceAdam.prepare`)
— and the kernel repeats torch's op order and rounding per element. Which multiply-adds torch's build fused and which square root /
division it emitted is measured, not assumed: :func:`calibrated_variant` runs torch's own Adam
and every kernel variant over a few steps of random data on the device and keeps the one that is
bit for bit torch's (``None`` if none is — the callers then keep torch's optimizer).
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Optional

import torch

from . import _native as nat

_VARIANTS: Dict[str, Optional[int]] = {}


def calibrated_variant(device, steps: int = 4, n: int = 1 << 16) -> Optional[int]:
    """The hgd_adam_step variant that reproduces torch.optim.Adam(lr=…) bit for bit on this
    device (checked over ``steps`` steps of random data with lr, betas and eps that exercise every
    op), or None. Cached per device; ``HGD_ADAM_VARIANT`` in the environment forces one."""
    device = torch.device(device)
    key = str(device)
    if key in _VARIANTS:
        return _VARIANTS[key]
    env = os.environ.get("HGD_ADAM_VARIANT")
    if env is not None:
        _VARIANTS[key] = int(env) if int(env) >= 0 else None
        return _VARIANTS[key]
    g = torch.Generator(device=device).manual_seed(1234)
    p0 = [torch.randn(n, device=device, generator=g), torch.randn(n // 2 + 3, device=device,
                                                                  generator=g) * 1e-3]
    grads = [[torch.randn_like(p) * (10.0 ** (k % 3 - 2)) for p in p0] for k in range(steps)]
    ref = [p.clone().requires_grad_(True) for p in p0]
    opt = torch.optim.Adam(ref, lr=3e-3, betas=(0.9, 0.999), eps=1e-8)
    for k in range(steps):
        for p, gr in zip(ref, grads[k]):
            p.grad = gr.clone()
        opt.step()
    found = None
    for variant in range(32):
        mine = [p.clone().requires_grad_(True) for p in p0]
        ropt = ReferenceAdam(mine, lr=3e-3, betas=(0.9, 0.999), eps=1e-8, variant=variant)
        for k in range(steps):
            for p, gr in zip(mine, grads[k]):
                p.grad = gr.clone()
            ropt.step()
        if all(torch.equal(a, b) for a, b in zip(mine, ref)) and all(
                torch.equal(ropt.state[a]["exp_avg"], opt.state[b]["exp_avg"]) and
                torch.equal(ropt.state[a]["exp_avg_sq"], opt.state[b]["exp_avg_sq"])
                for a, b in zip(mine, ref)):
            found = variant
            break
    _VARIANTS[key] = found
    return found


_TABLE_ROWS = 512  # steps of scalars computed ahead (rebuilt when used up or lr changes)


class ReferenceAdam(torch.optim.Adam):
    """torch.optim.Adam (same param groups, state and state_dict; lr, betas and eps as given, no
    weight decay / amsgrad / maximize) whose :meth:`step` is :meth:`prepare` (host: the step
    counters) then :meth:`launch` (the kernel). The per-step scalars are computed on the host
    exactly as torch computes them, for the next 512 steps at a time, into a device table; the
    launch reads the row of its step and advances a device row index, so a HIP graph holding
    :meth:`launch` steps through the table by itself and :meth:`prepare` before a replay only
    counts (and rebuilds the table when it is used up or a learning rate changed). Bitwise
    torch's Adam with the calibrated ``variant``."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, variant: int = None):
        super().__init__(params, lr=lr, betas=betas, eps=eps, foreach=True)
        for group in self.param_groups:
            if group["weight_decay"] or group["amsgrad"] or group["maximize"]:
                raise ValueError("ReferenceAdam: weight decay, amsgrad and maximize are not "
                                 "implemented")
        self.variant = variant
        self._table = None     # device [_TABLE_ROWS, count, 6] scalars
        self._row_dev = None   # device int32: the row the next launch reads
        self._row = 0          # the same, as the host counts it
        self._key = None       # (params, hyper-parameters, first step) the table was built for
        self._stage = None     # (pinned source of the last table copy, its event)
        self._captured = False  # a HIP graph holds a launch(): the table must not move

    def _params(self):
        return [p for group in self.param_groups for p in group["params"] if p.grad is not None]

    def _init_state(self, params):
        for p in params:
            st = self.state[p]
            if len(st) == 0:  # torch's _init_group: a CPU float32 step counter, zero moments
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)

    def _hyper(self, p):
        for group in self.param_groups:
            if any(q is p for q in group["params"]):
                return float(group["lr"]), group["betas"], group["eps"]
        raise KeyError("ReferenceAdam: parameter not in any group")

    def _build_table(self, params, dev):
        """Rows k = 0 .. _TABLE_ROWS-1: the floats torch's foreach kernels receive at each
        parameter's step count + k (1 − β1, β2, 1 − β2, sqrt(1 − β2^t), eps, −lr/(1 − β1^t))."""
        base = [self.state[p]["step"].item() for p in params]
        hyper = [self._hyper(p) for p in params]
        rows = []
        for k in range(_TABLE_ROWS):
            for t0, (lr, (beta1, beta2), eps) in zip(base, hyper):
                t = t0 + k
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                rows.append((1 - beta1, beta2, 1 - beta2, bc2 ** 0.5, eps, (lr / bc1) * -1))
        if self._stage is not None:
            self._stage[1].synchronize()  # the previous table copy has run
        src = torch.tensor(rows, dtype=torch.float64).to(torch.float32).reshape(
            _TABLE_ROWS, len(params), 6).pin_memory()
        if self._table is None or self._table.shape[1] != len(params):
            if self._captured:
                raise RuntimeError("ReferenceAdam: the set of parameters with a gradient changed "
                                   "after a HIP graph captured launch(); the graph would read a "
                                   "freed scalar table")
            self._table = torch.empty((_TABLE_ROWS, len(params), 6), dtype=torch.float32,
                                      device=dev)
            self._row_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self._table.copy_(src, non_blocking=True)  # ordered after every launch already queued
        self._row_dev.zero_()
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._stage = (src, ev)
        self._row = 0
        return tuple(base), tuple(hyper)

    @torch.no_grad()
    def prepare(self) -> None:
        """One step's host half: every step counter + 1 (float32 on the CPU, as torch's
        _foreach_add_), and the scalar table rebuilt if it is used up, a learning rate changed or
        the counters moved otherwise (a loaded state)."""
        params = self._params()
        if not params:
            return
        self._init_state(params)
        steps = [self.state[p]["step"] for p in params]
        torch._foreach_add_(steps, 1.0)
        hyper = tuple(self._hyper(p) for p in params)
        key = self._key
        expect_first = None if key is None else key[2][0] + self._row
        if (key is None or self._row >= _TABLE_ROWS or key[0] != tuple(id(p) for p in params)
                or key[1] != hyper or steps[0].item() != expect_first):
            base, hyper = self._build_table(params, params[0].device)
            self._key = (tuple(id(p) for p in params), hyper, base)
        self._row += 1

    @torch.no_grad()
    def launch(self) -> None:
        """One step's device half: hgd_adam_step over every parameter with a gradient (the
        pointers of the parameters' current .grad and moments), reading and advancing the device
        row of the scalar table."""
        params = self._params()
        if self._key is None or self._key[0] != tuple(id(p) for p in params):
            raise RuntimeError("ReferenceAdam.launch: the parameters with a gradient are not the "
                               "ones prepare() built the scalar table for")
        if torch.cuda.is_current_stream_capturing():
            self._captured = True
        arr = (nat.AdamTensor * len(params))()
        for k, p in enumerate(params):
            st = self.state[p]
            arr[k].param, arr[k].grad = p.data_ptr(), p.grad.data_ptr()
            arr[k].exp_avg, arr[k].exp_avg_sq = st["exp_avg"].data_ptr(), st["exp_avg_sq"].data_ptr()
            arr[k].n = p.numel()
        variant = self.variant if self.variant is not None else calibrated_variant(params[0].device)
        if variant is None:
            raise nat.HGDNativeError("ReferenceAdam: no hgd_adam_step variant reproduces this "
                                     "torch build's Adam; use torch.optim.Adam")
        nat.check(nat.load().hgd_adam_step(ctypes.cast(arr, ctypes.c_void_p), len(params),
                                           self._table.data_ptr(), self._row_dev.data_ptr(),
                                           int(variant), nat.stream_handle(params[0].device)),
                  "hgd_adam_step")

    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        if not self._params():
            return loss
        self.prepare()
        self.launch()
        return loss
