"""The reference's optimizer, capturable: ``torch.optim.Adam(params, lr=…)`` (model/graph/HCCF.py:33)
with its step as ONE libhgd kernel (``hgd_adam_step``) that a HIP graph can hold.

torch's device Adam (the multi-tensor, non-capturable form) rounds its per-step bias corrections
on the host in double and hands them to six foreach kernels as float scalars; a capturable Adam
rounds them on the device instead, so its steps differ from the reference's from the first one
(``scripts/diag/diag_adam_bitwise.py``). Here the host computes the same doubles exactly as torch
does (:meth:`ReferenceAdam.prepare`, once per step, before the launch or the graph replay) and
writes their floats into a small device buffer the kernel reads; the kernel repeats torch's op
order and rounding per element. Which multiply-adds torch's build fused and which square root /
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


class ReferenceAdam(torch.optim.Adam):
    """torch.optim.Adam (same param groups, state and state_dict; lr, betas and eps as given, no
    weight decay / amsgrad / maximize) whose :meth:`step` is :meth:`prepare` (host: the step
    counts and the per-step scalars, copied to the device) then :meth:`launch` (the one kernel).
    In a captured training step the graph holds :meth:`launch`; :meth:`prepare` runs before each
    replay. Bitwise torch's Adam with the calibrated ``variant``."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, variant: int = None):
        super().__init__(params, lr=lr, betas=betas, eps=eps, foreach=True)
        for group in self.param_groups:
            if group["weight_decay"] or group["amsgrad"] or group["maximize"]:
                raise ValueError("ReferenceAdam: weight decay, amsgrad and maximize are not "
                                 "implemented")
        self.variant = variant
        self._dev = None          # device [count, 6] scalars (the kernel's; fixed address)
        self._ring = []           # pinned host copies [(buffer, event of its last copy)]
        self._ring_i = 0

    def _params(self):
        return [p for group in self.param_groups for p in group["params"] if p.grad is not None]

    def _init_state(self, params):
        for p in params:
            st = self.state[p]
            if len(st) == 0:  # torch's _init_group: a CPU float32 step counter, zero moments
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)

    @torch.no_grad()
    def prepare(self) -> None:
        """One step's host half: every step counter + 1 and the six floats per tensor torch's
        foreach kernels would receive, written to the device buffer the kernel reads (ordered
        on the current stream before the launch / replay)."""
        params = self._params()
        if not params:
            return
        self._init_state(params)
        rows = []
        for group in self.param_groups:
            lr = float(group["lr"])
            beta1, beta2 = group["betas"]
            for p in group["params"]:
                if p.grad is None:
                    continue
                st = self.state[p]
                st["step"] += 1  # float32 on the CPU, as torch._foreach_add_(steps, 1)
                t = st["step"].item()
                bc1 = 1 - beta1 ** t
                bc2 = 1 - beta2 ** t
                rows.append((1 - beta1, beta2, 1 - beta2, bc2 ** 0.5, group["eps"],
                             (lr / bc1) * -1))
        dev = params[0].device
        if self._dev is None or self._dev.shape[0] != len(rows):
            self._dev = torch.empty((len(rows), 6), dtype=torch.float32, device=dev)
            self._ring = [(torch.empty((len(rows), 6), dtype=torch.float32, pin_memory=True),
                           None) for _ in range(4)]
        # a ring of pinned sources: the host may run steps ahead of the device, so a source is
        # rewritten only once the copy that last read it has run
        host, ev = self._ring[self._ring_i]
        if ev is not None:
            ev.synchronize()
        host.copy_(torch.tensor(rows, dtype=torch.float64))  # each double → its float
        self._dev.copy_(host, non_blocking=True)
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream(dev))
        self._ring[self._ring_i] = (host, ev)
        self._ring_i = (self._ring_i + 1) % len(self._ring)

    @torch.no_grad()
    def launch(self) -> None:
        """One step's device half: hgd_adam_step over every parameter with a gradient (the
        pointers of the parameters' current .grad, moments and scalars buffer)."""
        params = self._params()
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
                                           self._dev.data_ptr(), int(variant),
                                           nat.stream_handle(params[0].device)),
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
