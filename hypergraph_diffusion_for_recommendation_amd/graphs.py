"""A whole training step replayed from one HIP graph (hipGraph via torch.cuda.CUDAGraph).

The carriers' steps at dataset scale are launch-bound: HCCF's Yelp-shaped step (HCCF.py:79-97)
is ~340 kernels whose device time (≈2.3 ms) is below what the host needs to issue them through
Python and autograd, plus the host reads that size the next op (the drop-edge kept counts, the
InfoNCE node counts). With ``SpAdjDropEdge(capture_safe=True)`` (device mask from a device seed
counter, capacity-sized structures), :func:`~.functional.unique_long_n` and
``contrast_loss(..., count=...)`` (batch counts read by the kernels) and a capturable optimizer
(``torch.optim.Adam(capturable=True)``) nothing in the step reads the device from the host, so
the step is captured once and replayed: one launch per step, fresh drop-edge masks per replay
(the seed counter advances on the device).

Use: run the first steps eagerly (they are real training steps, and they allocate the optimizer
state and the library handles), then :class:`CapturedStep` records the step once (recording
executes nothing) and every later batch is copied into its static inputs and replayed.
"""
from __future__ import annotations

import gc
from typing import Callable, Sequence

import torch


class CapturedStep:
    """``step(*inputs)`` recorded into one graph over static copies of ``inputs``; calling the
    object copies new inputs in place and replays. ``step`` must be capture-safe (no host reads
    of device data, static shapes) and have run eagerly at least once before — and nothing may
    still hold an output of those eager runs that carries their autograd graph (a loss kept for
    logging keeps the parameters' AccumulateGrad nodes, bound to the eager stream, alive into
    the capture, where they break it: keep ``loss.detach()``)."""

    def __init__(self, step: Callable, example_inputs: Sequence[torch.Tensor],
                 before_replay: Callable = None):
        # before_replay: host work each replay needs first, e.g. SpAdjDropEdge.refill (the
        # reference's CPU keep-masks of the step, drawn into the buffers the graph reads)
        self.before_replay = before_replay
        self.static = [t.detach().clone() for t in example_inputs]
        # free eager autograd graphs still held by reference cycles: their AccumulateGrad nodes
        # would otherwise carry the eager stream into the capture
        gc.collect()
        torch.cuda.synchronize(self.static[0].device)
        self.graph = torch.cuda.CUDAGraph()
        # thread-local capture: a host thread of the harness (e.g. a keep-mask prefetch worker
        # allocating pinned memory) must not invalidate the capture
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            out = step(*self.static)
        # keep the outputs' storage, not their autograd graph: a captured loss would hold the
        # parameters' AccumulateGrad nodes (bound to the capture stream) alive, and a later eager
        # step (a short last batch) would accumulate through them from another stream — torch's
        # "AccumulateGrad node's stream does not match" warning and an extra sync
        self.out = _detached(out)

    def __call__(self, *inputs: torch.Tensor):
        for dst, src in zip(self.static, inputs):
            dst.copy_(src)
        if self.before_replay is not None:
            self.before_replay()
        self.graph.replay()
        return self.out


def _detached(x):
    if isinstance(x, torch.Tensor):
        return x.detach()
    if isinstance(x, (tuple, list)):
        return type(x)(_detached(v) for v in x)
    return x
