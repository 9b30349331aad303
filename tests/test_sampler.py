"""CPU: the native pairwise sampler (hgd_py_shuffle / hgd_sample_pairwise behind
sampler.next_batch_pairwise) against the restated reference sampler (util/sampler.py:237-264):
identical batches, identical in-place shuffle of training_data, identical Python random state
afterwards — bit for bit, over several epochs and an early stop."""
import random
from collections import defaultdict
from types import SimpleNamespace

import numpy as np
import pytest

from oracle import hgd_oracle as O


def _data(n_records, n_users, n_items, seed, item_skew=False):
    """An Interaction-like object (data/ui_graph.py:43-64): raw ids, first-appearance maps,
    training_set_u, duplicates allowed in training_data."""
    rng = np.random.default_rng(seed)
    users = rng.integers(0, n_users, n_records) * 7 + 3
    items = (rng.zipf(1.3, n_records) % n_items if item_skew
             else rng.integers(0, n_items, n_records)) * 5 + 11
    td = [[int(u), int(i), 1.0] for u, i in zip(users, items)]
    user, item = {}, {}
    tsu = defaultdict(dict)
    for u, i, r in td:
        user.setdefault(u, len(user))
        item.setdefault(i, len(item))
        tsu[u][i] = r
    return SimpleNamespace(training_data=td, user=user, item=item, training_set_u=tsu)


def _lib_or_skip():
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    try:
        nat.load()
    except nat.HGDNativeError as e:  # pragma: no cover - the build runs before the suite
        pytest.skip(str(e))


@pytest.mark.parametrize("n_records,n_users,n_items,batch,n_negs,skew",
                         [(3, 2, 40, 4, 1, False), (1000, 50, 64, 128, 1, False),
                          (5000, 300, 257, 2048, 2, True), (3000, 40, 1000, 4096, 1, False),
                          (777, 30, 33, 100, 3, True)])
def test_native_sampler_bit_exact(n_records, n_users, n_items, batch, n_negs, skew):
    _lib_or_skip()
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    d_ref = _data(n_records, n_users, n_items, 5, skew)
    d_nat = _data(n_records, n_users, n_items, 5, skew)
    random.seed(20)
    ref = [list(O.next_batch_pairwise(d_ref, batch, n_negs)) for _ in range(3)]
    ref_state = random.getstate()
    random.seed(20)
    got = [[tuple(t.tolist() for t in b) for b in next_batch_pairwise(d_nat, batch, n_negs)]
           for _ in range(3)]
    assert random.getstate() == ref_state
    assert d_nat.training_data == d_ref.training_data
    for e in range(3):
        assert len(got[e]) == len(ref[e])
        for (gu, gi, gj), (ru, ri, rj) in zip(got[e], ref[e]):
            assert gu == ru and gi == ri and gj == rj
    # the Python stream continues identically
    assert random.random() == (random.setstate(ref_state) or random.random())


def test_native_sampler_early_stop_and_external_reshuffle():
    """Batches are drawn lazily (the random stream after an early break matches the reference);
    an externally reordered training_data list is picked up."""
    _lib_or_skip()
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    d_ref = _data(4000, 100, 300, 9)
    d_nat = _data(4000, 100, 300, 9)
    random.seed(1)
    it = O.next_batch_pairwise(d_ref, 512)
    ref_first = [next(it) for _ in range(2)]
    ref_state = random.getstate()
    random.seed(1)
    it = next_batch_pairwise(d_nat, 512)
    got_first = [tuple(t.tolist() for t in next(it)) for _ in range(2)]
    assert random.getstate() == ref_state
    assert [tuple(b) for b in ref_first] == got_first
    # someone else reorders the list between epochs: the sampler follows the list
    d_ref.training_data.reverse()
    d_nat.training_data.reverse()
    random.seed(2)
    ref = list(O.next_batch_pairwise(d_ref, 1000))
    random.seed(2)
    got = [tuple(t.tolist() for t in b) for b in next_batch_pairwise(d_nat, 1000)]
    assert [tuple(b) for b in ref] == got


def test_native_sampler_rejects_saturated_user():
    _lib_or_skip()
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    from hypergraph_diffusion_for_recommendation_amd.sampler import next_batch_pairwise
    d = SimpleNamespace(training_data=[[1, 5, 1.0], [1, 6, 1.0]], user={1: 0},
                        item={5: 0, 6: 1}, training_set_u={1: {5: 1.0, 6: 1.0}})
    with pytest.raises(nat.HGDNativeError):
        list(next_batch_pairwise(d, 2))   # the reference would loop forever


@pytest.mark.parametrize("n,keep,skip", [(0, 0.7, 0), (1, 0.7, 0), (624, 0.5, 3),
                                         (625, 0.3, 623), (2_340_001, 0.7, 17), (5000, 0.999, 1)])
def test_torch_cpu_keep_mask_matches_torch_rand(n, keep, skip):
    """SpAdjDropEdge's CPU mask (HCCF.py:223) drawn natively: the same mask and the same
    generator position as torch.rand on the default CPU generator."""
    _lib_or_skip()
    import torch
    from hypergraph_diffusion_for_recommendation_amd.layers import (_native_cpu_mask_ok,
                                                                    torch_cpu_keep_mask)
    assert _native_cpu_mask_ok()
    torch.manual_seed(n + skip)
    torch.rand(skip)
    st = torch.get_rng_state()
    ref = ((torch.rand(n) + keep).floor()).type(torch.bool)
    ref_next = torch.rand(16)
    torch.set_rng_state(st)
    got, kept = torch_cpu_keep_mask(n, keep)
    assert got.dtype == torch.uint8 and torch.equal(got.bool(), ref)
    assert kept == int(ref.sum())
    assert torch.equal(torch.rand(16), ref_next)


def test_torch_cpu_keep_mask_prefetch_keeps_the_stream():
    """The prefetched draw is used only when nothing else drew from the generator in between:
    interleaved torch.rand calls, changed sizes / rates and reseeds all give torch's own masks."""
    _lib_or_skip()
    import torch
    from hypergraph_diffusion_for_recommendation_amd.layers import torch_cpu_keep_mask

    def ref_mask(n, keep):
        return ((torch.rand(n) + keep).floor()).type(torch.bool)

    plan = [(3000, 0.7, None), (3000, 0.7, None), (3000, 0.7, "rand"), (3000, 0.5, None),
            (1000, 0.5, None), (1000, 0.5, "seed"), (1000, 0.5, None), (3000, 0.7, None)]
    torch.manual_seed(123)
    want = []
    for n, keep, between in plan:
        want.append(ref_mask(n, keep))
        if between == "rand":
            torch.rand(5)
        elif between == "seed":
            torch.manual_seed(7)
    want_next = torch.rand(8)
    torch.manual_seed(123)
    for (n, keep, between), w in zip(plan, want):
        got, kept = torch_cpu_keep_mask(n, keep)
        assert torch.equal(got.bool(), w) and kept == int(w.sum())
        if between == "rand":
            torch.rand(5)
        elif between == "seed":
            torch.manual_seed(7)
    assert torch.equal(torch.rand(8), want_next)


@pytest.mark.parametrize("spec", [[(2_470_000, 0.5)] * 3, [(1000, 0.7), (5, 0.7), (70_000, 0.7)],
                                  [(3000, 0.5), (3000, 0.9)]])
def test_step_masks_one_draw_equals_per_call_draws(spec):
    """SpAdjDropEdge.refill's step draw: calls at one rate come from ONE split draw of Σn words,
    bit-identical to the per-call draws (torch.rand(n) and the native draw take one generator
    word per element) and leaving the generator in the same state."""
    import torch

    from hypergraph_diffusion_for_recommendation_amd.layers import (_draw_keep_mask,
                                                                    _draw_step_masks,
                                                                    _native_cpu_mask_ok)
    if not _native_cpu_mask_ok():
        pytest.skip("native torch CPU generator layout not recognised")
    torch.manual_seed(123)
    torch.rand(17)  # start mid-block
    st = torch.get_rng_state()
    got, end = _draw_step_masks(st.clone(), spec)
    state = st.clone()
    for (n, keep), g in zip(spec, got):
        ref, _, state = _draw_keep_mask(state, n, keep)
        assert torch.equal(g, ref), (n, keep)
    assert torch.equal(end, state)
    torch.set_rng_state(st)
    for (n, keep), g in zip(spec, got):  # and the reference's own calls
        assert torch.equal(g.bool(), ((torch.rand(n) + keep).floor()).type(torch.bool))
    assert torch.equal(torch.get_rng_state(), end)
