"""hgd_unique_* / functional.unique_long: torch.unique(x.long()) as HCCF's loss calls it every
step (model/graph/HCCF.py:65-66) — bit-exact (sorted int64 keys) against torch.unique on the
same tensor, over the range-bitmap path (LDS-private and global bitmaps) and the radix-sort path
taken beyond a 2^24 key range."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _ref(x):
    return torch.unique(x.cpu().long())


@pytest.mark.parametrize("shape,scale", [((4096, 64), 1.0), ((4096, 64), 3.0), ((1, 1), 1.0),
                                         ((513, 7), 40.0), ((2048, 32), 5000.0)])
def test_unique_of_truncated_embeddings(dev, shape, scale):
    from hypergraph_diffusion_for_recommendation_amd import unique_long
    g = torch.Generator(device=dev).manual_seed(int(scale * 10) + shape[0])
    x = torch.randn(shape, device=dev, generator=g) * scale
    got = unique_long(x)
    assert got.dtype == torch.int64
    assert torch.equal(got.cpu(), _ref(x))


def test_unique_int64_paths(dev):
    from hypergraph_diffusion_for_recommendation_amd import unique_long
    rng = np.random.default_rng(0)
    cases = {
        "small_range": rng.integers(-5, 6, size=100_000),
        "lds_boundary": rng.integers(0, 1024 * 32, size=50_000),       # exactly 1024 words
        "global_bitmap": rng.integers(-10**6, 10**6, size=300_000),    # > 1024 words
        "cap_minus_one": np.array([7, 7 + (1 << 24) - 1, 100, 7]),     # widest bitmap range
        "cap": np.array([7, 7 + (1 << 24), 100]),                      # one past: sort path
        "wide": rng.integers(-2**62, 2**62, size=200_000),             # sort path
        "extremes": np.array([-2**63, 2**63 - 1, 0, -2**63, 5]),       # span overflows int64
        "single": np.array([42]),
        "dups": np.full(1000, -3),
    }
    for name, a in cases.items():
        t = torch.from_numpy(a.astype(np.int64)).to(dev)
        got = unique_long(t)
        assert torch.equal(got.cpu(), torch.unique(t.cpu())), name


def test_unique_empty_and_special_floats(dev):
    from hypergraph_diffusion_for_recommendation_amd import unique_long
    assert unique_long(torch.empty(0, device=dev)).numel() == 0
    assert unique_long(torch.empty(0, dtype=torch.int64, device=dev)).numel() == 0
    x = torch.tensor([1.9, -1.9, -0.5, 0.5, 2.0, -2.0, 3e9, -3e9], device=dev)
    assert unique_long(x).cpu().tolist() == sorted({1, -1, 0, 2, -2, 3000000000, -3000000000})
    # NaN / inf / out of int64 range → INT64_MIN (documented; C++ leaves the cast undefined)
    y = torch.tensor([float("nan"), float("inf"), -float("inf"), 1e30, 4.0], device=dev)
    assert unique_long(y).cpu().tolist() == [-2**63, 4]


def test_unique_rejects_other_dtypes(dev):
    from hypergraph_diffusion_for_recommendation_amd import unique_long
    with pytest.raises(ValueError):
        unique_long(torch.zeros(4, dtype=torch.int32, device=dev))
    with pytest.raises(ValueError):
        unique_long(torch.zeros(4))


def test_unique_range_feeds_contrast_loss_bounds(dev):
    """unique_long attaches the key range; contrast_loss uses it for its IndexError check (and
    falls back to reading the nodes when they were modified in place)."""
    from hypergraph_diffusion_for_recommendation_amd import contrast_loss, unique_long
    E = torch.randn(10, 16, device=dev)
    nodes = unique_long(torch.tensor([-3.5, 2.2, 9.9, 0.1], device=dev))
    assert nodes._hgd_range[:2] == (-3, 9)
    loss = contrast_loss(E, E.clone(), nodes, 0.2)
    assert torch.isfinite(loss)
    bad = unique_long(torch.tensor([1.0, 10.0], device=dev))
    with pytest.raises(IndexError):
        contrast_loss(E, E.clone(), bad, 0.2)
    ok = unique_long(torch.tensor([1.0, 2.0], device=dev))
    ok[1] = 12  # in-place change: the cached range is ignored, the check reads the values
    with pytest.raises(IndexError):
        contrast_loss(E, E.clone(), ok, 0.2)


def _dev_unique(t):
    from hypergraph_diffusion_for_recommendation_amd.functional import unique_long_n
    vals, count = unique_long_n(t)
    k = int(count.item())
    assert vals.numel() == t.numel() and not vals[k:].any()
    return vals[:k]


def test_device_complete_unique_paths(dev):
    """hgd_unique_dev_* (functional.unique_long_n, the captured step's unique): the bitmap window
    [min, min + 2^24) plus the far keys merged on the device — the LDS sort of up to 4,096 far
    keys and the in-workspace bitonic network beyond — against torch.unique, bit-exact."""
    rng = np.random.default_rng(1)
    cases = {
        "small_range": rng.integers(-5, 6, size=100_000),
        "global_bitmap": rng.integers(-10**6, 10**6, size=300_000),
        "cap_minus_one": np.array([7, 7 + (1 << 24) - 1, 100, 7]),
        "one_far_key": np.array([7, 7 + (1 << 24), 100, 7 + (1 << 24)]),
        "far_lds": np.concatenate([rng.integers(0, 50, 10_000),
                                   rng.integers(1 << 40, (1 << 40) + 3000, 3000)]),
        "far_global": rng.integers(-2**62, 2**62, size=200_000),   # ~all keys far: bitonic path
        "extremes": np.array([-2**63, 2**63 - 1, 0, -2**63, 5]),
        "single": np.array([42]),
        "dups": np.full(1000, -3),
    }
    for name, a in cases.items():
        print("device-complete unique case:", name, flush=True)
        t = torch.from_numpy(a.astype(np.int64)).to(dev)
        assert torch.equal(_dev_unique(t).cpu(), torch.unique(t.cpu())), name


def test_device_complete_unique_of_floats(dev):
    """Truncated embeddings (HCCF.py:65-66), including a NaN that drags the window to INT64_MIN
    (every other key becomes a far key)."""
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(4096, 64, device=dev, generator=g) * 3.0
    assert torch.equal(_dev_unique(x).cpu(), _ref(x))
    y = x.clone()
    y[5, 7] = float("nan")
    want = _ref(y)  # the host cast maps NaN to INT64_MIN too
    assert want[0] == -2**63
    assert torch.equal(_dev_unique(y).cpu(), want)


def test_device_unique_group_equals_single_lists(dev):
    """hgd_unique_dev_group (functional.unique_long_n_group: several lists per launch, HCCF's
    anchor and positive lists): each list's nodes and count bitwise as unique_long_n gives them
    one at a time — float and int64 lists mixed, different sizes, a far-key list, a NaN list,
    a capacity cut by n_rows (count clamped, tail zero) and more lists than one group holds."""
    from hypergraph_diffusion_for_recommendation_amd.functional import (unique_long_n,
                                                                         unique_long_n_group)
    g = torch.Generator(device=dev).manual_seed(5)
    emb = torch.randn(4096, 64, device=dev, generator=g) * 3.0
    nan = emb.clone()
    nan[1, 2] = float("nan")
    ids = torch.randint(-50, 900, (5000,), device=dev, generator=g)
    far = torch.tensor([3, 3 + (1 << 30), 9, -(1 << 40)], device=dev)
    xs = [emb, ids, nan, far, emb[:100], ids[:7]]
    rows = [None, 900, None, None, 4, None]   # emb[:100] has ~13 distinct ids > 2·4: cut to 8
    got = unique_long_n_group(xs, rows)
    for k, (x, r) in enumerate(zip(xs, rows)):
        want_n, want_c = _single(x, r)
        assert torch.equal(unique_long_n(x, r)[0], want_n), k
        n, c = got[k]
        assert torch.equal(n, want_n) and torch.equal(c, want_c), k
        live = int(c)
        assert not n[live:].any(), k


def _single(x, n_rows):
    """The round-3 unique_long_n: the single-list C entry point, the clamp and the zeroed tail
    done by torch ops — the reference the grouped path must reproduce."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    x = x.detach().contiguous().view(-1)
    n = x.numel()
    out = torch.empty(n, dtype=torch.int64, device=x.device)
    wsb = lib.hgd_unique_workspace_size(n)
    buf = torch.empty(256 + wsb, dtype=torch.uint8, device=x.device)
    fn = lib.hgd_unique_dev_trunc_f32 if x.dtype == torch.float32 else lib.hgd_unique_dev_i64
    nat.check(fn(x.data_ptr(), n, out.data_ptr(), buf.data_ptr(), buf.data_ptr() + 256, wsb,
                 nat.stream_handle(x.device)), "hgd_unique_dev")
    count = buf[:8].view(torch.int64).clone()
    cap = n if n_rows is None else max(1, min(n, 2 * int(n_rows)))
    out = out[:cap]
    count = torch.clamp_max(count, cap)
    live = torch.arange(cap, device=x.device) < count
    return torch.where(live, out, torch.zeros((), dtype=torch.int64, device=x.device)), count
