"""CPU: the user-row partition of the sharded path (contiguous, degree-balanced
user ranges). Host logic only; no device calls."""
import numpy as np
import pytest

from hypergraph_diffusion_for_recommendation_amd.sharded_encoders import shard_bounds


def _ranges(n, world, deg=None):
    return [shard_bounds(n, world, r, deg) for r in range(world)]


@pytest.mark.parametrize("n,world", [(10, 3), (7, 8), (1000, 8), (0, 2)])
def test_equal_count_split(n, world):
    rs = _ranges(n, world)
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    sizes = [b - a for a, b in rs]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("seed,world", [(0, 2), (1, 3), (2, 8)])
def test_degree_balanced_split(seed, world):
    rng = np.random.default_rng(seed)
    n = 5000
    deg = rng.zipf(1.6, size=n).clip(max=2000)  # heavy-tailed interaction counts
    rs = _ranges(n, world, deg)
    assert rs[0][0] == 0 and rs[-1][1] == n
    assert all(a[1] == b[0] and a[0] <= a[1] for a, b in zip(rs, rs[1:]))
    w = deg + 1
    share = [int(w[a:b].sum()) for a, b in rs]
    target = w.sum() / world
    # every rank within one user's weight of its share
    assert max(abs(s - target) for s in share) <= w.max() + 1
    # and better balanced than the equal-count split on this skew
    eq = [int(w[a:b].sum()) for a, b in _ranges(n, world)]
    assert max(share) <= max(eq)


def test_one_heavy_user_and_empty_ranks():
    deg = np.zeros(6, np.int64)
    deg[2] = 10_000
    rs = _ranges(6, 4, deg)
    assert rs[0][0] == 0 and rs[-1][1] == 6
    assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
    owner = [r for r, (a, b) in enumerate(rs) if a <= 2 < b]
    assert len(owner) == 1


def test_degree_length_checked():
    with pytest.raises(ValueError):
        shard_bounds(5, 2, 0, np.ones(4))


@pytest.mark.parametrize("world", [1, 2, 3, 4, 7, 8])
@pytest.mark.parametrize("count", [0, 4, 12, 64, 1000, 4 * 1_000_003, 32 * 1_000_000])
def test_p2p_block_and_gather_arithmetic(world, count):
    """hgd_p2p_allreduce's block split (host entry points of the arithmetic its kernels use, no
    device calls): the reduce blocks of the N ranks tile [0, count) in rank order with whole
    float4s, and every rank's gather visits each float4 outside its own block exactly once,
    from the rank that reduced it. Large counts are checked at the block edges only."""
    import ctypes

    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    lib = nat.load()
    lo, hi = ctypes.c_int64(), ctypes.c_int64()
    blocks = []
    for q in range(world):
        assert lib.hgd_p2p_block_range(count, world, q, ctypes.byref(lo), ctypes.byref(hi)) == 0
        blocks.append((lo.value, hi.value))
    assert blocks[0][0] == 0 and blocks[-1][1] == count
    assert all(a[1] == b[0] and a[0] <= a[1] and a[0] % 4 == 0 for a, b in zip(blocks, blocks[1:]))
    j, owner = ctypes.c_int64(), ctypes.c_int32()
    n4 = count // 4
    for rank in range(world):
        own = (blocks[rank][0] // 4, blocks[rank][1] // 4)
        rest = n4 - (own[1] - own[0])
        idx = range(rest) if rest <= 4096 else sorted({0, 1, rest // 2, rest - 2, rest - 1,
                                                        max(own[0] - 1, 0), min(own[0], rest - 1)})
        seen = []
        for i in idx:
            assert lib.hgd_p2p_gather_index(count, world, rank, i, ctypes.byref(j),
                                            ctypes.byref(owner)) == 0
            assert not (own[0] <= j.value < own[1])
            q = owner.value
            assert q != rank and blocks[q][0] // 4 <= j.value < blocks[q][1] // 4
            seen.append(j.value)
        if rest <= 4096:
            assert sorted(seen) == [x for x in range(n4) if not own[0] <= x < own[1]]
        if rest > 0:  # one past the end is rejected
            assert lib.hgd_p2p_gather_index(count, world, rank, rest, ctypes.byref(j),
                                            ctypes.byref(owner)) != 0
            assert b"out of range" in lib.hgd_get_last_error_string()
    # a successful call clears the process-wide last error again
    assert lib.hgd_p2p_block_range(count, world, 0, ctypes.byref(lo), ctypes.byref(hi)) == 0
    assert lib.hgd_get_last_error_string() == b""
