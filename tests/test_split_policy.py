"""CPU: the long-row split policy (incidence.auto_split; the C handle's auto_split in
csrc/handle.hip restates it). Large structures split rows above pow2_floor(nnz / 8192) nonzeros,
clamped to [128, 2048], into chunks of half that (at most 512); small ones are cut for
occupancy. The headline graph keeps its 2,048 / 512 plan; a skewed catalogue of the plugin
epoch's size gets 128 / 64 (scripts/bench_skewed_hop.py)."""
import pytest

from hypergraph_diffusion_for_recommendation_amd.incidence import (DEFAULT_SPLIT_CHUNK,
                                                                   DEFAULT_SPLIT_THRESHOLD,
                                                                   TARGET_GROUPS, auto_split)


@pytest.mark.parametrize("n_rows,nnz,want", [
    (10_000_000, 100_000_000, (2048, 512)),   # headline H (users)
    (1_000_000, 100_000_000, (2048, 512)),    # headline Hᵀ (items)
    (69_716, 1_670_314, (128, 64)),           # Zipf Yelp-shaped norm_adj
    (69_716, 2_474_518, (256, 128)),          # uniform Yelp-shaped norm_adj
    (144_242, 4_480_000, (512, 256)),         # Amazon-shaped
    (20_000, 100_000, (128, 64)),             # floor
    (3_706, 1_000_000, (128, 64)),            # small row count: the occupancy rule
])
def test_auto_split_values(n_rows, nnz, want):
    assert auto_split(n_rows, nnz) == want


def test_auto_split_shape():
    for n_rows in (TARGET_GROUPS, 10 * TARGET_GROUPS):
        prev = 0
        for nnz in [2 ** k for k in range(10, 34)]:
            t, c = auto_split(n_rows, nnz)
            assert 128 <= t <= DEFAULT_SPLIT_THRESHOLD and t & (t - 1) == 0
            assert c == min(t // 2, DEFAULT_SPLIT_CHUNK)
            assert t >= prev  # never shrinks as the structure grows
            prev = t
            assert t <= max(128, nnz // 8192)
