"""Host logic of the source-blocked hop selection (incidence.spmm_blocks): which hops run as
hgd_spmm_blocked and in how many blocks. No GPU: the structures are CPU tensors that are never
launched on."""
import pytest
import torch

from hypergraph_diffusion_for_recommendation_amd.incidence import CSR, spmm_blocks


def _csr(n_rows, n_cols, nnz=10, ascending=True):
    rowptr = torch.zeros(n_rows + 1, dtype=torch.int64)
    rowptr[-1] = nnz
    s = CSR(rowptr, torch.zeros(nnz, dtype=torch.int32), n_rows, n_cols, split_threshold=0)
    s.cols_ascending = ascending
    return s


@pytest.fixture(autouse=True)
def _no_env(monkeypatch):
    monkeypatch.delenv("HGD_SPMM_BLOCKS", raising=False)


def test_size_rule_follows_the_gathered_table():
    # the bench's hop into items gathers the 10 M-row user table
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 64) == 4     # 2.56 GB
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 128) == 8    # 5.12 GB
    # rows wider than 128 run blocked as 128-column passes: the table of one pass decides
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 256) == 8
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 1024) == 8
    assert spmm_blocks(_csr(1_000_000, 2_000_000), 256) == 2  # 1.02 GB < 1 GiB
    assert spmm_blocks(_csr(1_000_000, 1_000_000), 256) == 0  # 512 MB < 512 MiB
    assert spmm_blocks(_csr(1_000_000, 100_000_000), 64) == 16  # clamped
    # the hop into users gathers the 256 MB item table: one pass
    assert spmm_blocks(_csr(10_000_000, 1_000_000), 64) == 0
    # the 512 MiB and 1 GiB steps
    assert spmm_blocks(_csr(10, (1 << 29) // 256 - 1), 64) == 0
    assert spmm_blocks(_csr(10, (1 << 29) // 256), 64) == 2
    assert spmm_blocks(_csr(10, (1 << 30) // 256 - 1), 64) == 2
    assert spmm_blocks(_csr(10, (1 << 30) // 256), 64) == 4  # at least 4 blocks
    # the sharded hop's 32-column slices: a 5 M-user shard (N = 2) 2 blocks, 2.5 M (N = 4) none
    assert spmm_blocks(_csr(1_000_000, 5_000_000), 32) == 2
    assert spmm_blocks(_csr(1_000_000, 2_500_000), 32) == 0
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 32) == 4   # 1.28 GB: measured best at 4


def test_only_for_ascending_unsplit_plain_structures(monkeypatch):
    big = 10_000_000
    assert spmm_blocks(_csr(1000, big, ascending=False), 64) == 0
    assert spmm_blocks(_csr(1000, big, nnz=0), 64) == 0
    s = _csr(1000, big)
    s.plan.flags = 1  # the segmented walk
    assert spmm_blocks(s, 64) == 0
    s = _csr(1000, big)
    s.plan.threshold, s.plan.n_heavy = 16, 3  # split rows
    assert spmm_blocks(s, 64) == 0
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "5")  # forcing never overrides the structure rules
    assert spmm_blocks(_csr(1000, big, ascending=False), 64) == 0


def test_environment_override(monkeypatch):
    small = _csr(100, 1000)
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "3")
    assert spmm_blocks(small, 8) == 3
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "1")
    assert spmm_blocks(small, 8) == 0
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "0")
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 64) == 0
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "auto")
    assert spmm_blocks(_csr(1_000_000, 10_000_000), 64) == 4
    monkeypatch.setenv("HGD_SPMM_BLOCKS", "65")
    with pytest.raises(ValueError):
        spmm_blocks(small, 8)


def test_blocked_implementation_bytes():
    from hypergraph_diffusion_for_recommendation_amd import profiling
    nnz, R, d = 1000, 100, 64
    plain = profiling.impl_bytes(nnz, R, d, True, True)
    assert profiling.impl_bytes(nnz, R, d, True, True, blocks=1) == plain
    four = profiling.impl_bytes(nnz, R, d, True, True, blocks=4)
    # + 3 Y writes and 3 Y reads, + 3 row-scale reads, block starts (R·5·8) for rowptr (R+1)·8
    assert four - plain == 6 * R * 4 * d + 3 * R * 4 + R * 5 * 8 - (R + 1) * 8


def test_library_size_rule():
    """hgd_spmm_blocks_for, the one size rule both hosts use (host-only, no device)."""
    from hypergraph_diffusion_for_recommendation_amd import _native as nat
    f = nat.load().hgd_spmm_blocks_for
    assert f(0, 64) == 0 and f(10_000_000, 0) == 0
    assert f(10_000_000, 64) == 4 and f(10_000_000, 128) == 8 and f(10_000_000, 512) == 8
    # table / 640 MiB exactly halfway: rounded half to even (4.5 -> 4, 5.5 -> 6)
    assert f(int(4.5 * (640 << 20)) // 256, 64) == 4
    assert f(int(5.5 * (640 << 20)) // 256, 64) == 6
    assert f(int(6.4 * (640 << 20)) // 256, 64) == 6
    assert f(int(6.6 * (640 << 20)) // 256, 64) == 7
