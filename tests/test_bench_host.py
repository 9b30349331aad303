"""bench.py's host-side logic on the CPU: the N > 1 self-check default, the same-run parity gate
(row rule of tests/_ref64.check_rows) against the reference's torch.sparse.mm calls, the CPU
baseline's bounded prefix sample, and the gathering of per-rank checks over gloo."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

import bench  # noqa: E402


@pytest.mark.parametrize("argv,world,want", [([], 1, False), (["--gpus", "2"], 2, True),
                                             (["--gpus", "8"], 8, True),
                                             (["--gpus", "2", "--no-check"], 2, False),
                                             (["--check"], 1, True)])
def test_check_on_by_default_above_one_rank(argv, world, want):
    assert bench.check_enabled(bench.parse(argv), world) is want


def _graph(U=300, I=40, E=3000, seed=0):
    rng = np.random.default_rng(seed)
    key = np.unique(rng.integers(0, U, E) * I + rng.integers(0, I, E))
    return torch.from_numpy(np.stack([key // I, key % I]))


def test_parity_gate_accepts_reference_and_names_a_bad_row():
    U, I, d = 300, 40, 16
    idx = _graph(U, I)
    g = torch.Generator().manual_seed(1)
    X, dY = torch.randn(U, d, generator=g), torch.randn(U, d, generator=g)
    Y, dX, s = bench.cpu_reference(idx, X, dY, U, I)
    assert Y.shape == (U, d) and dX.shape == (U, d) and s >= 0
    ok = bench.parity_gate(Y.clone(), dX.clone(), Y, dX, s)
    assert ok["ok"] and ok["max_row_ratio_Y"] == 0.0 and ok["rows"] == U
    # a 1e-6 relative wobble passes, a 1e-4 one on one row fails and is located
    Yb = Y * (1 + 1e-6)
    assert bench.parity_gate(Yb, dX, Y, dX, s)["ok"]
    row = int(Y.abs().amax(1).argmax())
    Yb = Y.clone()
    Yb[row] += 1e-4 * Y[row].abs().max()
    bad = bench.parity_gate(Yb, dX, Y, dX, s)
    assert not bad["ok"] and bad["worst_row_Y"] == row and bad["rows_over_Y"] == 1
    # an all-zero reference row (a user without interactions) must come out exactly zero
    zero = int((Y.abs().amax(1) == 0).nonzero()[0]) if bool((Y.abs().amax(1) == 0).any()) else None
    Yz = Y.clone()
    if zero is None:
        Yz[0] = 0.0
        Yr = Yz.clone()
        zero = 0
    else:
        Yr = Y
    Yz[zero, 0] = 1e-30
    assert not bench.parity_gate(Yz, dX, Yr, dX, s)["ok"]


def test_row_parity_blocks_equal_one_pass():
    g = torch.Generator().manual_seed(2)
    ref = torch.randn(1000, 8, generator=g)
    got = ref + 1e-7 * torch.randn(1000, 8, generator=g)
    assert bench.row_parity(got, ref, block=64)[:3] == bench.row_parity(got, ref, block=4096)[:3]


def test_cpu_baseline_times_a_prefix_sample_of_the_same_graph():
    U, I, d = 400, 50, 8
    idx = _graph(U, I, 4000)
    X, dY = torch.randn(U, d), torch.randn(U, d)
    out = bench.cpu_baseline(idx, X, dY, U, I, d, "t", full_s=0.5, frac=0.25)
    n = int((idx[0] < 100).sum())
    assert f"{n} edges" in out["sample"] and "median of 5 after 2" in out["sample"]
    assert out["kind"] == "port" and out["value"] > 0 and out["single_thread"]["cores"] == 1
    assert out["full_size"]["value"] == round(idx.shape[1] / 0.5 / 1e6, 3)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = {"Y": {"ok": True, "max_rel_err": 1e-7 * (rank + 1)},
                "dX": {"ok": rank != 1, "max_rel_err": 2e-7}, "wall_s": 3.0 + rank}
        q.put(bench.gather_checks(mine, world, shared_device=False))
    finally:
        dist.destroy_process_group()


def test_gather_checks_over_gloo_fails_if_any_rank_fails():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(2, _free_port(), q), nprocs=2, join=True,
                       start_method="spawn")
    got = [q.get(timeout=60) for _ in range(2)]
    for c in got:
        assert c["ok"] is False and c["ranks_checked"] == 2 and c["ranks_in_parallel"]
        assert c["max_rel_err_Y"] == pytest.approx(2e-7) and c["wall_s"] == 4.0


def _first_step_worker(rank, world, port, corrupt, q):
    """One rank of a CPU rehearsal of bench.py's N > 1 check: this rank's checked step and first
    timed step against the same reference rows, the rehearsal hook applied, gathered."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if corrupt is not None:
        os.environ["HGD_BENCH_CORRUPT_FIRST_STEP"] = str(corrupt)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(10 + rank)
        Y_ref, dX_ref = torch.randn(50, 8, generator=g), torch.randn(50, 8, generator=g)
        mag_Y, mag_dX = Y_ref.abs() + 1.0, dX_ref.abs() + 1.0
        Y, dX = Y_ref * (1 + 1e-7), dX_ref.clone()  # the checked step: within the bound
        first = bench.corrupt_first_step((Y_ref.clone(), dX_ref.clone()), rank)
        check = bench.check_rows(Y, dX, Y_ref, dX_ref, mag_Y, mag_dX, first)
        got = bench.gather_checks(check, world, shared_device=False)
        q.put((rank, got, bench.line_status(got, None)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("corrupt", [None, 1])
def test_corrupted_first_step_fails_the_line_over_gloo(corrupt):
    """VERDICT r05 'Next' 1: a first timed step that is wrong on ONE rank (rank 1, by the
    HGD_BENCH_CORRUPT_FIRST_STEP hook) fails the gathered check on every rank and the run's exit
    status, while the step after timing alone would have passed."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_first_step_worker, args=(2, _free_port(), corrupt, q), nprocs=2,
                       join=True, start_method="spawn")
    got = [q.get(timeout=60) for _ in range(2)]
    for rank, c, rc in got:
        assert c["max_rel_err_Y"] < 1e-5 and c["max_rel_err_dX"] == 0.0
        fs = c["first_step"]
        if corrupt is None:
            assert c["ok"] and fs["ok"] and fs["failed_ranks"] == [] and rc == 0
        else:
            assert not c["ok"] and not fs["ok"] and fs["failed_ranks"] == [1] and rc == 1
            assert fs["max_rel_err_Y"] > 0.5


def test_parity_gate_holds_the_first_step_too():
    U, I, d = 300, 40, 16
    idx = _graph(U, I)
    g = torch.Generator().manual_seed(3)
    X, dY = torch.randn(U, d, generator=g), torch.randn(U, d, generator=g)
    Y, dX, s = bench.cpu_reference(idx, X, dY, U, I)
    ok = bench.parity_gate(Y.clone(), dX.clone(), Y, dX, s, first=(Y.clone(), dX.clone()))
    assert ok["ok"] and ok["first_step"]["ok"] and bench.line_status(None, ok) == 0
    Yf = Y.clone()
    Yf[5] += 1.0
    bad = bench.parity_gate(Y.clone(), dX.clone(), Y, dX, s, first=(Yf, dX.clone()))
    assert not bad["ok"] and not bad["first_step"]["ok"] and bad["first_step"]["worst_row_Y"] == 5
    assert bad["rows_over_Y"] == 0 and bench.line_status(None, bad) == 1


def test_host_cpus_reports_the_thread_choice():
    h = bench.host_cpus()
    assert h["os_cpu_count"] >= 1 and 1 <= h["affinity"] <= h["os_cpu_count"]
    assert 1 <= h["threads"] <= h["affinity"]
    if h["cgroup_cpu_quota"]:
        assert h["threads"] <= h["cgroup_cpu_quota"]
