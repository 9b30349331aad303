"""bench.py's ``--transport auto`` decision (choose_transport) on two gloo ranks on the CPU: the
ranks must agree — the peer exchange is used only if it worked on EVERY rank, matched the
all-reduce's result and was faster; any failure or mismatch on one rank keeps RCCL on all of
them and is reported. The transports are stand-ins (timed sleeps, fixed results); the decision
logic and its collectives are bench.py's own."""
import os
import socket
import sys
import time

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _FakeP2P:
    def __init__(self, fail):
        self.fail = fail

    def wait(self):
        pass

    def check(self):
        if self.fail == "check":
            raise RuntimeError("hgd_p2p: a wait timed out")


class _FakeShard:
    def __init__(self, rank, case):
        self.rank, self.case = rank, case
        self.transport = "rccl"
        self._p2p = _FakeP2P(case if rank == 1 else None)


def _worker(rank, world, port, case, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, ROOT)
        import bench
        torch.cuda.synchronize = lambda *a, **k: None  # CPU stand-in: nothing queued
        sh = _FakeShard(rank, case)
        Y = torch.linspace(-1.0, 1.0, 64).reshape(8, 8)

        p2p_steps = [0]
        rccl_steps = [0]

        def eager_step():
            if sh.transport == "p2p":
                p2p_steps[0] += 1
                if case == "raise" and rank == 1:
                    raise RuntimeError("P2PExchange: rank 1: hgd_p2p_open: did not return")
                if case == "raise_timed" and rank == 1 and p2p_steps[0] == 2:
                    # the first TIMED step (the checked step passed): the other rank is
                    # already inside timed()'s collectives
                    raise RuntimeError("hgd_p2p_poll: a wait timed out on this rank")
                time.sleep(0.002 if case != "slower" else 0.02)
                y = Y * (1.0 + 1e-3) if case == "mismatch" and rank == 0 else Y
                return y, Y.clone()
            time.sleep(0.01)
            rccl_steps[0] += 1
            if case == "first_rccl_off" and rccl_steps[0] == 1:
                # the one-device gloo rehearsal's flake: the first all-reduce step after the
                # warm-up barrier is off; the reference is the last timed all-reduce step
                return Y * 1.5, Y.clone()
            return Y.clone(), Y.clone()

        out = bench.choose_transport(sh, eager_step, torch.device("cpu"), lambda m: None, n=2)
        if case == "first_rccl_off":  # reported, and it fails the run whatever is chosen
            assert out["rccl_first_vs_last_rel_diff"] > 0.4, out
            assert out["rccl_first_step_ok"] is False and bench.line_status(None, None, out) == 1
        else:
            assert out["rccl_first_step_ok"] is True and bench.line_status(None, None, out) == 0
        q.put((rank, out["chosen"], out.get("p2p_failed_on_some_rank", False),
               "p2p_error" in out, sh.transport))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case,chosen,failed", [("ok", "p2p", False), ("slower", "rccl", False),
                                                ("raise", "rccl", True), ("check", "rccl", True),
                                                ("mismatch", "rccl", True),
                                                ("raise_timed", "rccl", True),
                                                ("first_rccl_off", "p2p", False)])
def test_auto_transport_decision_is_agreed(case, chosen, failed):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    mp.start_processes(_worker, args=(2, _free_port(), case, q), nprocs=2, join=True,
                       start_method="spawn")
    got = sorted(q.get(timeout=60) for _ in range(2))
    for rank, ch, fail, has_err, transport in got:
        assert ch == chosen and transport == chosen, (case, rank, ch, transport)
        assert fail == failed, (case, rank, fail)
    if case in ("raise", "raise_timed"):  # the failing rank reports its error
        assert got[1][3]
