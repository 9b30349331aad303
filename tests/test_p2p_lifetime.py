"""sharded.P2PExchange's lifetime on the CPU, with a stand-in for libhgd's hgd_p2p_* calls whose
"slots" are host memory: the handle is destroyed only after a COLLECTIVE close() (no peer reads
its segments any more) AND once torch has released the storage of every slot view handed out
(nat.float_view's DLPack deleter) — never inside that deleter, which only queues it for the next
safe point. An exchange — or the ShardedIncidence that owns it — dropped without close() keeps
its segments mapped until a later collective close() in the process covers it
(tests/test_gpu_p2p.py repeats this on the device with hipMemGetInfo)."""
import ctypes
import gc

import pytest
import torch

from hypergraph_diffusion_for_recommendation_amd import _native as nat
from hypergraph_diffusion_for_recommendation_amd import sharded


class _FakeLib:
    def __init__(self, floats):
        self.buf = (ctypes.c_float * floats)()
        self.destroyed = 0

    def hgd_p2p_create(self, world, rank, count, slots, out):
        out._obj.value = 1
        return 0

    def hgd_p2p_set_timeout(self, h, t):
        return 0

    def hgd_p2p_export(self, h, buf):
        return 0

    def hgd_p2p_open(self, h, blob):
        return 0

    def hgd_p2p_slot(self, h, k):
        return ctypes.addressof(self.buf) + 4 * 64 * int(k)

    def hgd_p2p_destroy(self, h):
        self.destroyed += 1


@pytest.fixture
def fake(monkeypatch):
    lib = _FakeLib(64 * 4)
    monkeypatch.setattr(nat, "load", lambda: lib)
    return lib


def _exchange():
    return sharded.P2PExchange(64, 2, "cpu", setup_timeout_s=10.0)


@pytest.fixture(autouse=True)
def _no_sync(monkeypatch):
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    sharded.release_pending_p2p()
    with sharded._PLOCK:
        sharded._ABANDONED.clear()


def test_close_waits_for_every_slot_view_and_never_destroys_in_the_deleter(fake):
    ex = _exchange()
    live0 = nat.live_views()
    v = ex.slot(0, 8, 8)
    w = v[2:4]  # shares v's storage
    v.fill_(1.0)
    ex.close()
    with pytest.raises(RuntimeError, match="closed"):
        ex.slot(0, 8, 8)
    assert fake.destroyed == 0
    del v
    gc.collect()
    assert fake.destroyed == 0 and bool((w == 1.0).all())  # w still reads live memory
    del w
    gc.collect()
    assert fake.destroyed == 0  # due, but the deleter only queued it
    assert nat.live_views() == live0
    assert sharded.release_pending_p2p() == 1 and fake.destroyed == 1
    ex.close()  # idempotent
    ex.release()
    assert fake.destroyed == 1


def test_close_without_live_views_destroys_at_once(fake):
    ex = _exchange()
    ex.slot(0, 8, 8).fill_(1.0)  # the view is gone by the time close() runs
    gc.collect()
    ex.close()
    assert fake.destroyed == 1


def test_dropped_exchange_stays_mapped_until_a_collective_close(fake):
    ex = _exchange()
    ex.slot(0, 8, 8).fill_(2.0)
    ex.slot(1, 4, 16)
    del ex
    gc.collect()
    assert fake.destroyed == 0 and sharded.abandoned_p2p() == 1  # a peer may still read it
    other = _exchange()
    other.close()  # collective: covers the dropped exchange too
    assert fake.destroyed == 2 and sharded.abandoned_p2p() == 0


def test_dropped_sharded_incidence_keeps_its_exchange_mapped(fake):
    sh = sharded.ShardedIncidence.__new__(sharded.ShardedIncidence)
    sh._p2p = _exchange()
    sh._p2p.slot(0, 8, 8)
    del sh
    gc.collect()
    assert fake.destroyed == 0 and sharded.abandoned_p2p() == 1
    _exchange().close()
    assert fake.destroyed == 2


def test_a_close_over_another_group_leaves_a_dropped_exchange_mapped(fake):
    ex = _exchange()
    ex.slot(0, 8, 8)
    del ex
    gc.collect()
    other = sharded.P2PExchange(64, 2, "cpu", group=object(), setup_timeout_s=10.0)
    other.world = 1  # the stand-in group has one rank: no barrier
    other.close()
    assert fake.destroyed == 1 and sharded.abandoned_p2p() == 1  # only `other`'s own
    _exchange().close()  # a close over the default group covers it
    assert fake.destroyed == 3 and sharded.abandoned_p2p() == 0


def test_context_manager_closes(fake):
    with _exchange() as ex:
        ex.slot(0, 8, 8)
    gc.collect()
    sharded.release_pending_p2p()
    assert fake.destroyed == 1 and ex.h is None
