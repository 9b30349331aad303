"""sharded.P2PExchange's lifetime on the CPU, with a stand-in for libhgd's hgd_p2p_* calls whose
"slots" are host memory: the handle is destroyed once a release was requested AND torch has
released the storage of every slot view handed out (nat.float_view's DLPack deleter), so a view
held past close() never points at freed memory, and an exchange — or the ShardedIncidence that
owns it — dropped without close() still frees its segments (tests/test_gpu_p2p.py repeats this
on the device with hipMemGetInfo)."""
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


def test_release_waits_for_every_slot_view(fake):
    ex = _exchange()
    live0 = nat.live_views()
    v = ex.slot(0, 8, 8)
    w = v[2:4]  # shares v's storage
    v.fill_(1.0)
    ex.release()
    with pytest.raises(RuntimeError, match="closed"):
        ex.slot(0, 8, 8)
    assert fake.destroyed == 0
    del v
    gc.collect()
    assert fake.destroyed == 0 and bool((w == 1.0).all())  # w still reads live memory
    del w
    gc.collect()
    assert fake.destroyed == 1 and nat.live_views() == live0
    ex.release()  # idempotent
    assert fake.destroyed == 1


def test_dropped_exchange_is_destroyed(fake):
    ex = _exchange()
    ex.slot(0, 8, 8).fill_(2.0)
    ex.slot(1, 4, 16)
    del ex
    gc.collect()
    assert fake.destroyed == 1


def test_dropped_sharded_incidence_destroys_its_exchange(fake):
    sh = sharded.ShardedIncidence.__new__(sharded.ShardedIncidence)
    sh._p2p = _exchange()
    sh._p2p.slot(0, 8, 8)
    del sh
    gc.collect()
    assert fake.destroyed == 1


def test_context_manager_closes(fake, monkeypatch):
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    with _exchange() as ex:
        ex.slot(0, 8, 8)
    assert fake.destroyed == 1 and ex.h is None
