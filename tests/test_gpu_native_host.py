"""The plain-C host example (examples/hgconv2_host.c) runs hgconv2 through the C ABI on the GPU
and matches its own float64 host computation (the C program checks and exits non-zero on a
mismatch)."""
import subprocess

import pytest

pytestmark = pytest.mark.gpu


def test_c_host_hgconv2(tmp_path):
    from tests._native_host import build
    exe = build(tmp_path / "hgconv2_host")
    if exe is None:
        pytest.skip("gcc not available")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "hgconv2_host ok" in r.stdout


def test_c_host_conv2hop_objects(tmp_path):
    """examples/conv2hop_objects.c: incidence object, one-rank RCCL communicator, sharded conv
    forward + backward against the host float64 computation."""
    import os
    from tests._native_host import build
    exe = build(tmp_path / "conv2hop_objects", "conv2hop_objects.c")
    if exe is None:
        pytest.skip("gcc not available")
    env = dict(os.environ, WORLD_SIZE="1", RANK="0")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "conv2hop_objects ok" in r.stdout


def test_c_host_conv2hop_objects_over_p2p(tmp_path):
    """The same C host with HGD_TRANSPORT=p2p: two processes share the device, the peer-exchange
    handles travel through files, hgd_comm_create_p2p carries the conv's exchange; every rank's
    rows match the float64 host computation of the whole graph."""
    import os
    from tests._native_host import build
    exe = build(tmp_path / "conv2hop_objects", "conv2hop_objects.c")
    if exe is None:
        pytest.skip("gcc not available")
    procs = []
    for rank in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(rank), HGD_TRANSPORT="p2p",
                   HGD_COMM_ID_FILE=str(tmp_path / "p2p_handle"))
        procs.append(subprocess.Popen([exe], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env))
    for p in procs:
        out, err = p.communicate(timeout=180)
        assert p.returncode == 0, err + out
        assert "conv2hop_objects ok" in out and "(p2p)" in out
