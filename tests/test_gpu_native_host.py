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
