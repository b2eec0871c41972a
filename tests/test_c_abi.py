"""The C ABI driven from plain C (honu_amd/c_abi_demo.c: the MarshalBatch /
DecodeBatch flow a cgo shim runs, no Python or torch in the process): it
refuses to run without a gfx950 device and, on one, marshals and decodes
synthetic batches with every status, field and payload digest checked."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "honu_amd", "c_abi_demo")


def _gpu():
    torch = pytest.importorskip("torch")
    return torch.cuda.device_count() > 0


def test_c_demo_refuses_without_gpu():
    if not os.path.exists(DEMO):
        pytest.skip("c_abi_demo not built")
    if _gpu():
        pytest.skip("GPU present")
    r = subprocess.run([DEMO, "0", "16"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "gfx950" in r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("shape,n", [(0, 4096), (4, 2048), (2, 256)], ids=["small", "mixed", "large"])
def test_c_demo_marshal_decode(shape, n):
    assert os.path.exists(DEMO), "honu_amd/c_abi_demo not built (make -C honu_amd)"
    r = subprocess.run([DEMO, str(shape), str(n)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert r.stdout.startswith("ok:")
