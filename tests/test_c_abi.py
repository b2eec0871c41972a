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


@pytest.mark.gpu
@pytest.mark.parametrize("form", ["inplace", "table"])
@pytest.mark.parametrize("shape,n", [(2, 512), (0, 20000)], ids=["large", "small"])
def test_c_demo_count_sized_tables_vs_oracle(tmp_path, oracle_lib, shape, n, form):
    """The binding's DecodeBatch flow: ACL / region tables
    sized by the batch's entry counts through the retry on the totals the
    first call reports, not by record bytes. Table forms (acl_inplace 0,
    regions_inplace 0): the first call's caps are one entry per record, so the
    retry always runs. In-place forms (the defaults): the generator's lists
    need no table entry, so one call with empty tables is enough, and the
    demo rebuilds every ACL entry and region from the records arena.
    Everything the zero-copy decode returned is bit-exact with the oracle's
    decode of the same records, and the tables take their exact entry
    counts: a small fraction of the records arena (nothing in place)."""
    import numpy as np
    from honu_amd.metadata import ACL_DTYPE, INFO_DTYPE, META_DTYPE
    r = subprocess.run([DEMO, str(shape), str(n), str(tmp_path), form], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr
    assert ("decode calls 2," if form == "table" else "decode calls 1,") in r.stdout
    rd = lambda name, dt: np.fromfile(tmp_path / name, dtype=dt)  # noqa: E731
    rec, off = rd("rec.bin", np.uint8), rd("off.bin", np.uint64)
    inpl = form == "inplace"
    ometa, oinfo, oacl, oreg, _, otot = oracle_lib.decode_batch(rec, off, False, inpl, inpl)
    assert inpl == (int(otot[0]) + int(otot[1]) == 0)
    assert np.array_equal(rd("tot.bin", np.uint64), otot)
    assert rd("meta.bin", META_DTYPE).tobytes() == ometa.tobytes()
    assert rd("info.bin", INFO_DTYPE).tobytes() == oinfo.tobytes()
    assert rd("acl.bin", ACL_DTYPE).tobytes() == oacl.tobytes()
    assert rd("reg.bin", np.uint32).tobytes() == oreg.tobytes()
    table_bytes = 20 * int(otot[0]) + 4 * int(otot[1])
    assert f"table bytes {table_bytes} " in r.stdout
    assert table_bytes < 0.5 * len(rec)  # byte-sized tables would be 24x the arena
