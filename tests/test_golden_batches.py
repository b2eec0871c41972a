"""Committed golden batches (tests/golden/batches, written by
tests/make_golden_batches.py from the oracle): the files match their SHA-256
manifest; the generator + oracle still reproduce them bit for bit (CPU); the
GPU path reproduces them without consulting the oracle (-m gpu)."""
import hashlib
import json
import os

import numpy as np
import pytest

import make_golden_batches as mk

BATCHES = mk.OUT
MANIFEST = json.load(open(os.path.join(BATCHES, "manifest.json")))


def _file(name, suf):
    with open(os.path.join(BATCHES, f"{name}.{suf}.bin"), "rb") as fh:
        return fh.read()


@pytest.mark.parametrize("name", mk.NAMES)
def test_fixture_files_match_manifest(name):
    for suf, digest in MANIFEST[name]["sha256"].items():
        assert hashlib.sha256(_file(name, suf)).hexdigest() == digest, suf


@pytest.mark.parametrize("name", mk.NAMES)
def test_oracle_and_generator_reproduce_fixture(oracle_lib, name):
    files, tot = mk.outputs(name)
    assert tot == MANIFEST[name]["totals"]
    for suf, data in files.items():
        assert hashlib.sha256(data).hexdigest() == MANIFEST[name]["sha256"][suf], suf


@pytest.mark.gpu
@pytest.mark.parametrize("name", mk.NAMES)
def test_gpu_reproduces_fixture(name):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd import object as hobj
    from honu_amd.metadata import ACL_DTYPE, INFO_DTYPE, META_DTYPE
    rec = np.frombuffer(_file(name, "records"), np.uint8)
    off = np.frombuffer(_file(name, "offsets"), "<u8").astype(np.uint64)
    n = len(off) - 1
    c = hobj.Codec(0, max(n, 1))
    try:
        if name in mk.ENCODE:
            r = c.marshal(hobj.DeviceBatch.from_host(mk.encode_input(mk.ENCODE[name]), c.torch_device))
            torch.cuda.synchronize()
            out, goff, st = r.host()
            assert (st == 0).all() and np.array_equal(goff, off)
            assert out.tobytes() == rec.tobytes()
        d_rec = hobj._dev_bytes(rec if len(rec) else np.zeros(1, np.uint8), c.torch_device)
        d_off = hobj._dev_bytes(off, c.torch_device)
        # both list forms (totals: ACL, regions, data bytes of the in-place
        # forms, then the table forms' ACL entries and regions), both decodes
        # (single launch, split)
        for inplace, sfx in ((1, ""), (0, "_table")):
            hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"acl_inplace", inplace), "param")
            hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"regions_inplace", inplace), "param")
            for rv in (6, 5):
                hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"record_variant", rv), "param")
                meta, info, acl, reg, _, tot = c.decode(d_rec, d_off, n, rec_bytes=int(off[-1])).host()
                want = MANIFEST[name]["totals"]
                assert [int(x) for x in tot] == (want[:3] if inplace else [want[3], want[4], want[2]])
                assert meta.tobytes() == np.frombuffer(_file(name, "rows" + sfx), META_DTYPE).tobytes()
                assert info.tobytes() == np.frombuffer(_file(name, "info"), INFO_DTYPE).tobytes()
                assert acl.tobytes() == np.frombuffer(_file(name, "acl" + sfx), ACL_DTYPE).tobytes()
                assert reg.tobytes() == _file(name, "regions" + sfx)
    finally:
        c.close()
