"""BASELINE-size batches compared with the CPU oracle byte for byte.

configs[1] is 1M Small records encoded + decoded on one GPU; the other parity
tests compare at most a few thousand records byte-exact and check the big
batches through digests. Here the whole 1M Small batch (≈3.6 GB of records)
goes through the default batch calls (size pass + scan + encode + payload
copy; the single-launch decode, which honu_decode_batch picks from 48 K
records, both zero-copy and materialising) and every output is compared with
oracle.marshal_batch / oracle.decode_batch: the records arena, offsets and
statuses, all 352-byte rows, record info, the ACL and region tables, the
totals and every materialised payload. A 128 K Medium batch (≈3.4 GB) does the
same with 25 KB payloads.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from honu_amd import object as hobj  # noqa: E402
from honu_amd.workload import gen_host_batch  # noqa: E402


@pytest.mark.parametrize("shape,n", [("small", 1 << 20), ("medium", 1 << 17)])
def test_full_size_batch_bit_exact(oracle_lib, shape, n):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    hb = gen_host_batch(23, shape, 0, n)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert (ost == 0).all()
    c = hobj.Codec(0, n)
    try:
        enc = c.marshal(hobj.DeviceBatch.from_host(hb, c.torch_device))
        out, off, st = enc.host()
        assert np.array_equal(st, ost)
        assert np.array_equal(off, ooff)
        assert out.tobytes() == oout.tobytes()
        del out
        for materialize in (False, True):
            ometa, oinfo, oacl, oreg, odata, otot = oracle_lib.decode_batch(oout, ooff, materialize)
            dec = c.decode(enc.out, enc.out_off, n, materialize=materialize,
                           acl_cap=int(otot[0]), regions_cap=int(otot[1]),
                           data_cap=int(otot[2]), rec_bytes=int(ooff[-1]))
            meta, info, acl, reg, data, tot = dec.host()
            assert np.array_equal(tot, otot)
            assert meta.tobytes() == ometa.tobytes()
            assert info.tobytes() == oinfo.tobytes()
            assert acl.tobytes() == oacl[: int(otot[0])].tobytes()
            assert reg.tobytes() == oreg[: int(otot[1])].tobytes()
            if materialize:
                # every payload where Data() put it, equal to the source bytes
                doff = info["data_off"].astype(np.int64)
                dlen = info["data_len"].astype(np.int64)
                src = hb.payload_off.astype(np.int64)
                assert np.array_equal(dlen, np.diff(src))
                mark = np.zeros(len(data) + 1, np.int8)  # +1 at a payload's start, -1 past it
                np.add.at(mark, doff[dlen > 0], 1)
                np.add.at(mark, (doff + dlen)[dlen > 0], -1)
                inside = np.cumsum(mark, dtype=np.int8)[: len(data)].astype(bool)
                assert int(inside.sum()) == int(src[-1])
                assert np.array_equal(data[inside], hb.payload[: int(src[-1])])
            del dec, meta, info, acl, reg, data
            torch.cuda.synchronize()
    finally:
        c.close()
