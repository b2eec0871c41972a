"""bench.py --mode decode (configs[2]: Object.Metadata() + Object.Data() over
one resident records arena) against the CPU oracle, byte for byte.

DecodeBench encodes every chunk into one records arena, then runs the
zero-copy decode over the whole batch in one call and the materialising decode
chunk by chunk (two streams, two data slots). Here both legs run on a few
thousand records split into several chunks, and every output is compared with
oracle.decode_batch of the same arena: the whole-batch rows, record info and
ACL / region tables (zero copy: spans and Data() subslices are offsets into
the arena), then every chunk's rows, info, tables and materialised payloads."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import bench  # noqa: E402
from honu_amd.workload import gen_host_batch  # noqa: E402


def _host(t, nbytes, dtype=np.uint8):
    return t[:nbytes].cpu().numpy().view(dtype)


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


# chunks of >= 48 K records take the single-launch decode, smaller ones the
# split kernels (honu_decode_batch's choice)
@pytest.mark.parametrize("shape,n,chunks", [("small", 100000, 2), ("small", 20000, 4),
                                            ("mixed", 1500, 4), ("large", 200, 4)])
def test_decode_mode_bit_exact(oracle_lib, shape, n, chunks):
    seed = 11
    args = bench.parse_args(["--records", str(n), "--shape", shape, "--min-chunks", str(chunks),
                             "--seed", str(seed), "--mode", "decode", "--steps", "1",
                             "--warmup", "0"])
    b = bench.Bench(args, 0, 0, pipeline=False)
    assert len(b.chunks) == chunks
    db = bench.DecodeBench(b)
    assert db.encode_ok
    # the arena is the oracle's encoding of the same records
    hb = gen_host_batch(seed, shape, 0, n)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert (ost == 0).all()
    assert db.total == int(ooff[-1])
    assert np.array_equal(_host(db.rec_off, 8 * (n + 1), np.uint64), ooff)
    assert _host(db.arena, db.total).tobytes() == oout.tobytes()

    # zero copy, whole batch in one call (the single-launch decode from 48 K records)
    res = db.run(1, 0)
    assert res["verified"] is True
    assert res["zero_copy"]["records"] == n
    ometa, oinfo, oacl, oreg, _, otot = oracle_lib.decode_batch(oout, ooff, False)
    # run() ends with the materialising check pass, which rewrote rows with
    # chunk-relative list offsets: decode the whole batch once more
    db._zero_copy_once(torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    assert np.array_equal(_host(db.totals, 24, np.uint64), otot)
    assert _host(db.dmeta, 352 * n).tobytes() == ometa.tobytes()
    assert _host(db.dinfo, 32 * n).tobytes() == oinfo.tobytes()
    assert _host(db.dacl, 20 * int(otot[0])).tobytes() == oacl.tobytes()
    assert _host(db.dreg, 4 * int(otot[1])).tobytes() == oreg.tobytes()
    assert db.check_zero_copy()

    # materialising, chunk by chunk, checked as each chunk drains
    def check(a, z, sl):
        m = z - a
        cm, ci, ca, cr, cd, ct = oracle_lib.decode_batch(oout, ooff[a:z + 1], True)
        assert _host(db.dmeta[352 * a:], 352 * m).tobytes() == cm.tobytes()
        assert _host(db.dinfo[32 * a:], 32 * m).tobytes() == ci.tobytes()
        assert np.array_equal(_host(sl.totals, 24, np.uint64), ct)
        assert _host(sl.dacl, 20 * int(ct[0])).tobytes() == ca.tobytes()
        assert _host(sl.dreg, 4 * int(ct[1])).tobytes() == cr.tobytes()
        data = _host(sl.data, int(ct[2]))  # payloads; the alignment gaps are not written
        for i in range(m):
            o, ln = int(ci[i]["data_off"]), int(ci[i]["data_len"])
            assert data[o:o + ln].tobytes() == cd[o:o + ln].tobytes(), a + i
        assert db._check_chunk(a, z, sl)
        return True

    assert db.materialise_pass(check=check)
    db.release()
