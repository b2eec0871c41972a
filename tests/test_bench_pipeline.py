"""The bench's exact timed pipeline against the CPU oracle, byte for byte.

bench.py times a pipelined form of the codec that no other test drives: per
chunk, the size pass + scan, the header/tail encoder and the decode parse /
tables run on one stream while the payload copies run on a second stream, the
encode copy starting after the scan so it writes payload bytes into the same
16-byte chunks the header/tail encoder is writing around them; two output
slots alternate across chunks and across steps. Here Bench itself runs that
pipeline on small batches split into 5 chunks for 2 steps (with the
single-launch decode and with the split parse + tables), and every chunk of
every step is compared with oracle.marshal_batch / oracle.decode_batch once it
has drained (while the next chunk runs): encoded bytes, offsets, statuses,
full 352-byte rows, record info, ACL and region tables and every materialised
payload."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

import bench  # noqa: E402
from honu_amd import _lib  # noqa: E402
from honu_amd.metadata import HostBatch  # noqa: E402
from honu_amd.workload import gen_host_batch  # noqa: E402


def _host(t, nbytes, dtype=np.uint8):
    return t[:nbytes].cpu().numpy().view(dtype)


@pytest.fixture(autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("decode", ["fused", "split"])
@pytest.mark.parametrize("after,beside,ms,cs", [("scan", "encode", 1, 1), ("meta", "encode", 1, 1),
                                                ("scan", "decode", 1, 1), ("scan", "encode", 2, 1),
                                                ("scan", "decode", 2, 1), ("scan", "encode", 2, 2),
                                                ("scan", "decode", 2, 2)])
@pytest.mark.parametrize("shape,n", [("small", 4000), ("mixed", 1200), ("large", 160)])
def test_bench_pipeline_bit_exact(oracle_lib, shape, n, after, decode, beside, ms, cs):
    seed = 7
    args = bench.parse_args(["--records", str(n), "--shape", shape, "--min-chunks", "5",
                             "--encode-copy-after", after, "--seed", str(seed),
                             "--decode", decode, "--meta-beside", beside, "--meta-streams", str(ms),
                             "--copy-streams", str(cs)])
    b = bench.Bench(args, 0, 0)
    assert len(b.chunks) >= 5 and len(b.slots) == 2 and len(b.sms) == ms
    assert (b.sd is b.sc) == (cs == 1)
    hb = gen_host_batch(seed, shape, 0, n)  # the same records the device generator made
    seen = []

    def check(a, z, sl):
        m = z - a
        sub = HostBatch(hb.meta[a:z], hb.var, hb.acl, hb.regions, hb.payload,
                        hb.payload_off[a:z + 1])
        oout, ooff, ost = oracle_lib.marshal_batch(sub)
        assert (ost == 0).all()
        assert np.array_equal(_host(sl.status, 4 * m, np.int32), ost)
        assert np.array_equal(_host(sl.out_off, 8 * (m + 1), np.uint64), ooff)
        assert _host(sl.out, int(ooff[-1])).tobytes() == oout.tobytes(), (a, z)
        ometa, oinfo, oacl, oreg, odata, otot = oracle_lib.decode_batch(oout, ooff, True)
        assert np.array_equal(_host(sl.totals, 24, np.uint64), otot)
        assert _host(sl.dmeta, 352 * m).tobytes() == ometa.tobytes()
        assert _host(sl.dinfo, 32 * m).tobytes() == oinfo.tobytes()
        assert _host(sl.dacl, 20 * int(otot[0])).tobytes() == oacl.tobytes()
        assert _host(sl.dreg, 4 * int(otot[1])).tobytes() == oreg.tobytes()
        data = _host(sl.data, int(otot[2]))
        for i in range(m):
            o, ln = int(oinfo[i]["data_off"]), int(oinfo[i]["data_len"])
            assert data[o:o + ln].tobytes() == odata[o:o + ln].tobytes(), (a + i)
        # the bench's own device-side check agrees
        assert b._verify_chunk(a, z, sl)
        seen.append((a, z, sl))
        return True

    for _ in range(2):
        assert b.step(check=check)
    torch.cuda.synchronize()
    assert [x[:2] for x in seen] == b.chunks * 2
    # slots alternate across chunks and across steps (5 chunks: step 2 starts on slot 1)
    slots = [id(x[2]) for x in seen]
    assert all(p != q for p, q in zip(slots, slots[1:]))


@pytest.mark.parametrize("slots", [2, 3])
@pytest.mark.parametrize("shape,n", [("small", 4000), ("mixed", 1200)])
def test_bench_copy_order_ahead(oracle_lib, shape, n, slots):
    """--copy-order ahead: chunk k's decode copy is issued after chunk k+1's
    encode copy (and the last one by flush()); every chunk still decodes to
    the oracle's bytes, with 2 and 3 slots in rotation."""
    seed = 11
    args = bench.parse_args(["--records", str(n), "--shape", shape, "--min-chunks", "5",
                             "--seed", str(seed), "--copy-order", "ahead", "--slots", str(slots)])
    b = bench.Bench(args, 0, 0)
    assert b.ahead and len(b.slots) == slots
    hb = gen_host_batch(seed, shape, 0, n)
    seen = []

    def check(a, z, sl):
        sub = HostBatch(hb.meta[a:z], hb.var, hb.acl, hb.regions, hb.payload,
                        hb.payload_off[a:z + 1])
        oout, ooff, _ = oracle_lib.marshal_batch(sub)
        assert _host(sl.out, int(ooff[-1])).tobytes() == oout.tobytes(), (a, z)
        _, oinfo, _, _, odata, otot = oracle_lib.decode_batch(oout, ooff, True)
        data = _host(sl.data, int(otot[2]))
        for i in range(z - a):
            o, ln = int(oinfo[i]["data_off"]), int(oinfo[i]["data_len"])
            assert data[o:o + ln].tobytes() == odata[o:o + ln].tobytes(), (a + i)
        assert b._verify_chunk(a, z, sl)
        seen.append((a, z))
        return True

    for _ in range(2):  # the timed form (decode copies one chunk behind), then a checked step
        b.step()
    assert b.pending_dec is not None
    b.flush()
    assert b.pending_dec is None
    for _ in range(2):
        assert b.step(check=check)
    torch.cuda.synchronize()
    assert seen == b.chunks * 2
    assert b.verify()


@pytest.mark.parametrize("shape,n", [("mixed", 1500), ("small", 4000)])
def test_bench_encode_only_bit_exact(oracle_lib, shape, n):
    """--mode encode (configs[3]: size pass, scan, header/tail encoder and
    payload copy, no decode), the pipeline the default line's mixed_encode
    leg times: every chunk's records equal oracle.marshal_batch's, and the
    bench's own verification (zero-copy decode of each chunk, row and payload
    digests) passes."""
    seed = 5
    args = bench.parse_args(["--records", str(n), "--shape", shape, "--min-chunks", "4",
                             "--seed", str(seed), "--mode", "encode"])
    b = bench.Bench(args, 0, 0, encode_only=True)
    assert len(b.chunks) >= 4
    hb = gen_host_batch(seed, shape, 0, n)
    seen = []

    def check(a, z, sl):
        sub = HostBatch(hb.meta[a:z], hb.var, hb.acl, hb.regions, hb.payload,
                        hb.payload_off[a:z + 1])
        oout, ooff, ost = oracle_lib.marshal_batch(sub)
        assert np.array_equal(_host(sl.status, 4 * (z - a), np.int32), ost)
        assert np.array_equal(_host(sl.out_off, 8 * (z - a + 1), np.uint64), ooff)
        assert _host(sl.out, int(ooff[-1])).tobytes() == oout.tobytes(), (a, z)
        seen.append((a, z))
        return True

    for _ in range(2):
        b.step()
    for _ in range(2):
        assert b.step(check=check)
    torch.cuda.synchronize()
    assert seen == b.chunks * 2
    assert b.verify()


def test_bench_verify_detects_corruption():
    """_verify_chunk (honu_verify_decoded + digests) flags one wrong byte in a
    decoded ObjectID, span, ACL entry (in place in the records arena: its
    flag, a ClientID byte, its Permissions; or in the table), region (in
    place: a byte of its uvarint in the records arena; or in the table) or
    payload."""
    args = bench.parse_args(["--records", "600", "--shape", "small", "--min-chunks", "1"])
    b = bench.Bench(args, 0, 0)
    (a, z), = b.chunks
    sl = b._issue(a, z, False)
    torch.cuda.synchronize()
    assert b._verify_chunk(a, z, sl)
    m = z - a
    rows = _host(sl.dmeta, 352 * m, np.uint8).copy().reshape(m, 352)
    tot = _host(sl.totals, 24, np.uint64)

    def flip(t, k):
        v = t[k:k + 1].clone()
        t[k:k + 1] = v ^ 0x5A
        torch.cuda.synchronize()
        ok = b._verify_chunk(a, z, sl)
        t[k:k + 1] = v
        torch.cuda.synchronize()
        return ok

    i = 17
    mime = int(rows[i, 208:216].view(np.uint64)[0])
    assert not flip(sl.dmeta, 352 * i + 96)          # ObjectID byte
    assert not flip(sl.dmeta, 352 * i + 11)          # padding must stay zero
    assert not flip(sl.out, mime)                    # a MIME span byte in the records arena
    from honu_amd.metadata import ACL_INPLACE
    pr, acl_off, nacl = (int(rows[i, 0:4].view(np.uint32)[0]), int(rows[i, 320:328].view(np.uint64)[0]),
                         int(rows[i, 328:336].view(np.uint64)[0]))
    assert nacl and pr & ACL_INPLACE and int(tot[0]) == 0  # the generator writes no nil entry
    for k in (0, 1, 17):  # the 2nd entry's flag, a ClientID byte, the Permissions byte
        assert not flip(sl.out, acl_off + 18 * (nacl // 2) + k)
    from honu_amd.metadata import REGIONS_INPLACE
    nreg = rows[:, 344:352].copy().view(np.uint64)[:, 0]
    j = int(np.flatnonzero(nreg > 1)[0])
    pr = int(rows[j, 0:4].view(np.uint32)[0])
    assert pr & REGIONS_INPLACE and int(tot[1]) == 0  # every region list in place
    reg_off = int(rows[j, 336:344].view(np.uint64)[0])
    assert not flip(sl.out, reg_off)                 # the first region's uvarint
    for x in b.slots:  # the table forms
        _lib.check(b.lib.honu_ctx_set_param(x.codec.ctx, b"acl_inplace", 0), "param")
        _lib.check(b.lib.honu_ctx_set_param(x.codec.ctx, b"regions_inplace", 0), "param")
    sl = b._issue(a, z, False)
    torch.cuda.synchronize()
    assert b._verify_chunk(a, z, sl)
    tot = _host(sl.totals, 24, np.uint64)
    assert not flip(sl.dacl, 20 * (int(tot[0]) // 2) + 3)
    assert not flip(sl.dreg, 4 * (int(tot[1]) // 2))
    info = _host(sl.dinfo, 32 * m, np.uint64).reshape(m, 4)
    assert not flip(sl.data, int(info[i, 0]) + 5)    # a payload byte
    assert b._verify_chunk(a, z, sl)


def test_encode_payloads_respects_out_cap(oracle_lib):
    """honu_encode_payloads run without the header/tail encoder's capacity
    verdict (another stream) writes nothing past out_cap."""
    from honu_amd import object as hobj
    hb = gen_host_batch(3, "small", 0, 200)
    oout, ooff, _ = oracle_lib.marshal_batch(hb)
    codec = hobj.Codec(0, 1024)
    d = hobj.DeviceBatch.from_host(hb, codec.torch_device)
    total = int(ooff[-1])
    cap = int(ooff[120]) + 7  # record 120 does not fit
    out = torch.full((total + 4096,), 0xEE, dtype=torch.uint8, device=codec.torch_device)
    off = torch.from_numpy(ooff.view(np.uint8).copy()).to(codec.torch_device)
    st = torch.zeros(4 * 200, dtype=torch.uint8, device=codec.torch_device)  # size pass: all OK
    _lib.check(codec.lib.honu_encode_payloads(codec.ctx, _lib.ptr(d.payload),
                                              _lib.ptr(d.payload_off), 200, _lib.ptr(out), cap,
                                              _lib.ptr(off), _lib.ptr(st), codec.stream), "copy")
    torch.cuda.synchronize()
    h = out.cpu().numpy()
    assert (h[cap:] == 0xEE).all()
    # the records that fit got their payload bytes
    for i in (0, 50, 119):
        s = int(ooff[i])
        plen = int(hb.payload_off[i + 1] - hb.payload_off[i])
        hl = 1 + len(oracle_lib.put_uvarint(plen))
        assert h[s + hl:s + hl + plen].tobytes() == oout[s + hl:s + hl + plen].tobytes()
    codec.close()


@pytest.mark.parametrize("units", [1, 0], ids=["units_pair", "plain_pair"])
@pytest.mark.parametrize("corpus", ["random", "small", "large"])
def test_encode_pairs_bit_exact(oracle_lib, corpus, units):
    """The two forms of the split encode, each phase on its own stream as the
    bench runs them: honu_encode_records_units + honu_encode_payloads_units
    (the encoder writes each payload's partial end 64-byte units, the copy the
    whole ones; ABI 5) and honu_encode_records + honu_encode_payloads. Every
    record's bytes equal oracle.marshal_batch's, with empty, tiny, unit-
    aligned and unit-straddling payloads (random corpus: nil metas, empty
    data, every frame size) and the output arena at several 64-byte phases."""
    from corpora import random_metas
    from honu_amd import object as hobj
    from honu_amd.metadata import pack_batch
    if corpus == "random":
        metas, datas = random_metas(300, 91)
        # payload lengths around the unit: 0..130 bytes, and a few long ones
        datas = [None if d is None else bytes((j * 7 + k) & 0xFF for k in range((j * 37) % 131 if j % 5 else 4096 + j))
                 for j, d in enumerate(datas)]
        hb = pack_batch(metas, datas)
    else:
        hb = gen_host_batch(4, corpus, 0, 300 if corpus == "small" else 40)
    n = len(hb.meta)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    codec = hobj.Codec(0, 1024)
    d = hobj.DeviceBatch.from_host(hb, codec.torch_device)
    L = codec.lib
    total = int(ooff[-1])
    sizes = codec._empty(8 * (n + 1))
    st = codec._empty(4 * n)
    codec.encode_sizes(d, sizes, st)
    codec.scan(sizes, n, sizes)
    side = torch.cuda.Stream(codec.torch_device)
    for phase in (0, 16, 48):  # the arena's start against the 64-byte units
        buf = torch.full((total + 256,), 0xEE, dtype=torch.uint8, device=codec.torch_device)
        out = buf[phase:]
        ev = torch.cuda.Event()
        ev.record(torch.cuda.current_stream())
        side.wait_event(ev)
        P = _lib.ptr
        if units:
            _lib.check(L.honu_encode_records_units(codec.ctx, P(d.meta), P(d.var), P(d.acl), P(d.regions),
                                                   P(d.payload), P(d.payload_off), n, P(out), total,
                                                   P(sizes), P(st), codec.stream), "records_units")
            _lib.check(L.honu_encode_payloads_units(codec.ctx, P(d.payload), P(d.payload_off), n, P(out),
                                                    total, P(sizes), P(st), side.cuda_stream), "payloads_units")
        else:
            _lib.check(L.honu_encode_records(codec.ctx, P(d.meta), P(d.var), P(d.acl), P(d.regions),
                                             P(d.payload_off), n, P(out), total, P(sizes), P(st),
                                             codec.stream), "records")
            _lib.check(L.honu_encode_payloads(codec.ctx, P(d.payload), P(d.payload_off), n, P(out), total,
                                              P(sizes), P(st), side.cuda_stream), "payloads")
        torch.cuda.synchronize()
        assert np.array_equal(_host(st, 4 * n, np.int32), ost)
        assert np.array_equal(_host(sizes, 8 * (n + 1), np.uint64), ooff)
        h = out.cpu().numpy()
        for i in range(n):
            if ost[i] == 0:
                a, z = int(ooff[i]), int(ooff[i + 1])
                assert h[a:z].tobytes() == oout[a:z].tobytes(), (phase, i)
    codec.close()


def test_bench_serial_verify(oracle_lib):
    """--serial (one stream, one output slot): each chunk is checked before
    the next one reuses the slot, and the bench's own verification passes."""
    args = bench.parse_args(["--records", "3000", "--shape", "small", "--min-chunks", "3",
                             "--serial"])
    b = bench.Bench(args, 0, 0)
    assert len(b.slots) == 1 and len(b.chunks) == 3
    b.step()
    assert b.verify()
