"""Parity of the gfx950 path (through the C ABI) with the CPU oracle.

Bit-exact: encoded record bytes, offsets and statuses; decoded rows, record
info, ACL/region tables, materialised payloads and keys — on generated batches
of every benchmark shape, on the reference's fixture, on the reference's
decoder error vectors and on a fuzzed corpus of malformed records. Full-size
batches are checked through size-independent properties (payload digests
survive encode -> decode; a sample of records equals the oracle's bytes).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from corpora import malformed_corpus, mutant_corpus, random_metas  # noqa: E402
from fixtures import load_object_fixture, py_uvarint  # noqa: E402
from honu_amd import object as hobj  # noqa: E402
from honu_amd.metadata import META_DTYPE, normalize, pack_batch, unpack_row  # noqa: E402
from honu_amd.workload import gen_host_batch, gen_meta  # noqa: E402


@pytest.fixture(scope="module", params=[(6, 2, 1, 1), (5, 0, 1, 1), (6, 1, 1, 1), (6, 2, 0, 0), (5, 2, 0, 0),
                                        (6, 2, 1, 0), (5, 2, 0, 1)],
                ids=["fused", "split", "fork", "fused_table", "split_table", "fused_regtable",
                     "split_acltable"])
def codec(request):
    """Both metadata decodes of the product library with both list forms, and
    both placements of the encoder's ACL lists: the single-launch decode
    (fused.hip) at every batch size and the split decode kernels (windowed
    lane parse, group fill); ACL and region lists returned in place
    (acl_inplace 1 and regions_inplace 1, the defaults) or every list in the
    ACL and region tables ("_table"), or one list kind in its table
    ("_regtable": the round-5 default, "_acltable"). The default picks the
    decode by batch size; the bench pipeline and large-batch tests run it.
    The encoder is the lane encoder + group ACL lists (lane.hip, grp.hip):
    "split" runs the lists' kernel after the lane encoder (encode_fork 0),
    "fork" on the context's own stream beside it, placing the lists itself
    (encode_fork 1; the default 2 forks only when lane_blocks caps the
    encoder's grid, as the bench does for large records)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = hobj.Codec(0, 1 << 18)
    rv, fork, inplace, reg_inplace = request.param
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"record_variant", rv), "param")
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"encode_fork", fork), "param")
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"acl_inplace", inplace), "param")
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"regions_inplace", reg_inplace), "param")
    c.acl_inplace = bool(inplace)
    c.regions_inplace = bool(reg_inplace)
    yield c
    c.close()


def dev(a, codec):
    return hobj._dev_bytes(np.ascontiguousarray(a), codec.torch_device)


def gpu_marshal(codec, hb):
    r = codec.marshal(hobj.DeviceBatch.from_host(hb, codec.torch_device))
    torch.cuda.synchronize()
    return r.host()


def gpu_decode(codec, rec, off, materialize=False):
    n = len(off) - 1
    d = codec.decode(dev(rec if len(rec) else np.zeros(1, np.uint8), codec), dev(off, codec), n,
                     materialize=materialize, rec_bytes=int(off[-1]))
    torch.cuda.synchronize()
    return d.host()


def assert_decode_equal(oracle_lib, codec, rec, off, materialize=False):
    meta, info, acl, reg, data, tot = gpu_decode(codec, rec, off, materialize)
    ometa, oinfo, oacl, oreg, odata, otot = oracle_lib.decode_batch(
        rec, off, materialize, getattr(codec, "acl_inplace", True), getattr(codec, "regions_inplace", True))
    n = len(off) - 1
    assert np.array_equal(tot, otot)
    assert info.tobytes() == oinfo.tobytes()
    bad = [i for i in range(n) if meta[i].tobytes() != ometa[i].tobytes()]
    assert not bad, (bad[:5], meta[bad[0]], ometa[bad[0]])
    assert acl.tobytes() == oacl.tobytes()
    assert reg.tobytes() == oreg.tobytes()
    if materialize:
        for i in range(n):
            if oinfo[i]["data_status"] == 0 and oinfo[i]["data_len"]:
                o, ln = int(oinfo[i]["data_off"]), int(oinfo[i]["data_len"])
                assert data[o:o + ln].tobytes() == odata[o:o + ln].tobytes(), i
    return meta, info, acl, reg, data


# --------------------------------------------------------------------------
def test_fixture_object(codec, oracle_lib):
    """TestObject (object_test.go:23-45) through the GPU."""
    meta, data = load_object_fixture()
    obj = hobj.Marshal(meta, data)
    assert len(obj) == 1264
    out, off, st = oracle_lib.marshal_batch(pack_batch([meta], [data]))
    assert bytes(obj) == out.tobytes()
    assert obj.StorageVersion() == 1
    assert obj.Metadata() == normalize(meta)
    assert obj.Data() == data
    assert obj.Tombstone() is False
    key = obj.Key()
    assert key == bytes([1]) + bytes(16) + (12).to_bytes(8, "big") + (8).to_bytes(4, "big")
    tomb = hobj.Marshal(meta, None)
    assert tomb.Tombstone() is True and tomb.Data() is None


def test_nil_and_malformed_objects(codec):
    """TestNil / TestMalformed (object_test.go:60-83)."""
    with pytest.raises(hobj.ErrBadVersion):
        hobj.Object(b"").Metadata()
    with pytest.raises(hobj.ErrBadVersion):
        hobj.Object(b"").Data()
    assert hobj.Object(b"").Tombstone() is False
    with pytest.raises(hobj.ErrMalformed):
        hobj.Object(b"\x01").Metadata()
    with pytest.raises(hobj.ErrMalformed):
        hobj.Object(b"\x01").Data()
    with pytest.raises(hobj.GoPanic):
        hobj.Marshal(None, b"x")


@pytest.mark.parametrize("shape,n", [("small", 3000), ("medium", 500), ("large", 96),
                                     ("xlarge", 6), ("mixed", 800)])
def test_encode_parity(codec, oracle_lib, shape, n):
    hb = gen_host_batch(21, shape, 5000, n)
    out, off, st = gpu_marshal(codec, hb)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert np.array_equal(st, ost) and (st == 0).all()
    assert np.array_equal(off, ooff)
    assert out.tobytes() == oout.tobytes()


@pytest.mark.parametrize("materialize", [False, True])
@pytest.mark.parametrize("shape,n", [("small", 3000), ("large", 64), ("mixed", 600)])
def test_decode_parity(codec, oracle_lib, shape, n, materialize):
    hb = gen_host_batch(22, shape, 0, n)
    rec, off, st = oracle_lib.marshal_batch(hb)
    meta, info, acl, reg, data = assert_decode_equal(oracle_lib, codec, rec, off, materialize)
    assert (info["meta_status"] == 0).all()
    for i in range(0, n, max(1, n // 50)):
        src = normalize(unpack_row(hb.meta[i], hb.var, hb.acl, hb.regions))
        assert unpack_row(meta[i], rec, acl, reg) == src


def test_malformed_corpus_parity(codec, oracle_lib):
    objs = malformed_corpus(oracle_lib)
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    rec = np.frombuffer(b"".join(objs) + b"\0", np.uint8)[: int(off[-1])]
    meta, info, *_ = assert_decode_equal(oracle_lib, codec, rec, off, materialize=True)
    statuses = set(info["meta_status"].tolist())
    assert {0, 1, 2, 3, 4, 5, 6, 7, 8} <= statuses, statuses


def test_keys_parity(codec, oracle_lib):
    hb = gen_host_batch(23, "small", 0, 500)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    objs = [rec[int(off[i]):int(off[i + 1])].tobytes() for i in range(500)] + [b"\x01\x00\x00", b""]
    off2 = np.zeros(len(objs) + 1, np.uint64)
    off2[1:] = np.cumsum([len(o) for o in objs])
    rec2 = np.frombuffer(b"".join(objs), np.uint8)
    d = codec.decode(dev(rec2, codec), dev(off2, codec), len(objs), rec_bytes=int(off2[-1]))
    keys, kst = codec.keys(d)
    torch.cuda.synchronize()
    keys = hobj._to_host(keys, 29 * len(objs), np.uint8).reshape(-1, 29)
    kst = hobj._to_host(kst, 4 * len(objs), np.int32)
    meta, info, *_ = d.host()
    for i in range(len(objs)):
        st, k = oracle_lib.key(meta[i:i + 1], int(info[i]["meta_status"]))
        assert st == kst[i] and (st != 0 or k == keys[i].tobytes()), i
    assert kst[-2] == 8 and kst[-1] == 1  # nil Version panics; empty object: ErrBadVersion


def test_encode_input_errors(codec, oracle_lib):
    """Rows the encoder refuses (HONU_ERR_INPUT / PANIC), as the oracle: a
    span or list outside its arena, and a carried ACL list length
    (HONU_ACL_SIZED) outside [count, 18 count] (the size
    pass) or inside it but not the list's length (the list kernel, which reads
    every entry: the record keeps the range its carried length sized and
    reports HONU_ERR_INPUT; its bytes are unspecified). A row without the bit
    is sized from the table as before."""
    from honu_amd.metadata import ACL_SIZED
    meta, data = load_object_fixture()
    hb = pack_batch([meta, None, meta, meta, meta, meta, meta, meta],
                    [data, b"a", b"", data, data, b"zz", data, b""])
    assert int(hb.meta[0]["present"]) & ACL_SIZED and int(hb.meta[0]["acl_bytes"]) == 36
    hb.meta[2]["mime"]["off"] = 10**9          # span outside the var arena
    hb.meta[3]["acl_count"] = 10**6            # list outside the ACL table
    hb.meta[4]["acl_bytes"] = 19               # a lying length: 2 entries, not 1 present + 1 nil
    hb.meta[5]["acl_bytes"] = 37               # outside [2, 36]
    hb.meta[6]["present"] = int(hb.meta[6]["present"]) & ~ACL_SIZED  # no carried length: the table is read
    hb.meta[7]["acl_bytes"] = 1                # below the count
    out, off, st = gpu_marshal(codec, hb)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert st.tolist() == ost.tolist() == [0, 8, 10, 10, 10, 10, 0, 10]
    assert np.array_equal(off, ooff)
    lie = slice(int(off[4]), int(off[5]))
    assert lie.stop - lie.start == int(off[1]) - int(off[0]) - 17  # sized by 19 bytes, not 36
    g, o = out.copy(), oout.copy()
    g[lie] = 0
    o[lie] = 0
    assert g.tobytes() == o.tobytes()


def test_decode_capacity(codec, oracle_lib):
    hb = gen_host_batch(24, "small", 0, 64)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    n = 64
    d = codec.decode(dev(rec, codec), dev(off, codec), n, materialize=True, acl_cap=10,
                     regions_cap=10, data_cap=4096, rec_bytes=int(off[-1]))
    torch.cuda.synchronize()
    meta, info, acl, reg, data, tot = d.host()
    # the generator writes no nil ACL entry: in place, no list needs the table
    assert (int(tot[0]) == 0 if codec.acl_inplace else int(tot[0]) > 10) and int(tot[2]) > 4096
    assert int(tot[1]) == 0 if codec.regions_inplace else int(tot[1]) > 10
    # (lists in place take no table entry: no record fails the small caps)
    if codec.acl_inplace and codec.regions_inplace:
        assert (info["meta_status"] == 0).all()
    else:
        assert (info["meta_status"] == 9).any()
    assert (info["data_status"] == 9).any()
    ok = info["data_status"] == 0
    assert (info["data_off"][ok] + info["data_len"][ok] <= 4096).all()


def test_device_payload_and_digest(codec):
    meta, var, acl, reg, off = gen_meta(31, "mixed", 77, 300)
    hb = gen_host_batch(31, "mixed", 77, 300)
    d_off = dev(off, codec)
    d_pay = codec._empty(int(off[-1]))
    hobj._lib.check(codec.lib.honu_gen_payload(codec.ctx, 31, 77, 300, hobj._lib.ptr(d_off),
                                               hobj._lib.ptr(d_pay), codec.stream), "gen")
    dig = codec._empty(8 * 300)
    hobj._lib.check(codec.lib.honu_digest_records(codec.ctx, hobj._lib.ptr(d_pay),
                                                  hobj._lib.ptr(d_off), 0, 300,
                                                  hobj._lib.ptr(dig), codec.stream), "digest")
    torch.cuda.synchronize()
    pay = hobj._to_host(d_pay, int(off[-1]), np.uint8)
    assert pay.tobytes() == hb.payload[: int(off[-1])].tobytes()
    from honu_amd.workload import digest_host
    dg = hobj._to_host(dig, 8 * 300, np.uint64)
    for i in range(0, 300, 7):
        assert int(dg[i]) == digest_host(pay[int(off[i]):int(off[i + 1])].tobytes())


def test_full_size_property_large(codec, oracle_lib):
    """4096 Large records (~0.8 GB) generated on the device: payload digests
    survive encode -> materialising decode; sampled records equal the oracle's."""
    n = 4096
    meta, var, acl, reg, off = gen_meta(41, "large", 0, n)
    D = lambda a: dev(a, codec)  # noqa: E731
    db = hobj.DeviceBatch(D(meta), D(var), len(var), D(acl), len(acl), D(reg), len(reg),
                          codec._empty(int(off[-1])), D(off), n)
    L = hobj._lib
    L.check(codec.lib.honu_gen_payload(codec.ctx, 41, 0, n, L.ptr(db.payload_off),
                                       L.ptr(db.payload), codec.stream), "gen")
    enc = codec.marshal(db)
    dec = codec.decode(enc.out, enc.out_off, n, materialize=True)
    lens = torch.from_numpy(np.diff(off).astype(np.uint64).view(np.int64)).to(codec.torch_device)
    dsrc, ddst = codec._empty(8 * n), codec._empty(8 * n)
    L.check(codec.lib.honu_digest_records(codec.ctx, L.ptr(db.payload), L.ptr(db.payload_off), 0,
                                          n, L.ptr(dsrc), codec.stream), "digest")
    info_t = dec.info.view(torch.int64)[: 4 * n].view(n, 4)
    doff = info_t[:, 0].contiguous()
    dlen = info_t[:, 1].contiguous()
    L.check(codec.lib.honu_digest_records(codec.ctx, L.ptr(dec.data), L.ptr(doff), L.ptr(dlen), n,
                                          L.ptr(ddst), codec.stream), "digest")
    torch.cuda.synchronize()
    assert torch.equal(dlen.cpu(), lens.cpu())
    assert torch.equal(dsrc[: 8 * n].cpu(), ddst[: 8 * n].cpu())
    _, info, *_ = dec.host()
    assert (info["meta_status"] == 0).all() and (info["data_status"] == 0).all()
    sample = [0, 1, 17, 1023, 2048, n - 1]
    hb = gen_host_batch(41, "large", 0, n)
    oout, ooff, _ = oracle_lib.marshal_batch(hb)
    out, goff, _ = enc.host()
    assert np.array_equal(goff, ooff)
    for i in sample:
        assert out[int(goff[i]):int(goff[i + 1])].tobytes() == oout[int(ooff[i]):int(ooff[i + 1])].tobytes()


def _odd_metas(seed=11, n=48):
    """Records outside the generator's envelope: tails beyond one 2 KiB LDS
    window (long frames, hundreds of ACL entries), nil ACL entries, more than
    8 regions, multi-byte region varints, empty and nil lists."""
    from honu_amd.metadata import (AccessControl, Compression, Encryption, Metadata, Publisher,
                                   Scalar, SchemaVersion, Version)
    rng = np.random.default_rng(seed)
    metas, datas = [], []
    for i in range(n):
        kind = i % 6
        nacl = [0, 3, 130, 300, 17, 64][kind]
        acl = None if nacl == 0 else [
            None if (kind in (1, 3, 4) and j % 7 == 3) else
            AccessControl(rng.bytes(16), int(rng.integers(0, 256))) for j in range(nacl)]
        regs = [int(x) for x in rng.integers(0, [2**7, 2**14, 2**21, 2**32, 2**32, 2**10][kind],
                                              [0, 5, 9, 40, 8, 12][kind])]
        sig = rng.bytes([0, 32, 5000, 300, 2100, 1][kind])
        m = Metadata(
            ObjectID=rng.bytes(16), CollectionID=rng.bytes(16),
            Version=Version(Scalar(int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63))),
                            int(rng.integers(0, 2**32)), Scalar(7, 9) if kind % 2 else None,
                            bool(kind & 2), int(rng.integers(-2**62, 2**62))),
            Schema=SchemaVersion("S" * [0, 3, 700, 20, 5, 1][kind], 1, 2**20, 3) if kind else None,
            MIME="m" * [0, 10, 3000, 17, 40, 2][kind], Owner=rng.bytes(16), Group=rng.bytes(16),
            Permissions=int(rng.integers(0, 256)), ACL=acl,
            WriteRegions=regs if kind != 0 else None,
            Publisher=Publisher(rng.bytes(16), rng.bytes(16), rng.bytes(16),
                                "UA" * [0, 5, 900, 1, 3, 7][kind]) if kind != 5 else None,
            Encryption=Encryption("k" * 22, rng.bytes(32), rng.bytes(32), sig, 1, 2, 4)
            if kind != 1 else None,
            Compression=Compression(1, int(rng.integers(-5, 10))) if kind % 3 else None,
            Flags=int(rng.integers(0, 256)), Created=int(rng.integers(0, 2**62)),
            Modified=int(rng.integers(0, 2**62)))
        metas.append(m)
        datas.append(rng.bytes(int(rng.integers(0, 3000))) if i % 5 else None)
    return metas, datas


def test_long_tails_and_nil_entries_parity(codec, oracle_lib):
    metas, datas = _odd_metas()
    hb = pack_batch(metas, datas)
    out, off, st = gpu_marshal(codec, hb)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert np.array_equal(st, ost) and (st == 0).all()
    assert np.array_equal(off, ooff)
    assert out.tobytes() == oout.tobytes()
    tails = np.diff(off.astype(np.int64))
    assert tails.max() > 3 * 2048  # several stage windows
    for materialize in (False, True):
        meta, info, acl, reg, data = assert_decode_equal(oracle_lib, codec, oout, ooff, materialize)
        assert (info["meta_status"] == 0).all()
    for i in range(len(metas)):
        assert unpack_row(meta[i], oout, acl, reg) == normalize(metas[i]), i


@pytest.mark.parametrize("lens", ["tiny", "edges", "skew", "long", "mixed"])
@pytest.mark.parametrize("copy_variant", [0, -1, 1, 6, 11, 12, 13, 44, 46],
                         ids=["default", "steal_off", "unroll8", "sweep", "nt_load", "nt_store", "unaligned",
                              "no_tails", "short_tails"])
def test_copy_engine_parity(oracle_lib, copy_variant, lens):
    """The payload copy engine on awkward length mixes: payloads of 0-40 bytes
    (head/tail bytes only), lengths around multiples of 16, and a skewed mix of
    a few 300 KiB payloads among thousands of short ones (a wave range then
    spans a long segment and many short ones), segments of 16-100 KB ("long":
    the range tails taken from the counter) and a Mixed-like batch ("mixed":
    average >= 64 KB, so the short-segment class and the range tails at
    once). The default copy and, with the A/B build
    (HONU_LIB_PATH=honu_amd/libhonu_codec_ab.so; skipped on the product
    library), its measured variants: unroll 8, the sweep form, non-temporal
    loads / stores, unaligned loads, no range tails (44), the short class's
    run tails too (46); "steal_off": the
    product copy with the context param copy_steal 0. Encoded bytes and
    materialised payloads are bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rng = np.random.default_rng(5)
    n = 5000
    if lens == "tiny":
        ln = rng.integers(0, 41, n)
    elif lens == "edges":
        ln = (rng.integers(1, 200, n) * 16 + rng.integers(-2, 3, n)).clip(0)
    elif lens == "long":
        ln = rng.integers(16 << 10, 100 << 10, n)  # 58 KB on average
    elif lens == "mixed":
        ln = rng.integers(512, 4608, n)
        big = rng.random(n) < 0.3
        ln[big] = rng.integers(128 << 10, 400 << 10, int(big.sum()))  # 81 KB on average
    else:
        ln = rng.integers(0, 3000, n)
        ln[rng.integers(0, n, 12)] = 300 << 10
    base = gen_host_batch(9, "small", 0, n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(ln)
    pay = rng.integers(0, 256, int(off[-1]) + 1, dtype=np.uint8)
    from honu_amd.metadata import HostBatch
    hb = HostBatch(base.meta, base.var, base.acl, base.regions, pay, off)
    c = hobj.Codec(0, n)
    try:
        if copy_variant < 0:  # the range tails off (honu_codec.h "copy_steal")
            v = ctypes.c_int64(-1)
            hobj._lib.check(c.lib.honu_ctx_get_param(c.ctx, b"copy_steal", ctypes.byref(v)), "param")
            assert v.value == 1  # the default
            assert c.lib.honu_ctx_set_param(c.ctx, b"copy_steal", 2) != 0
            hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"copy_steal", 0), "param")
            hobj._lib.check(c.lib.honu_ctx_get_param(c.ctx, b"copy_steal", ctypes.byref(v)), "param")
            assert v.value == 0
        elif c.lib.honu_ctx_set_param(c.ctx, b"copy_variant", copy_variant) != 0:
            pytest.skip("A/B copy variant: not in the product library")
        out, goff, st = gpu_marshal(c, hb)
        oout, ooff, ost = oracle_lib.marshal_batch(hb)
        assert np.array_equal(st, ost) and np.array_equal(goff, ooff)
        assert out.tobytes() == oout.tobytes()
        assert_decode_equal(oracle_lib, c, oout, ooff, materialize=True)
    finally:
        c.close()


def test_payload_length_varint_boundaries(oracle_lib):
    """Payload lengths at every uvarint-length boundary of the header
    (object.go:35: 1 -> 5 bytes of length), up to a 256 MiB + 5 B payload:
    encoded bytes, offsets, the Data() descriptors and the materialised
    payloads are bit-exact; digests cover the big records."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    lens = [0, 1, 127, 128, 16383, 16384, (1 << 21) - 1, 1 << 21, (1 << 28) - 1, (1 << 28) + 5]
    n = len(lens)
    base = gen_host_batch(13, "small", 0, n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    rng = np.random.default_rng(13)
    pay = rng.integers(0, 256, int(off[-1]) + 1, dtype=np.uint8)
    from honu_amd.metadata import HostBatch
    hb = HostBatch(base.meta, base.var, base.acl, base.regions, pay, off)
    c = hobj.Codec(0, n)
    try:
        out, goff, st = gpu_marshal(c, hb)
        oout, ooff, ost = oracle_lib.marshal_batch(hb)
        assert np.array_equal(st, ost) and (st == 0).all() and np.array_equal(goff, ooff)
        assert out.tobytes() == oout.tobytes()
        for i, ln in enumerate(lens):  # header: 01 | uvarint(len)
            r = out[int(goff[i]):int(goff[i + 1])]
            assert r[0] == 1 and bytes(r[1:1 + py_uvarint_len(ln)]) == py_uvarint(ln)
        meta, info, acl, reg, data = assert_decode_equal(oracle_lib, c, oout, ooff, materialize=True)
        assert (info["meta_status"] == 0).all() and (info["data_status"] == 0).all()
        assert list(info["data_len"]) == lens
        assert list(info["tombstone"]) == [1] + [0] * (n - 1)
    finally:
        c.close()


def py_uvarint_len(x):
    return len(py_uvarint(x))


def test_decode_data_without_metadata(oracle_lib):
    """honu_decode_data: Object.Data() materialised without Metadata(): the
    record info's data fields, StorageVersion and Tombstone equal the oracle's
    full decode (meta_status is HONU_UNPARSED), data offsets equal the ones
    the materialising decode assigns, payload bytes are bit-exact — on a batch
    with corrupted and truncated records; then a data arena too small for the
    batch gives HONU_ERR_CAPACITY exactly for the payloads past it."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    hb = gen_host_batch(17, "mixed", 0, 700)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    objs = [rec[int(off[i]):int(off[i + 1])].tobytes() for i in range(700)]
    rng = np.random.default_rng(17)
    for i in range(0, 700, 23):
        b = bytearray(objs[i])
        b[int(rng.integers(0, min(len(b), 6)))] ^= 0xFF  # header bytes: version / length
        objs[i] = bytes(b[: int(rng.integers(0, len(b) + 1))])
    objs += [b"", b"\x01", b"\x01\x00", b"\x01\x00\x00", b"\x02\x00\x00"]
    n = len(objs)
    roff = np.zeros(n + 1, np.uint64)
    roff[1:] = np.cumsum([len(o) for o in objs])
    arena = np.frombuffer(b"".join(objs), np.uint8)
    _, oinfo, _, _, odata, otot = oracle_lib.decode_batch(arena, roff, True)
    c = hobj.Codec(0, n)
    try:
        L = hobj._lib
        d_rec, d_off = dev(arena, c), dev(roff, c)
        cap = int(otot[2]) + 64
        d_info, d_data, d_tot = c._empty(32 * n), c._empty(cap), c._empty(8)
        L.check(c.lib.honu_decode_data(c.ctx, L.ptr(d_rec), L.ptr(d_off), n, L.ptr(d_info),
                                       L.ptr(d_data), cap, L.ptr(d_tot), c.stream), "decode_data")
        torch.cuda.synchronize()
        info = hobj._to_host(d_info, 32 * n, np.uint8).view(oinfo.dtype)
        data = hobj._to_host(d_data, cap, np.uint8)
        assert int(hobj._to_host(d_tot, 8, np.uint64)[0]) == int(otot[2])
        for f in ("data_off", "data_len", "data_status", "storage_version", "tombstone"):
            assert np.array_equal(info[f], oinfo[f]), f
        assert (info["meta_status"] == 11).all()
        assert len(set(oinfo["data_status"].tolist())) >= 3
        for i in range(n):
            if oinfo[i]["data_status"] == 0 and oinfo[i]["data_len"]:
                o, ln = int(oinfo[i]["data_off"]), int(oinfo[i]["data_len"])
                assert data[o:o + ln].tobytes() == odata[o:o + ln].tobytes(), i
        # a smaller arena: exactly the payloads ending past it fail with CAPACITY
        small = int(otot[2]) // 2
        L.check(c.lib.honu_decode_data(c.ctx, L.ptr(d_rec), L.ptr(d_off), n, L.ptr(d_info),
                                       L.ptr(d_data), small, 0, c.stream), "decode_data")
        torch.cuda.synchronize()
        info2 = hobj._to_host(d_info, 32 * n, np.uint8).view(oinfo.dtype)
        ok = oinfo["data_status"] == 0
        past = ok & (oinfo["data_off"] + oinfo["data_len"] > small) & (oinfo["data_len"] > 0)
        assert (info2["data_status"][past] == 9).all() and past.any()
        keep = ok & ~past
        assert np.array_equal(info2["data_off"][keep], oinfo["data_off"][keep])
    finally:
        c.close()


def test_extreme_values_parity(codec, oracle_lib):
    from fixtures import extreme_metas
    metas, datas = extreme_metas()
    hb = pack_batch(metas, datas)
    out, off, st = gpu_marshal(codec, hb)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert np.array_equal(st, ost) and (st == 0).all()
    assert np.array_equal(off, ooff)
    assert out.tobytes() == oout.tobytes()
    for materialize in (False, True):
        meta, info, acl, reg, data = assert_decode_equal(oracle_lib, codec, oout, ooff, materialize)
        assert (info["meta_status"] == 0).all()
    for i in range(len(metas)):
        assert unpack_row(meta[i], oout, acl, reg) == normalize(metas[i]), i


def test_decode_parse_full_waves(codec, oracle_lib):
    """A batch of 2^17 + 77 records (many grid-stride rounds of the window
    parse and group fill, a partial last wave): bit-exact rows, info and tables."""
    n = (1 << 17) + 77
    hb = gen_host_batch(23, "small", 0, n)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    meta, info, acl, reg, data, tot = gpu_decode(codec, rec, off)
    ometa, oinfo, oacl, oreg, odata, otot = oracle_lib.decode_batch(rec, off, False, codec.acl_inplace,
                                                                    codec.regions_inplace)
    assert np.array_equal(tot, otot) and info.tobytes() == oinfo.tobytes()
    assert meta.tobytes() == ometa.tobytes()
    assert acl.tobytes() == oacl.tobytes() and reg.tobytes() == oreg.tobytes()


@pytest.mark.parametrize("rv", [0, 6], ids=["split", "fused"])
def test_hip_graph_capture_replay(oracle_lib, rv):
    """The ABI's calls neither allocate nor synchronise (include/honu_codec.h),
    so a whole marshal + decode + keys sequence is captured into one hipGraph
    (torch.cuda.CUDAGraph over the capturing stream) and replayed: outputs are
    recomputed from the device inputs at every replay, bit-exact. With the
    single-launch decode the look-back's epoch lives in device memory, so
    replays of the same launch arguments stay correct."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = hobj._lib
    n = 1500
    hb = gen_host_batch(37, "mixed", 0, n)
    oout, ooff, _ = oracle_lib.marshal_batch(hb)
    ometa, oinfo, oacl, oreg, odata, otot = oracle_lib.decode_batch(oout, ooff, True)
    c = hobj.Codec(0, n)
    L.check(c.lib.honu_ctx_set_param(c.ctx, b"record_variant", rv), "param")
    try:
        db = hobj.DeviceBatch.from_host(hb, c.torch_device)
        total = int(ooff[-1])
        out_off, status, out = c._empty(8 * (n + 1)), c._empty(4 * n), c._empty(total)
        meta, info, totals = c._empty(352 * n), c._empty(32 * n), c._empty(32)
        acl_cap, reg_cap, data_cap = total, total, total + 16 * n
        acl, reg, data = c._empty(20 * acl_cap), c._empty(4 * reg_cap), c._empty(data_cap)
        keys, kst = c._empty(29 * n), c._empty(4 * n)

        def seq():
            c.encode_sizes(db, out_off, status)
            c.scan(out_off, n, out_off)
            c.encode(db, out, total, out_off, status)
            L.check(c.lib.honu_decode_batch(c.ctx, L.ptr(out), L.ptr(out_off), n, L.ptr(meta),
                                            L.ptr(info), L.ptr(acl), acl_cap, L.ptr(reg), reg_cap,
                                            L.ptr(data), data_cap, L.ptr(totals), c.stream), "decode")
            L.check(c.lib.honu_decode_keys(c.ctx, L.ptr(meta), L.ptr(info), n, L.ptr(keys),
                                           L.ptr(kst), c.stream), "keys")

        seq()  # warm up outside the capture (module loading)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            seq()
        for t in (out, meta, info, acl, reg, data, keys, totals):
            t.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert hobj._to_host(out, total, np.uint8).tobytes() == oout.tobytes()
        assert hobj._to_host(meta, 352 * n, np.uint8).tobytes() == ometa.tobytes()
        assert hobj._to_host(info, 32 * n, np.uint8).tobytes() == oinfo.tobytes()
        assert np.array_equal(hobj._to_host(totals, 24, np.uint64), otot)
        na, nr, nd = (int(x) for x in otot)
        assert hobj._to_host(acl, 20 * na, np.uint8).tobytes() == oacl.tobytes()
        assert hobj._to_host(reg, 4 * nr, np.uint8).tobytes() == oreg.tobytes()
        assert hobj._to_host(data, nd, np.uint8).tobytes() == odata[:nd].tobytes()
        # the replay reads the inputs again: a changed payload byte shows up
        p = int(hb.payload_off[7])
        db.payload[p:p + 1].bitwise_xor_(torch.tensor([0xFF], dtype=torch.uint8,
                                                      device=c.torch_device))
        g.replay()
        torch.cuda.synchronize()
        got = hobj._to_host(out, total, np.uint8)
        diff = np.nonzero(got != oout)[0]
        assert len(diff) == 1 and got[diff[0]] == oout[diff[0]] ^ 0xFF
    finally:
        c.close()


def test_decode_fuzz_mutations(codec, oracle_lib):
    """20,000 mutants of valid records (byte flips, varint-byte rewrites to
    0x80/0xff/0x00/0x01, insertions, deletions and truncations inside the
    Metadata tail), decoded bit-exact against the oracle: rows, record info
    (every status), ACL/region tables and materialised payloads."""
    arena, o = mutant_corpus(oracle_lib)
    meta, info, acl, reg, data = assert_decode_equal(oracle_lib, codec, arena, o, materialize=True)
    assert len(set(info["meta_status"].tolist())) >= 5


def test_encode_fuzz_random_metadata(codec, oracle_lib):
    """3,000 random Metadata (every sub-struct present or nil, frames of 0-400
    bytes around the 1/2-byte length boundary, nil ACL entries, region and
    integer values of every varint width, negative times): encoded bytes
    bit-exact vs the oracle, and decoded back to the same fields."""
    metas, datas = random_metas(3000, 77)
    hb = pack_batch(metas, datas)
    out, off, st = gpu_marshal(codec, hb)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert np.array_equal(st, ost) and (st == 0).all()
    assert np.array_equal(off, ooff) and out.tobytes() == oout.tobytes()
    meta, info, acl, reg, data = assert_decode_equal(oracle_lib, codec, oout, ooff, materialize=True)
    assert (info["meta_status"] == 0).all()
    for i in range(0, 3000, 7):
        assert unpack_row(meta[i], oout, acl, reg) == normalize(metas[i]), i


def test_concurrent_contexts_on_streams(oracle_lib):
    """Two contexts on two streams, their batches in flight together (the ABI:
    calls on distinct streams are concurrent, one context per stream): both
    encodes and decodes bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = hobj._lib
    runs = []
    for seed, shape in ((61, "small"), (62, "mixed")):
        n = 1200
        hb = gen_host_batch(seed, shape, 0, n)
        oout, ooff, _ = oracle_lib.marshal_batch(hb)
        c = hobj.Codec(0, n)
        db = hobj.DeviceBatch.from_host(hb, c.torch_device)
        total = int(ooff[-1])
        bufs = dict(out_off=c._empty(8 * (n + 1)), status=c._empty(4 * n), out=c._empty(total),
                    meta=c._empty(352 * n), info=c._empty(32 * n), acl=c._empty(20 * total),
                    reg=c._empty(4 * total), totals=c._empty(32))
        runs.append((c, db, n, total, bufs, oout, ooff, torch.cuda.Stream()))
    torch.cuda.synchronize()
    for c, db, n, total, b, _, _, s in runs:  # issue both before waiting for either
        with torch.cuda.stream(s):
            c.encode_sizes(db, b["out_off"], b["status"])
            c.scan(b["out_off"], n, b["out_off"])
            c.encode(db, b["out"], total, b["out_off"], b["status"])
            L.check(c.lib.honu_decode_batch(c.ctx, L.ptr(b["out"]), L.ptr(b["out_off"]), n,
                                            L.ptr(b["meta"]), L.ptr(b["info"]), L.ptr(b["acl"]),
                                            total, L.ptr(b["reg"]), total, 0, 0, L.ptr(b["totals"]),
                                            c.stream), "decode")
    torch.cuda.synchronize()
    for c, db, n, total, b, oout, ooff, _ in runs:
        assert hobj._to_host(b["out"], total, np.uint8).tobytes() == oout.tobytes()
        ometa, oinfo, *_ = oracle_lib.decode_batch(oout, ooff, False)
        assert hobj._to_host(b["meta"], 352 * n, np.uint8).tobytes() == ometa.tobytes()
        assert hobj._to_host(b["info"], 32 * n, np.uint8).tobytes() == oinfo.tobytes()
        c.close()


def test_encode_writer_drain_bounds(codec, oracle_lib):
    """The lane encoder's LDS ring (lane.h LaneWriterT) holds 8 chunks between
    drains; its drain placement assumes at most ~112 bytes per lane in between.
    Records at that bound: every varint at its widest (10-byte VIDs and times,
    5-byte PIDs, schema numbers and region ids), frames 63/64/65/128 bytes long
    around the 64-byte run batches, up to 40 regions, empty frames right after
    full batches, and payload lengths 0..15 so the tail starts at every phase
    of the 16-byte grid. Encoded bytes bit-exact vs the oracle."""
    from honu_amd.metadata import (AccessControl, Compression, Encryption, Metadata, Publisher,
                                   Scalar, SchemaVersion, Version)
    rng = np.random.default_rng(41)
    M32, M64, MIN64 = 2**32 - 1, 2**64 - 1, -2**63
    LENS = [0, 1, 63, 64, 65, 128]
    metas, datas = [], []
    for i in range(6 * 16 * 3):
        ln = LENS[i % 6]
        metas.append(Metadata(
            ObjectID=rng.bytes(16), CollectionID=rng.bytes(16),
            Version=Version(Scalar(M32, M64), M32, Scalar(M32, M64), True, MIN64),
            Schema=SchemaVersion("s" * LENS[(i + 1) % 6], M32, M32, M32),
            MIME="m" * LENS[(i + 2) % 6], Owner=rng.bytes(16), Group=rng.bytes(16), Permissions=255,
            ACL=[AccessControl(rng.bytes(16), 7) for _ in range(i % 3)] or None,
            WriteRegions=[M32] * ((i * 7) % 41) or None,
            Publisher=Publisher(rng.bytes(16), rng.bytes(16), rng.bytes(ln) or None, "u" * LENS[(i + 3) % 6]),
            Encryption=Encryption("k" * LENS[(i + 4) % 6], rng.bytes(LENS[(i + 5) % 6]) or None,
                                  None, rng.bytes(ln) or None, 5, 1, 4),
            Compression=Compression(1, MIN64), Flags=255, Created=MIN64, Modified=2**63 - 1))
        datas.append(rng.bytes((i // 6) % 16) or None)
    hb = pack_batch(metas, datas)
    out, off, st = gpu_marshal(codec, hb)
    oout, ooff, ost = oracle_lib.marshal_batch(hb)
    assert np.array_equal(st, ost) and (st == 0).all()
    assert np.array_equal(off, ooff) and out.tobytes() == oout.tobytes()


def test_hbm_probe_modes(codec):
    """honu_hbm_probe (bench.py's achievable-rate denominator): the three copy
    forms move every byte (sizes not a multiple of a wave's chunk), the write
    form fills the buffer, bad arguments are refused."""
    L = hobj._lib
    for nbytes in (16, 4096 + 48, (3 << 20) + 16 * 77):
        a = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=codec.torch_device)
        for mode in (2, 3, 4):
            for bpc in (0, 1, 4):
                b = torch.zeros_like(a)
                L.check(codec.lib.honu_hbm_probe(codec.ctx, mode, L.ptr(a), L.ptr(b), nbytes, bpc,
                                                 codec.stream), "probe")
                torch.cuda.synchronize()
                assert torch.equal(a, b), (nbytes, mode, bpc)
        b = torch.zeros_like(a)
        L.check(codec.lib.honu_hbm_probe(codec.ctx, 1, None, L.ptr(b), nbytes, 2, codec.stream), "probe")
        L.check(codec.lib.honu_hbm_probe(codec.ctx, 0, L.ptr(a), None, nbytes, 2, codec.stream), "probe")
        torch.cuda.synchronize()
        assert int((b.view(torch.int32)[2::4] == 1).sum()) == nbytes // 16
    assert codec.lib.honu_hbm_probe(codec.ctx, 7, None, None, 16, 1, codec.stream) != 0


def test_environment_is_ignored(oracle_lib, monkeypatch):
    """The product library takes its configuration from honu_ctx_set_param
    only: HONU_* variables set in the process before the
    context is created change neither its parameters nor its outputs (the ACL
    lists still come back in place with HONU_ACL_INPLACE=0). The A/B build
    reads them (HONU_LIB_PATH set: skipped)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import os
    if os.environ.get("HONU_LIB_PATH"):
        pytest.skip("A/B build")
    env = {"HONU_ACL_INPLACE": "0", "HONU_RECORD_VARIANT": "5", "HONU_LANE_BLOCKS": "3",
           "HONU_COPY_BLOCKS": "1", "HONU_ENCODE_FORK": "0", "HONU_GUARD_BLOCKS": "7",
           "HONU_INLINE_RECOVERY": "1", "HONU_RECORD_BLOCKS": "1"}
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    c = hobj.Codec(0, 4096)
    try:
        got = {}
        for name in ("acl_inplace", "record_variant", "lane_blocks", "encode_fork", "guard_blocks",
                     "inline_recovery"):
            v = ctypes.c_int64(-1)
            hobj._lib.check(c.lib.honu_ctx_get_param(c.ctx, name.encode(), ctypes.byref(v)), "param")
            got[name] = v.value
        assert got == {"acl_inplace": 1, "record_variant": 0, "lane_blocks": 0, "encode_fork": 2,
                       "guard_blocks": 0, "inline_recovery": 0}
        hb = gen_host_batch(71, "small", 0, 300)
        rec, off, _ = oracle_lib.marshal_batch(hb)
        meta, info, acl, reg, data, tot = gpu_decode(c, rec, off)
        ometa, oinfo, oacl, oreg, _, otot = oracle_lib.decode_batch(rec, off, False)
        assert meta.tobytes() == ometa.tobytes() and np.array_equal(tot, otot)
        assert (meta["present"] & (1 << 8)).any()  # HONU_ACL_INPLACE
    finally:
        c.close()


def test_copy_counter_lines_concurrent(oracle_lib):
    """The range tails' counters (copy.hip): payload copies of one
    context issued back to back on two streams at once, each into its own
    records arena, with payloads averaging >= 16 KB so every launch takes
    tails from a counter. Every copy call counts on a line of its own, so no
    launch skips a tail another took: every arena bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = hobj._lib
    n = 1500
    rng = np.random.default_rng(19)
    base = gen_host_batch(19, "small", 0, n)
    off = np.zeros(n + 1, np.uint64)
    off[1:] = np.cumsum(rng.integers(16 << 10, 60 << 10, n))
    pay = rng.integers(0, 256, int(off[-1]) + 1, dtype=np.uint8)
    from honu_amd.metadata import HostBatch
    hb = HostBatch(base.meta, base.var, base.acl, base.regions, pay, off)
    oout, ooff, _ = oracle_lib.marshal_batch(hb)
    total = int(ooff[-1])
    c = hobj.Codec(0, n)
    try:
        db = hobj.DeviceBatch.from_host(hb, c.torch_device)
        out_off, status = c._empty(8 * (n + 1)), c._empty(4 * n)
        c.encode_sizes(db, out_off, status)
        c.scan(out_off, n, out_off)
        outs = [c._empty(total) for _ in range(8)]
        for o in outs:  # headers and tails (plain form), then only the copies race
            L.check(c.lib.honu_encode_records(c.ctx, L.ptr(db.meta), L.ptr(db.var), L.ptr(db.acl),
                                              L.ptr(db.regions), L.ptr(db.payload_off), n, L.ptr(o),
                                              total, L.ptr(out_off), L.ptr(status), c.stream), "records")
        torch.cuda.synchronize()
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]
        for rep in range(3):
            for k, o in enumerate(outs):
                s = streams[k % 2]
                L.check(c.lib.honu_encode_payloads(c.ctx, L.ptr(db.payload), L.ptr(db.payload_off), n,
                                                   L.ptr(o), total, L.ptr(out_off), L.ptr(status),
                                                   s.cuda_stream), "payloads")
        torch.cuda.synchronize()
        for o in outs:
            assert hobj._to_host(o, total, np.uint8).tobytes() == oout.tobytes()
    finally:
        c.close()


def test_encode_forms_not_mixed_and_null_payload(oracle_lib):
    """The payload-unit pair and the plain pair complete different bytes
    (honu_codec.h): a payload call of the other form than the context's last
    records call is refused (HONU_E_ARG) instead of leaving bytes unwritten
    with every status OK. honu_encode of a batch whose payloads are all empty
    accepts a null payload arena."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    L = hobj._lib
    n = 200
    hb = gen_host_batch(29, "small", 0, n)
    oout, ooff, _ = oracle_lib.marshal_batch(hb)
    total = int(ooff[-1])
    c = hobj.Codec(0, n)
    try:
        db = hobj.DeviceBatch.from_host(hb, c.torch_device)
        out_off, status, out = c._empty(8 * (n + 1)), c._empty(4 * n), c._empty(total)
        c.encode_sizes(db, out_off, status)
        c.scan(out_off, n, out_off)
        args = (c.ctx, L.ptr(db.meta), L.ptr(db.var), L.ptr(db.acl), L.ptr(db.regions))
        L.check(c.lib.honu_encode_records(*args, L.ptr(db.payload_off), n, L.ptr(out), total,
                                          L.ptr(out_off), L.ptr(status), c.stream), "records")
        assert c.lib.honu_encode_payloads_units(c.ctx, L.ptr(db.payload), L.ptr(db.payload_off), n,
                                                L.ptr(out), total, L.ptr(out_off), L.ptr(status),
                                                c.stream) == -1
        L.check(c.lib.honu_encode_payloads(c.ctx, L.ptr(db.payload), L.ptr(db.payload_off), n, L.ptr(out),
                                           total, L.ptr(out_off), L.ptr(status), c.stream), "payloads")
        torch.cuda.synchronize()
        assert hobj._to_host(out, total, np.uint8).tobytes() == oout.tobytes()
        L.check(c.lib.honu_encode_records_units(*args, L.ptr(db.payload), L.ptr(db.payload_off), n,
                                                L.ptr(out), total, L.ptr(out_off), L.ptr(status),
                                                c.stream), "records_units")
        assert c.lib.honu_encode_payloads(c.ctx, L.ptr(db.payload), L.ptr(db.payload_off), n, L.ptr(out),
                                          total, L.ptr(out_off), L.ptr(status), c.stream) == -1
        # every payload empty (tombstones): a null payload arena is accepted
        from honu_amd.metadata import HostBatch
        eoff = np.zeros(n + 1, np.uint64)
        eb = HostBatch(hb.meta, hb.var, hb.acl, hb.regions, np.zeros(1, np.uint8), eoff)
        eout, eooff, _ = oracle_lib.marshal_batch(eb)
        etotal = int(eooff[-1])
        edb = hobj.DeviceBatch.from_host(eb, c.torch_device)
        eo, est, eoo = c._empty(etotal), c._empty(4 * n), c._empty(8 * (n + 1))
        L.check(c.lib.honu_marshal_batch(c.ctx, L.ptr(edb.meta), L.ptr(edb.var), edb.var_len,
                                         L.ptr(edb.acl), edb.acl_len, L.ptr(edb.regions), edb.regions_len,
                                         None, L.ptr(edb.payload_off), n, L.ptr(eo), etotal, L.ptr(eoo),
                                         L.ptr(est), c.stream), "marshal null payload")
        torch.cuda.synchronize()
        assert (hobj._to_host(est, 4 * n, np.int32) == 0).all()
        assert hobj._to_host(eo, etotal, np.uint8).tobytes() == eout.tobytes()
    finally:
        c.close()
