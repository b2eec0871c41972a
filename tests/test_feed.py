"""The read feed: pinned double-buffered batches decoded on the GPU, checked
batch by batch against the oracle (-m gpu); on a CPU-only host it refuses to
start (no CPU fallback)."""
import numpy as np
import pytest

from honu_amd import _lib
from honu_amd.workload import gen_host_batch


def _records(oracle_lib, n=3000, seed=31):
    hb = gen_host_batch(seed, "small", 0, n)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    objs = [rec[int(off[i]):int(off[i + 1])].tobytes() for i in range(n)]
    rng = np.random.default_rng(seed)
    for i in range(0, n, 37):  # malformed records in the stream
        b = bytearray(objs[i])
        b[int(rng.integers(0, len(b)))] ^= 0xFF
        objs[i] = bytes(b[: int(rng.integers(0, len(b) + 1))])
    return objs


def test_feed_refuses_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from honu_amd.feed import RecordFeed
    with pytest.raises(_lib.HonuError):
        RecordFeed(0, 16, 1 << 16)


def _raw_copy(v):
    """Byte-exact copy (np.array(copy=True) skips the padding of structured
    dtypes, and rows are compared bytewise)."""
    return np.frombuffer(np.ascontiguousarray(v).view(np.uint8).tobytes(), v.dtype).reshape(v.shape)


def _copy(res):
    """Results are views of pinned buffers reused by the next fill: copy."""
    return {k: (_raw_copy(v) if isinstance(v, np.ndarray) else v) for k, v in vars(res).items()}


def _drive(feed, objs):
    """The cursor loop: append until full, submit, collect the previous batch
    (its slot is the one the next appends go to)."""
    prev, cur, out = None, [], []
    for o in objs:
        if feed.append(o) == 9:
            t = feed.submit()
            if prev is not None:
                out.append((prev[1], _copy(feed.wait(prev[0]))))
            prev, cur = (t, cur), []
            assert feed.append(o) == 0
        cur.append(o)
    t = feed.submit()
    if prev is not None:
        out.append((prev[1], _copy(feed.wait(prev[0]))))
    out.append((cur, _copy(feed.wait(t))))
    return out


@pytest.mark.gpu
def test_feed_matches_oracle(oracle_lib):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.feed import RecordFeed
    objs = _records(oracle_lib)
    feed = RecordFeed(0, batch_records=700, batch_bytes=1 << 20)
    nb = 0
    for chunk, r in _drive(feed, objs):
        n = len(chunk)
        assert len(r["rec_off"]) == n + 1
        off = np.zeros(n + 1, np.uint64)
        off[1:] = np.cumsum([len(o) for o in chunk])
        assert np.array_equal(r["rec_off"], off)
        assert r["records"].tobytes() == b"".join(chunk)
        meta, info, acl, reg, _, tot = oracle_lib.decode_batch(r["records"], off)
        assert r["info"].tobytes() == info.tobytes()
        assert r["meta"].tobytes() == meta.tobytes()
        assert r["acl"].tobytes() == acl.tobytes()
        assert r["regions"].tobytes() == reg.tobytes()
        for i in range(n):
            st, key = oracle_lib.key(meta[i], int(info[i]["meta_status"]))
            assert int(r["key_status"][i]) == st
            assert r["keys"][i].tobytes() == key
        nb += 1
    assert nb >= 4
    feed.close()


@pytest.mark.gpu
def test_feed_headers_only(oracle_lib):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.feed import RecordFeed
    objs = _records(oracle_lib, n=1500, seed=32) + [b"", b"\x01", b"\x01\x00", b"\x02\x00\x00"]
    feed = RecordFeed(0, batch_records=400, batch_bytes=1 << 20, headers_only=True)
    for chunk, r in _drive(feed, objs):
        off = r["rec_off"]
        _, info, *_ = oracle_lib.decode_batch(r["records"], off)
        for f in ("data_off", "data_len", "data_status", "storage_version", "tombstone"):
            assert np.array_equal(r["info"][f], info[f]), f
        assert (r["info"]["meta_status"] == 11).all()
        assert r["meta"] is None
    feed.close()


# --------------------------------------------------------------------------
# Write feed (honu_put_feed_*): object.Marshal batched for the Put path
# --------------------------------------------------------------------------
def test_put_feed_refuses_without_gpu():
    torch = pytest.importorskip("torch")
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from honu_amd.feed import PutFeed
    with pytest.raises(_lib.HonuError):
        PutFeed(0, 16, 1 << 16)


def _drive_put(feed, hb):
    """append_batch until full, submit, collect the previous batch."""
    first, prev, out = 0, None, []
    while first < len(hb):
        st, got = feed.append_batch(hb, first)
        assert got > 0 or st == 0
        span = (first, first + got)
        first += got
        t = feed.submit()
        if prev is not None:
            r = feed.wait(prev[0])
            out.append((prev[1], r.objects()))
        prev = (t, span)
    r = feed.wait(prev[0])
    out.append((prev[1], r.objects()))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("shape", ["small", "mixed"])
def test_put_feed_matches_oracle(oracle_lib, shape):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.feed import PutFeed
    n = 2500
    hb = gen_host_batch(51, shape, 0, n)
    rec, off, st = oracle_lib.marshal_batch(hb)
    feed = PutFeed(0, batch_records=600, batch_bytes=6 << 20)
    got = {}
    batches = _drive_put(feed, hb)
    for (a, b), objs in batches:
        assert len(objs) == b - a
        for i, o in zip(range(a, b), objs):
            got[i] = o
    assert len(batches) >= 4 and len(got) == n
    for i in range(n):
        assert got[i] == rec[int(off[i]):int(off[i + 1])].tobytes(), i
    feed.close()


@pytest.mark.gpu
def test_put_feed_single_records_and_errors(oracle_lib):
    """append() of Metadata mirrors: records outside the generator's envelope
    (long tails, nil ACL entries), nil payloads (tombstones), Marshal(nil, …)
    (HONU_ERR_PANIC), a span outside its arena (HONU_ERR_INPUT, nothing
    appended) and a record larger than the batch (HONU_ERR_CAPACITY)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_gpu_parity import _odd_metas
    from honu_amd.feed import PutFeed
    from honu_amd.metadata import pack_batch
    metas, datas = _odd_metas(seed=12, n=36)
    metas.append(None)
    datas.append(b"x")
    feed = PutFeed(0, batch_records=64, batch_bytes=4 << 20)
    for m, d in zip(metas, datas):
        assert feed.append(m, d) == 0
    assert feed.pending == len(metas)
    hb = pack_batch(metas[:-1], datas[:-1])
    rec, off, _ = oracle_lib.marshal_batch(hb)
    r = feed.wait(feed.submit())
    objs = r.objects()
    for i in range(len(metas) - 1):
        assert objs[i] == rec[int(off[i]):int(off[i + 1])].tobytes(), i
    assert objs[-1] == 8  # HONU_ERR_PANIC: Marshal(nil, data)
    # a span outside the var arena: refused, nothing appended
    one = pack_batch([metas[1]], [b"abc"])
    row = one.meta.copy()
    row["mime"]["off"] = len(one.var) + 5
    row["mime"]["len"] = 3
    st = feed.lib.honu_put_feed_append(feed.feed, row.ctypes.data, one.var.ctypes.data,
                                       len(one.var), one.acl.ctypes.data, len(one.acl),
                                       one.regions.ctypes.data, len(one.regions), b"abc", 3)
    assert st == 10 and feed.pending == 0
    # larger than a whole batch
    assert feed.append(metas[1], b"\0" * (5 << 20)) == 9
    # submit without wait on both slots -> the third submit is refused
    assert feed.append(metas[2], b"y") == 0
    t1 = feed.submit()
    assert feed.append(metas[2], b"z") == 0
    t2 = feed.submit()
    with pytest.raises(_lib.HonuError):
        feed.submit()
    for t, d in ((t1, b"y"), (t2, b"z")):
        o, oo, _ = oracle_lib.marshal_batch(pack_batch([metas[2]], [d]))
        assert feed.wait(t).objects() == [o[: int(oo[1])].tobytes()]
    feed.close()


@pytest.mark.gpu
def test_feed_append_batch(oracle_lib):
    """honu_feed_append_batch (a cursor page at a time) gives the same batches
    as per-record appends."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.feed import RecordFeed
    objs = _records(oracle_lib, n=1200, seed=33)
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    arena = np.frombuffer(b"".join(objs) or b"\0", np.uint8)
    feed = RecordFeed(0, batch_records=500, batch_bytes=1 << 20)
    first = 0
    while first < len(objs):
        st, got = feed.append_batch(arena, off, first)
        assert got > 0 and (st == 9 or first + got == len(objs))
        r = _copy(feed.wait(feed.submit()))
        chunk = objs[first:first + got]
        assert r["records"].tobytes() == b"".join(chunk)
        meta, info, *_ = oracle_lib.decode_batch(r["records"], r["rec_off"])
        assert r["info"].tobytes() == info.tobytes() and r["meta"].tobytes() == meta.tobytes()
        first += got
    feed.close()


@pytest.mark.gpu
def test_feed_acl_table_overflow(oracle_lib):
    """A nil-entry flood (1 byte per ACL entry) needs more table entries than
    the feed holds (batch_bytes/8 + 1024): the flooded record gets
    HONU_ERR_CAPACITY, acl_n never exceeds the table and acl_needed reports
    what the batch needed; the records before it decode as the oracle says."""
    from honu_amd.feed import RecordFeed
    from honu_amd.metadata import ACL_INPLACE, Metadata, pack_batch
    flood = Metadata(ACL=[None] * 60000)
    hb = gen_host_batch(5, "small", 0, 4)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    objs = [rec[int(off[i]):int(off[i + 1])].tobytes() for i in range(4)]
    frec, foff, fst = oracle_lib.marshal_batch(pack_batch([flood], [b"x" * 10]))
    assert fst[0] == 0
    objs.append(frec.tobytes())
    feed = RecordFeed(0, 64, 1 << 17)
    for o in objs:
        assert feed.append(o) == 0
    res = feed.wait(feed.submit())
    cap = (1 << 17) // 8 + 1024
    # the generated records' lists have every entry present: returned in
    # place (HONU_ACL_INPLACE), they take no table entries
    good = 0
    assert all(int(res.meta[i]["present"]) & ACL_INPLACE for i in range(4) if res.meta[i]["acl_count"])
    assert res.acl_needed == good + 60000
    assert len(res.acl) == min(res.acl_needed, cap) <= cap
    assert res.info["meta_status"][4] == 9  # HONU_ERR_CAPACITY
    assert (res.info["meta_status"][:4] == 0).all()
    ometa, oinfo, oacl, oreg, _, _ = oracle_lib.decode_batch(rec, off)
    assert res.acl[:good].tobytes() == oacl.tobytes()
    assert res.meta[:4].tobytes() == ometa.tobytes()
    feed.close()
