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
    return {k: (None if v is None else _raw_copy(v)) for k, v in vars(res).items()}


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
