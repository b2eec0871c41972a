"""System objects (object/system.go:10-45 with metadata.Collection, Index,
Field): the oracle against the reference's known answers (CPU), and the GPU
kernels against the oracle (-m gpu)."""
import numpy as np
import pytest

from fixtures import (collection_from_json, field_from_json, index_from_json, load_json,
                      py_marshal_system)
from honu_amd.metadata import AccessControl, Compression, Encryption, Publisher, Scalar, \
    SchemaVersion, Version
from honu_amd.system import (COLLECTION_DTYPE, INDEX_DTYPE, Collection, Field, Index,
                             normalize_collection, pack_system_batch, unpack_collection)


def random_collection(rng, big=False):
    """A Collection with every optional part present or nil at random."""
    def ulid():
        return rng.bytes(16)

    def maybe(p=0.8):
        return rng.random() < p

    def text(lo, hi):
        return "".join(chr(int(c)) for c in rng.integers(32, 127, int(rng.integers(lo, hi))))

    def field():
        return Field(text(0, 12), int(rng.integers(0, 9)), ulid())

    sz = 40 if big else 1
    c = Collection(ID=ulid(), Name=text(0, 20 * sz), Owner=ulid(), Group=ulid(),
                   Permissions=int(rng.integers(0, 256)), Flags=int(rng.integers(0, 256)),
                   Created=int(rng.integers(-2**62, 2**62)), Modified=int(rng.integers(0, 2**62)))
    if maybe():
        c.Version = Version(Scalar(int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63))),
                            int(rng.integers(0, 2**32)),
                            Scalar(int(rng.integers(0, 2**32)), int(rng.integers(0, 2**63)))
                            if maybe() else None, bool(maybe(0.3)), int(rng.integers(-2**62, 2**62)))
    if maybe():
        c.ACL = [AccessControl(ulid(), int(rng.integers(0, 256))) if maybe(0.85) else None
                 for _ in range(int(rng.integers(0, 20 * sz)))]
    if maybe():
        c.WriteRegions = [int(x) for x in rng.integers(0, 2**32, int(rng.integers(0, 12)))]
    if maybe():
        c.Publisher = Publisher(ulid(), ulid(), rng.bytes(int(rng.choice([0, 4, 16]))),
                                text(0, 30))
    if maybe():
        c.Schema = SchemaVersion(text(0, 16), int(rng.integers(0, 2**32)),
                                 int(rng.integers(0, 300)), int(rng.integers(0, 5)))
    if maybe():
        c.Encryption = Encryption(text(0, 22), rng.bytes(int(rng.integers(0, 40))),
                                  rng.bytes(int(rng.integers(0, 40))),
                                  rng.bytes(int(rng.integers(0, 300 * sz))),
                                  int(rng.integers(0, 6)), int(rng.integers(0, 6)),
                                  int(rng.integers(0, 6)))
    if maybe():
        c.Compression = Compression(int(rng.integers(0, 5)), int(rng.integers(-10, 10)))
    if maybe():
        c.Indexes = [Index(ulid(), text(0, 16), int(rng.integers(0, 8)),
                           field() if maybe() else None, field() if maybe() else None)
                     if maybe(0.85) else None for _ in range(int(rng.integers(0, 6 * sz)))]
    return c


def random_batch(seed, n, big_every=0):
    rng = np.random.default_rng(seed)
    cols = [None if i % 17 == 5 else random_collection(rng, big_every and i % big_every == 0)
            for i in range(n)]
    return cols


# --------------------------------------------------------------------------
# known answers (CPU, oracle)
# --------------------------------------------------------------------------
def test_size_known_answers(oracle_lib):
    """TestCollection / TestIndex / TestField static and fixture sizes
    (collection_test.go:12-29, index_test.go:12-25, field_test.go:12-22)."""
    sb = pack_system_batch([Collection()])
    assert oracle_lib.collection_size(sb.rows[0], sb.acl, sb.index) == 115
    fx = collection_from_json(load_json("meta_collection.json"))
    sb = pack_system_batch([fx])
    assert oracle_lib.collection_size(sb.rows[0], sb.acl, sb.index) == 637
    empty = np.zeros(1, INDEX_DTYPE)
    empty["present"] = 1
    assert oracle_lib.index_size(empty[0]) == 29
    ix = pack_system_batch([Collection(Indexes=[index_from_json(load_json("meta_index.json"))])])
    assert oracle_lib.index_size(ix.index[0]) == 104
    assert oracle_lib.field_size(0) == 27
    assert oracle_lib.field_size(len(field_from_json(load_json("meta_field.json")).Name)) == 36


@pytest.mark.parametrize("name", ["object_collection.json", "meta_collection.json"])
def test_system_serialize_round_trip(oracle_lib, name):
    """TestSystemSerialize (system_test.go:12-35): MarshalSystem then
    UnmarshalSystem gives back the collection; bytes match the independent
    Python restatement."""
    c = collection_from_json(load_json(name))
    sb = pack_system_batch([c])
    out, off, st = oracle_lib.system_marshal_batch(sb)
    assert st[0] == 0
    assert out.tobytes() == py_marshal_system(c)
    rows, st, acl, reg, idx, tot = oracle_lib.system_decode_batch(out, off)
    assert st[0] == 0
    assert unpack_collection(rows[0], out, acl, reg, idx) == normalize_collection(c)


def test_oracle_matches_python_restatement(oracle_lib):
    cols = random_batch(3, 300, big_every=25)
    out, off, st = oracle_lib.system_marshal_batch(pack_system_batch(cols))
    assert (st == 0).all()
    for i, c in enumerate(cols):
        assert out[int(off[i]):int(off[i + 1])].tobytes() == py_marshal_system(c), i
    rows, st, acl, reg, idx, tot = oracle_lib.system_decode_batch(out, off)
    assert (st == 0).all()
    for i, c in enumerate(cols):
        assert unpack_collection(rows[i], out, acl, reg, idx) == normalize_collection(c), i


def test_decode_error_vectors(oracle_lib):
    """UnmarshalSystem on short and malformed objects (system.go:40-44)."""
    cases = [
        (b"", 8),                      # obj[1:-1]: slice bounds panic
        (b"\x01", 8),                  # obj[1:0]
        (b"\x01\x00", 3),              # empty window: DecodeBool -> io.EOF
        (b"\x01\x00\x00", 0),          # nil collection
        (b"\x07\x00\x00", 0),          # the version byte is not checked
        (b"\x01\x02\x00", 6),          # bad struct flag
        (b"\x01\x01" + bytes(8) + b"\x00", 4),  # ID needs 16 bytes
        (b"\x01\x01" + bytes(16) + b"\xff" * 10 + b"\x00", 5),  # name length overflows
    ]
    recs = [c for c, _ in cases]
    off = np.zeros(len(recs) + 1, np.uint64)
    off[1:] = np.cumsum([len(r) for r in recs])
    rec = np.frombuffer(b"".join(recs) + b"\0", np.uint8)[: int(off[-1])]
    rows, st, *_ = oracle_lib.system_decode_batch(rec, off)
    assert st.tolist() == [s for _, s in cases]
    assert not rows["present"].any()


def test_headless_collection_decode(oracle_lib):
    """lani.Unmarshal(raw, &Collection{}) as store.go:367 calls it on a raw
    bbolt value (Collection.Decode from byte 0, collection.go:240-356):
    lani.Marshal(c)'s bytes -- the system object without its version byte,
    struct flag and trailing nil-metadata flag (system.go:17-28) -- decode to
    c; a whole system object is decoded with its first two bytes read as the
    start of the ID; short values give the DecodeULID errors
    (decode.go:209-221)."""
    cols = random_batch(11, 120, big_every=30)
    cols = [c for c in cols if c is not None] + [
        collection_from_json(load_json("object_collection.json"))]
    out, off, st = oracle_lib.system_marshal_batch(pack_system_batch(cols))
    bodies = [out[int(off[i]) + 2:int(off[i + 1]) - 1].tobytes() for i in range(len(cols))]
    boff = np.zeros(len(bodies) + 1, np.uint64)
    boff[1:] = np.cumsum([len(b) for b in bodies])
    brec = np.frombuffer(b"".join(bodies), np.uint8)
    rows, st, acl, reg, idx, _ = oracle_lib.system_decode_batch(brec, boff, headless=True)
    assert (st == 0).all()
    for i, c in enumerate(cols):
        assert unpack_collection(rows[i], brec, acl, reg, idx) == normalize_collection(c), i
    raw = out[int(off[-2]):int(off[-1])].tobytes()  # the fixture's system object, as stored
    cases = [b"", b"\x01\x00\x00", bytes(15), raw]
    coff = np.zeros(len(cases) + 1, np.uint64)
    coff[1:] = np.cumsum([len(b) for b in cases])
    crec = np.frombuffer(b"".join(cases), np.uint8)
    rows, st, *_ = oracle_lib.system_decode_batch(crec, coff, headless=True)
    assert st[:3].tolist() == [3, 4, 4]  # io.EOF, io.ErrUnexpectedEOF x2
    # the stored fixture: ID = raw[0:16] (01 01 + the real ID's first 14
    # bytes); the Name length is the uvarint of the real ID's last two bytes
    # (8c 4a -> 9484), longer than what is left: io.ErrUnexpectedEOF
    # (decode.go:46-48)
    assert raw[:2] == b"\x01\x01" and raw[16:18] == b"\x8c\x4a"
    assert st[3] == 4


# --------------------------------------------------------------------------
# GPU vs oracle
# --------------------------------------------------------------------------
def _corpus(oracle_lib, seed=4):
    rng = np.random.default_rng(seed)
    cols = random_batch(seed, 64, big_every=9)
    out, off, _ = oracle_lib.system_marshal_batch(pack_system_batch(cols))
    objs = [out[int(off[i]):int(off[i + 1])].tobytes() for i in range(len(cols))]
    bad = [b"", b"\x01", b"\x01\x00", b"\x01\x02\x00"]
    for v in objs[:6]:
        bad += [v[:k] for k in range(0, len(v), max(1, len(v) // 60))]
    for v in objs:
        for _ in range(12):
            b = bytearray(v)
            for _k in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            bad.append(bytes(b))
    bad += [rng.integers(0, 256, int(rng.integers(0, 80)), dtype=np.uint8).tobytes()
            for _ in range(100)]
    return objs + bad


@pytest.mark.gpu
def test_gpu_system_encode_parity(oracle_lib):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.system import marshal_system_batch
    cols = random_batch(5, 500, big_every=20) + [
        collection_from_json(load_json("object_collection.json")),
        collection_from_json(load_json("meta_collection.json"))]
    out, off, st = marshal_system_batch(cols)
    oout, ooff, ost = oracle_lib.system_marshal_batch(pack_system_batch(cols))
    assert np.array_equal(st, ost) and (st == 0).all()
    assert np.array_equal(off, ooff)
    assert out.tobytes() == oout.tobytes()


@pytest.mark.gpu
def test_gpu_system_decode_parity(oracle_lib):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.system import decode_system_batch
    objs = _corpus(oracle_lib)
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    rec = np.frombuffer(b"".join(objs) + b"\0", np.uint8)[: int(off[-1])]
    rows, st, acl, reg, idx, tot = decode_system_batch(rec, off)
    orows, ost, oacl, oreg, oidx, otot = oracle_lib.system_decode_batch(rec, off)
    assert np.array_equal(tot, otot)
    assert st.tolist() == ost.tolist()
    assert rows.tobytes() == orows.tobytes()
    assert acl.tobytes() == oacl.tobytes()
    assert reg.tobytes() == oreg.tobytes()
    assert idx.tobytes() == oidx.tobytes()
    assert {0, 3, 4, 5, 6, 7, 8} <= set(st.tolist())


@pytest.mark.gpu
def test_gpu_headless_collection_decode_parity(oracle_lib):
    """honu_collection_decode_batch (lani.Unmarshal(raw, &Collection{}),
    store.go:367) against the oracle on whole system objects, their
    lani.Marshal bodies and the malformed corpus."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.system import decode_system_batch
    objs = _corpus(oracle_lib, seed=6)
    objs += [o[2:-1] for o in objs[:64] if len(o) > 3]
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    rec = np.frombuffer(b"".join(objs) + b"\0", np.uint8)[: int(off[-1])]
    rows, st, acl, reg, idx, tot = decode_system_batch(rec, off, headless=True)
    orows, ost, oacl, oreg, oidx, otot = oracle_lib.system_decode_batch(rec, off, headless=True)
    assert np.array_equal(tot, otot)
    assert st.tolist() == ost.tolist()
    assert rows.tobytes() == orows.tobytes()
    assert acl.tobytes() == oacl.tobytes()
    assert reg.tobytes() == oreg.tobytes()
    assert idx.tobytes() == oidx.tobytes()
    assert 0 in set(st.tolist()) and len(set(st.tolist())) >= 4


@pytest.mark.gpu
def test_gpu_marshal_unmarshal_system_api():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd import object as hobj
    from honu_amd.system import MarshalSystem, UnmarshalSystem
    c = collection_from_json(load_json("object_collection.json"))
    obj = MarshalSystem(c)
    assert obj == py_marshal_system(c)
    assert UnmarshalSystem(obj) == normalize_collection(c)
    assert MarshalSystem(None) == b"\x01\x00\x00"
    assert UnmarshalSystem(b"\x01\x00\x00") == Collection()
    with pytest.raises(hobj.GoPanic):
        UnmarshalSystem(b"\x01")
    with pytest.raises(hobj.EOFError_):
        UnmarshalSystem(b"\x01\x00")
    from honu_amd.system import Unmarshal
    assert Unmarshal(obj[2:-1], Collection()) == normalize_collection(c)
    into = Collection(Name="stale")  # decoded in place, as lani.Unmarshal(raw, &c)
    assert Unmarshal(obj[2:-1], into) is into and into == normalize_collection(c)
    with pytest.raises(hobj.GoPanic):  # store.go:155: a nil *Collection
        Unmarshal(obj, None)
    with pytest.raises(hobj.ErrUnexpectedEOF):
        Unmarshal(b"\x01\x00\x00", Collection())
