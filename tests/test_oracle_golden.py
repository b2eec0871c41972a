"""Pin the CPU oracle against the reference's own known-answer tests.

Every test names the reference test it restates. These run on the CPU only;
the GPU path is then checked against this oracle (tests/test_gpu_parity.py).
"""
import numpy as np
import pytest

from fixtures import (load_json, load_object_fixture, metadata_from_json, py_marshal, py_uvarint,
                      py_varint)
from honu_amd.metadata import (HAS_META, REGIONS_INPLACE, Metadata, Scalar, Version, normalize,
                               pack_batch, unpack_row)


def marshal(oracle_lib, meta, data):
    hb = pack_batch([meta], [data])
    out, off, st = oracle_lib.marshal_batch(hb)
    return int(st[0]), bytes(out[int(off[0]):int(off[1])])


def decode(oracle_lib, obj: bytes, materialize=False):
    rec = np.frombuffer(obj, np.uint8) if obj else np.zeros(0, np.uint8)
    off = np.array([0, len(obj)], np.uint64)
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(rec, off, materialize)
    return meta[0], info[0], acl, reg, data, rec


# --------------------------------------------------------------------------
# object_test.go
# --------------------------------------------------------------------------
def test_object_fixture_1264_bytes(oracle_lib):
    """TestObject (object_test.go:23-45): the fixture object is 1264 bytes and round trips."""
    meta, data = load_object_fixture()
    assert len(data) == 860
    st, obj = marshal(oracle_lib, meta, data)
    assert st == 0
    assert len(obj) == 1264
    assert obj[0] == 1  # StorageVersion
    # independent restatement agrees byte for byte
    assert obj == py_marshal(meta, data)
    m, info, acl, reg, _, rec = decode(oracle_lib, obj)
    assert info["meta_status"] == 0 and info["data_status"] == 0
    assert unpack_row(m, rec, acl, reg) == normalize(meta)
    assert bytes(rec[int(info["data_off"]):int(info["data_off"]) + int(info["data_len"])]) == data
    assert not info["tombstone"]
    st, key = oracle_lib.key(m, 0)
    assert st == 0 and key[0] == 1 and key[1:17] == bytes(16)
    assert key[17:25] == (12).to_bytes(8, "big") and key[25:29] == (8).to_bytes(4, "big")


def test_object_fixture_byte_map(oracle_lib):
    """SURVEY App. C.1 byte map of the 1264-byte object."""
    meta, data = load_object_fixture()
    _, o = marshal(oracle_lib, meta, data)
    assert o[0:3] == b"\x01\xdc\x06"                                   # version, uv(860)
    assert o[3:863] == data
    assert o[863] == 1 and o[864:896] == bytes(32)                   # meta flag, oid, collection
    assert o[896:907] == bytes.fromhex("01080cdaadad0101030b00")     # Version 8.12 r=2840282 parent 3.11
    assert o[907:916] == bytes.fromhex("8098f6a6ab93dc8c30")         # zz(1732962599000000000)
    assert o[916:928] == b"\x01\x07Weather\x01\x03\x00"               # Schema 1.3.0
    assert o[928:945] == b"\x10application/json"                      # MIME
    assert o[977] == 23                                              # Permissions
    assert o[978] == 2 and o[979] == 1 and o[996] == 84 and o[997] == 1 and o[1014] == 76
    assert o[1015:1020] == b"\x01\xda\xad\xad\x01"                    # WriteRegions [2840282]
    assert o[1020] == 1 and o[1053] == 16                             # Publisher, IP frame len
    assert o[1054:1070] == bytes(10) + b"\xff\xff\x0a\x2a\x0a\x7b"
    assert o[1070:1080] == b"\x09PyHonu v1"
    assert o[1080:1082] == b"\x01\x1c"                                # Encryption, PKID len 28
    assert o[1239:1242] == b"\x05\x00\x04"                            # sealing, enc (typo -> 0), sig
    assert o[1242:1245] == b"\x01\x01\x12"                            # GZIP level 9
    assert o[1245] == 42                                             # Flags
    assert o[1246:1255] == o[907:916] == o[1255:1264]                 # Created, Modified


def test_tombstone(oracle_lib):
    """TestTombstone (object_test.go:47-58)."""
    meta, _ = load_object_fixture()
    st, obj = marshal(oracle_lib, meta, None)
    assert st == 0 and obj[1] == 0
    m, info, *_ = decode(oracle_lib, obj)
    assert info["tombstone"] == 1
    assert info["data_status"] == 0 and info["data_len"] == 0
    assert info["meta_status"] == 0


def test_nil_object(oracle_lib):
    """TestNil (object_test.go:60-71)."""
    m, info, *_ = decode(oracle_lib, b"")
    assert info["storage_version"] == 0
    assert info["meta_status"] == 1 and info["data_status"] == 1  # ErrBadVersion
    assert info["tombstone"] == 0


def test_malformed(oracle_lib):
    """TestMalformed (object_test.go:73-83) and the dataLength window rule."""
    for obj in (b"\x01", b"\x01\x00", b"\x01\x80\x01"):
        _, info, *_ = decode(oracle_lib, obj)
        assert info["meta_status"] == 2 and info["data_status"] == 2, obj  # ErrMalformed
        assert info["tombstone"] == 0
    # {01 00 00}: window o[1:2] = {00} -> tombstone, metadata nil flag -> &Metadata{}
    m, info, *_ = decode(oracle_lib, b"\x01\x00\x00")
    assert info["tombstone"] == 1 and info["meta_status"] == 0 and m["present"] == 0


def test_marshal_nil_metadata_panics(oracle_lib):
    st, obj = marshal(oracle_lib, None, b"abc")
    assert st == 8 and obj == b""


# --------------------------------------------------------------------------
# lani/encode_test.go and decode_test.go known answers
# --------------------------------------------------------------------------
@pytest.mark.parametrize("v,size", [(127, 1), (16383, 2), (2097151, 3), (268435455, 4),
                                    (4294967295, 5)])
def test_uvarint32_sizes(oracle_lib, v, size):
    """encode_test.go:270-293"""
    assert len(oracle_lib.put_uvarint(v)) == size


@pytest.mark.parametrize("v,size", [(127, 1), (16383, 2), (2097151, 3), (268435455, 4),
                                    (34359738367, 5), (4398046511103, 6), (562949953421311, 7),
                                    (72057594037927928, 8), (9223372036854775807, 9),
                                    (18446744073709551615, 10)])
def test_uvarint64_sizes(oracle_lib, v, size):
    """encode_test.go:295-322"""
    b = oracle_lib.put_uvarint(v)
    assert len(b) == size and b == py_uvarint(v)
    assert oracle_lib.uvarint(b) == (v, size)


@pytest.mark.parametrize("v,size", [(-9223372036854775807, 10), (-72057594037927928, 9),
                                    (-562949953421311, 8), (-4398046511103, 7), (-34359738367, 6),
                                    (-268435455, 5), (-2097151, 4), (-16383, 3), (-127, 2),
                                    (-32, 1), (0, 1), (32, 1), (127, 2), (16383, 3),
                                    (2097151, 4), (268435455, 5), (34359738367, 6),
                                    (4398046511103, 7), (562949953421311, 8),
                                    (72057594037927928, 9), (9223372036854775807, 10)])
def test_varint_sizes(oracle_lib, v, size):
    """encode_test.go:324-362"""
    b = oracle_lib.put_varint(v)
    assert len(b) == size and b == py_varint(v)
    assert oracle_lib.varint(b) == (v, size)


def test_uvarint_overflow_and_short(oracle_lib):
    """Go binary.Uvarint: overflow at the 10th byte > 1; 0 for a short buffer."""
    assert oracle_lib.uvarint(b"\xff" * 9 + b"\x02")[1] == -10
    assert oracle_lib.uvarint(b"\xff" * 9 + b"\x01") == (2**64 - 1, 10)
    assert oracle_lib.uvarint(b"\xff" * 11)[1] == -11
    assert oracle_lib.uvarint(b"\xff\xff")[1] == 0


def test_scalar_binary(oracle_lib):
    """lamport/scalar_test.go:74-79: Scalar{42,198} -> 2a c6 01."""
    assert oracle_lib.put_uvarint(42) + oracle_lib.put_uvarint(198) == b"\x2a\xc6\x01"
    m = Metadata(Version=Version(Scalar(42, 198)))
    _, o = marshal(oracle_lib, m, None)
    # 01 00 | 01 | oid cid | 01 <scalar> ...
    assert o[36:39] == b"\x2a\xc6\x01"


def test_frames_and_single_bytes(oracle_lib):
    """encode_test.go:95-154 frames (2+len for 145 B, 1+len under 128) and
    :236-268 single bytes; :389-395 zero time; :397-405 nil struct."""
    teapot = ("I'm a little teapot short and stout, here is my handle, here is my spout. "
              "When I'm feeling steamed I jump and shout; tip me over and pour me out!")
    assert len(teapot) == 145
    m = Metadata(MIME=teapot, Permissions=0x42, Flags=0x2A)
    _, o = marshal(oracle_lib, m, None)
    # 01 00 01 oid(16) cid(16) 00(version nil) 00(schema nil) = 37 bytes, then MIME
    assert o[37:39] == py_uvarint(145) and o[39:184] == teapot.encode()
    assert o[184 + 32] == 0x42                         # Permissions
    assert o[-3:] == b"\x2a\x00\x00"                    # Flags, zero Created/Modified
    assert o[35] == 0x00                                # nil Version = 1 byte
    m.MIME = "hello world"
    _, o = marshal(oracle_lib, m, None)
    assert o[37:49] == b"\x0bhello world"


def _tail_record(tail: bytes) -> bytes:
    """A tombstone record whose Metadata tail is `tail` (01 00 | tail)."""
    return b"\x01\x00" + tail


def _mime_record(frame: bytes) -> bytes:
    # meta flag, oid, cid, nil version, nil schema, then the MIME frame
    return _tail_record(b"\x01" + bytes(32) + b"\x00\x00" + frame)


@pytest.mark.parametrize("frame,status", [
    (b"", 3),                                   # decode_test.go:44-49 Decode(nil) -> EOF
    (b"\xff\xff", 5),                           # :51-56 ErrNoLength
    (b"\xff\x12\x23\x42\xf2\x21", 4),           # :58-63 ErrUnexpectedEOF
    (b"\x00", 3),                               # :65-70 nil frame ok; Owner then hits EOF
    (b"\x05abc", 4),
    (b"\xff" * 9 + b"\x7f", 5),                 # 10th byte > 1: Uvarint overflow
    (b"\xff" * 9 + b"\x01", 8),                 # rl >= 2^63: int(rl) < 0 -> makeslice panic
    (b"\xff" * 8 + b"\x7f", 8),                 # d.i + rl overflows int -> makeslice panic
    (b"\xff" * 7 + b"\x7f", 4),                 # rl < 2^63 - d.i, past the end
])
def test_decoder_frame_vectors(oracle_lib, frame, status):
    _, info, *_ = decode(oracle_lib, _mime_record(frame))
    assert info["meta_status"] == status


def test_bad_bool(oracle_lib):
    """decode_test.go:175-182: bool byte f2 -> ErrParseBoolean."""
    _, info, *_ = decode(oracle_lib, b"\x01\x00\xf2")
    assert info["meta_status"] == 6
    _, info, *_ = decode(oracle_lib, _tail_record(b"\x01" + bytes(32) + b"\x02"))
    assert info["meta_status"] == 6


def test_ulid_eof(oracle_lib):
    """DecodeULID (decode.go:209-221): EOF at the end, UnexpectedEOF mid-ULID."""
    _, info, *_ = decode(oracle_lib, _tail_record(b"\x01"))
    assert info["meta_status"] == 3
    _, info, *_ = decode(oracle_lib, _tail_record(b"\x01" + bytes(5)))
    assert info["meta_status"] == 4


def test_panics_on_huge_counts(oracle_lib):
    base = b"\x01" + bytes(32) + b"\x00\x00\x00" + bytes(32) + b"\x07"  # .. MIME nil, owner, group, perms
    # ACL count 2^45 + 1 -> make([]*AccessControl) panics; 2^45 decodes entries until EOF
    _, info, *_ = decode(oracle_lib, _tail_record(base + py_uvarint(2**45 + 1)))
    assert info["meta_status"] == 8
    _, info, *_ = decode(oracle_lib, _tail_record(base + py_uvarint(2**45)))
    assert info["meta_status"] == 3
    # Regions count 2^46 + 1 panics
    _, info, *_ = decode(oracle_lib, _tail_record(base + b"\x00" + py_uvarint(2**46 + 1)))
    assert info["meta_status"] == 8
    # payload length beyond the record: Data() and Metadata() both panic (slice out of range)
    _, info, *_ = decode(oracle_lib, b"\x01\x05\x00\x00")
    assert info["meta_status"] == 8 and info["data_status"] == 8
    # payload length >= 2^63: int(rl) < 0 -> ErrMalformed
    _, info, *_ = decode(oracle_lib, b"\x01" + b"\xff" * 9 + b"\x01\x00")
    assert info["meta_status"] == 2 and info["data_status"] == 2


def test_uint32_window(oracle_lib):
    """DecodeUint32 reads at most 5 bytes and truncates (decode.go:127-146)."""
    base = b"\x01" + bytes(32) + b"\x00\x00\x00" + bytes(32) + b"\x07\x00"  # ... perms, ACL 0
    tail = b"\x00\x00\x00\x00" + b"\x2a" + b"\x00\x00"
    ok = _tail_record(base + b"\x01\xff\xff\xff\xff\x7f" + tail)
    rec = np.frombuffer(ok, np.uint8)
    off = np.array([0, len(ok)], np.uint64)
    # the table form: the truncated value in the region table
    m, info, acl, reg, _, _ = oracle_lib.decode_batch(rec, off, False, regions_inplace=False)
    assert info[0]["meta_status"] == 0 and list(reg) == [0xFFFFFFFF]
    # in place (the default): the 5-byte uvarint in the record, read back the same way
    m, info, acl, reg, *_ = decode(oracle_lib, ok)
    assert info["meta_status"] == 0 and len(reg) == 0 and m["present"] & REGIONS_INPLACE
    assert int(m["regions_off"]) == len(ok) - len(tail) - 5
    assert unpack_row(m, rec).WriteRegions == [0xFFFFFFFF]
    bad = _tail_record(base + b"\x01\xff\xff\xff\xff\xff\x01" + tail)
    _, info, *_ = decode(oracle_lib, bad)
    assert info["meta_status"] == 7


# --------------------------------------------------------------------------
# metadata/*_test.go Size() fixtures (generic_test.go:33-44)
# --------------------------------------------------------------------------
def _row(meta):
    return pack_batch([meta], [None]).meta[0:1]


def test_size_bounds(oracle_lib):
    m = metadata_from_json(load_json("meta_metadata.json"))
    assert oracle_lib.size_bound(0, _row(m)) == 557         # metadata_test.go:28
    assert oracle_lib.size_bound(1, _row(m)) == 42          # version_test.go:25
    assert oracle_lib.size_bound(2, _row(m)) == 32          # schema_test.go:20
    assert oracle_lib.size_bound(3, _row(m)) == 17          # acls_test.go:17
    assert oracle_lib.size_bound(4, _row(m)) == 77          # provenance_test.go:22
    assert oracle_lib.size_bound(5, _row(m)) == 197         # encryption_test.go:24
    assert oracle_lib.size_bound(6, _row(m)) == 11          # compression_test.go:20
    z = Metadata()
    assert oracle_lib.size_bound(0, _row(z)) == 121         # metadataStaticSize
    zv = Metadata(Version=Version())
    assert oracle_lib.size_bound(1, _row(zv)) == 27         # version_test.go:14-20
    # every encoded Metadata fits its Size() bound (object.go:27 Grow)
    _, o = marshal(oracle_lib, m, None)
    assert len(o) - 3 <= 557


def test_metadata_fixture_roundtrip(oracle_lib):
    """generic_test.go:46-58 TestSerialization of metadata.json through an object."""
    m = metadata_from_json(load_json("meta_metadata.json"))
    st, o = marshal(oracle_lib, m, b"payload")
    assert st == 0 and o == py_marshal(m, b"payload")
    row, info, acl, reg, _, rec = decode(oracle_lib, o)
    assert unpack_row(row, rec, acl, reg) == normalize(m)
    assert int(row["present"]) & HAS_META
