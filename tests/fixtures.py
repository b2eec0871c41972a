"""Load the reference's JSON fixtures the way Go's encoding/json does for the
metadata types, and a second, independent pure-Python restatement of the
lani/object encoder used to cross-check the C oracle (test infrastructure).

The fixture files themselves are committed under tests/golden/ (copied data,
not source). JSON semantics reproduced here:
  - ULIDs: Crockford base32 text (go.rtnl.ai/ulid UnmarshalText)
  - lamport.Scalar: "PID.VID" (lamport/scalar.go:153-171; VID parsed as
    ParseUint(..., 10, 32) like the reference)
  - region.Region: name, upper-cased, '-' -> '_' (region/region.go:52-59)
  - time.Time: RFC 3339 -> UnixNano
  - []byte: standard base64; net.IP: ParseIP -> 16-byte form for IPv4
  - enums by name (encryption.go:127-145, compression.go:69-85)
  - Encryption.EncryptionAlgorithm's tag is the typo "encryption_algoirthm"
    (encryption.go:32): the fixtures' "encryption_algorithm" key does not
    match it, so the field stays PLAINTEXT (0).
"""
from __future__ import annotations

import base64
import datetime as _dt
import json
import os
import numpy as np

from honu_amd.metadata import (AccessControl, Compression, Encryption, Metadata, Publisher, Scalar,
                               SchemaVersion, Version)

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Only the region names the fixtures use (ids from pkg/region/values.go).
REGION_IDS = {
    "GCP_US_CENTRAL_1A": 2840280,
    "GCP_US_CENTRAL_1C": 2840282,
    "GCP_US_EAST_1B": 2840291,
    "GCP_US_EAST_1C": 2840292,
    "GCP_US_WEST_1A": 2840330,
    "GCP_US_WEST_1B": 2840331,
}
ENC_ALGS = {"PLAINTEXT": 0, "AES256_GCM": 1, "AES192_GCM": 2, "AES128_GCM": 3, "HMAC_SHA256": 4,
            "RSA_OEAP_SHA512": 5}
CMP_ALGS = {"NONE": 0, "GZIP": 1, "COMPRESS": 2, "DEFLATE": 3, "BROTLI": 4}

_CROCKFORD = "0123456789ABCDEFGHJKMNPQRSTVWXYZ"


def ulid_parse(s: str) -> bytes:
    s = s.upper()
    if len(s) != 26:
        raise ValueError("bad ULID length")
    v = 0
    for ch in s:
        v = (v << 5) | _CROCKFORD.index(ch)
    if v >> 128:
        raise ValueError("ULID overflow")
    return v.to_bytes(16, "big")


def scalar_parse(s: str) -> Scalar:
    pid, vid = s.split(".")
    return Scalar(int(pid), int(vid))


def region_parse(s: str) -> int:
    return REGION_IDS[s.strip().upper().replace("-", "_")]


def time_parse(s: str) -> int:
    t = _dt.datetime.strptime(s, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=_dt.timezone.utc)
    return int(t.timestamp()) * 1_000_000_000


def ip_parse(s: str) -> bytes:
    parts = [int(x) for x in s.split(".")]
    return bytes(10) + b"\xff\xff" + bytes(parts)


def _get(d: dict, key: str):
    """encoding/json matches object keys to field tags case-insensitively."""
    for k, v in d.items():
        if k.lower() == key.lower():
            return v
    return None


def _common_from_json(m, d: dict):
    """Fields Metadata and Collection share, decoded as encoding/json does."""
    v = _get(d, "version")
    if v is not None:
        m.Version = Version(scalar_parse(_get(v, "scalar")), region_parse(_get(v, "region")),
                            scalar_parse(_get(v, "parent")) if _get(v, "parent") else None,
                            bool(_get(v, "tombstone") or False),
                            time_parse(_get(v, "created")) if _get(v, "created") else 0)
    s = _get(d, "schema")
    if s is not None:
        m.Schema = SchemaVersion(_get(s, "name") or "", _get(s, "major") or 0,
                                 _get(s, "minor") or 0, _get(s, "patch") or 0)
    m.Owner = ulid_parse(_get(d, "owner"))
    m.Group = ulid_parse(_get(d, "group"))
    m.Permissions = _get(d, "permissions") or 0
    if _get(d, "acl") is not None:
        m.ACL = [AccessControl(ulid_parse(_get(a, "client_id")), _get(a, "permissions") or 0)
                 for a in _get(d, "acl")]
    if _get(d, "write_regions") is not None:
        m.WriteRegions = [region_parse(r) for r in _get(d, "write_regions")]
    p = _get(d, "publisher")
    if p is not None:
        m.Publisher = Publisher(ulid_parse(_get(p, "publisher_id")), ulid_parse(_get(p, "client_id")),
                                ip_parse(_get(p, "ipaddr")), _get(p, "user_agent") or "")
    e = _get(d, "encryption")
    if e is not None:
        b64 = lambda k: base64.b64decode(_get(e, k)) if _get(e, k) else None  # noqa: E731
        m.Encryption = Encryption(
            _get(e, "public_key_id") or "", b64("encryption_key"), b64("hmac_secret"),
            b64("signature"), ENC_ALGS[_get(e, "sealing_algorithm") or "PLAINTEXT"],
            ENC_ALGS[_get(e, "encryption_algoirthm") or "PLAINTEXT"],  # tag typo, encryption.go:32
            ENC_ALGS[_get(e, "signature_algorithm") or "PLAINTEXT"])
    c = _get(d, "compression")
    if c is not None:
        m.Compression = Compression(CMP_ALGS[_get(c, "algorithm") or "NONE"], _get(c, "level") or 0)
    m.Flags = _get(d, "flags") or 0
    m.Created = time_parse(_get(d, "created")) if _get(d, "created") else 0
    m.Modified = time_parse(_get(d, "modified")) if _get(d, "modified") else 0


def field_from_json(d: dict):
    """metadata.Field (field.go:12-16); FieldType by name, upper-cased (:99-107)."""
    from honu_amd.system import FIELD_TYPES, Field
    t = (_get(d, "type") or "STRING").strip().upper()
    return Field(_get(d, "name") or "", FIELD_TYPES.index(t),
                 ulid_parse(_get(d, "collection")) if _get(d, "collection") else bytes(16))


def index_from_json(d: dict):
    """metadata.Index (index.go:16-22); IndexType by name, upper-cased (:122-130)."""
    from honu_amd.system import INDEX_TYPES, Index
    t = (_get(d, "type") or "UNKNOWN").strip().upper()
    return Index(ulid_parse(_get(d, "id")), _get(d, "name") or "", INDEX_TYPES.index(t),
                 field_from_json(_get(d, "field")) if _get(d, "field") is not None else None,
                 field_from_json(_get(d, "ref")) if _get(d, "ref") is not None else None)


def collection_from_json(d: dict):
    """metadata.Collection (collection.go:16-33) as encoding/json fills it."""
    from honu_amd.system import Collection
    c = Collection()
    c.ID = ulid_parse(_get(d, "id"))
    c.Name = _get(d, "name") or ""
    _common_from_json(c, d)
    if _get(d, "indexes") is not None:
        c.Indexes = [index_from_json(x) for x in _get(d, "indexes")]
    return c


def metadata_from_json(d: dict) -> Metadata:
    m = Metadata()
    if _get(d, "oid"):
        m.ObjectID = ulid_parse(_get(d, "oid"))
    if _get(d, "collection"):
        m.CollectionID = ulid_parse(_get(d, "collection"))
    m.MIME = _get(d, "mime") or ""
    _common_from_json(m, d)
    return m


def load_json(name: str) -> dict:
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def load_object_fixture():
    """loadObjectFixture (object_test.go:85-93): metadata.json + data.json bytes."""
    meta = metadata_from_json(load_json("object_metadata.json"))
    with open(os.path.join(GOLDEN, "object_data.json"), "rb") as f:
        data = f.read()
    return meta, data


# --------------------------------------------------------------------------
# independent pure-Python restatement of the encoder (cross-check only)
# --------------------------------------------------------------------------
def py_uvarint(x: int) -> bytes:
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


def py_varint(x: int) -> bytes:
    ux = (x << 1) & 0xFFFFFFFFFFFFFFFF
    if x < 0:
        ux ^= 0xFFFFFFFFFFFFFFFF
    return py_uvarint(ux)


def _frame(b) -> bytes:
    b = b or b""
    if isinstance(b, str):
        b = b.encode("utf-8", "surrogateescape")
    return py_uvarint(len(b)) + b


def py_marshal(m: Metadata, data: bytes) -> bytes:
    """object.Marshal restated directly from Appendix A of SURVEY.md."""
    o = bytearray(b"\x01") + _frame(data) + b"\x01"
    o += m.ObjectID + m.CollectionID
    if m.Version is None:
        o += b"\x00"
    else:
        v = m.Version
        o += b"\x01" + py_uvarint(v.Scalar.PID) + py_uvarint(v.Scalar.VID) + py_uvarint(v.Region)
        o += (b"\x01" + py_uvarint(v.Parent.PID) + py_uvarint(v.Parent.VID)) if v.Parent else b"\x00"
        o += (b"\x01" if v.Tombstone else b"\x00") + py_varint(v.Created)
    if m.Schema is None:
        o += b"\x00"
    else:
        s = m.Schema
        o += b"\x01" + _frame(s.Name) + py_uvarint(s.Major) + py_uvarint(s.Minor) + py_uvarint(s.Patch)
    o += _frame(m.MIME) + m.Owner + m.Group + bytes([m.Permissions])
    acl = m.ACL or []
    o += py_uvarint(len(acl))
    for a in acl:
        o += b"\x00" if a is None else b"\x01" + a.ClientID + bytes([a.Permissions])
    reg = m.WriteRegions or []
    o += py_uvarint(len(reg)) + b"".join(py_uvarint(r) for r in reg)
    if m.Publisher is None:
        o += b"\x00"
    else:
        p = m.Publisher
        o += b"\x01" + p.PublisherID + p.ClientID + _frame(p.IPAddress) + _frame(p.UserAgent)
    if m.Encryption is None:
        o += b"\x00"
    else:
        e = m.Encryption
        o += (b"\x01" + _frame(e.PublicKeyID) + _frame(e.EncryptionKey) + _frame(e.HMACSecret) +
              _frame(e.Signature) + bytes([e.SealingAlgorithm, e.EncryptionAlgorithm,
                                           e.SignatureAlgorithm]))
    if m.Compression is None:
        o += b"\x00"
    else:
        o += b"\x01" + bytes([m.Compression.Algorithm]) + py_varint(m.Compression.Level)
    o += bytes([m.Flags]) + py_varint(m.Created) + py_varint(m.Modified)
    return bytes(o)



def py_marshal_system(c) -> bytes:
    """object.MarshalSystem(collection) restated directly from
    collection.go:137-237 / index.go:58-86 / field.go:42-60 (cross-check only)."""
    if c is None:
        return b"\x01\x00\x00"
    o = bytearray(b"\x01\x01") + c.ID + _frame(c.Name)
    if c.Version is None:
        o += b"\x00"
    else:
        v = c.Version
        o += b"\x01" + py_uvarint(v.Scalar.PID) + py_uvarint(v.Scalar.VID) + py_uvarint(v.Region)
        o += (b"\x01" + py_uvarint(v.Parent.PID) + py_uvarint(v.Parent.VID)) if v.Parent else b"\x00"
        o += (b"\x01" if v.Tombstone else b"\x00") + py_varint(v.Created)
    o += c.Owner + c.Group + bytes([c.Permissions])
    acl = c.ACL or []
    o += py_uvarint(len(acl))
    for a in acl:
        o += b"\x00" if a is None else b"\x01" + a.ClientID + bytes([a.Permissions])
    reg = c.WriteRegions or []
    o += py_uvarint(len(reg)) + b"".join(py_uvarint(r) for r in reg)
    if c.Publisher is None:
        o += b"\x00"
    else:
        p = c.Publisher
        o += b"\x01" + p.PublisherID + p.ClientID + _frame(p.IPAddress) + _frame(p.UserAgent)
    if c.Schema is None:
        o += b"\x00"
    else:
        s = c.Schema
        o += b"\x01" + _frame(s.Name) + py_uvarint(s.Major) + py_uvarint(s.Minor) + py_uvarint(s.Patch)
    if c.Encryption is None:
        o += b"\x00"
    else:
        e = c.Encryption
        o += (b"\x01" + _frame(e.PublicKeyID) + _frame(e.EncryptionKey) + _frame(e.HMACSecret) +
              _frame(e.Signature) + bytes([e.SealingAlgorithm, e.EncryptionAlgorithm,
                                           e.SignatureAlgorithm]))
    if c.Compression is None:
        o += b"\x00"
    else:
        o += b"\x01" + bytes([c.Compression.Algorithm]) + py_varint(c.Compression.Level)
    o += bytes([c.Flags])
    idx = c.Indexes or []
    o += py_uvarint(len(idx))
    for x in idx:
        if x is None:
            o += b"\x00"
            continue
        o += b"\x01" + x.ID + _frame(x.Name) + bytes([x.Type])
        for f in (x.Field, x.Ref):
            o += b"\x00" if f is None else b"\x01" + _frame(f.Name) + bytes([f.Type]) + f.Collection
    o += py_varint(c.Created) + py_varint(c.Modified) + b"\x00"
    return bytes(o)


def extreme_metas(n=96, seed=29):
    """Every varint at its widest and narrowest: PID/region/schema numbers at
    0 and 2^32-1 (5 bytes), VIDs at 2^64-1 (10 bytes), times and compression
    levels at INT64_MIN / INT64_MAX / -1 / 1 (zig-zag 10 bytes and 1 byte),
    frame lengths at 0, 127, 128 and 16384, region ids at every varint width,
    permission and flag bytes at 0 and 255."""
    from honu_amd.metadata import (AccessControl, Compression, Encryption, Metadata, Publisher,
                                   Scalar, SchemaVersion, Version)
    rng = np.random.default_rng(seed)
    U32, U64, I64 = [0, 1, 127, 128, 2**32 - 1], [0, 2**63, 2**64 - 1], [-2**63, 2**63 - 1, -1, 1, 0]
    LENS = [0, 1, 127, 128, 16384]
    pick = lambda xs, i: xs[i % len(xs)]  # noqa: E731
    metas, datas = [], []
    for i in range(n):
        ln = pick(LENS, i // 3)
        metas.append(Metadata(
            ObjectID=rng.bytes(16), CollectionID=rng.bytes(16),
            Version=Version(Scalar(pick(U32, i), pick(U64, i)), pick(U32, i + 1),
                            Scalar(pick(U32, i + 2), pick(U64, i + 1)) if i % 2 else None,
                            bool(i % 3 == 0), pick(I64, i)),
            Schema=SchemaVersion("s" * pick(LENS, i), pick(U32, i), pick(U32, i + 3), pick(U32, i + 4))
            if i % 4 else None,
            MIME="m" * ln, Owner=rng.bytes(16), Group=rng.bytes(16), Permissions=255 * (i % 2),
            ACL=[AccessControl(rng.bytes(16), 255 * (j % 2)) for j in range(i % 5)] or None,
            WriteRegions=[pick(U32, i + j) for j in range(i % 4)] if i % 6 else None,
            Publisher=Publisher(rng.bytes(16), rng.bytes(16), rng.bytes(pick(LENS, i + 1)) or None,
                                "u" * pick(LENS, i + 2)) if i % 3 else None,
            Encryption=Encryption("k" * pick(LENS, i + 3), rng.bytes(pick(LENS, i + 4)) or None,
                                  rng.bytes(pick(LENS, i)) or None, rng.bytes(pick(LENS, i + 1)) or None,
                                  i % 6, (i + 1) % 6, (i + 2) % 6) if i % 5 else None,
            Compression=Compression(i % 5, pick(I64, i + 1)) if i % 7 else None,
            Flags=255 * ((i + 1) % 2), Created=pick(I64, i + 2), Modified=pick(I64, i + 3)))
        datas.append(rng.bytes(pick(LENS, i)) if i % 9 else None)
    return metas, datas
