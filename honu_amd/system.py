"""System objects: the host mirror of object.MarshalSystem / UnmarshalSystem
(pkg/store/object/system.go:10-45) for metadata.Collection
(metadata/collection.go:16-33) with its Index / Field lists (index.go:16-22,
field.go:12-16), over the gfx950 batch kernels (honu_system_* in
include/honu_codec.h).

Wire form: 0x01 | EncodeStruct(collection) | 0x00 (nil metadata);
UnmarshalSystem decodes obj[1 : len-1] without checking the version byte.
"""
from __future__ import annotations

import copy
from dataclasses import dataclass, field, fields
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .metadata import (ACL_DTYPE, HAS_META, SPAN, AccessControl, Compression, Encryption,
                       Publisher, SchemaVersion, Version, _b2s, _s2b, _ulid, acl_table,
                       pack_common, unpack_common)

HAS_COLLECTION = HAS_META

COLLECTION_DTYPE = np.dtype(
    {
        "names": [
            "present", "permissions", "flags", "tombstone", "compression_alg",
            "sealing_alg", "encryption_alg", "signature_alg", "region", "vid", "pid",
            "parent_pid", "parent_vid", "version_created", "schema_major", "schema_minor",
            "schema_patch", "compression_level", "created", "modified", "id", "owner", "group",
            "publisher_id", "client_id", "name", "schema_name", "ip_address", "user_agent",
            "public_key_id", "encryption_key", "hmac_secret", "signature", "acl_off",
            "acl_count", "regions_off", "regions_count", "index_off", "index_count",
        ],
        "formats": [
            "<u4", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "<u4", "<u8", "<u4", "<u4", "<u8",
            "<i8", "<u4", "<u4", "<u4", "<i8", "<i8", "<i8", ("u1", 16), ("u1", 16), ("u1", 16),
            ("u1", 16), ("u1", 16), SPAN, SPAN, SPAN, SPAN, SPAN, SPAN, SPAN, SPAN,
            "<u8", "<u8", "<u8", "<u8", "<u8", "<u8",
        ],
        "offsets": [
            0, 4, 5, 6, 7, 8, 9, 10, 12, 16, 24, 28, 32, 40, 48, 52, 56, 64, 72, 80, 96, 112,
            128, 144, 160, 192, 208, 224, 240, 256, 272, 288, 304, 320, 328, 336, 344, 352, 360,
        ],
        "itemsize": 368,
    }
)

INDEX_DTYPE = np.dtype(
    {
        "names": ["present", "type", "has_field", "field_type", "has_ref", "ref_type", "id",
                  "field_collection", "ref_collection", "name", "field_name", "ref_name"],
        "formats": ["u1", "u1", "u1", "u1", "u1", "u1", ("u1", 16), ("u1", 16), ("u1", 16),
                    SPAN, SPAN, SPAN],
        "offsets": [0, 1, 2, 3, 4, 5, 16, 32, 48, 64, 80, 96],
        "itemsize": 112,
    }
)

# IndexType (index.go:26-35) and FieldType (field.go:20-30)
INDEX_TYPES = ("UNKNOWN", "UNIQUE", "INDEX", "FOREIGN_KEY", "VECTOR", "SEARCH", "COLUMN", "BLOOM")
FIELD_TYPES = ("STRING", "BLOB", "ULID", "UUID", "INT", "UINT", "FLOAT", "TIME", "VECTOR")


@dataclass
class Field:  # metadata/field.go:12-16
    Name: str = ""
    Type: int = 0
    Collection: bytes = bytes(16)


@dataclass
class Index:  # metadata/index.go:16-22
    ID: bytes = bytes(16)
    Name: str = ""
    Type: int = 0
    Field: Optional[Field] = None
    Ref: Optional[Field] = None


@dataclass
class Collection:  # metadata/collection.go:16-33
    ID: bytes = bytes(16)
    Name: str = ""
    Version: Optional[Version] = None
    Owner: bytes = bytes(16)
    Group: bytes = bytes(16)
    Permissions: int = 0
    ACL: Optional[List[Optional[AccessControl]]] = None
    WriteRegions: Optional[List[int]] = None
    Publisher: Optional[Publisher] = None
    Schema: Optional[SchemaVersion] = None
    Encryption: Optional[Encryption] = None
    Compression: Optional[Compression] = None
    Flags: int = 0
    Indexes: Optional[List[Optional[Index]]] = None
    Created: int = 0
    Modified: int = 0


class SystemHostBatch:
    """Collections in the C layout (rows + var arena + ACL/region/index tables)."""

    def __init__(self, rows, var, acl, regions, index):
        self.rows, self.var, self.acl, self.regions, self.index = rows, var, acl, regions, index

    def __len__(self):
        return len(self.rows)


def pack_system_batch(cols: Sequence[Optional[Collection]]) -> SystemHostBatch:
    """Flatten collections (None = MarshalSystem(nil)) into rows + arenas."""
    n = len(cols)
    rows = np.zeros(n, COLLECTION_DTYPE)
    var = bytearray()
    acl_rows: list = []
    regions: list = []
    idx_rows: list = []

    def span(b: bytes):
        off = len(var)
        var.extend(b)
        return (off, len(b)) if b else (0, 0)

    for i, c in enumerate(cols):
        if c is None:
            continue
        r = rows[i]
        r["id"] = np.frombuffer(_ulid(c.ID), np.uint8)
        r["name"] = span(_s2b(c.Name))
        pr = HAS_COLLECTION | pack_common(r, c, span, acl_rows, regions)
        if c.Indexes:
            r["index_off"], r["index_count"] = len(idx_rows), len(c.Indexes)
            for x in c.Indexes:
                idx_rows.append(None if x is None else (
                    _ulid(x.ID), span(_s2b(x.Name)), x.Type,
                    None if x.Field is None else (span(_s2b(x.Field.Name)), x.Field.Type,
                                                  _ulid(x.Field.Collection)),
                    None if x.Ref is None else (span(_s2b(x.Ref.Name)), x.Ref.Type,
                                                _ulid(x.Ref.Collection))))
        r["present"] = pr
    index = np.zeros(len(idx_rows), INDEX_DTYPE)
    for j, x in enumerate(idx_rows):
        if x is None:
            continue
        e = index[j]
        e["present"] = 1
        e["id"] = np.frombuffer(x[0], np.uint8)
        e["name"], e["type"] = x[1], x[2]
        if x[3] is not None:
            e["has_field"], e["field_name"], e["field_type"] = 1, x[3][0], x[3][1]
            e["field_collection"] = np.frombuffer(x[3][2], np.uint8)
        if x[4] is not None:
            e["has_ref"], e["ref_name"], e["ref_type"] = 1, x[4][0], x[4][1]
            e["ref_collection"] = np.frombuffer(x[4][2], np.uint8)
    return SystemHostBatch(rows, np.frombuffer(bytes(var) or b"\0", np.uint8).copy(),
                           acl_table(acl_rows), np.asarray(regions, np.uint32), index)


def unpack_collection(row, arena, acl=None, regions=None, index=None) -> Collection:
    """Rebuild a Collection from a decoded row (spans index `arena`); a row
    without HAS_COLLECTION is the untouched &Collection{} of a nil flag."""
    c = Collection()
    if not int(row["present"]) & HAS_COLLECTION:
        return c
    arena = memoryview(arena)

    def sb_of(sp) -> Optional[bytes]:
        off, ln = int(sp["off"]), int(sp["len"])
        return bytes(arena[off:off + ln]) if ln else None

    def sb(name):
        return sb_of(row[name])

    def ss(name) -> str:
        b = sb(name)
        return _b2s(b) if b else ""

    c.ID = bytes(row["id"])
    c.Name = ss("name")
    unpack_common(row, c, sb, ss, acl, regions)
    nx = int(row["index_count"])
    if nx:
        c.Indexes = []
        base = int(row["index_off"])
        for j in range(nx):
            e = index[base + j]
            if not e["present"]:
                c.Indexes.append(None)
                continue
            name = lambda sp: _b2s(sb_of(sp) or b"")  # noqa: E731
            c.Indexes.append(Index(
                bytes(e["id"]), name(e["name"]), int(e["type"]),
                Field(name(e["field_name"]), int(e["field_type"]), bytes(e["field_collection"]))
                if e["has_field"] else None,
                Field(name(e["ref_name"]), int(e["ref_type"]), bytes(e["ref_collection"]))
                if e["has_ref"] else None))
    return c


def normalize_collection(c: Optional[Collection]) -> Collection:
    """What a MarshalSystem/UnmarshalSystem round trip turns a Collection into
    (Go decoder rules: empty frames -> nil/"", empty ACL/Indexes -> nil,
    WriteRegions -> a (possibly empty) slice); nil -> &Collection{}."""
    if c is None:
        return Collection()
    c = copy.deepcopy(c)
    if not c.ACL:
        c.ACL = None
    if not c.Indexes:
        c.Indexes = None
    c.WriteRegions = list(c.WriteRegions or [])
    if c.Publisher is not None:
        c.Publisher.IPAddress = c.Publisher.IPAddress or None
        c.Publisher.UserAgent = c.Publisher.UserAgent or ""
    if c.Encryption is not None:
        e = c.Encryption
        e.EncryptionKey = e.EncryptionKey or None
        e.HMACSecret = e.HMACSecret or None
        e.Signature = e.Signature or None
    return c


# --------------------------------------------------------------------------
# GPU batch API
# --------------------------------------------------------------------------
def _dev(a, codec):
    from .object import _dev_bytes
    return _dev_bytes(np.ascontiguousarray(a), codec.torch_device)


def marshal_system_batch(cols: Sequence[Optional[Collection]], codec=None):
    """[MarshalSystem(c) ...] on the GPU -> (records arena, offsets[n+1], status[n])."""
    from .object import _to_host, default_codec
    codec = codec or default_codec()
    hb = pack_system_batch(cols)
    n = len(hb)
    rows, var, acl = _dev(hb.rows, codec), _dev(hb.var, codec), _dev(hb.acl, codec)
    reg, idx = _dev(hb.regions, codec), _dev(hb.index, codec)
    off = codec._empty(8 * (n + 1))
    st = codec._empty(4 * n)
    L, P = codec.lib, _lib.ptr
    _lib.check(L.honu_system_sizes(codec.ctx, P(rows), len(hb.var), P(acl), len(hb.acl), P(reg),
                                   len(hb.regions), P(idx), len(hb.index), n, P(off), P(st),
                                   codec.stream), "honu_system_sizes")
    codec.scan(off, n, off)
    total = int(off.view(__import__("torch").int64)[n].item())
    out = codec._empty(total)
    _lib.check(L.honu_system_encode(codec.ctx, P(rows), P(var), P(acl), P(reg), P(idx), n,
                                    P(out), total, P(off), P(st), codec.stream),
               "honu_system_encode")
    return (_to_host(out, total, np.uint8), _to_host(off, 8 * (n + 1), np.uint64),
            _to_host(st, 4 * n, np.int32))


def decode_system_batch(rec: np.ndarray, rec_off: np.ndarray, codec=None, headless=False):
    """UnmarshalSystem(obj, &Collection{}) for a CSR batch on the GPU ->
    (rows, status, acl table, region table, index table, totals[3])."""
    from .object import _to_host, default_codec
    codec = codec or default_codec()
    n = len(rec_off) - 1
    nbytes = int(rec_off[-1]) if n >= 0 else 0
    d_rec = _dev(rec if len(rec) else np.zeros(1, np.uint8), codec)
    d_off = _dev(np.asarray(rec_off, np.uint64), codec)
    cap = max(nbytes, 1)  # every entry takes >= 1 byte of its record
    rows = codec._empty(COLLECTION_DTYPE.itemsize * n)
    st = codec._empty(4 * n)
    acl = codec._empty(ACL_DTYPE.itemsize * cap)
    reg = codec._empty(4 * cap)
    idx = codec._empty(INDEX_DTYPE.itemsize * cap)
    tot = codec._empty(32)
    P = _lib.ptr
    fn = codec.lib.honu_collection_decode_batch if headless else codec.lib.honu_system_decode_batch
    _lib.check(fn(codec.ctx, P(d_rec), P(d_off), n, P(rows), P(st), P(acl), cap, P(reg), cap,
                  P(idx), cap, P(tot), codec.stream), "honu collection decode")
    t = _to_host(tot, 24, np.uint64)
    return (_to_host(rows, COLLECTION_DTYPE.itemsize * n, COLLECTION_DTYPE),
            _to_host(st, 4 * n, np.int32), _to_host(acl, ACL_DTYPE.itemsize * int(t[0]), ACL_DTYPE),
            _to_host(reg, 4 * int(t[1]), np.uint32),
            _to_host(idx, INDEX_DTYPE.itemsize * int(t[2]), INDEX_DTYPE), t)


def MarshalSystem(c: Optional[Collection]) -> bytes:
    """object.MarshalSystem (system.go:10-31) for one collection."""
    from .object import _ERRORS, HonuCodecError
    out, off, st = marshal_system_batch([c])
    if st[0]:
        raise _ERRORS.get(int(st[0]), HonuCodecError)(f"status {int(st[0])}")
    return bytes(out[int(off[0]):int(off[1])])


def UnmarshalSystem(obj: bytes) -> Collection:
    """object.UnmarshalSystem(obj, &metadata.Collection{}) (system.go:33-45);
    Go errors raise (GoPanic where the reference panics)."""
    from .object import _ERRORS, HonuCodecError
    rec = np.frombuffer(bytes(obj), np.uint8)
    rows, st, acl, reg, idx, _ = decode_system_batch(rec, np.array([0, len(obj)], np.uint64))
    if st[0]:
        raise _ERRORS.get(int(st[0]), HonuCodecError)(f"status {int(st[0])}")
    return unpack_collection(rows[0], rec, acl, reg, idx)


def Unmarshal(raw: bytes, c: Optional[Collection] = None) -> Collection:
    """lani.Unmarshal(raw, c) with c a *metadata.Collection (lani/lani.go:29-33):
    Collection.Decode from byte 0 of raw, as pkg/store calls it on raw bbolt
    values (store.go:155, :367). Decodes INTO c, as the Go decoder assigns
    every field of *c (collection.go:242-356), and returns c. c=None is
    store.go:155's nil pointer, on which the reference panics. On an error c is
    left as it was (Go may have assigned a prefix of the fields; callers
    discard c on error)."""
    from .object import _ERRORS, GoPanic, HonuCodecError
    if c is None:
        raise GoPanic("Collection.Decode on a nil *Collection (store.go:155)")
    rec = np.frombuffer(bytes(raw), np.uint8)
    rows, st, acl, reg, idx, _ = decode_system_batch(rec, np.array([0, len(raw)], np.uint64),
                                                     headless=True)
    if st[0]:
        raise _ERRORS.get(int(st[0]), HonuCodecError)(f"status {int(st[0])}")
    out = unpack_collection(rows[0], rec, acl, reg, idx)
    for f in fields(out):
        setattr(c, f.name, getattr(out, f.name))
    return c
