"""Host mirror of pkg/store/metadata (+ lamport.Scalar, region.Regions) and the
packing of Go-shaped values into the fixed-row batch layout of
include/honu_codec.h (honu_meta, honu_acl).

Field names follow the Go structs (metadata/metadata.go:17-35, version.go:15-23,
schema.go:11-16, acls.go:12-15, provenance.go:14-19, encryption.go:25-33,
compression.go:25-28, lamport/scalar.go:25-28). Times are Go UnixNano with
0 meaning time.Time{} (lani/encode.go:201-206). Go nil slices/pointers are None.
String fields hold str (utf-8, surrogateescape so any byte string round-trips).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

# --------------------------------------------------------------------------
# numpy views of the C structs (offsets pinned by tests/test_abi.py)
# --------------------------------------------------------------------------
SPAN = np.dtype([("off", "<u8"), ("len", "<u8")])

META_DTYPE = np.dtype(
    {
        "names": [
            "present", "permissions", "flags", "tombstone", "compression_alg",
            "sealing_alg", "encryption_alg", "signature_alg", "region", "vid", "pid",
            "parent_pid", "parent_vid", "version_created", "schema_major", "schema_minor",
            "schema_patch", "compression_level", "created", "modified", "acl_bytes", "object_id",
            "collection_id", "owner", "group", "publisher_id", "client_id", "schema_name",
            "mime", "ip_address", "user_agent", "public_key_id", "encryption_key",
            "hmac_secret", "signature", "acl_off", "acl_count", "regions_off", "regions_count",
        ],
        "formats": [
            "<u4", "u1", "u1", "u1", "u1", "u1", "u1", "u1", "<u4", "<u8", "<u4", "<u4", "<u8",
            "<i8", "<u4", "<u4", "<u4", "<i8", "<i8", "<i8", "<u8", ("u1", 16), ("u1", 16), ("u1", 16),
            ("u1", 16), ("u1", 16), ("u1", 16), SPAN, SPAN, SPAN, SPAN, SPAN, SPAN, SPAN, SPAN,
            "<u8", "<u8", "<u8", "<u8",
        ],
        "offsets": [
            0, 4, 5, 6, 7, 8, 9, 10, 12, 16, 24, 28, 32, 40, 48, 52, 56, 64, 72, 80, 88, 96, 112,
            128, 144, 160, 176, 192, 208, 224, 240, 256, 272, 288, 304, 320, 328, 336, 344,
        ],
        "itemsize": 352,
    }
)

ACL_DTYPE = np.dtype(
    {"names": ["client_id", "permissions", "present"], "formats": [("u1", 16), "u1", "u1"],
     "offsets": [0, 16, 17], "itemsize": 20}
)

INFO_DTYPE = np.dtype(
    {"names": ["data_off", "data_len", "data_status", "meta_status", "storage_version",
               "tombstone"],
     "formats": ["<u8", "<u8", "<i4", "<i4", "u1", "u1"],
     "offsets": [0, 8, 16, 20, 24, 25], "itemsize": 32}
)

HAS_META = 1 << 0
HAS_VERSION = 1 << 1
HAS_PARENT = 1 << 2
HAS_SCHEMA = 1 << 3
HAS_PUBLISHER = 1 << 4
HAS_ENCRYPTION = 1 << 5
HAS_COMPRESSION = 1 << 6
REGIONS_NONNIL = 1 << 7
ACL_INPLACE = 1 << 8  # decode output: the ACL list in place in the records arena (honu_codec.h)
REGIONS_INPLACE = 1 << 9  # decode output: the region list in place in the records arena
ACL_SIZED = 1 << 10  # encode input: acl_bytes holds the ACL list's encoded length (honu_codec.h)

SPAN_FIELDS = ("schema_name", "mime", "ip_address", "user_agent", "public_key_id",
               "encryption_key", "hmac_secret", "signature")


def _s2b(s) -> bytes:
    if s is None:
        return b""
    if isinstance(s, (bytes, bytearray, memoryview)):
        return bytes(s)
    return s.encode("utf-8", "surrogateescape")


def _b2s(b: bytes) -> str:
    return b.decode("utf-8", "surrogateescape")


# --------------------------------------------------------------------------
# Go-shaped values
# --------------------------------------------------------------------------
@dataclass
class Scalar:  # lamport/scalar.go:25-28
    PID: int = 0
    VID: int = 0


@dataclass
class Version:  # metadata/version.go:15-23
    Scalar: Scalar = field(default_factory=Scalar)
    Region: int = 0
    Parent: Optional[Scalar] = None
    Tombstone: bool = False
    Created: int = 0


@dataclass
class SchemaVersion:  # metadata/schema.go:11-16
    Name: str = ""
    Major: int = 0
    Minor: int = 0
    Patch: int = 0


@dataclass
class AccessControl:  # metadata/acls.go:12-15
    ClientID: bytes = bytes(16)
    Permissions: int = 0


@dataclass
class Publisher:  # metadata/provenance.go:14-19
    PublisherID: bytes = bytes(16)
    ClientID: bytes = bytes(16)
    IPAddress: Optional[bytes] = None
    UserAgent: str = ""


@dataclass
class Encryption:  # metadata/encryption.go:25-33
    PublicKeyID: str = ""
    EncryptionKey: Optional[bytes] = None
    HMACSecret: Optional[bytes] = None
    Signature: Optional[bytes] = None
    SealingAlgorithm: int = 0
    EncryptionAlgorithm: int = 0
    SignatureAlgorithm: int = 0


@dataclass
class Compression:  # metadata/compression.go:25-28
    Algorithm: int = 0
    Level: int = 0


@dataclass
class Metadata:  # metadata/metadata.go:17-35
    ObjectID: bytes = bytes(16)
    CollectionID: bytes = bytes(16)
    Version: Optional[Version] = None
    Schema: Optional[SchemaVersion] = None
    MIME: str = ""
    Owner: bytes = bytes(16)
    Group: bytes = bytes(16)
    Permissions: int = 0
    ACL: Optional[List[Optional[AccessControl]]] = None
    WriteRegions: Optional[List[int]] = None
    Publisher: Optional[Publisher] = None
    Encryption: Optional[Encryption] = None
    Compression: Optional[Compression] = None
    Flags: int = 0
    Created: int = 0
    Modified: int = 0


# Enum values (encryption.go:18-23, compression.go:15-23)
PLAINTEXT, AES256_GCM, AES192_GCM, AES128_GCM, HMAC_SHA256, RSA_OEAP_SHA512 = range(6)
NONE, GZIP, COMPRESS, DEFLATE, BROTLI = range(5)


# --------------------------------------------------------------------------
# packing
# --------------------------------------------------------------------------
class HostBatch:
    """A batch in the C layout, in host memory (numpy arrays)."""

    def __init__(self, meta, var, acl, regions, payload, payload_off):
        self.meta = meta
        self.var = var
        self.acl = acl
        self.regions = regions
        self.payload = payload
        self.payload_off = payload_off

    def __len__(self):
        return len(self.meta)


def pack_common(r, m, span, acl_rows: list, regions: list) -> int:
    """Fill the row fields Metadata and Collection share (Version, Schema,
    Owner, Group, Permissions, ACL, WriteRegions, Publisher, Encryption,
    Compression, Flags, Created, Modified); returns their presence bits."""
    pr = 0
    if m.Version is not None:
        v = m.Version
        pr |= HAS_VERSION
        r["pid"], r["vid"], r["region"] = v.Scalar.PID, v.Scalar.VID, v.Region
        r["tombstone"] = 1 if v.Tombstone else 0
        r["version_created"] = v.Created
        if v.Parent is not None:
            pr |= HAS_PARENT
            r["parent_pid"], r["parent_vid"] = v.Parent.PID, v.Parent.VID
    if m.Schema is not None:
        pr |= HAS_SCHEMA
        r["schema_name"] = span(_s2b(m.Schema.Name))
        r["schema_major"], r["schema_minor"], r["schema_patch"] = (
            m.Schema.Major, m.Schema.Minor, m.Schema.Patch)
    r["owner"] = np.frombuffer(_ulid(m.Owner), np.uint8)
    r["group"] = np.frombuffer(_ulid(m.Group), np.uint8)
    r["permissions"] = m.Permissions
    if m.ACL:
        r["acl_off"], r["acl_count"] = len(acl_rows), len(m.ACL)
        for a in m.ACL:
            acl_rows.append(None if a is None else (_ulid(a.ClientID), a.Permissions))
        if "acl_bytes" in r.dtype.names:  # honu_meta: the list's encoded length, as the
            # binding's flatten carries it (HONU_ACL_SIZED: the size pass reads no entry)
            r["acl_bytes"] = sum(1 if a is None else 18 for a in m.ACL)
            pr |= ACL_SIZED
    if m.WriteRegions:
        r["regions_off"], r["regions_count"] = len(regions), len(m.WriteRegions)
        regions.extend(m.WriteRegions)
    if m.Publisher is not None:
        p = m.Publisher
        pr |= HAS_PUBLISHER
        r["publisher_id"] = np.frombuffer(_ulid(p.PublisherID), np.uint8)
        r["client_id"] = np.frombuffer(_ulid(p.ClientID), np.uint8)
        r["ip_address"] = span(_s2b(p.IPAddress))
        r["user_agent"] = span(_s2b(p.UserAgent))
    if m.Encryption is not None:
        e = m.Encryption
        pr |= HAS_ENCRYPTION
        r["public_key_id"] = span(_s2b(e.PublicKeyID))
        r["encryption_key"] = span(_s2b(e.EncryptionKey))
        r["hmac_secret"] = span(_s2b(e.HMACSecret))
        r["signature"] = span(_s2b(e.Signature))
        r["sealing_alg"], r["encryption_alg"], r["signature_alg"] = (
            e.SealingAlgorithm, e.EncryptionAlgorithm, e.SignatureAlgorithm)
    if m.Compression is not None:
        pr |= HAS_COMPRESSION
        r["compression_alg"], r["compression_level"] = m.Compression.Algorithm, m.Compression.Level
    r["flags"] = m.Flags
    r["created"], r["modified"] = m.Created, m.Modified
    return pr


def acl_table(acl_rows: list) -> np.ndarray:
    acl = np.zeros(len(acl_rows), ACL_DTYPE)
    for j, a in enumerate(acl_rows):
        if a is not None:
            acl[j]["client_id"] = np.frombuffer(a[0], np.uint8)
            acl[j]["permissions"] = a[1]
            acl[j]["present"] = 1
    return acl


def pack_batch(metas: Sequence[Optional[Metadata]], datas: Sequence[Optional[bytes]]) -> HostBatch:
    """Flatten (meta, data) pairs into rows + arenas. A None meta is Marshal(nil, …)."""
    if len(metas) != len(datas):
        raise ValueError("metas and datas differ in length")
    n = len(metas)
    rows = np.zeros(n, META_DTYPE)
    var = bytearray()
    acl_rows: list = []
    regions: list = []

    def span(b: bytes):
        off = len(var)
        var.extend(b)
        return (off, len(b)) if b else (0, 0)

    for i, m in enumerate(metas):
        r = rows[i]
        if m is None:
            continue
        r["object_id"] = np.frombuffer(_ulid(m.ObjectID), np.uint8)
        r["collection_id"] = np.frombuffer(_ulid(m.CollectionID), np.uint8)
        r["mime"] = span(_s2b(m.MIME))
        r["present"] = HAS_META | pack_common(r, m, span, acl_rows, regions)

    acl = acl_table(acl_rows)
    payload_off = np.zeros(n + 1, np.uint64)
    pay = bytearray()
    for i, d in enumerate(datas):
        payload_off[i] = len(pay)
        if d:
            pay.extend(d)
    payload_off[n] = len(pay)
    return HostBatch(rows, np.frombuffer(bytes(var) or b"\0", np.uint8).copy(), acl,
                     np.asarray(regions, np.uint32), np.frombuffer(bytes(pay) or b"\0", np.uint8).copy(),
                     payload_off)


def _ulid(b) -> bytes:
    b = bytes(b)
    if len(b) != 16:
        raise ValueError("ULID must be 16 bytes")
    return b


def unpack_row(row, arena, acl_table=None, regions_table=None) -> Metadata:
    """Rebuild a Metadata from a decoded row; spans index `arena`, lists the
    decoded tables, or `arena` for an ACL list returned in place
    (ACL_INPLACE: entry j = the 18 bytes 01 | ClientID | Permissions at
    acl_off + 18 j) or a region list returned in place (REGIONS_INPLACE: the
    uvarints from regions_off). Mirrors the nil/empty rules of the Go decoder
    (lani/decode.go:37-39, metadata.go:254, region.go:160)."""
    pr = int(row["present"])
    m = Metadata()
    if not pr & HAS_META:
        return m  # Metadata() of a nil-flagged object: &Metadata{} (object.go:76-82)
    arena = memoryview(arena)

    def sb(name) -> Optional[bytes]:
        off, ln = int(row[name]["off"]), int(row[name]["len"])
        return bytes(arena[off:off + ln]) if ln else None

    def ss(name) -> str:
        b = sb(name)
        return _b2s(b) if b else ""

    m.ObjectID = bytes(row["object_id"])
    m.CollectionID = bytes(row["collection_id"])
    m.MIME = ss("mime")
    unpack_common(row, m, sb, ss, acl_table, regions_table, arena)
    return m


def acl_inplace_entries(arena, off: int, count: int) -> list:
    """The AccessControl list of a row returned in place (ACL_INPLACE):
    what Metadata.Decode builds from those bytes (metadata.go:254-266,
    acls.go:41-51), each entry copied out of the records arena."""
    arena = memoryview(arena)
    out = []
    for j in range(count):
        e = bytes(arena[off + 18 * j: off + 18 * j + 18])
        if len(e) != 18 or e[0] != 1:
            raise ValueError("in-place ACL entry %d is not a present entry" % j)
        out.append(AccessControl(e[1:17], e[17]))
    return out


def regions_inplace_values(arena, off: int, count: int) -> list:
    """The WriteRegions of a row returned in place (REGIONS_INPLACE): what
    Regions.Decode builds from those bytes (region.go:154-169), each uvarint
    read as lani.DecodeUint32 does (at most 5 bytes, truncated to uint32,
    decode.go:127-146; the GPU decode has validated every one of them)."""
    arena = memoryview(arena)
    out, p = [], off
    for j in range(count):
        v, sh = 0, 0
        for k in range(5):
            b = arena[p + k]
            v |= (b & 0x7F) << sh
            sh += 7
            if not b & 0x80:
                break
        else:
            raise ValueError("in-place region %d is not a 5-byte uvarint" % j)
        out.append(v & 0xFFFFFFFF)
        p += k + 1
    return out


def unpack_common(row, m, sb, ss, acl_table, regions_table, arena=None):
    """Inverse of pack_common on a decoded row (Go decoder nil/empty rules)."""
    pr = int(row["present"])
    if pr & HAS_VERSION:
        m.Version = Version(Scalar(int(row["pid"]), int(row["vid"])), int(row["region"]),
                            Scalar(int(row["parent_pid"]), int(row["parent_vid"]))
                            if pr & HAS_PARENT else None,
                            bool(row["tombstone"]), int(row["version_created"]))
    if pr & HAS_SCHEMA:
        m.Schema = SchemaVersion(ss("schema_name"), int(row["schema_major"]),
                                 int(row["schema_minor"]), int(row["schema_patch"]))
    m.Owner = bytes(row["owner"])
    m.Group = bytes(row["group"])
    m.Permissions = int(row["permissions"])
    na = int(row["acl_count"])
    if na and pr & ACL_INPLACE:
        m.ACL = acl_inplace_entries(arena, int(row["acl_off"]), na)
    elif na:
        m.ACL = []
        base = int(row["acl_off"])
        for j in range(na):
            a = acl_table[base + j]
            m.ACL.append(AccessControl(bytes(a["client_id"]), int(a["permissions"]))
                         if a["present"] else None)
    nr = int(row["regions_count"])
    if nr and pr & REGIONS_INPLACE:
        m.WriteRegions = regions_inplace_values(arena, int(row["regions_off"]), nr)
    elif pr & REGIONS_NONNIL or nr:
        base = int(row["regions_off"])
        m.WriteRegions = [int(x) for x in regions_table[base:base + nr]] if nr else []
    if pr & HAS_PUBLISHER:
        m.Publisher = Publisher(bytes(row["publisher_id"]), bytes(row["client_id"]),
                                sb("ip_address"), ss("user_agent"))
    if pr & HAS_ENCRYPTION:
        m.Encryption = Encryption(ss("public_key_id"), sb("encryption_key"), sb("hmac_secret"),
                                  sb("signature"), int(row["sealing_alg"]),
                                  int(row["encryption_alg"]), int(row["signature_alg"]))
    if pr & HAS_COMPRESSION:
        m.Compression = Compression(int(row["compression_alg"]), int(row["compression_level"]))
    m.Flags = int(row["flags"])
    m.Created = int(row["created"])
    m.Modified = int(row["modified"])


def normalize(m: Optional[Metadata]) -> Optional[Metadata]:
    """What a Go round trip turns a Metadata into: empty frames become nil/"",
    empty ACL becomes nil, WriteRegions becomes a (possibly empty) slice."""
    if m is None:
        return None
    import copy
    m = copy.deepcopy(m)
    if not m.ACL:
        m.ACL = None
    m.WriteRegions = list(m.WriteRegions or [])
    if m.Publisher is not None:
        m.Publisher.IPAddress = m.Publisher.IPAddress or None
        m.Publisher.UserAgent = m.Publisher.UserAgent or ""
    if m.Encryption is not None:
        e = m.Encryption
        e.EncryptionKey = e.EncryptionKey or None
        e.HMACSecret = e.HMACSecret or None
        e.Signature = e.Signature or None
    return m
