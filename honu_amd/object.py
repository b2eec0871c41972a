"""Host mirror of pkg/store/object over the gfx950 batch codec.

Reference API (pkg/store/object/object.go):
    Marshal(meta, data) (Object, error)            :24-45
    Object.StorageVersion() uint8                  :47-52
    Object.Key() (keys.Key, error)                 :57-64
    Object.Metadata() (*metadata.Metadata, error)  :66-83
    Object.Data() ([]byte, error)                  :85-99
    Object.Tombstone() bool                        :103-112
Errors are raised as the Python counterparts of the Go sentinels
(object/errors.go:6-7, lani/errors.go:6-10, io.EOF, io.ErrUnexpectedEOF);
inputs on which Go panics raise GoPanic.

Every codec operation runs on the GPU through the C ABI (Codec). The
per-record mirror functions are batches of one, kept for API parity; the batch
methods (Codec.marshal / Codec.decode) are the point of the library.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np

from . import _lib
from .metadata import (ACL_DTYPE, INFO_DTYPE, META_DTYPE, HostBatch, Metadata, pack_batch,
                       unpack_row)

StorageVersion = 1  # object.go:14

# --------------------------------------------------------------------------
# status codes (include/honu_codec.h) and the Go sentinels they stand for
# --------------------------------------------------------------------------
OK, BAD_VERSION, MALFORMED, EOF, UNEXPECTED_EOF, NO_LENGTH, PARSE_BOOLEAN, PARSE_VARINT, \
    PANIC, CAPACITY, INPUT = range(11)


class HonuCodecError(Exception):
    status = -1


class ErrBadVersion(HonuCodecError):  # object/errors.go:6
    status = BAD_VERSION


class ErrMalformed(HonuCodecError):  # object/errors.go:7
    status = MALFORMED


class EOFError_(HonuCodecError):  # io.EOF
    status = EOF


class ErrUnexpectedEOF(HonuCodecError):  # io.ErrUnexpectedEOF
    status = UNEXPECTED_EOF


class ErrNoLength(HonuCodecError):  # lani/errors.go:8
    status = NO_LENGTH


class ErrParseBoolean(HonuCodecError):  # lani/errors.go:9
    status = PARSE_BOOLEAN


class ErrParseVarInt(HonuCodecError):  # lani/errors.go:10
    status = PARSE_VARINT


class GoPanic(HonuCodecError):  # the reference panics on this input
    status = PANIC


class ErrCapacity(HonuCodecError):
    status = CAPACITY


class ErrInput(HonuCodecError):
    status = INPUT


_ERRORS = {c.status: c for c in (ErrBadVersion, ErrMalformed, EOFError_, ErrUnexpectedEOF,
                                 ErrNoLength, ErrParseBoolean, ErrParseVarInt, GoPanic,
                                 ErrCapacity, ErrInput)}


def raise_status(st: int):
    if st != OK:
        raise _ERRORS.get(int(st), HonuCodecError)(f"status {int(st)}")


# --------------------------------------------------------------------------
# device plumbing (torch is used for device memory and streams only)
# --------------------------------------------------------------------------
def _torch():
    import torch
    return torch


def _dev_bytes(a: np.ndarray, device):
    torch = _torch()
    a = np.ascontiguousarray(a)
    t = torch.empty(max(a.nbytes, 16), dtype=torch.uint8, device=device)
    if a.nbytes:
        src = a.view(np.uint8).reshape(-1)
        if not src.flags.writeable:
            src = src.copy()
        t[: a.nbytes].copy_(torch.from_numpy(src))
    return t


def _to_host(t, nbytes: int, dtype) -> np.ndarray:
    raw = t[:nbytes].cpu().numpy() if nbytes else np.zeros(0, np.uint8)
    return raw.view(dtype)


@dataclass
class DeviceBatch:
    """Encode input on the device, C layout (rows + arenas + CSR payload)."""
    meta: object
    var: object
    var_len: int
    acl: object
    acl_len: int
    regions: object
    regions_len: int
    payload: object
    payload_off: object
    n: int

    @classmethod
    def from_host(cls, hb: HostBatch, device="cuda"):
        return cls(_dev_bytes(hb.meta, device), _dev_bytes(hb.var, device), len(hb.var),
                   _dev_bytes(hb.acl, device), len(hb.acl), _dev_bytes(hb.regions, device),
                   len(hb.regions), _dev_bytes(hb.payload, device),
                   _dev_bytes(hb.payload_off, device), len(hb.meta))


@dataclass
class EncodeResult:
    out: object        # device uint8 records arena
    out_off: object    # device uint64[n+1]
    status: object     # device int32[n]
    n: int

    def host(self):
        total = int(self.out_off.view(_torch().int64)[self.n].item())
        off = _to_host(self.out_off, 8 * (self.n + 1), np.uint64)
        st = _to_host(self.status, 4 * self.n, np.int32)
        return _to_host(self.out, total, np.uint8), off, st


@dataclass
class DecodeResult:
    meta: object       # device honu_meta[n]
    info: object       # device honu_record_info[n]
    acl: object        # device honu_acl table
    regions: object    # device uint32 table
    data: object       # device data arena or None (zero copy)
    totals: object     # device u64[3]: ACL entries, regions, data bytes
    n: int

    def host(self):
        tot = _to_host(self.totals, 24, np.uint64)
        meta = _to_host(self.meta, 352 * self.n, META_DTYPE)
        info = _to_host(self.info, 32 * self.n, INFO_DTYPE)
        acl = _to_host(self.acl, 20 * int(tot[0]), ACL_DTYPE)
        reg = _to_host(self.regions, 4 * int(tot[1]), np.uint32)
        data = _to_host(self.data, int(tot[2]), np.uint8) if self.data is not None else None
        return meta, info, acl, reg, data, tot


class Codec:
    """A device context of the batch codec (one per GPU / stream family)."""

    def __init__(self, device: int = 0, max_records: int = 1 << 16):
        torch = _torch()
        self.lib = _lib.load()
        self.device = device
        self.torch_device = torch.device("cuda", device)
        err = _lib.I32(0)
        torch.cuda.set_device(device)
        self.ctx = self.lib.honu_ctx_create(device, max_records, _lib.C.byref(err))
        if not self.ctx:
            _lib.check(err.value or -4, "honu_ctx_create")
        self.max_records = max_records

    def close(self):
        if getattr(self, "ctx", None):
            self.lib.honu_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream(self) -> int:
        return _torch().cuda.current_stream(self.torch_device).cuda_stream

    def _empty(self, nbytes: int):
        torch = _torch()
        return torch.empty(max(int(nbytes), 16), dtype=torch.uint8, device=self.torch_device)

    # ---- encode ---------------------------------------------------------
    def encode_sizes(self, b: DeviceBatch, sizes, status):
        _lib.check(self.lib.honu_encode_sizes(
            self.ctx, _lib.ptr(b.meta), b.var_len, _lib.ptr(b.acl), b.acl_len,
            _lib.ptr(b.regions), b.regions_len, _lib.ptr(b.payload_off), b.n, _lib.ptr(sizes),
            _lib.ptr(status), self.stream), "honu_encode_sizes")

    def scan(self, inp, n, out):
        _lib.check(self.lib.honu_exclusive_scan(self.ctx, _lib.ptr(inp), n, _lib.ptr(out),
                                                self.stream), "honu_exclusive_scan")

    def encode(self, b: DeviceBatch, out, out_cap, out_off, status):
        _lib.check(self.lib.honu_encode(
            self.ctx, _lib.ptr(b.meta), _lib.ptr(b.var), b.var_len, _lib.ptr(b.acl), b.acl_len,
            _lib.ptr(b.regions), b.regions_len, _lib.ptr(b.payload), _lib.ptr(b.payload_off),
            b.n, _lib.ptr(out), out_cap, _lib.ptr(out_off), _lib.ptr(status), self.stream),
            "honu_encode")

    def marshal(self, b: DeviceBatch) -> EncodeResult:
        """object.Marshal over the batch; sizes the output arena (one sync)."""
        out_off = self._empty(8 * (b.n + 1))
        status = self._empty(4 * b.n)
        self.encode_sizes(b, out_off, status)
        self.scan(out_off, b.n, out_off)
        total = int(out_off.view(_torch().int64)[b.n].item())
        out = self._empty(total)
        self.marshal_into(b, out, total, out_off, status)
        return EncodeResult(out, out_off, status, b.n)

    def marshal_into(self, b: DeviceBatch, out, out_cap, out_off, status):
        """honu_marshal_batch into a caller-sized arena: the single-launch
        size/offset/header/tail kernel + the payload copy (record_variant 0),
        or the split phases."""
        _lib.check(self.lib.honu_marshal_batch(
            self.ctx, _lib.ptr(b.meta), _lib.ptr(b.var), b.var_len, _lib.ptr(b.acl), b.acl_len,
            _lib.ptr(b.regions), b.regions_len, _lib.ptr(b.payload), _lib.ptr(b.payload_off),
            b.n, _lib.ptr(out), out_cap, _lib.ptr(out_off), _lib.ptr(status), self.stream),
            "honu_marshal_batch")

    # ---- decode ---------------------------------------------------------
    def decode(self, rec, rec_off, n: int, materialize: bool = False,
               acl_cap: Optional[int] = None, regions_cap: Optional[int] = None,
               data_cap: Optional[int] = None, rec_bytes: Optional[int] = None) -> DecodeResult:
        """Object.Metadata() + Object.Data() over a CSR batch of records."""
        if rec_bytes is None:
            rec_bytes = int(rec_off.view(_torch().int64)[n].item())
        # every ACL entry / region takes >= 1 byte of its record
        acl_cap = rec_bytes if acl_cap is None else acl_cap
        regions_cap = rec_bytes if regions_cap is None else regions_cap
        meta = self._empty(352 * n)
        info = self._empty(32 * n)
        acl = self._empty(20 * acl_cap)
        reg = self._empty(4 * regions_cap)
        totals = self._empty(32)
        data = None
        if materialize:
            data_cap = rec_bytes + 16 * n if data_cap is None else data_cap
            data = self._empty(data_cap)
        _lib.check(self.lib.honu_decode_batch(
            self.ctx, _lib.ptr(rec), _lib.ptr(rec_off), n, _lib.ptr(meta), _lib.ptr(info),
            _lib.ptr(acl), acl_cap, _lib.ptr(reg), regions_cap, _lib.ptr(data),
            data_cap or 0, _lib.ptr(totals), self.stream), "honu_decode_batch")
        return DecodeResult(meta, info, acl, reg, data, totals, n)

    def keys(self, d: DecodeResult):
        keys = self._empty(29 * d.n)
        st = self._empty(4 * d.n)
        _lib.check(self.lib.honu_decode_keys(self.ctx, _lib.ptr(d.meta), _lib.ptr(d.info), d.n,
                                             _lib.ptr(keys), _lib.ptr(st), self.stream),
                   "honu_decode_keys")
        return keys, st


_default: Optional[Codec] = None


def default_codec() -> Codec:
    global _default
    if _default is None:
        _default = Codec(0, 1 << 16)
    return _default


# --------------------------------------------------------------------------
# batch helpers on host values
# --------------------------------------------------------------------------
def marshal_batch(metas: Sequence[Optional[Metadata]], datas: Sequence[Optional[bytes]],
                  codec: Optional[Codec] = None):
    """[object.Marshal(m, d) ...] -> (list of Object | exception)."""
    codec = codec or default_codec()
    hb = pack_batch(metas, datas)
    res = codec.marshal(DeviceBatch.from_host(hb, codec.torch_device))
    out, off, st = res.host()
    objs: List[object] = []
    for i in range(len(metas)):
        if st[i] != OK:
            objs.append(_ERRORS.get(int(st[i]), HonuCodecError)(f"status {int(st[i])}"))
        else:
            objs.append(Object(bytes(out[int(off[i]):int(off[i + 1])])))
    return objs


def decode_batch(objs: Sequence[bytes], codec: Optional[Codec] = None):
    """[(meta|exc, data|exc, tombstone)] for each object, decoded on the GPU."""
    codec = codec or default_codec()
    n = len(objs)
    off = np.zeros(n + 1, np.uint64)
    buf = bytearray()
    for i, o in enumerate(objs):
        off[i] = len(buf)
        buf.extend(o)
    off[n] = len(buf)
    arena = np.frombuffer(bytes(buf) or b"\0", np.uint8)
    rec = _dev_bytes(arena, codec.torch_device)
    rec_off = _dev_bytes(off, codec.torch_device)
    d = codec.decode(rec, rec_off, n, rec_bytes=len(buf))
    meta, info, acl, reg, _, _ = d.host()
    out = []
    for i in range(n):
        ms, ds = int(info[i]["meta_status"]), int(info[i]["data_status"])
        m = unpack_row(meta[i], arena, acl, reg) if ms == OK else _ERRORS.get(ms, HonuCodecError)()
        if ds == OK:
            ln = int(info[i]["data_len"])
            o = int(info[i]["data_off"])
            data = bytes(arena[o:o + ln]) if ln else None
        else:
            data = _ERRORS.get(ds, HonuCodecError)()
        out.append((m, data, bool(info[i]["tombstone"])))
    return out


# --------------------------------------------------------------------------
# per-record mirror of the reference API
# --------------------------------------------------------------------------
def Marshal(meta: Optional[Metadata], data: Optional[bytes]) -> "Object":
    (r,) = marshal_batch([meta], [data])
    if isinstance(r, Exception):
        raise r
    return r


class Object(bytes):
    """object.Object: the encoded record bytes."""

    def StorageVersion(self) -> int:  # object.go:47-52
        return self[0] if len(self) else 0

    def _decoded(self):
        return decode_batch([bytes(self)])[0]

    def Metadata(self) -> Metadata:  # object.go:66-83
        m, _, _ = self._decoded()
        if isinstance(m, Exception):
            raise m
        return m

    def Data(self) -> Optional[bytes]:  # object.go:85-99
        _, d, _ = self._decoded()
        if isinstance(d, Exception):
            raise d
        return d

    def Tombstone(self) -> bool:  # object.go:103-112
        return self._decoded()[2]

    def Key(self) -> bytes:  # object.go:57-64 -> keys.New (keys/keys.go:42-51)
        codec = default_codec()
        arena = np.frombuffer(bytes(self) or b"\0", np.uint8)
        rec = _dev_bytes(arena, codec.torch_device)
        rec_off = _dev_bytes(np.array([0, len(self)], np.uint64), codec.torch_device)
        d = codec.decode(rec, rec_off, 1, rec_bytes=len(self))
        keys, st = codec.keys(d)
        s = int(_to_host(st, 4, np.int32)[0])
        raise_status(s)
        return bytes(_to_host(keys, 29, np.uint8))
