"""The read feed (include/honu_codec.h, "Read feed"): batches of stored
records — what a bbolt cursor scan yields (iterator/cursor.go:31-38) — are
appended into pinned host memory and decoded on the GPU while the next batch
fills. Results are numpy views of the feed's pinned buffers, valid until the
slot is refilled (one more submit)."""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Optional

import numpy as np

from . import _lib
from .metadata import ACL_DTYPE, INFO_DTYPE, META_DTYPE

HEADERS = 1  # HONU_FEED_HEADERS


class _Result(C.Structure):
    _fields_ = [("n", C.c_uint64), ("records", C.c_void_p), ("rec_off", C.c_void_p),
                ("meta", C.c_void_p), ("info", C.c_void_p), ("acl", C.c_void_p),
                ("acl_n", C.c_uint64), ("regions", C.c_void_p), ("regions_n", C.c_uint64),
                ("keys", C.c_void_p), ("key_status", C.c_void_p),
                ("acl_needed", C.c_uint64), ("regions_needed", C.c_uint64)]


def _view(ptr, count, dtype):
    dtype = np.dtype(dtype)
    if not ptr or not count:
        return np.zeros(0, dtype)
    buf = (C.c_uint8 * (count * dtype.itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype)


@dataclass
class FeedResult:
    records: np.ndarray          # the batch's records arena (spans index it)
    rec_off: np.ndarray          # n + 1
    meta: Optional[np.ndarray]   # honu_meta rows (None in headers mode)
    info: np.ndarray             # honu_record_info
    acl: Optional[np.ndarray]
    regions: Optional[np.ndarray]
    keys: Optional[np.ndarray]   # (n, 29) uint8
    key_status: Optional[np.ndarray]
    acl_needed: int = 0          # table entries the batch needed (> len(acl): overflow)
    regions_needed: int = 0


class RecordFeed:
    def __init__(self, device: int = 0, batch_records: int = 1 << 16,
                 batch_bytes: int = 64 << 20, headers_only: bool = False):
        self.lib = _lib.load()
        err = _lib.I32(0)
        self.headers_only = headers_only
        self.feed = self.lib.honu_feed_create(device, batch_records, batch_bytes,
                                              HEADERS if headers_only else 0, C.byref(err))
        if not self.feed:
            _lib.check(err.value or -4, "honu_feed_create")

    def close(self):
        if getattr(self, "feed", None):
            self.lib.honu_feed_destroy(self.feed)
            self.feed = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def append(self, rec: bytes) -> int:
        """0 on success, HONU_ERR_CAPACITY (9) when the batch is full."""
        st = self.lib.honu_feed_append(self.feed, rec, len(rec))
        if st not in (0, 9):
            _lib.check(st, "honu_feed_append")
        return st

    def append_batch(self, arena: np.ndarray, off: np.ndarray, first: int = 0):
        """Append records first.. of a CSR arena until the batch is full.
        Returns (status, records appended)."""
        n = len(off) - 1 - first
        got = C.c_uint64(0)
        st = self.lib.honu_feed_append_batch(self.feed, arena.ctypes.data,
                                             off[first:].ctypes.data if n else None, n,
                                             C.byref(got))
        if st not in (0, 9):
            _lib.check(st, "honu_feed_append_batch")
        return st, got.value

    @property
    def pending(self) -> int:
        return self.lib.honu_feed_pending(self.feed)

    def submit(self) -> int:
        t = C.c_uint64(0)
        _lib.check(self.lib.honu_feed_submit(self.feed, C.byref(t)), "honu_feed_submit")
        return t.value

    def wait(self, ticket: int) -> FeedResult:
        r = _Result()
        _lib.check(self.lib.honu_feed_wait(self.feed, ticket, C.byref(r)), "honu_feed_wait")
        n = r.n
        off = _view(r.rec_off, n + 1, np.uint64)
        nbytes = int(off[n]) if n else 0
        hdr = self.headers_only
        return FeedResult(
            _view(r.records, nbytes, np.uint8), off,
            None if hdr else _view(r.meta, n, META_DTYPE), _view(r.info, n, INFO_DTYPE),
            None if hdr else _view(r.acl, r.acl_n, ACL_DTYPE),
            None if hdr else _view(r.regions, r.regions_n, np.uint32),
            None if hdr else _view(r.keys, 29 * n, np.uint8).reshape(n, 29),
            None if hdr else _view(r.key_status, n, np.int32),
            int(r.acl_needed), int(r.regions_needed))


# --------------------------------------------------------------------------
# Write feed (include/honu_codec.h, "Write feed"): object.Marshal for a
# store's Put path, batched through pinned memory and the GPU encoder.
# --------------------------------------------------------------------------
class _PutResult(C.Structure):
    _fields_ = [("n", C.c_uint64), ("records", C.c_void_p), ("rec_off", C.c_void_p),
                ("status", C.c_void_p)]


@dataclass
class PutResult:
    records: np.ndarray   # encoded records back to back (views of pinned memory)
    rec_off: np.ndarray   # n + 1
    status: np.ndarray    # n, honu_status per record

    def objects(self):
        """Marshal's result per record: bytes, or the status code on failure."""
        return [int(s) if s else self.records[int(self.rec_off[i]):int(self.rec_off[i + 1])].tobytes()
                for i, s in enumerate(self.status)]


class PutFeed:
    """object.Marshal(meta, data) over batches: append() one record (a
    metadata.Metadata mirror or None + payload bytes or None), append_batch()
    a whole host batch (HostBatch), submit() a batch, wait() for its records.
    Results are views of pinned buffers, valid until the slot is refilled."""

    def __init__(self, device: int = 0, batch_records: int = 1 << 16, batch_bytes: int = 64 << 20):
        self.lib = _lib.load()
        err = _lib.I32(0)
        self.feed = self.lib.honu_put_feed_create(device, batch_records, batch_bytes, C.byref(err))
        if not self.feed:
            _lib.check(err.value or -4, "honu_put_feed_create")

    def close(self):
        if getattr(self, "feed", None):
            self.lib.honu_put_feed_destroy(self.feed)
            self.feed = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def append(self, meta, data: Optional[bytes]) -> int:
        """0 on success, HONU_ERR_CAPACITY (9) when the batch is full."""
        from .metadata import pack_batch
        hb = pack_batch([meta], [data])
        d = bytes(data) if data else b""
        st = self.lib.honu_put_feed_append(
            self.feed, hb.meta.ctypes.data, hb.var.ctypes.data, len(hb.var),
            hb.acl.ctypes.data if len(hb.acl) else None, len(hb.acl),
            hb.regions.ctypes.data if len(hb.regions) else None, len(hb.regions),
            d or None, len(d))
        if st not in (0, 9):
            _lib.check(st, "honu_put_feed_append")
        return st

    def append_batch(self, hb, first: int = 0):
        """Append records first.. of a HostBatch until the batch is full.
        Returns (status, records appended)."""
        n = len(hb) - first
        got = C.c_uint64(0)
        st = self.lib.honu_put_feed_append_batch(
            self.feed, hb.meta[first:].ctypes.data if n else None, n,
            hb.var.ctypes.data, len(hb.var), hb.acl.ctypes.data if len(hb.acl) else None,
            len(hb.acl), hb.regions.ctypes.data if len(hb.regions) else None, len(hb.regions),
            hb.payload.ctypes.data, hb.payload_off[first:].ctypes.data, C.byref(got))
        if st not in (0, 9):
            _lib.check(st, "honu_put_feed_append_batch")
        return st, got.value

    @property
    def pending(self) -> int:
        return self.lib.honu_put_feed_pending(self.feed)

    def submit(self) -> int:
        t = C.c_uint64(0)
        _lib.check(self.lib.honu_put_feed_submit(self.feed, C.byref(t)), "honu_put_feed_submit")
        return t.value

    def wait(self, ticket: int) -> PutResult:
        r = _PutResult()
        _lib.check(self.lib.honu_put_feed_wait(self.feed, ticket, C.byref(r)), "honu_put_feed_wait")
        n = r.n
        off = _view(r.rec_off, n + 1, np.uint64)
        return PutResult(_view(r.records, int(off[n]) if n else 0, np.uint8), off,
                         _view(r.status, n, np.int32))
