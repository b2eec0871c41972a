"""TEST INFRASTRUCTURE ONLY: ctypes binding of the CPU oracle (libhonu_oracle.so).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / CPU baseline; honu_amd never does.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# HONU_ORACLE_LIB: an alternative build of the same oracle (the ASan/UBSan
# one, oracle/Makefile `sanitize`)
LIB_PATH = os.environ.get("HONU_ORACLE_LIB") or os.path.join(_HERE, "libhonu_oracle.so")
_lib = None
P, U64, I32 = C.c_void_p, C.c_uint64, C.c_int32


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        build()
    lib = C.CDLL(LIB_PATH)
    protos = {
        "oracle_put_uvarint": (C.c_int, [P, U64]),
        "oracle_uvarint": (C.c_int, [P, U64, P]),
        "oracle_put_varint": (C.c_int, [P, C.c_int64]),
        "oracle_varint": (C.c_int, [P, U64, P]),
        "oracle_size_bound": (C.c_int64, [C.c_int, P]),
        "oracle_marshal": (C.c_int, [P, P, U64, P, U64, P, U64, P, U64, P, U64, P]),
        "oracle_decode": (None, [P, U64, U64, P, P, P, U64, P, U64, P, P, C.c_int]),
        "oracle_marshal_batch": (C.c_int, [P, P, U64, P, U64, P, U64, P, P, U64, P, U64, P, P]),
        "oracle_decode_batch": (C.c_int, [P, P, U64, P, P, P, U64, P, U64, P, U64, P, C.c_int]),
        "oracle_key": (C.c_int, [P, I32, P]),
        "oracle_field_size": (C.c_int64, [U64]),
        "oracle_index_size": (C.c_int64, [P]),
        "oracle_collection_size": (C.c_int64, [P, P, P]),
        "oracle_system_marshal_batch": (C.c_int, [P, P, U64, P, U64, P, U64, P, U64, U64, P, U64,
                                                  P, P]),
        "oracle_system_decode_batch": (C.c_int, [P, P, U64, P, P, P, U64, P, U64, P, U64, P]),
        "oracle_collection_decode_batch": (C.c_int, [P, P, U64, P, P, P, U64, P, U64, P, U64, P]),
    }
    for name, (res, args) in protos.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _p(a):
    return 0 if a is None else a.ctypes.data


def put_uvarint(x: int) -> bytes:
    buf = (C.c_uint8 * 10)()
    k = load().oracle_put_uvarint(buf, x)
    return bytes(buf[:k])


def uvarint(b: bytes):
    out = C.c_uint64(0)
    k = load().oracle_uvarint(b, len(b), C.byref(out))
    return out.value, k


def put_varint(x: int) -> bytes:
    buf = (C.c_uint8 * 10)()
    k = load().oracle_put_varint(buf, x)
    return bytes(buf[:k])


def varint(b: bytes):
    out = C.c_int64(0)
    k = load().oracle_varint(b, len(b), C.byref(out))
    return out.value, k


def size_bound(which: int, row) -> int:
    row = np.ascontiguousarray(row)
    return load().oracle_size_bound(which, _p(row))


def marshal_batch(hb):
    """(records arena, out_off[n+1], status[n]) for a honu_amd.metadata.HostBatch."""
    lib = load()
    n = len(hb.meta)
    out_off = np.zeros(n + 1, np.uint64)
    status = np.zeros(n, np.int32)
    lib.oracle_marshal_batch(_p(hb.meta), _p(hb.var), len(hb.var), _p(hb.acl), len(hb.acl),
                             _p(hb.regions), len(hb.regions), _p(hb.payload), _p(hb.payload_off),
                             n, None, 0, _p(out_off), _p(status))
    total = int(out_off[n])
    out = np.zeros(max(total, 1), np.uint8)
    lib.oracle_marshal_batch(_p(hb.meta), _p(hb.var), len(hb.var), _p(hb.acl), len(hb.acl),
                             _p(hb.regions), len(hb.regions), _p(hb.payload), _p(hb.payload_off),
                             n, _p(out), total, _p(out_off), _p(status))
    return out[:total], out_off, status


def forms(acl_inplace: bool = True, regions_inplace: bool = True) -> int:
    """The oracle's `forms` bits (honu_oracle.h ORACLE_*_INPLACE)."""
    return (1 if acl_inplace else 0) | (2 if regions_inplace else 0)


def decode_batch(rec: np.ndarray, rec_off: np.ndarray, materialize: bool = False,
                 acl_inplace: bool = True, regions_inplace: bool = True):
    """(meta rows, info, acl table, region table, data arena | None, totals[3]).

    acl_inplace (the product's default, context param "acl_inplace"): an ACL
    list whose entries are all present comes back in place (HONU_ACL_INPLACE,
    acl_off absolute in `rec`), only lists with a nil entry in the table.
    regions_inplace (the default, context param "regions_inplace"): every
    non-empty region list comes back in place (HONU_REGIONS_INPLACE,
    regions_off absolute in `rec`), the region table stays empty."""
    from honu_amd.metadata import ACL_DTYPE, INFO_DTYPE, META_DTYPE
    lib = load()
    n = len(rec_off) - 1
    rec = np.ascontiguousarray(rec, np.uint8)
    if rec.size == 0:
        rec = np.zeros(1, np.uint8)
    rec_off = np.ascontiguousarray(rec_off, np.uint64)
    nbytes = int(rec_off[-1]) if n >= 0 else 0
    meta = np.zeros(max(n, 1), META_DTYPE)
    info = np.zeros(max(n, 1), INFO_DTYPE)
    acl = np.zeros(nbytes + 1, ACL_DTYPE)  # lazily zeroed; a nil entry is 1 byte
    reg = np.zeros(nbytes + 1, np.uint32)
    data = np.zeros(nbytes + 16 * n + 16, np.uint8) if materialize else None
    totals = np.zeros(3, np.uint64)
    lib.oracle_decode_batch(_p(rec), _p(rec_off), n, _p(meta), _p(info), _p(acl), len(acl),
                            _p(reg), len(reg), _p(data), 0 if data is None else len(data),
                            _p(totals), forms(acl_inplace, regions_inplace))
    return (meta[:n], info[:n], acl[: int(totals[0])], reg[: int(totals[1])],
            None if data is None else data[: int(totals[2])], totals)


class CycleWorkspace:
    """Output arrays of one marshal + materialising decode of a HostBatch,
    allocated once (tables sized by the batch's ACL entry and region counts,
    the data arena by its payload bytes) so that a timing loop measures the
    codec, not allocation and page faults. cycle() re-encodes the batch into
    `out` and decodes it into the tables; returns the encoded bytes."""

    def __init__(self, hb):
        from honu_amd.metadata import ACL_DTYPE, INFO_DTYPE, META_DTYPE
        self.hb = hb
        self.lib = load()
        n = len(hb.meta)
        self.n = n
        self.out_off = np.zeros(n + 1, np.uint64)
        self.status = np.zeros(max(n, 1), np.int32)
        self._marshal(None, 0)  # size pass: out_off
        self.total = int(self.out_off[n])
        self.out = np.zeros(max(self.total, 1), np.uint8)
        self.meta = np.zeros(max(n, 1), META_DTYPE)
        self.info = np.zeros(max(n, 1), INFO_DTYPE)
        nacl = int(hb.meta["acl_count"].astype(np.int64).sum()) if n else 0
        nreg = int(hb.meta["regions_count"].astype(np.int64).sum()) if n else 0
        self.acl = np.zeros(nacl + 1, ACL_DTYPE)
        self.reg = np.zeros(nreg + 1, np.uint32)
        pay = np.diff(np.asarray(hb.payload_off, np.int64)) if n else np.zeros(0, np.int64)
        self.data = np.zeros(int(((pay + 15) // 16 * 16).sum()) + 16, np.uint8)
        self.totals = np.zeros(3, np.uint64)
        for a in (self.out, self.meta, self.info, self.acl, self.reg, self.data):
            a.view(np.uint8).reshape(-1)[::4096] = 0  # fault the pages in before timing

    def _marshal(self, out, cap):
        hb = self.hb
        return self.lib.oracle_marshal_batch(
            _p(hb.meta), _p(hb.var), len(hb.var), _p(hb.acl), len(hb.acl), _p(hb.regions),
            len(hb.regions), _p(hb.payload), _p(hb.payload_off), self.n, _p(out), cap,
            _p(self.out_off), _p(self.status))

    def cycle(self) -> int:
        self._marshal(self.out, self.total)
        self.lib.oracle_decode_batch(_p(self.out), _p(self.out_off), self.n, _p(self.meta),
                                     _p(self.info), _p(self.acl), len(self.acl), _p(self.reg),
                                     len(self.reg), _p(self.data), len(self.data), _p(self.totals),
                                     forms())  # the product's default forms (lists in place)
        return self.total


def key(row, meta_status: int):
    out = (C.c_uint8 * 29)()
    row = np.ascontiguousarray(row)
    st = load().oracle_key(_p(row), meta_status, out)
    return st, bytes(out)


def system_marshal_batch(sb):
    """MarshalSystem over a honu_amd.system.SystemHostBatch -> (out, off, status)."""
    lib = load()
    n = len(sb.rows)
    out_off = np.zeros(n + 1, np.uint64)
    status = np.zeros(n, np.int32)
    args = (_p(sb.rows), _p(sb.var), len(sb.var), _p(sb.acl), len(sb.acl), _p(sb.regions),
            len(sb.regions), _p(sb.index), len(sb.index), n)
    lib.oracle_system_marshal_batch(*args, None, 0, _p(out_off), _p(status))
    total = int(out_off[n])
    out = np.zeros(max(total, 1), np.uint8)
    lib.oracle_system_marshal_batch(*args, _p(out), total, _p(out_off), _p(status))
    return out[:total], out_off, status


def system_decode_batch(rec: np.ndarray, rec_off: np.ndarray, headless: bool = False):
    """UnmarshalSystem(obj, &Collection{}) -> (rows, status, acl, regions, index, totals);
    headless: lani.Unmarshal(obj, &Collection{}) instead (store.go:367)."""
    from honu_amd.metadata import ACL_DTYPE
    from honu_amd.system import COLLECTION_DTYPE, INDEX_DTYPE
    lib = load()
    n = len(rec_off) - 1
    rec = np.ascontiguousarray(rec, np.uint8)
    if rec.size == 0:
        rec = np.zeros(1, np.uint8)
    rec_off = np.ascontiguousarray(rec_off, np.uint64)
    nbytes = int(rec_off[-1]) if n >= 0 else 0
    rows = np.zeros(max(n, 1), COLLECTION_DTYPE)
    status = np.zeros(max(n, 1), np.int32)
    acl = np.zeros(nbytes + 1, ACL_DTYPE)
    reg = np.zeros(nbytes + 1, np.uint32)
    idx = np.zeros(nbytes + 1, INDEX_DTYPE)
    totals = np.zeros(3, np.uint64)
    fn = lib.oracle_collection_decode_batch if headless else lib.oracle_system_decode_batch
    fn(_p(rec), _p(rec_off), n, _p(rows), _p(status), _p(acl), len(acl), _p(reg), len(reg),
       _p(idx), len(idx), _p(totals))
    return (rows[:n], status[:n], acl[: int(totals[0])], reg[: int(totals[1])],
            idx[: int(totals[2])], totals)


def collection_size(row, acl, index) -> int:
    """Collection.Size() (collection.go:81-135) of a packed row."""
    lib = load()
    row = np.ascontiguousarray(row)
    acl = np.ascontiguousarray(acl) if len(acl) else np.zeros(1, acl.dtype)
    index = np.ascontiguousarray(index) if len(index) else np.zeros(1, index.dtype)
    return lib.oracle_collection_size(_p(row), _p(acl), _p(index))


def index_size(row) -> int:
    return load().oracle_index_size(_p(np.ascontiguousarray(row)))


def field_size(name_len: int) -> int:
    return load().oracle_field_size(name_len)
