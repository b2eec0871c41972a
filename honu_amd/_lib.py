"""ctypes binding of the C ABI (include/honu_codec.h) in libhonu_codec.so.

The library is loaded lazily and fails loudly: there is no CPU fallback for
any codec operation. torch is imported first so that its HIP runtime (same
soname, libamdhip64.so.7) is the one the library binds to; the process then
has a single HIP runtime shared by torch allocations/streams and our kernels.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("HONU_LIB_PATH") or os.path.join(_HERE, "libhonu_codec.so")  # override: A/B builds

_lib = None

P = C.c_void_p
U64 = C.c_uint64
I32 = C.c_int32

# name: (restype, argtypes)
_PROTOS = {
    "honu_abi_version": (C.c_uint32, []),
    "honu_sizeof_meta": (U64, []),
    "honu_sizeof_acl": (U64, []),
    "honu_sizeof_record_info": (U64, []),
    "honu_sizeof_collection": (U64, []),
    "honu_sizeof_index": (U64, []),
    "honu_status_string": (C.c_char_p, [I32]),
    "honu_last_error": (C.c_char_p, []),
    "honu_ctx_create": (P, [C.c_int, U64, C.POINTER(I32)]),
    "honu_ctx_destroy": (None, [P]),
    "honu_ctx_max_records": (U64, [P]),
    "honu_ctx_set_param": (I32, [P, C.c_char_p, C.c_int64]),
    "honu_ctx_get_param": (I32, [P, C.c_char_p, P]),
    "honu_ctx_reset": (I32, [P, P]),
    "honu_encode_sizes": (I32, [P, P, U64, P, U64, P, U64, P, U64, P, P, P]),
    "honu_exclusive_scan": (I32, [P, P, U64, P, P]),
    "honu_encode": (I32, [P, P, P, U64, P, U64, P, U64, P, P, U64, P, U64, P, P, P]),
    "honu_encode_records": (I32, [P, P, P, P, P, P, U64, P, U64, P, P, P]),
    "honu_encode_payloads": (I32, [P, P, P, U64, P, U64, P, P, P]),
    "honu_encode_records_units": (I32, [P, P, P, P, P, P, P, U64, P, U64, P, P, P]),
    "honu_encode_payloads_units": (I32, [P, P, P, U64, P, U64, P, P, P]),
    "honu_decode_tables": (I32, [P, P, U64, P, P, P, U64, P, U64, P, U64, P, P]),
    "honu_decode_payloads": (I32, [P, P, U64, P, P, P, P]),
    "honu_marshal_batch": (I32, [P, P, P, U64, P, U64, P, U64, P, P, U64, P, U64, P, P, P]),
    "honu_decode_parse": (I32, [P, P, P, U64, P, P, P]),
    "honu_decode_fill": (I32, [P, P, P, U64, P, P, P, U64, P, U64, P, U64, P, P]),
    "honu_decode_batch": (I32, [P, P, P, U64, P, P, P, U64, P, U64, P, U64, P, P]),
    "honu_decode_records": (I32, [P, P, P, U64, P, P, P, U64, P, U64, I32, U64, P, P]),
    "honu_decode_keys": (I32, [P, P, P, U64, P, P, P]),
    "honu_decode_headers": (I32, [P, P, P, U64, P, P]),
    "honu_decode_data": (I32, [P, P, P, U64, P, P, U64, P, P]),
    "honu_decode_data_place": (I32, [P, P, P, U64, P, U64, P, P]),
    "honu_decode_data_copy": (I32, [P, P, U64, P, P, P]),
    "honu_system_sizes": (I32, [P, P, U64, P, U64, P, U64, P, U64, U64, P, P, P]),
    "honu_system_encode": (I32, [P, P, P, P, P, P, U64, P, U64, P, P, P]),
    "honu_system_marshal_batch": (I32, [P, P, P, U64, P, U64, P, U64, P, U64, U64, P, U64, P, P,
                                        P]),
    "honu_system_decode_batch": (I32, [P, P, P, U64, P, P, P, U64, P, U64, P, U64, P, P]),
    "honu_collection_decode_batch": (I32, [P, P, P, U64, P, P, P, U64, P, U64, P, U64, P, P]),
    "honu_feed_create": (P, [C.c_int, U64, U64, C.c_uint32, C.POINTER(I32)]),
    "honu_feed_destroy": (None, [P]),
    "honu_feed_append": (I32, [P, P, U64]),
    "honu_feed_append_batch": (I32, [P, P, P, U64, C.POINTER(U64)]),
    "honu_feed_reserve": (P, [P, U64, C.POINTER(I32)]),
    "honu_feed_pending": (U64, [P]),
    "honu_feed_submit": (I32, [P, C.POINTER(U64)]),
    "honu_feed_wait": (I32, [P, U64, P]),
    "honu_put_feed_create": (P, [C.c_int, U64, U64, C.POINTER(I32)]),
    "honu_put_feed_destroy": (None, [P]),
    "honu_put_feed_append": (I32, [P, P, P, U64, P, U64, P, U64, P, U64]),
    "honu_put_feed_append_batch": (I32, [P, P, U64, P, U64, P, U64, P, U64, P, P, C.POINTER(U64)]),
    "honu_put_feed_pending": (U64, [P]),
    "honu_put_feed_submit": (I32, [P, C.POINTER(U64)]),
    "honu_put_feed_wait": (I32, [P, U64, P]),
    "honu_gen_totals": (None, [U64, I32, U64, U64, P]),
    "honu_gen_meta": (None, [U64, I32, U64, U64, P, P, P, P, P]),
    "honu_gen_payload_host": (None, [U64, U64, U64, P, P]),
    "honu_gen_payload": (I32, [P, U64, U64, U64, P, P, P]),
    "honu_digest_records": (I32, [P, P, P, P, U64, P, P]),
    "honu_digest_host": (U64, [P, U64]),
    "honu_hbm_probe": (I32, [P, I32, P, P, U64, C.c_uint32, P]),
    "honu_verify_decoded": (I32, [P, P, P, P, P, P, P, P, P, P, P, U64, P, P]),
    "honu_host_alloc": (P, [U64]),
    "honu_host_free": (None, [P]),
    "honu_device_alloc": (P, [U64]),
    "honu_device_free": (None, [P]),
    "honu_memcpy_h2d": (I32, [P, P, U64, P]),
    "honu_memcpy_d2h": (I32, [P, P, U64, P]),
    "honu_stream_sync": (I32, [P]),
}

EXPORTS = tuple(_PROTOS)


class HonuError(RuntimeError):
    pass


def load():
    """Load libhonu_codec.so (raises ImportError if it was not built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
            "(hipcc --offload-arch=gfx950). honu_amd has no CPU fallback.")
    try:  # share torch's HIP runtime (see module docstring)
        import torch  # noqa: F401
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    lib = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
    for name, (res, args) in _PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(status: int, what: str = ""):
    if status != 0:
        lib = load()
        msg = lib.honu_last_error().decode(errors="replace")
        raise HonuError(f"{what}: {lib.honu_status_string(status).decode()} ({status}) {msg}")


def ptr(x) -> int:
    """Device or host address of a torch tensor / numpy array (0 for None)."""
    if x is None:
        return 0
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if hasattr(x, "ctypes"):
        return x.ctypes.data
    return int(x)
