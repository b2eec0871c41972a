"""honu_amd — MI355X-native (gfx950) batch implementation of Honu's
object-record codec (rotationalio/honu pkg/store/object + lani + metadata).

The codec itself lives in libhonu_codec.so (HIP kernels + C ABI,
include/honu_codec.h). This package is the host-side mirror of the reference
interface: `metadata` (Go structs <-> batch rows) and `object` (Marshal,
Object.Metadata/Data/Tombstone/Key, and the batch Codec).
"""
from . import metadata  # noqa: F401
from .metadata import (AccessControl, Compression, Encryption, Metadata, Publisher, Scalar,  # noqa: F401
                       SchemaVersion, Version)


def __getattr__(name):  # object API loads the HIP library lazily
    if name in ("object", "Codec", "Marshal", "Object", "marshal_batch", "decode_batch"):
        import importlib
        _object = importlib.import_module(__name__ + ".object")
        return _object if name == "object" else getattr(_object, name)
    raise AttributeError(name)
