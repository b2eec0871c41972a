"""Corpora shared by the GPU parity tests and the CPU oracle tests (the
latter also run against the ASan/UBSan oracle build): the reference's decoder
error vectors, truncations and byte flips of valid records, structure-aware
mutants, and random Metadata."""
import numpy as np

from fixtures import load_object_fixture, py_uvarint
from honu_amd.metadata import pack_batch
from honu_amd.workload import gen_host_batch


def _tail_record(tail):
    return b"\x01\x00" + tail


def malformed_corpus(oracle_lib, seed=5):
    """Reference decoder vectors + truncations + byte flips of valid records."""
    rng = np.random.default_rng(seed)
    base = b"\x01" + bytes(32) + b"\x00\x00\x00" + bytes(32) + b"\x07"
    objs = [b"", b"\x01", b"\x01\x00", b"\x01\x00\x00", b"\x01\x80\x01", b"\x02\x00\x00",
            b"\x01\x00\xf2", b"\x01\x05\x00\x00", b"\x01" + b"\xff" * 9 + b"\x01\x00",
            _tail_record(b"\x01"), _tail_record(b"\x01" + bytes(5)),
            _tail_record(base + py_uvarint(2**45 + 1)), _tail_record(base + py_uvarint(2**45)),
            _tail_record(base + b"\x00" + py_uvarint(2**46 + 1)),
            _tail_record(base + b"\x00\x01\xff\xff\xff\xff\x7f" + bytes(7)),
            _tail_record(base + b"\x00\x01\xff\xff\xff\xff\xff\x01" + bytes(7))]
    for fr in (b"", b"\xff\xff", b"\xff\x12\x23\x42\xf2\x21", b"\x00", b"\x05abc",
               b"\xff" * 9 + b"\x7f", b"\xff" * 9 + b"\x01", b"\xff" * 8 + b"\x7f",
               b"\xff" * 7 + b"\x7f"):
        objs.append(_tail_record(b"\x01" + bytes(32) + b"\x00\x00" + fr))
    hb = gen_host_batch(9, "small", 0, 24)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    valid = [rec[int(off[i]):int(off[i + 1])].tobytes() for i in range(24)]
    meta, _ = load_object_fixture()
    fx = oracle_lib.marshal_batch(pack_batch([meta], [b"xyz"]))[0].tobytes()
    valid.append(fx)
    for v in valid[:4] + [fx]:  # every truncation point of the metadata tail
        for cut in range(0, len(v), 1 if len(v) < 2000 else 7):
            objs.append(v[:cut])
    for v in valid:
        for _ in range(40):
            b = bytearray(v)
            for _k in range(int(rng.integers(1, 4))):
                pos = int(rng.integers(0, len(b)))
                b[pos] = int(rng.integers(0, 256))
            objs.append(bytes(b))
    for _ in range(200):
        objs.append(rng.integers(0, 256, int(rng.integers(0, 64)), dtype=np.uint8).tobytes())
    return objs



def mutant_corpus(oracle_lib, n=20000, seed=2024):
    """n structure-aware mutants of valid Small records: byte flips, varint
    bytes rewritten to 0x80/0xff/0x00/0x01, insertions, deletions and
    truncations inside the Metadata tail. Returns (arena, off)."""
    rng = np.random.default_rng(seed)
    hb = gen_host_batch(55, "small", 0, 400)
    rec, off, _ = oracle_lib.marshal_batch(hb)
    valid = [rec[int(off[i]):int(off[i + 1])].tobytes() for i in range(400)]
    objs = []
    for k in range(n):
        v = bytearray(valid[k % 400])
        hdr = 1 + len(py_uvarint(int(hb.payload_off[k % 400 + 1] - hb.payload_off[k % 400])))
        tail0 = hdr + int(hb.payload_off[k % 400 + 1] - hb.payload_off[k % 400])
        kind = k % 5
        pos = int(rng.integers(tail0, len(v)))
        if kind == 0:
            v[pos] ^= int(rng.integers(1, 256))
        elif kind == 1:
            v[pos] = int(rng.choice([0x80, 0xFF, 0x00, 0x01]))
        elif kind == 2:
            v[pos:pos] = rng.integers(0, 256, int(rng.integers(1, 4)), dtype=np.uint8).tobytes()
        elif kind == 3:
            del v[pos:pos + int(rng.integers(1, 4))]
        else:
            v = v[:pos]
        objs.append(bytes(v))
    o = np.zeros(len(objs) + 1, np.uint64)
    o[1:] = np.cumsum([len(x) for x in objs])
    arena = np.frombuffer(b"".join(objs), np.uint8)
    return arena, o


def random_metas(n, seed):
    """n random Metadata (every sub-struct nil or present, frames around the
    varint length boundaries, nil ACL entries, every integer width) and
    payloads."""
    from honu_amd.metadata import (AccessControl, Compression, Encryption, Metadata, Publisher,
                                   Scalar, SchemaVersion, Version)
    rng = np.random.default_rng(seed)
    ri = lambda bits: int(rng.integers(0, 2**bits, dtype=np.uint64)) if bits < 64 else \
        int(rng.integers(0, 2**63)) * 2 + int(rng.integers(0, 2))  # noqa: E731
    rs = lambda: int(rng.integers(-2**62, 2**62)) * int(rng.choice([1, 2]))  # noqa: E731
    ln = lambda: int(rng.choice([0, 1, 5, 127, 128, 129, int(rng.integers(0, 400))]))  # noqa: E731
    p = lambda q: rng.random() < q  # noqa: E731
    metas, datas = [], []
    for _ in range(n):
        w = lambda: int(rng.choice([7, 14, 21, 28, 32]))  # noqa: E731
        metas.append(Metadata(
            ObjectID=rng.bytes(16), CollectionID=rng.bytes(16),
            Version=Version(Scalar(ri(w()), ri(int(rng.choice([7, 35, 63, 64])))), ri(w()),
                            Scalar(ri(w()), ri(40)) if p(.5) else None, p(.5), rs()) if p(.8) else None,
            Schema=SchemaVersion("x" * ln(), ri(w()), ri(w()), ri(w())) if p(.7) else None,
            MIME="m" * ln(), Owner=rng.bytes(16), Group=rng.bytes(16),
            Permissions=int(rng.integers(0, 256)),
            ACL=[AccessControl(rng.bytes(16), int(rng.integers(0, 256))) if p(.9) else None
                 for _ in range(int(rng.integers(0, 40)))] or None,
            WriteRegions=[ri(w()) for _ in range(int(rng.integers(0, 13)))] if p(.8) else None,
            Publisher=Publisher(rng.bytes(16), rng.bytes(16), rng.bytes(ln()) or None, "u" * ln())
            if p(.7) else None,
            Encryption=Encryption("k" * ln(), rng.bytes(ln()) or None, rng.bytes(ln()) or None,
                                  rng.bytes(ln()) or None, int(rng.integers(0, 256)),
                                  int(rng.integers(0, 256)), int(rng.integers(0, 256))) if p(.7) else None,
            Compression=Compression(int(rng.integers(0, 256)), rs()) if p(.7) else None,
            Flags=int(rng.integers(0, 256)), Created=rs() if p(.9) else 0, Modified=rs() if p(.9) else 0))
        datas.append(rng.bytes(int(rng.integers(0, 3000))) if p(.9) else None)
    return metas, datas
