#!/usr/bin/env python3
"""Writes the committed golden batches under tests/golden/batches/ (test
infrastructure: the CPU oracle is the producer, the fixtures are data).

Each fixture is a batch of records with the outputs the reference semantics
give for it, as raw little-endian files plus a SHA-256 manifest:
  <name>.records.bin / .offsets.bin   encoded records (CSR, u64 offsets)
  <name>.rows.bin / .info.bin         decoded honu_meta rows / honu_record_info
  <name>.acl.bin / .regions.bin       decoded ACL / region tables
    (the default forms: ACL lists with every entry present returned in place,
    HONU_ACL_INPLACE, and every region list in place, HONU_REGIONS_INPLACE;
    only lists with a nil ACL entry in a table)
  <name>.rows_table.bin / .acl_table.bin / .regions_table.bin   the same rows
    and tables with every list in its table (context params acl_inplace 0,
    regions_inplace 0)
  totals (manifest): ACL entries, regions, data bytes of the default forms,
    then the table forms' ACL entries and regions
Encode fixtures regenerate their input from the seeded generator (or
tests/fixtures.py:extreme_metas); decode fixtures carry malformed records.

  python tests/make_golden_batches.py        # (re)write the fixtures
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)
OUT = os.path.join(HERE, "golden", "batches")

ENCODE = {  # name -> generator parameters
    "small64": {"seed": 101, "shape": "small", "first": 0, "n": 64},
    "medium8": {"seed": 103, "shape": "medium", "first": 7, "n": 8},
    "extreme40": {"extreme_metas": {"n": 40, "seed": 29}},
    "large4": {"seed": 105, "shape": "large", "first": 11, "n": 4},
    "mixed12": {"seed": 106, "shape": "mixed", "first": 3, "n": 12},
}


def encode_input(params):
    from honu_amd.metadata import pack_batch
    from honu_amd.workload import gen_host_batch
    if "extreme_metas" in params:
        from fixtures import extreme_metas
        return pack_batch(*extreme_metas(**params["extreme_metas"]))
    p = params
    return gen_host_batch(p["seed"], p["shape"], p["first"], p["n"])


def malformed_records():
    """The reference's decoder vectors, every 5th truncation of the fixture
    object, byte flips of generated records and random short records."""
    from fixtures import load_object_fixture, py_uvarint
    from honu_amd.metadata import pack_batch
    from oracle import oracle
    rng = np.random.default_rng(7)
    tail = lambda t: b"\x01\x00" + t  # noqa: E731
    base = b"\x01" + bytes(32) + b"\x00\x00\x00" + bytes(32) + b"\x07"
    objs = [b"", b"\x01", b"\x01\x00", b"\x01\x00\x00", b"\x01\x80\x01", b"\x02\x00\x00",
            b"\x01\x00\xf2", b"\x01\x05\x00\x00", b"\x01" + b"\xff" * 9 + b"\x01\x00",
            tail(b"\x01"), tail(base + py_uvarint(2**45 + 1)),
            tail(base + b"\x00\x01\xff\xff\xff\xff\x7f" + bytes(7))]
    for fr in (b"", b"\xff\xff", b"\xff\x12\x23\x42\xf2\x21", b"\x00", b"\x05abc",
               b"\xff" * 9 + b"\x7f", b"\xff" * 9 + b"\x01"):
        objs.append(tail(b"\x01" + bytes(32) + b"\x00\x00" + fr))
    meta, _ = load_object_fixture()
    fx = oracle.marshal_batch(pack_batch([meta], [b"xyz"]))[0].tobytes()
    objs += [fx[:cut] for cut in range(0, len(fx), 5)]
    from honu_amd.workload import gen_host_batch
    rec, off, _ = oracle.marshal_batch(gen_host_batch(104, "small", 0, 6))
    for i in range(6):
        v = rec[int(off[i]):int(off[i + 1])].tobytes()
        for _ in range(10):
            b = bytearray(v)
            for _k in range(int(rng.integers(1, 4))):
                b[int(rng.integers(0, len(b)))] = int(rng.integers(0, 256))
            objs.append(bytes(b))
    objs += [rng.integers(0, 256, int(rng.integers(0, 48)), dtype=np.uint8).tobytes()
             for _ in range(60)]
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    return np.frombuffer(b"".join(objs), np.uint8).copy(), off


def outputs(name):
    """{file suffix: bytes} of a fixture, produced by the oracle."""
    from oracle import oracle
    oracle.build()
    oracle.load()
    if name in ENCODE:
        rec, off, st = oracle.marshal_batch(encode_input(ENCODE[name]))
        assert (st == 0).all()
    else:
        rec, off = malformed_records()
    meta, info, acl, reg, _, tot = oracle.decode_batch(rec, off, False)
    tmeta, tinfo, tacl, treg, _, ttot = oracle.decode_batch(rec, off, False, acl_inplace=False,
                                                            regions_inplace=False)
    assert tinfo.tobytes() == info.tobytes() and len(reg) == 0
    return {"records": rec.tobytes(), "offsets": off.astype("<u8").tobytes(),
            "rows": meta.tobytes(), "info": info.tobytes(), "acl": acl.tobytes(),
            "regions": reg.astype("<u4").tobytes(), "rows_table": tmeta.tobytes(),
            "acl_table": tacl.tobytes(), "regions_table": treg.astype("<u4").tobytes()}, \
        [int(x) for x in tot] + [int(ttot[0]), int(ttot[1])]


NAMES = list(ENCODE) + ["malformed"]


def main():
    os.makedirs(OUT, exist_ok=True)
    manifest = {}
    for name in NAMES:
        files, tot = outputs(name)
        entry = {"params": ENCODE.get(name, {"malformed_records": "tests/make_golden_batches.py"}),
                 "totals": tot, "sha256": {}}
        for suf, data in files.items():
            with open(os.path.join(OUT, f"{name}.{suf}.bin"), "wb") as fh:
                fh.write(data)
            entry["sha256"][suf] = hashlib.sha256(data).hexdigest()
        manifest[name] = entry
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1, sort_keys=True)
    print("wrote", ", ".join(NAMES))


if __name__ == "__main__":
    main()
