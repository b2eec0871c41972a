"""The CPU oracle over the adversarial corpora the GPU parity tests use (the
reference's decoder error vectors, truncations, byte flips, 20,000
structure-aware mutants, random Metadata), with invariants that hold whatever
the bytes: every status is a Go sentinel, a record that decodes OK has every
span, the payload and the ACL/region tables inside its own bytes / the
batch's totals, and random Metadata round-trip. tests/test_sanitizers.py runs
this file again against the ASan + UBSan build of the oracle."""
import numpy as np
import pytest

from corpora import malformed_corpus, mutant_corpus, random_metas
from honu_amd.metadata import ACL_INPLACE, SPAN_FIELDS, normalize, pack_batch, unpack_row

# both forms of the decoded ACL lists: in place (the default) and the table
FORMS = pytest.mark.parametrize("inplace", [True, False], ids=["acl_inplace", "acl_table"])


def _arena(objs):
    off = np.zeros(len(objs) + 1, np.uint64)
    off[1:] = np.cumsum([len(o) for o in objs])
    return np.frombuffer(b"".join(objs) + b"\0", np.uint8)[: int(off[-1])], off


def _check_bounds(meta, info, tot, off, rec=None, inplace=True):
    ok = info["meta_status"] == 0
    beg, end = off[:-1].astype(np.int64), off[1:].astype(np.int64)
    for f in SPAN_FIELDS:
        o, ln = meta[f]["off"].astype(np.int64), meta[f]["len"].astype(np.int64)
        inside = (ln == 0) | ((o >= beg) & (o + ln <= end))
        assert inside[ok].all(), f
    inpl = (meta["present"] & ACL_INPLACE) != 0
    assert inplace or not inpl.any()
    tab = ok & ~inpl
    acl_end = (meta["acl_off"] + meta["acl_count"]).astype(np.int64)
    reg_end = (meta["regions_off"] + meta["regions_count"]).astype(np.int64)
    assert (acl_end[tab] <= int(tot[0])).all() and (reg_end[ok] <= int(tot[1])).all()
    # an in-place list: inside its record, every entry flag 1 (18 bytes each)
    for i in np.flatnonzero(ok & inpl):
        a, n = int(meta[i]["acl_off"]), int(meta[i]["acl_count"])
        assert n > 0 and a >= beg[i] and a + 18 * n <= end[i], i
        if rec is not None:
            assert (rec[a:a + 18 * n:18] == 1).all(), i
    dok = info["data_status"] == 0
    assert (info["data_off"][dok] + info["data_len"][dok] <= int(tot[2])).all()
    assert set(info["meta_status"].tolist()) <= set(range(10))


@FORMS
def test_malformed_corpus(oracle_lib, inplace):
    rec, off = _arena(malformed_corpus(oracle_lib))
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(rec, off, True, inplace)
    assert {0, 1, 2, 3, 4, 5, 6, 7, 8} <= set(info["meta_status"].tolist())
    _check_bounds(meta, info, tot, off, rec, inplace)


@FORMS
def test_mutant_corpus(oracle_lib, inplace):
    rec, off = mutant_corpus(oracle_lib)
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(rec, off, True, inplace)
    assert len(set(info["meta_status"].tolist())) >= 5
    _check_bounds(meta, info, tot, off, rec, inplace)


@FORMS
def test_random_metadata_round_trip(oracle_lib, inplace):
    metas, datas = random_metas(1500, 77)
    out, off, st = oracle_lib.marshal_batch(pack_batch(metas, datas))
    assert (st == 0).all()
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(out, off, True, inplace)
    assert (info["meta_status"] == 0).all() and (info["data_status"] == 0).all()
    _check_bounds(meta, info, tot, off, out, inplace)
    if inplace:  # random_metas holds lists with and without nil entries
        inpl = (meta["present"] & ACL_INPLACE) != 0
        assert inpl.any() and ((meta["acl_count"] > 0) & ~inpl).any()
    for i in range(0, 1500, 5):
        assert unpack_row(meta[i], out, acl, reg) == normalize(metas[i]), i
        d = datas[i] or b""
        o, ln = int(info[i]["data_off"]), int(info[i]["data_len"])
        assert data[o:o + ln].tobytes() == d
