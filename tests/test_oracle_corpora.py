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
from honu_amd.metadata import (ACL_INPLACE, REGIONS_INPLACE, SPAN_FIELDS, normalize, pack_batch,
                               unpack_row)

# both forms of the decoded lists: in place (the default: ACL and region lists)
# and the tables (context params acl_inplace 0, regions_inplace 0)
FORMS = pytest.mark.parametrize("inplace", [True, False], ids=["lists_inplace", "lists_table"])


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
    rinpl = (meta["present"] & REGIONS_INPLACE) != 0
    assert not (rinpl & (meta["regions_count"] == 0)).any()  # only non-empty lists
    assert (rinpl[ok] == (inplace & (meta["regions_count"][ok] > 0))).all()
    acl_end = (meta["acl_off"] + meta["acl_count"]).astype(np.int64)
    reg_end = (meta["regions_off"] + meta["regions_count"]).astype(np.int64)
    assert (acl_end[tab] <= int(tot[0])).all() and (reg_end[ok & ~rinpl] <= int(tot[1])).all()
    assert not inplace or int(tot[1]) == 0
    # an in-place region list: inside its record (>= 1 byte per uvarint)
    for i in np.flatnonzero(ok & rinpl):
        a, n = int(meta[i]["regions_off"]), int(meta[i]["regions_count"])
        assert a >= beg[i] and a + n <= end[i], i
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
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(rec, off, True, inplace, inplace)
    assert {0, 1, 2, 3, 4, 5, 6, 7, 8} <= set(info["meta_status"].tolist())
    _check_bounds(meta, info, tot, off, rec, inplace)


@FORMS
def test_mutant_corpus(oracle_lib, inplace):
    rec, off = mutant_corpus(oracle_lib)
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(rec, off, True, inplace, inplace)
    assert len(set(info["meta_status"].tolist())) >= 5
    _check_bounds(meta, info, tot, off, rec, inplace)


@FORMS
def test_random_metadata_round_trip(oracle_lib, inplace):
    metas, datas = random_metas(1500, 77)
    out, off, st = oracle_lib.marshal_batch(pack_batch(metas, datas))
    assert (st == 0).all()
    meta, info, acl, reg, data, tot = oracle_lib.decode_batch(out, off, True, inplace, inplace)
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


def test_carried_acl_length(oracle_lib):
    """HONU_ACL_SIZED rows (the list's encoded length carried in acl_bytes,
    include/honu_codec.h): honest rows encode exactly as rows without the bit;
    a length outside [count, 18 count] is refused by the size pass (size 0),
    one inside it but wrong sizes the record by the carried length and fails
    with HONU_ERR_INPUT (range left unwritten by the oracle)."""
    from honu_amd.metadata import ACL_SIZED
    metas, datas = random_metas(300, 5)
    hb = pack_batch(metas, datas)
    sized = (hb.meta["present"] & ACL_SIZED) != 0
    assert sized.any() and (hb.meta["acl_count"][sized] > 0).all()
    out, off, st = oracle_lib.marshal_batch(hb)
    hb2 = pack_batch(metas, datas)
    hb2.meta["present"] &= ~np.uint32(ACL_SIZED)
    out2, off2, st2 = oracle_lib.marshal_batch(hb2)
    assert (st == 0).all() and np.array_equal(off, off2) and out.tobytes() == out2.tobytes()
    i, j = np.flatnonzero(sized)[:2]
    na = int(hb.meta[i]["acl_count"])
    hb.meta[i]["acl_bytes"] = int(hb.meta[i]["acl_bytes"]) + (1 if int(hb.meta[i]["acl_bytes"]) < 18 * na else -1)
    hb.meta[j]["acl_bytes"] = 18 * int(hb.meta[j]["acl_count"]) + 1
    out3, off3, st3 = oracle_lib.marshal_batch(hb)
    assert st3[i] == 10 and st3[j] == 10 and (np.delete(st3, [i, j]) == 0).all()
    d = np.diff(off3.astype(np.int64)) - np.diff(off.astype(np.int64))
    assert abs(d[i]) == 1 and d[j] == -int(np.diff(off.astype(np.int64))[j])
    assert not out3[int(off3[i]):int(off3[i + 1])].any()
