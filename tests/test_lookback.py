"""The single-launch decode's cross-tile scan (honu_amd/csrc/lookback.h) over
many launches: status words carry an 18-bit launch epoch kept in device memory
and are never cleared between launches, except when the epoch wraps. A wide
batch (many tiles) publishes words for every tile; 2^18 - 1 one-tile launches
then advance the epoch to its wrap, where the status array must be cleared: a
second wide batch with different counts decodes bit-exact only if no stale
word of the first one is taken for its own. Also: batches of 1..300 tiles in
a row, each checked against the oracle (every look-back window size).

Launches whose tiles all fit the resident waves take static tiles (one per
wave, no ticket atomics); larger ones take tickets. Every single-launch decode
ends in lookback.h lb_finish_blocks (a per-workgroup done count whose last
arrival advances the epoch, resets the ticket and clears misspec; lb_finish is
the scans' form). Both tile modes advance the same epoch: a test alternates
them, across an epoch wrap reached by static launches. Then the speculative
launches' recovery (late-failing records, nil ACL entries, a long unstaged list
under a capacity failure) and concurrent launches on two streams. The
speculation and tile tests run with three list forms (context params
acl_inplace and regions_inplace): both kinds of list in place, the default
(ACL lists whose speculated flags the launch gathers after its publish; tiles
with no table entry skip the look-back wait); every list in its table (ACL
flags checked by the table fill); and ACL lists in place with the regions in
their table (the round-5 default: every tile waits for its region offsets)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from honu_amd import object as hobj  # noqa: E402
from honu_amd.workload import gen_host_batch  # noqa: E402

EPOCHS = 1 << 18
FORMS = pytest.mark.parametrize("inplace", [1, 0, 2], ids=["lists_inplace", "lists_table", "regions_table"])
# form code -> (acl_inplace, regions_inplace)
FORM_PARAMS = {1: (1, 1), 0: (0, 0), 2: (1, 0)}


def _form(c, inplace):
    acl, reg = FORM_PARAMS[inplace]
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"acl_inplace", acl), "param")
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"regions_inplace", reg), "param")


def _oracle(oracle_lib, rec, off, inplace, materialize=False):
    acl, reg = FORM_PARAMS[inplace]
    return oracle_lib.decode_batch(rec, off, materialize, bool(acl), bool(reg))


def _speculative(c):
    """The single-launch decode with speculation on in every form (speculate
    1; the default 2 leaves the zero-copy in-place forms without it)."""
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"record_variant", 6), "param")
    hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"speculate", 1), "param")


def _nil_at(metas, datas, k, where):
    """k (meta, data) pairs from the random corpus whose ACL list is 40
    entries long with nil entries at the positions `where`. Mid-list nils
    (20) are only seen by the flag burst, so a speculative launch
    misspeculates on them; nils among the first entries (the walk's window
    holds them) or the last few (the window after the list) are caught by the
    walk itself (win.h HONU_GATHER_SKIP_WIN / _WIN2). (Any byte other than 1
    where the walk looks for a flag sends the list to the entry-by-entry walk,
    which is exact either way.)"""
    from dataclasses import replace
    from honu_amd.metadata import AccessControl
    out = []
    for m, d in zip(metas, datas):
        if len(out) == k:
            break
        if not (m.ACL and d):
            continue
        # Permissions 1 everywhere: after a nil entry, the speculated flag
        # positions of the later entries hold their Permissions bytes, so the
        # walk's look at the last flags passes and only the burst sees a
        # mid-list nil
        base = [AccessControl(a.ClientID, 1) for a in m.ACL if a is not None] or \
            [AccessControl(bytes(range(16)), 1)]
        acl = (base * 40)[:40]
        for w in where:
            acl[w] = None
        # six 5-byte region ids after the list: the record holds the 18 bytes
        # per entry a speculated list takes (17 more than a nil's 1), so the
        # list is speculated, not walked for want of room
        out.append((replace(m, ACL=acl, WriteRegions=[(1 << 28) + r for r in range(6)]), d))
    assert len(out) == k
    return out


def _splice(oracle_lib, rec, off, pairs, first):
    """rec/off of a batch with the encoded `pairs` replacing records spread
    evenly from index `first` on."""
    from honu_amd.metadata import pack_batch
    n = len(off) - 1
    r2, o2, st2 = oracle_lib.marshal_batch(pack_batch([m for m, _ in pairs], [d for _, d in pairs]))
    assert (st2 == 0).all()
    at = set(int(x) for x in np.linspace(first, n - 1, len(pairs)).astype(np.int64))
    pieces, noff, j = [], [0], 0
    for i in range(n):
        if i in at:
            r = r2[int(o2[j]):int(o2[j + 1])]
            j += 1
        else:
            r = rec[int(off[i]):int(off[i + 1])]
        pieces.append(r)
        noff.append(noff[-1] + len(r))
    return np.concatenate(pieces), np.array(noff, np.uint64)


def _dev(a, codec):
    return hobj._dev_bytes(np.ascontiguousarray(a), codec.torch_device)


class _Dec:
    """Preallocated honu_decode_records over one encoded batch."""

    def __init__(self, codec, rec, off, inplace=1):
        self.c, self.n = codec, len(off) - 1
        self.inplace = inplace
        self.rec, self.off = _dev(rec, codec), _dev(off, codec)
        cap = int(off[-1])
        self.acl_cap = self.reg_cap = cap
        e = codec._empty
        self.meta, self.info, self.tot = e(352 * self.n), e(32 * self.n), e(32)
        self.acl, self.reg = e(20 * cap), e(4 * cap)

    def __call__(self):
        L = hobj._lib
        _form(self.c, self.inplace)
        return self.c.lib.honu_decode_records(
            self.c.ctx, L.ptr(self.rec), L.ptr(self.off), self.n, L.ptr(self.meta),
            L.ptr(self.info), L.ptr(self.acl), self.acl_cap, L.ptr(self.reg), self.reg_cap, 0, 0,
            L.ptr(self.tot), self.c.stream)

    def check(self, oracle_lib, rec, off):
        torch.cuda.synchronize()
        ometa, oinfo, oacl, oreg, _, otot = _oracle(oracle_lib, rec, off, self.inplace)
        tot = self.tot[:24].cpu().numpy().view(np.uint64)
        assert np.array_equal(tot, otot)
        assert self.meta[:352 * self.n].cpu().numpy().tobytes() == ometa.tobytes()
        assert self.info[:32 * self.n].cpu().numpy().tobytes() == oinfo.tobytes()
        assert self.acl[:20 * int(otot[0])].cpu().numpy().tobytes() == oacl.tobytes()
        assert self.reg[:4 * int(otot[1])].cpu().numpy().tobytes() == oreg.tobytes()


@pytest.fixture(scope="module")
def codec():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = hobj.Codec(0, 64 * 400)
    yield c
    c.close()


@FORMS
def test_tile_counts(codec, oracle_lib, inplace):
    for tiles, seed in ((1, 1), (2, 2), (3, 3), (65, 4), (66, 5), (129, 6), (300, 7)):
        n = 64 * tiles - (seed % 3) * 7  # ragged last tile too
        rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(seed, "small", 0, n))
        d = _Dec(codec, rec, off, inplace)
        assert d() == 0
        d.check(oracle_lib, rec, off)


def test_epoch_wrap_clears_stale_words(codec, oracle_lib):
    wide1 = oracle_lib.marshal_batch(gen_host_batch(11, "small", 0, 64 * 200))
    wide2 = oracle_lib.marshal_batch(gen_host_batch(12, "small", 0, 64 * 200))
    tiny = oracle_lib.marshal_batch(gen_host_batch(13, "small", 0, 64))
    d1, d2, dt = _Dec(codec, *wide1[:2]), _Dec(codec, *wide2[:2]), _Dec(codec, *tiny[:2])
    # wherever the context's epoch stands, bring it to EPOCHS - 1 launches
    # before a wrap: one wide launch, then tiny ones up to the wrap
    assert d1() == 0
    d1.check(oracle_lib, *wide1[:2])
    for _ in range(EPOCHS - 1):
        assert dt() == 0
    # the epoch has wrapped (or is past it) exactly once since d1's words
    assert d2() == 0
    d2.check(oracle_lib, *wide2[:2])
    dt.check(oracle_lib, *tiny[:2])


def test_static_and_ticket_launches_alternate(oracle_lib):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    big_tiles = 2 * 4 * torch.cuda.get_device_properties(0).multi_processor_count + 40
    c = hobj.Codec(0, 64 * big_tiles)
    try:
        wide1 = oracle_lib.marshal_batch(gen_host_batch(21, "small", 0, 64 * big_tiles - 5))
        wide2 = oracle_lib.marshal_batch(gen_host_batch(22, "small", 0, 64 * big_tiles - 9))
        mid = oracle_lib.marshal_batch(gen_host_batch(23, "small", 0, 64 * 150 - 3))
        tiny = oracle_lib.marshal_batch(gen_host_batch(24, "small", 0, 64))
        d1, d2 = _Dec(c, *wide1[:2]), _Dec(c, *wide2[:2])
        dm, dt = _Dec(c, *mid[:2]), _Dec(c, *tiny[:2])
        for d, b in ((d1, wide1), (dm, mid), (d2, wide2), (dt, tiny), (d1, wide1), (dm, mid)):
            assert d() == 0
            d.check(oracle_lib, *b[:2])
        # static launches up to (and past) a wrap, then tickets over other data
        for _ in range(EPOCHS - 1):
            assert dt() == 0
        assert d2() == 0
        d2.check(oracle_lib, *wide2[:2])
        assert dm() == 0
        dm.check(oracle_lib, *mid[:2])
    finally:
        c.close()


def test_static_tiles_beside_a_copy_that_fills_the_chip(oracle_lib):
    """Static tiles rely on in-order workgroup dispatch (lookback.h): with a
    long copy on another stream holding the CUs, the decode's grid is not
    resident at once, and a wave may wait on a tile whose workgroup has not
    started. Dispatch in blockIdx order means that workgroup is dispatched
    first, so the launch completes; results stay bit-exact. Also
    honu_ctx_reset between launches."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    tiles = 2 * 4 * ncu - 3  # every tile has a resident wave slot: static tiles
    c = hobj.Codec(0, 64 * tiles)
    try:
        rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(31, "small", 0, 64 * tiles - 11))
        d = _Dec(c, rec, off)
        src = torch.empty(3 << 30, dtype=torch.uint8, device="cuda")
        dst = torch.empty_like(src)
        side = torch.cuda.Stream(priority=-1)
        for k in range(4):
            with torch.cuda.stream(side):
                dst.copy_(src)
                dst.copy_(src)
            assert d() == 0  # on the codec's stream, beside the copies
            torch.cuda.synchronize()
            d.check(oracle_lib, rec, off)
            if k == 1:
                assert c.lib.honu_ctx_reset(c.ctx, c.stream) == 0
        del src, dst
    finally:
        c.close()


@FORMS
@pytest.mark.parametrize("n,bad", [(140000, [77]), (140000, [5, 64 * 1500 + 3, 139999]),
                                   (5000, [1234])])
def test_speculative_publish_recovers(oracle_lib, n, bad, inplace):
    """Launches with more tiles than resident waves (here 2188 tiles) publish a
    tile's counts once its regions are read (fused.hip SpecPub). Records
    truncated by a few bytes fail in a later field (the Modified time), so
    their published counts were wrong: the guarded second launch must redo the
    batch, bit-exact with the oracle, and clear the flag (a clean batch
    decoded next on the same context is exact too). 5000 records: static
    tiles, no speculation."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(41, "small", 0, n))
    pieces, noff = [], [0]
    for i in range(n):
        r = rec[int(off[i]):int(off[i + 1])]
        if i in bad:
            r = r[:-3]
        pieces.append(r)
        noff.append(noff[-1] + len(r))
    brec = np.concatenate(pieces)
    boff = np.array(noff, np.uint64)
    c = hobj.Codec(0, n)
    try:
        _speculative(c)
        d = _Dec(c, brec, boff, inplace)
        assert d() == 0
        d.check(oracle_lib, brec, boff)
        info = d.info[:32 * n].cpu().numpy().view(np.int32).reshape(n, 8)
        assert all(info[i, 5] != 0 for i in bad)  # meta_status of the truncated records
        good = _Dec(c, rec, off, inplace)
        assert good() == 0
        good.check(oracle_lib, rec, off)
    finally:
        c.close()


@pytest.mark.parametrize("inline_rec,guard_blocks", [(1, 0), (0, 0), (0, 16)],
                         ids=["in_launch", "guard_launch", "small_guard"])
@FORMS
@pytest.mark.parametrize("n,k", [(140000, 1), (140000, 200), (100000, 1), (100000, 200)])
def test_speculative_acl_flags_recover(oracle_lib, n, k, inplace, inline_rec, guard_blocks):
    """Speculative launches also take every ACL list that fits its record as
    all present without gathering its entry flags in the walk; the table fill
    (table form) or the flag gather after the publish (in-place form, fused.hip
    flag_gather / flag_check) checks them. Records whose lists hold nil entries (the walk
    then read every later field at the wrong place) are spliced into a
    2188-tile batch (ticket tiles) or a 1563-tile one (static tiles): the check
    must raise misspec and the batch be decoded again, bit-exact with the
    oracle, by the guarded second launch (inline_recovery 0, the default), by
    a guarded launch of 16 one-wave workgroups (guard_blocks 16: ticket
    tiles over 16 waves, also after a static speculative launch), or by the launch's own
    recovery pass (inline_recovery 1; static tiles keep the guard); a clean
    batch decoded next on the same context is exact too."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from corpora import random_metas
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(43, "small", 0, n))
    metas, datas = random_metas(4 * k + 40, 77)
    brec, boff = _splice(oracle_lib, rec, off, _nil_at(metas, datas, k, [20]), 3)
    c = hobj.Codec(0, n)
    try:
        _speculative(c)
        hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"inline_recovery", inline_rec), "param")
        hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"guard_blocks", guard_blocks), "param")
        r0 = _get(c, b"recoveries")
        d = _Dec(c, brec, boff, inplace)
        assert d() == 0
        d.check(oracle_lib, brec, boff)
        assert _get(c, b"recoveries") == r0 + 1  # the guarded launch redid the batch
        good = _Dec(c, rec, off, inplace)
        assert good() == 0
        good.check(oracle_lib, rec, off)
    finally:
        c.close()


def _get(c, name):
    import ctypes as C
    v = C.c_int64(-1)
    hobj._lib.check(c.lib.honu_ctx_get_param(c.ctx, name, C.byref(v)), "get_param")
    return v.value


def test_speculation_backs_off_after_a_recovery(oracle_lib):
    """A recovery launch that ran sets the context's pinned word; the context's
    next 16 decode calls then run without speculation (honu_decode_records),
    and speculation resumes after them. Every call in the sequence, and a call
    with speculation switched off by honu_ctx_set_param("speculate", 0) over a
    batch that would misspeculate, is bit-exact with the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import ctypes as C
    n = 140000
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(45, "small", 0, n))
    bad = {9, 64 * 900 + 1}
    pieces, noff = [], [0]
    for i in range(n):
        r = rec[int(off[i]):int(off[i + 1])]
        pieces.append(r[:-3] if i in bad else r)
        noff.append(noff[-1] + len(pieces[-1]))
    brec, boff = np.concatenate(pieces), np.array(noff, np.uint64)
    c = hobj.Codec(0, n)

    def get(name):
        v = C.c_int64(-1)
        hobj._lib.check(c.lib.honu_ctx_get_param(c.ctx, name, C.byref(v)), "get_param")
        return v.value
    try:
        _speculative(c)
        d, good = _Dec(c, brec, boff), _Dec(c, rec, off)
        assert get(b"speculate") == 1 and get(b"speculate_backoff") == 0
        assert good() == 0
        good.check(oracle_lib, rec, off)
        assert get(b"speculate_backoff") == 0  # a clean speculative call: no recovery
        assert d() == 0
        d.check(oracle_lib, brec, boff)  # synchronizes: the recovery has run
        assert get(b"speculate_backoff") == 16
        for k in range(16):
            assert (good if k % 2 else d)() == 0
            assert get(b"speculate_backoff") == 15 - k
            if k in (0, 15):
                (good if k % 2 else d).check(oracle_lib, *((rec, off) if k % 2 else (brec, boff)))
        # the back-off is over: the next misspeculating call recovers again
        assert d() == 0
        d.check(oracle_lib, brec, boff)
        assert get(b"speculate_backoff") == 16
        hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"speculate", 0), "param")
        for _ in range(17):  # run the back-off out, then no speculation at all
            assert d() == 0
        d.check(oracle_lib, brec, boff)
        assert get(b"speculate") == 0 and get(b"speculate_backoff") == 0
    finally:
        c.close()


def test_concurrent_ticket_and_static_launches_on_two_streams(oracle_lib):
    """Two contexts decoding at once on their own streams: ticket-mode launches
    (2188 tiles: a workgroup takes its waves' first tiles with one atomic,
    fused.hip FUSED_WG_TICKET) beside each other and beside a static-tile
    launch. Each launch's grid fills the chip, so neither is resident at once;
    a wave only ever waits on tiles that running waves hold (tickets are taken
    by running waves, static tiles wait only on lower-numbered workgroups), so
    every launch completes, bit-exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    n_ticket, n_static = 140000, 64 * (2 * 4 * ncu) - 17
    b1 = oracle_lib.marshal_batch(gen_host_batch(51, "small", 0, n_ticket))
    b2 = oracle_lib.marshal_batch(gen_host_batch(52, "small", 0, n_ticket))
    b3 = oracle_lib.marshal_batch(gen_host_batch(53, "small", 0, n_static))
    c1, c2 = hobj.Codec(0, n_ticket), hobj.Codec(0, n_ticket)
    try:
        for c in (c1, c2):  # speculative ticket launches beside each other
            hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"speculate", 1), "param")
        d1, d2, d3 = _Dec(c1, *b1[:2]), _Dec(c2, *b2[:2]), _Dec(c2, *b3[:2])
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        torch.cuda.synchronize()
        for _ in range(3):
            with torch.cuda.stream(s1):
                assert d1() == 0
                assert d1() == 0
            with torch.cuda.stream(s2):
                assert d2() == 0  # beside d1's first launch
                assert d3() == 0  # static tiles, beside d1's second launch
            torch.cuda.synchronize()
        d1.check(oracle_lib, *b1[:2])
        d2.check(oracle_lib, *b2[:2])
        d3.check(oracle_lib, *b3[:2])
    finally:
        c1.close()
        c2.close()


@FORMS
def test_speculated_long_list_checked_under_capacity_failure(oracle_lib, inplace):
    """A speculated ACL list too long to be staged (1,200 entries: more than
    STAGE_SLOTS blocks) whose last entry is nil, in the last record of a
    2188-tile batch, with acl_cap one entry short of the batch's total so that
    this record fails the capacity check. Its suffix is crafted so that the
    walk, which took the list as all present (17 bytes too long), still parses
    the bytes after it (as 0 regions instead of 5): only the entry flags reveal
    the misspeculation. They must be checked although the record stores
    nothing, and the guarded launch then redoes the batch:
    totals, rows, info (CAPACITY for that record) and the tables equal the
    oracle's with the same caps."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from honu_amd.metadata import AccessControl, Metadata, pack_batch
    n = 140000
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(45, "small", 0, n - 1))
    acl = [AccessControl(bytes([(7 * j + k) & 0xFF for k in range(16)]), j & 0xFF) for j in range(1199)]
    m = Metadata(ObjectID=bytes(range(16)), MIME="x", ACL=acl + [None],
                 WriteRegions=[(1 << 21) + 1, 1 << 22, 1 << 23, 1 << 24, 0])
    r2, o2, st2 = oracle_lib.marshal_batch(pack_batch([m], [b"payload"]))
    assert (st2 == 0).all()
    assert r2[-7:].tobytes() == bytes(7)  # last region 0, then six zero bytes
    brec = np.concatenate([rec, r2])
    boff = np.concatenate([off, off[-1] + o2[1:]]).astype(np.uint64)
    ometa, oinfo, oacl, oreg, _, otot = _oracle(oracle_lib, brec, boff, inplace)
    assert int(ometa[-1]["regions_count"]) == 5 and int(ometa[-1]["acl_count"]) == 1200
    acl_cap, reg_cap = int(otot[0]) - 1, int(otot[1]) + 16
    c = hobj.Codec(0, n)
    try:
        _speculative(c)
        d = _Dec(c, brec, boff, inplace)
        d.acl_cap, d.reg_cap = acl_cap, reg_cap
        assert d() == 0
        torch.cuda.synchronize()
        tot = d.tot[:24].cpu().numpy().view(np.uint64)
        assert np.array_equal(tot, otot)
        assert d.meta[:352 * n].cpu().numpy().tobytes() == ometa.tobytes()
        # raw bytes (a numpy copy of a structured array need not keep its pad
        # bytes): the last record's meta_status (byte 20 of its 32) is CAPACITY
        want = bytearray(oinfo.tobytes())
        ms = oinfo.dtype.fields["meta_status"][1]
        want[32 * (n - 1) + ms:32 * (n - 1) + ms + 4] = (9).to_bytes(4, "little")  # HONU_ERR_CAPACITY
        assert d.info[:32 * n].cpu().numpy().tobytes() == bytes(want)
        nacl = int(otot[0]) - 1200  # the entries of every record before the last
        assert d.acl[:20 * nacl].cpu().numpy().tobytes() == oacl[:nacl].tobytes()
        # the capacity-failed record stores no regions either (in place: none at all)
        nreg = int(otot[1]) - (0 if FORM_PARAMS[inplace][1] else 5)
        assert d.reg[:4 * nreg].cpu().numpy().tobytes() == oreg[:nreg].tobytes()
    finally:
        c.close()


@pytest.mark.parametrize("inplace", [1, 0], ids=["lists_inplace", "lists_table"])
def test_speculate_auto(oracle_lib, inplace):
    """Context param speculate 2 (auto): speculation only where it hides a
    look-back wait. A zero-copy call with both list forms in place waits for
    nothing, so it decodes without speculation: a 2188-tile batch with nil ACL
    entries spliced in decodes bit-exact with no recovery launch; with the
    table forms the same call speculates and recovers once. The param reads
    back, and values outside 0..2 are refused."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from corpora import random_metas
    n = 140000
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(47, "small", 0, n))
    metas, datas = random_metas(200, 79)
    brec, boff = _splice(oracle_lib, rec, off, _nil_at(metas, datas, 20, [20]), 5)
    c = hobj.Codec(0, n)
    try:
        hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"record_variant", 6), "param")
        assert _get(c, b"speculate") == 2  # the default
        assert c.lib.honu_ctx_set_param(c.ctx, b"speculate", 3) != 0
        hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"speculate", 2), "param")
        assert _get(c, b"speculate") == 2
        r0 = _get(c, b"recoveries")
        d = _Dec(c, brec, boff, inplace)
        assert d() == 0
        d.check(oracle_lib, brec, boff)
        assert _get(c, b"recoveries") == r0 + (0 if inplace == 1 else 1)
    finally:
        c.close()


def _caught(t, prefix, na, first, checks=3):
    """Whether the walk itself sees a list's first nil entry (index `first`)
    without the flag burst (win.h): window 1, [t & ~63, +256) from the tail's
    start t, holds the first flags (a0; checks bit 0, HONU_GATHER_SKIP_WIN);
    the window after the speculated list end E, from E's 64-byte unit on, its
    last ones (tl; checks bit 1, HONU_GATHER_SKIP_WIN2). prefix: the tail's
    bytes before the list, na: its entries. checks: the library's
    "walk_flag_checks"."""
    ap = t + prefix
    w1 = t & ~63
    a0 = min(na, (w1 + 256 - ap + 17) // 18) if (checks & 1) and w1 <= ap < w1 + 256 else 0
    w2 = (ap + 18 * na) & ~63
    jb = max(a0, min(na, (w2 - ap + 17) // 18) if w2 > ap else 0)
    tl = na - jb if (checks & 2) and jb < na else 0
    return first < a0 or first >= na - tl


def _placed_batch(oracle_lib, rec, off, pairs, twins, first, want, checks, every=2311):
    """The batch rec/off with the nil-entry records `pairs` spliced in every
    `every` records, each one's payload lengthened by 0-63 bytes so that its
    tail starts where _caught(...) == want (the geometry the walk sees)."""
    from honu_amd.metadata import pack_batch
    r2, o2, _ = oracle_lib.marshal_batch(pack_batch([m for m, _ in twins], [d for _, d in twins]))
    meta, info = oracle_lib.decode_batch(r2, o2)[:2]
    geo = [(int(meta[j]["acl_off"]) - int(info[j]["data_off"]) - int(info[j]["data_len"]),
            int(meta[j]["acl_count"])) for j in range(len(twins))]
    n = len(off) - 1
    pieces, noff, k, placed = [], [0], 0, 0
    for i in range(n):
        r = None
        if i % every == 7 and k < len(pairs):
            (m, d), (prefix, na) = pairs[k], geo[k]
            k += 1
            for delta in range(64):
                dl = len(d) + delta
                t = noff[-1] + 1 + len(_uvarint(dl)) + dl
                if _caught(t, prefix, na, first, checks) == want:
                    d2 = (d * (dl // len(d) + 1))[:dl]
                    rr, oo, st = oracle_lib.marshal_batch(pack_batch([m], [d2]))
                    assert st[0] == 0
                    r = rr[:int(oo[1])]
                    placed += 1
                    break
        if r is None:
            r = rec[int(off[i]):int(off[i + 1])]
        pieces.append(r)
        noff.append(noff[-1] + len(r))
    return np.concatenate(pieces), np.array(noff, np.uint64), placed


def _uvarint(x):
    out = bytearray()
    while x >= 0x80:
        out.append((x & 0x7F) | 0x80)
        x >>= 7
    out.append(x)
    return bytes(out)


@FORMS
@pytest.mark.parametrize("where", [[0], [1, 12], [39], [37, 38], [0, 39], [20]],
                         ids=["first", "window", "last", "tail", "both_ends", "middle"])
def test_walk_catches_nil_entries_at_the_list_ends(oracle_lib, where, inplace):
    """Nil ACL entries the walk sees itself — among the first flags, which the
    window at the tail's start holds, or the last few, which the window after
    the list holds (win.h HONU_GATHER_SKIP_WIN / _WIN2) — send the list to
    the entry-by-entry walk at once: a speculative 2188-tile batch holding
    such records (placed so that the windows hold their first nil: _caught)
    decodes bit-exact with no recovery launch; with records whose first nil
    (index 20) only the flag burst sees, the batch recovers once. Without
    speculation: bit-exact, never a recovery."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from corpora import random_metas
    n = 140000
    rec, off, _ = oracle_lib.marshal_batch(gen_host_batch(49, "small", 0, n))
    metas, datas = random_metas(120, 81)
    c = hobj.Codec(0, 64)
    try:
        checks = _get(c, b"walk_flag_checks")  # which flags this build's walk checks itself
    finally:
        c.close()
    # the walk sees the first nil: among the first flags (every case but the
    # last-only and mid-list ones), or among the last ones when the build
    # checks those from the window after the list
    walk = (where[0] < 13 and bool(checks & 1)) or (where[0] > 36 and bool(checks & 2))
    pairs = _nil_at(metas, datas, 40, where)
    twins = _nil_at(metas, datas, 40, [])  # the same records, every entry present
    brec, boff, placed = _placed_batch(oracle_lib, rec, off, pairs, twins, min(where), walk, checks)
    assert placed >= 8
    for spec in (1, 0):
        c = hobj.Codec(0, n)
        try:
            hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"record_variant", 6), "param")
            hobj._lib.check(c.lib.honu_ctx_set_param(c.ctx, b"speculate", spec), "param")
            r0 = _get(c, b"recoveries")
            d = _Dec(c, brec, boff, inplace)
            assert d() == 0
            d.check(oracle_lib, brec, boff)
            assert _get(c, b"recoveries") == r0 + (1 if spec and not walk else 0)
        finally:
            c.close()
