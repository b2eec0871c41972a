#!/usr/bin/env python3
"""Benchmark: device-resident encode + decode of a 1M-record Large batch per GPU.

One step = object.Marshal of every record of the batch (object.go:24-45) followed
by Object.Metadata() + Object.Data() of every encoded record (object.go:66-99)
with the payloads materialised into a packed arena, all on the GPU through the
C ABI (include/honu_codec.h). Inputs (metadata rows + arenas + payload arena)
are resident in HBM before the timed region. 1M Large records in + out do not
fit one MI355X (≈197.6 GB of payload, ≈395 GB per direction pair), so the batch
is processed as device-resident chunks of --chunk records whose output buffers
are reused; every byte of every record is encoded and decoded each step.

Multi-GPU: weak scaling, one process per GPU, each rank encodes and decodes its
own shard of --records records (records are independent: no data-path
collective). `--gpus N` without a torchrun environment spawns the N ranks itself
(before anything touches the GPU) and fails if fewer than N devices are
visible; under torchrun WORLD_SIZE must equal --gpus. A barrier + synchronize
brackets the timed steps and the max time over ranks is reported; byte and
record totals are summed over ranks.

Prints ONE JSON line on rank 0 (see DESIGN.md for every field).
"""
from __future__ import annotations

import argparse
import ctypes
import gc
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from honu_amd import _lib  # noqa: E402
from honu_amd.object import Codec  # noqa: E402
from honu_amd.shard import weak_range  # noqa: E402
from honu_amd.workload import gen_meta  # noqa: E402

METRIC = "GiB/s + records/s device-resident encode+decode, 1M Large(~300KB) object batch"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def parse_args(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1,
                   help="ranks (one per GPU); without torchrun the ranks are spawned here")
    p.add_argument("--dry-run", action="store_true",
                   help="stop before any device work: ranks report their shard (launcher test)")
    p.add_argument("--shared-gpu", action="store_true",
                   help="rehearsal of the N > 1 code paths on a one-GPU box: every rank on GPU 0, "
                        "gloo instead of RCCL (the scatter staged through host memory); the "
                        "numbers are not a measurement")
    p.add_argument("--steps", type=int, default=3)
    p.add_argument("--warmup", type=int, default=1)
    p.add_argument("--records", type=int, default=1 << 20, help="records per GPU")
    p.add_argument("--shape", default="large")
    p.add_argument("--chunk-gib", type=float, default=12.0,
                   help="encoded bytes per device-resident chunk (output slots are sized by it)")
    p.add_argument("--min-chunks", type=int, default=-1,
                   help="at least this many chunks, so metadata and copies can overlap "
                        "(-1 = auto: 1 for batches under 8 GiB, where the launch tails of "
                        "extra chunks cost more than the overlap gains, else 4)")
    p.add_argument("--seed", type=int, default=1)
    p.add_argument("--cpu-seconds", type=float, default=20.0,
                   help="total CPU-baseline time, split between the 1-thread and all-core legs")
    p.add_argument("--cpu-records", type=int, default=2048)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--serial", action="store_true", help="one stream, no metadata/copy overlap")
    p.add_argument("--meta-blocks", type=int, default=2,
                   help="workgroups per CU for the per-record kernels (0 = library default)")
    p.add_argument("--lane-blocks", type=int, default=-1,
                   help="workgroups per CU for the lane/group metadata kernels while copies run "
                        "beside them (0 = no cap; -1 = auto: 2 when records average > 64 KiB, "
                        "where the copies dominate, else no cap)")
    p.add_argument("--meta-streams", type=int, default=2, choices=[1, 2],
                   help="metadata streams: 2 = one per output slot, so consecutive chunks' metadata "
                        "kernels (each slot has its own context) may run at once (round 4: Mixed "
                        "66.4 -> 58.3 ms/step, Small/Medium/Large unchanged within 0.5%%)")
    p.add_argument("--copy-streams", type=int, default=1, choices=[1, 2],
                   help="2: decode copies on a stream of their own, so a chunk's encode copy need "
                        "not wait behind the previous chunk's decode copy")
    p.add_argument("--copy-prio", type=int, default=1,
                   help="1: the copy stream gets high priority; 0: neither; -1: the metadata stream does")
    p.add_argument("--meta-beside", choices=["auto", "encode", "decode"], default="auto",
                   help="chunk k+1's metadata kernels start when its slot frees (beside chunk "
                        "k's encode copy) or once chunk k's encode copy is done (beside its "
                        "decode copy); auto: decode for records over 64 KiB on average")
    p.add_argument("--meta-cu-stride", type=int, default=0,
                   help="metadata kernels on the CUs i with i %% S == 0 only (a CU-masked stream); "
                        "0: every CU")
    p.add_argument("--copy-cu-mask", choices=["all", "rest"], default="rest",
                   help="with --meta-cu-stride: the copy stream on every CU or on the others only")
    p.add_argument("--encode-copy-after", choices=["scan", "meta"], default="scan",
                   help="start a chunk's encode payload copy after its sizes + scan, or after "
                        "its header/tail encoder too")
    p.add_argument("--decode", choices=["auto", "fused", "split"], default="auto",
                   help="Metadata decode of a chunk: the single-launch kernel (fused), parse + "
                        "tables (split), or by chunk size as honu_decode_batch (auto)")
    p.add_argument("--copy-blocks", type=int, default=0,
                   help="workgroups per CU of the payload copy engine (0 = library default)")
    p.add_argument("--mode", choices=["encdec", "decode", "encode"], default="encdec",
                   help="encdec: the encode + materialising decode step (the metric); decode: "
                        "configs[2] only, Metadata()+Data() of the whole batch from one resident "
                        "records arena (zero copy in one call + materialising in chunks); encode: "
                        "configs[3]'s step, object.Marshal of every record (size pass, the "
                        "per-record output-offset prefix scan, headers + tails, payload copy)")
    p.add_argument("--legs", default="auto",
                   help="encdec mode, comma list of extra legs after the main one: small (1M Small "
                        "encode + decode, configs[1]), mixed_encode (1M Mixed encode, configs[3]), "
                        "medium (1M Medium encode + decode), xlarge (--records/16 XLarge encode + "
                        "decode + chunk zero copy); auto: all four for the default Large line, none "
                        "otherwise; none: no legs")
    p.add_argument("--legs-at", choices=["first", "after_main", "end"], default="after_main",
                   help="when the shape legs run: first (before the main line, after the host path), "
                        "after_main (right after the main line, before the decode legs and their 207 GB "
                        "records arena; the default: 1M Small 3.96-4.23 against 4.21-4.35 ms after the "
                        "decode legs, profiles/r06/order3/) or end (after the decode legs)")
    p.add_argument("--host-path-at", choices=["first", "end"], default="first",
                   help="when the host-path leg runs: first (on a device nothing else has touched yet) "
                        "or end (after every other leg)")
    p.add_argument("--leg-pause", type=float, default=0.0,
                   help="seconds the device idles before each leg (a probe of whether a leg's time "
                        "depends on the load before it; 0: none)")
    p.add_argument("--guard-blocks", type=int, default=-1,
                   help="context param guard_blocks of the output slots: one-wave workgroups of the "
                        "single-launch decode's guarded launch (0: as many as the speculative launch "
                        "has waves; -1: the library default)")
    p.add_argument("--decode-prio", type=int, default=0, choices=[0, 1],
                   help="1: a chunk's single-launch decode (and its guarded launch) on a high-priority "
                        "stream of its slot, so the guard's workgroups are dispatched before the other "
                        "slot's metadata kernels when CUs free up")
    p.add_argument("--slots", type=int, default=2,
                   help="output slots (chunks in flight); 3 lets a chunk's encode run while the two "
                        "before it are still being decoded (with --copy-order ahead)")
    p.add_argument("--copy-order", choices=["chunk", "ahead"], default="chunk",
                   help="chunk: a chunk's decode copy right after its encode copy on the copy stream; "
                        "ahead: after the NEXT chunk's encode copy, so the copy stream does not wait "
                        "for a chunk's Metadata decode")
    p.add_argument("--enc-units", type=int, default=1, choices=[0, 1],
                   help="1: the payload-unit encode pair (honu_encode_records_units + "
                        "honu_encode_payloads_units: the encoder writes each payload's partial end "
                        "64-byte units, the copy the whole ones); 0: honu_encode_records + "
                        "honu_encode_payloads")
    p.add_argument("--decode-chain", type=int, default=1, choices=[0, 1],
                   help="with two metadata streams, a chunk's single-launch decode waits for the "
                        "previous chunk's (and its guarded launch): the guard never queues for "
                        "LDS behind the other slot's persistent decode")
    p.add_argument("--decode-leg", choices=["both", "zero_copy", "materialising"], default="both",
                   help="decode mode: run one leg only (PMC passes attribute a kernel's traffic "
                        "to one leg)")
    p.add_argument("--zc-forms", choices=["all", "default"], default="all",
                   help="decode legs: the zero-copy leg times the default list forms and, for "
                        "comparison, the table forms and speculation off (all), or the default forms "
                        "only (default: PMC passes, whose per-kernel averages would mix the forms)")
    p.add_argument("--zc-speculate", type=int, default=-1, choices=[-1, 0, 1, 2],
                   help="the zero-copy leg's context param speculate for the default forms (-1: the "
                        "library default)")
    p.add_argument("--no-host-path", action="store_true",
                   help="encdec mode: skip the host-path leg (PMC passes: its small launches "
                        "would mix into the copy kernels' per-launch averages)")
    p.add_argument("--no-decode-legs", action="store_true",
                   help="encdec mode: skip the whole-batch decode legs run after the timed steps")
    return p.parse_args(argv)


def P(t):
    return t.data_ptr()


class Slot:
    """Output buffers + codec context of one in-flight chunk."""

    def __init__(self, dev, chunk, out_cap, acl_cap, reg_cap, data_cap, pad=(0, 0)):
        E = lambda nb: torch.empty(int(nb), dtype=torch.uint8, device=dev)  # noqa: E731
        self.codec = Codec(dev.index, max_records=chunk)
        self.out_off, self.status = E(8 * (chunk + 1)), E(4 * chunk + 16)
        # pad: byte offsets of the records and data arenas inside their
        # allocations (multiples of 256), for placement experiments
        self.out = E(out_cap + pad[0])[pad[0]:]
        self.dmeta, self.dinfo = E(352 * chunk), E(32 * chunk)
        self.dacl, self.dreg, self.data = E(20 * acl_cap), E(4 * reg_cap), E(data_cap + pad[1])[pad[1]:]
        self.totals = E(32)
        self.free = None  # event: the slot's last copy finished


class Bench:
    def __init__(self, args, rank, device, pipeline=True, encode_only=False):
        """pipeline=False: inputs, chunks and sizes only (no payload arena, no
        output slots) for DecodeBench. encode_only: the step is object.Marshal
        of every record (configs[3]); the decode runs only in the check."""
        self.args = args
        self.encode_only = encode_only
        self.dev = torch.device("cuda", device)
        N = args.records
        self.N = N
        self.first, _ = weak_range(rank, int(os.environ.get("WORLD_SIZE", "1")), N)
        t0 = time.time()
        meta, var, acl, reg, off = gen_meta(args.seed, args.shape, self.first, N)
        self.host_meta = meta
        self.host_off = off
        self.gen_s = time.time() - t0
        # chunk boundaries by bytes (payload + ~1.1 KB of header/metadata per record)
        est = np.diff(off.astype(np.int64)) + 1100
        cum = np.concatenate([[0], np.cumsum(est)])
        # equal-byte chunks: enough that each fits --chunk-gib, at least --min-chunks
        min_chunks = args.min_chunks if args.min_chunks >= 0 else (1 if cum[-1] < 8 * 2**30 else 4)
        k = max(1, min_chunks, int(np.ceil(cum[-1] / (args.chunk_gib * 2**30))))
        k = min(k, N)
        cuts = np.searchsorted(cum, cum[-1] * np.arange(1, k) / k, side="left")
        bounds = sorted(set([0, N] + [int(c) for c in cuts if 0 < c < N]))
        self.chunks = list(zip(bounds[:-1], bounds[1:]))
        C = max(b - a for a, b in self.chunks)
        self.C = C
        self.codec = Codec(device, max_records=C)
        self.lib = self.codec.lib

        def D(a):
            a = np.ascontiguousarray(a)
            t = torch.empty(max(a.nbytes, 16), dtype=torch.uint8, device=self.dev)
            if a.nbytes:
                t[: a.nbytes].copy_(torch.from_numpy(a.view(np.uint8).reshape(-1)))
            return t

        self.meta, self.var, self.acl, self.reg, self.off = D(meta), D(var), D(acl), D(reg), D(off)
        self.var_len, self.acl_len, self.reg_len = len(var), len(acl), len(reg)
        self.payload_bytes = int(off[N])
        s0 = torch.cuda.current_stream(self.dev).cuda_stream
        self.payload = None
        if pipeline:
            self.payload = torch.empty(self.payload_bytes + 16, dtype=torch.uint8, device=self.dev)
            _lib.check(self.lib.honu_gen_payload(self.codec.ctx, args.seed, self.first, N,
                                                 P(self.off), P(self.payload), s0), "gen_payload")
        # sizing pass (untimed): exact record bytes of every chunk
        out_off = torch.empty(8 * (C + 1), dtype=torch.uint8, device=self.dev)
        status = torch.empty(4 * C + 16, dtype=torch.uint8, device=self.dev)
        self.rec_bytes = []
        for a, b in self.chunks:
            self._sizes(self.codec, a, b, out_off, status, s0)
            self.rec_bytes.append(int(out_off.view(torch.int64)[b - a].item()))
        del out_off, status
        self.total_rec_bytes = sum(self.rec_bytes)
        lens = np.diff(off.astype(np.int64))
        acl_n = meta["acl_count"].astype(np.int64)
        reg_n = meta["regions_count"].astype(np.int64)
        alloc = (lens + 15) // 16 * 16
        self.chunk_payload = [int(lens[a:b].sum()) for a, b in self.chunks]
        self.acl_cap = max(int(acl_n[a:b].sum()) for a, b in self.chunks) + 1
        self.reg_cap = max(int(reg_n[a:b].sum()) for a, b in self.chunks) + 1
        self.data_cap = max(int(alloc[a:b].sum()) for a, b in self.chunks) + 16
        self.out_cap = max(self.rec_bytes) + 16
        self.ncu = torch.cuda.get_device_properties(self.dev).multi_processor_count
        self._copy_form = {}
        if not pipeline:
            return
        nslots = 1 if args.serial else max(2, getattr(args, "slots", 2))
        self.slots = [Slot(self.dev, C, self.out_cap, self.acl_cap, self.reg_cap,
                           16 if encode_only else self.data_cap) for _ in range(nslots)]
        ncu = torch.cuda.get_device_properties(self.dev).multi_processor_count
        lane_blocks = args.lane_blocks
        if lane_blocks < 0:  # measured: tools/overlap_sweep.sh, tools/ab_env.sh, tools/args_ab.sh
            avg = self.total_rec_bytes / N
            # round 3: no cap below 64 KiB (1M Medium 1048-1050 uncapped vs 1032-1034
            # GiB/s capped at 4 per CU, profiles/r03/medium_lane_blocks_ab.txt)
            lane_blocks = 2 if avg > 65536 else 0
        self.lane_blocks = 0 if args.serial else lane_blocks
        # measured (profiles/r03/ab/meta_beside_ab.txt): 1M Large 1343-1347 -> 1377 GiB/s and
        # 1M Mixed 1194 -> 1213-1223 with the metadata beside the decode copy, 1M Medium
        # 1052-1078 -> 1048-1061
        self.meta_beside = args.meta_beside
        if self.meta_beside == "auto":
            self.meta_beside = "decode" if self.total_rec_bytes / N > 65536 else "encode"
        for sl in self.slots:
            if args.copy_blocks:
                _lib.check(self.lib.honu_ctx_set_param(sl.codec.ctx, b"copy_blocks",
                                                       args.copy_blocks * ncu), "param")
            if getattr(args, "guard_blocks", -1) >= 0:
                _lib.check(self.lib.honu_ctx_set_param(sl.codec.ctx, b"guard_blocks",
                                                       args.guard_blocks), "param")
        if not args.serial:
            for sl in self.slots:
                if args.meta_blocks:
                    _lib.check(self.lib.honu_ctx_set_param(sl.codec.ctx, b"record_blocks",
                                                           args.meta_blocks * ncu), "param")
                _lib.check(self.lib.honu_ctx_set_param(sl.codec.ctx, b"lane_blocks",
                                                       self.lane_blocks * ncu), "param")
        var, steal = ctypes.c_int64(0), ctypes.c_int64(0)
        c0 = self.slots[0].codec.ctx
        _lib.check(self.lib.honu_ctx_get_param(c0, b"copy_variant", ctypes.byref(var)), "param")
        _lib.check(self.lib.honu_ctx_get_param(c0, b"copy_steal", ctypes.byref(steal)), "param")
        self._copy_form = {"copy_variant": var.value, "copy_range_tails": bool(steal.value)}
        self.sm = torch.cuda.Stream(self.dev, priority=-1 if args.copy_prio < 0 else 0)  # metadata kernels
        # payload copies: the bandwidth-bound critical path, dispatched first
        self.sc = (torch.cuda.Stream(self.dev, priority=-1 if args.copy_prio > 0 else 0)
                   if nslots >= 2 else self.sm)
        if args.meta_cu_stride and nslots >= 2:  # metadata and copies on their own CUs
            S = args.meta_cu_stride
            self.sm = cu_masked_stream(self.dev, ncu, lambda i: i % S == 0)
            if args.copy_cu_mask == "rest":
                self.sc = cu_masked_stream(self.dev, ncu, lambda i: i % S != 0)
        # --meta-streams 2: slot k's metadata kernels on stream k (its own context)
        self.sms = [self.sm]
        if getattr(args, "meta_streams", 1) == 2 and nslots >= 2 and not args.meta_cu_stride:
            self.sms.append(torch.cuda.Stream(self.dev, priority=-1 if args.copy_prio < 0 else 0))
        # --copy-streams 2: decode copies on their own stream
        self.sd = self.sc
        if getattr(args, "copy_streams", 1) == 2 and nslots >= 2 and not args.meta_cu_stride:
            self.sd = torch.cuda.Stream(self.dev, priority=-1 if args.copy_prio > 0 else 0)
        # --decode-prio: one high-priority decode stream per metadata stream
        self.sdec = [torch.cuda.Stream(self.dev, priority=-1) for _ in self.sms] \
            if getattr(args, "decode_prio", 0) else None
        self.sv = torch.cuda.Stream(self.dev)  # verification of drained chunks
        self.events = None
        self.last = None
        self.nchunk = 0  # chunks issued so far, across steps: slots alternate globally
        self.enc_done = None  # the last issued chunk's encode copy (--meta-beside decode)
        self.dec_done = None  # the last issued chunk's single-launch decode (--decode-chain)
        # --copy-order ahead: the last chunk's decode copy, issued after the
        # next chunk's encode copy (flush() issues it)
        self.ahead = getattr(args, "copy_order", "chunk") == "ahead" and nslots >= 2 and not encode_only
        self.units = bool(getattr(args, "enc_units", 1))  # the payload-unit encode pair
        self.pending_dec = None
        torch.cuda.synchronize()

    def _sizes(self, codec, a, b, out_off, status, s):
        n = b - a
        L, c = self.lib, codec.ctx
        _lib.check(L.honu_encode_sizes(c, P(self.meta) + 352 * a, self.var_len, P(self.acl),
                                       self.acl_len, P(self.reg), self.reg_len, P(self.off) + 8 * a,
                                       n, P(out_off), P(status), s), "sizes")
        _lib.check(L.honu_exclusive_scan(c, P(out_off), n, P(out_off), s), "scan")

    def step(self, timed=False, check=None):
        """Chunk k: metadata work (sizes, scan, headers+tails, parse, tables) on
        stream sm, payload copies on stream sc; two slots so chunk k+1's metadata
        work overlaps chunk k's copies. The encode copy needs only the output
        offsets and statuses (sizes + scan): it writes the payload bytes, the
        metadata kernels write only the bytes around them (byte-exact stores at
        the shared 16-byte chunks), so it runs beside the header/tail encoder.

        check(a, b, slot) -> bool, when given, is called for chunk k once chunk
        k+1 has been issued (so chunks still overlap exactly as in the timed
        steps) and chunk k's slot has drained; it runs on its own stream and
        must finish before it returns (chunk k+2 reuses the slot). The result
        is the AND of its answers."""
        ok = True
        pending = None
        for a, b in self.chunks:
            sl = self._issue(a, b, timed)
            if check is not None:
                if len(self.slots) == 1:  # --serial: the next chunk reuses the one slot
                    ok &= self._check(check, (a, b, sl))
                    continue
                if pending is not None:
                    ok &= self._check(check, pending)
                pending = (a, b, sl)
        if check is not None:
            self.flush()
        if pending is not None:
            ok &= self._check(check, pending)
        torch.cuda.current_stream(self.dev).wait_stream(self.sc)
        torch.cuda.current_stream(self.dev).wait_stream(self.sd)
        for sm in self.sms + (self.sdec or []):
            torch.cuda.current_stream(self.dev).wait_stream(sm)
        return ok

    def flush(self):
        """--copy-order ahead: issue the decode copy still held back (the
        timed region issues its last one before it ends)."""
        dec, self.pending_dec = self.pending_dec, None
        if dec is not None:
            dec()

    def _check(self, check, pending):
        a, b, sl = pending
        sl.free.synchronize()  # chunk k's last copy done; chunk k+1 may still run
        with torch.cuda.stream(self.sv):
            return bool(check(a, b, sl))

    def _issue(self, a, b, timed):
        """Enqueue encode + materialising decode of records [a, b) into the
        next slot; returns the slot."""
        L = self.lib
        n = b - a
        # the slot after the previous chunk's, also across steps, so a step's
        # first chunk overlaps the previous step's last one
        k = self.nchunk % len(self.slots)
        sl = self.slots[k]
        sm, sc = self.sms[k % len(self.sms)], self.sc
        self.nchunk += 1
        c = sl.codec.ctx
        if sl.free is not None:
            sm.wait_event(sl.free)
        if self.meta_beside == "decode" and self.enc_done is not None:
            sm.wait_event(self.enc_done)
        ms = sm.cuda_stream
        if timed and self.encode_only:
            o0, o1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            o0.record(sm)
        self._sizes(sl.codec, a, b, sl.out_off, sl.status, ms)
        ev_off = torch.cuda.Event()
        ev_off.record(sm)
        if timed and self.encode_only:
            o1.record(sm)
        if self.units:  # the encoder also writes the payloads' partial end 64-byte units
            _lib.check(L.honu_encode_records_units(c, P(self.meta) + 352 * a, P(self.var), P(self.acl),
                                                   P(self.reg), P(self.payload), P(self.off) + 8 * a, n,
                                                   P(sl.out), self.out_cap, P(sl.out_off), P(sl.status), ms),
                       "encode_records_units")
        else:
            _lib.check(L.honu_encode_records(c, P(self.meta) + 352 * a, P(self.var), P(self.acl),
                                             P(self.reg), P(self.off) + 8 * a, n, P(sl.out),
                                             self.out_cap, P(sl.out_off), P(sl.status), ms),
                       "encode_records")
        if self.args.encode_copy_after == "meta":
            ev_off = torch.cuda.Event()
            ev_off.record(sm)
        if self.encode_only:
            return self._issue_encode_copy(a, b, sl, sm, timed, ev_off, (o0, o1) if timed else None)
        if self.fused_decode(n):  # parse + look-back + tables in one launch (fused.hip)
            # --decode-chain (default on): with two metadata streams the
            # previous chunk's decode (and its guarded launch) finishes first,
            # so the two slots' persistent decodes never share the chip
            # (measured equal to off: a guard waits for registers the other
            # slot's tail encoder holds, not for the other decode; DESIGN §3
            # "Round 5: the guard in one-wave workgroups")
            chain = self.args.decode_chain and len(self.sms) > 1
            dm = sm
            if self.sdec is not None:  # fork onto the slot's high-priority decode stream
                dm = self.sdec[k % len(self.sdec)]
                ev = torch.cuda.Event()
                ev.record(sm)
                dm.wait_event(ev)
            if chain and self.dec_done is not None:
                dm.wait_event(self.dec_done)
            _lib.check(L.honu_decode_records(c, P(sl.out), P(sl.out_off), n, P(sl.dmeta),
                                             P(sl.dinfo), P(sl.dacl), self.acl_cap, P(sl.dreg),
                                             self.reg_cap, 1, self.data_cap, P(sl.totals), dm.cuda_stream),
                       "decode_records")
            if chain:
                self.dec_done = torch.cuda.Event()
                self.dec_done.record(dm)
            if dm is not sm:  # join: the fill event below and the slot's next chunk follow it
                ev = torch.cuda.Event()
                ev.record(dm)
                sm.wait_event(ev)
        else:
            _lib.check(L.honu_decode_parse(c, P(sl.out), P(sl.out_off), n, P(sl.dmeta),
                                           P(sl.dinfo), ms), "decode_parse")
            _lib.check(L.honu_decode_tables(c, P(sl.out), n, P(sl.dmeta), P(sl.dinfo),
                                            P(sl.dacl), self.acl_cap, P(sl.dreg), self.reg_cap,
                                            P(sl.data), self.data_cap, P(sl.totals), ms),
                       "decode_tables")
        ev_fill = torch.cuda.Event()
        ev_fill.record(sm)
        cs = sc.cuda_stream
        sc.wait_event(ev_off)
        e0 = torch.cuda.Event(enable_timing=True) if timed else None
        e1 = torch.cuda.Event(enable_timing=True) if timed else None
        if timed:
            e0.record(sc)
        enc_copy = L.honu_encode_payloads_units if self.units else L.honu_encode_payloads
        _lib.check(enc_copy(c, P(self.payload), P(self.off) + 8 * a, n,
                            P(sl.out), self.out_cap, P(sl.out_off), P(sl.status),
                            cs), "encode_payloads")
        if timed:
            e1.record(sc)
        self.enc_done = torch.cuda.Event()
        self.enc_done.record(sc)
        enc_done = self.enc_done

        def dec():  # the decode copy: after this chunk's encode copy and its table fill
            sd = self.sd
            if sd is not sc:
                sd.wait_event(enc_done)
            sd.wait_event(ev_fill)
            e2 = torch.cuda.Event(enable_timing=True) if timed else None
            e3 = torch.cuda.Event(enable_timing=True) if timed else None
            if timed:
                e2.record(sd)
            _lib.check(L.honu_decode_payloads(c, P(sl.out), n, P(sl.dinfo), P(sl.data),
                                              P(sl.totals), sd.cuda_stream), "decode_payloads")
            if timed:
                e3.record(sd)
                self.events.append((a, b, e0, e1, e2, e3))
            sl.free = torch.cuda.Event()
            sl.free.record(sd)
        if self.ahead:  # the previous chunk's decode copy after this chunk's encode copy
            prev, self.pending_dec = self.pending_dec, dec
            if prev is not None:
                prev()
        else:
            dec()
        self.last = (a, b, sl)
        return sl

    def _issue_encode_copy(self, a, b, sl, sm, timed, ev_off, off_events):
        """encode_only: the payload copy of chunk [a, b) after its offsets; the
        slot frees when it is done."""
        L, n = self.lib, b - a
        sc = self.sc
        sc.wait_event(ev_off)
        e0 = torch.cuda.Event(enable_timing=True) if timed else None
        e1 = torch.cuda.Event(enable_timing=True) if timed else None
        if timed:
            e0.record(sc)
        enc_copy = L.honu_encode_payloads_units if self.units else L.honu_encode_payloads
        _lib.check(enc_copy(sl.codec.ctx, P(self.payload), P(self.off) + 8 * a, n,
                            P(sl.out), self.out_cap, P(sl.out_off), P(sl.status),
                            sc.cuda_stream), "encode_payloads")
        if timed:
            e1.record(sc)
            self.events.append((a, b, e0, e1) + tuple(off_events))
        ev = torch.cuda.Event()  # the slot frees once its header/tail encoder is done too
        ev.record(sm)
        sc.wait_event(ev)
        sl.free = torch.cuda.Event()
        sl.free.record(sc)
        self.last = (a, b, sl)
        return sl

    # The pipeline's own crossover, above honu_decode_batch's 48 K: beside the
    # other chunk's copies the split kernels are as fast on 62 K-record Large
    # chunks (box-dependent, -2 % to +4 % for the single launch) and keep the
    # encode copy faster (5.84 vs 5.63-5.67 TB/s, profiles/r02/crossover_static_tiles.txt)
    FUSED_DECODE_MIN = 128 << 10

    def copy_form(self):
        """The payload copy's form on the output slots' contexts, read when
        they were set up: the copy variant (0 in the product library) and
        whether the range tails (honu_codec.h "copy_steal") are on."""
        return self._copy_form

    def recoveries(self):
        """Recovery launches the output slots' single-launch decodes have run
        so far (honu_ctx_get_param "recoveries": a count the guarded launch
        increments when it runs; malformed input or nil ACL entries only, so
        it stays put on the bench's records). The timed steps report the
        difference across them."""
        total = 0
        for sl in self.slots:
            v = ctypes.c_int64(0)
            _lib.check(self.lib.honu_ctx_get_param(sl.codec.ctx, b"recoveries", ctypes.byref(v)), "param")
            total += v.value
        return total

    def fused_decode(self, n):
        # beside the decode copy the persistent single-launch grid costs the copy more
        # than it saves: 1M Mixed (262 K-record chunks) 1143-1146 GiB/s fused vs
        # 1267-1269 split (profiles/r03/ab/meta_beside_decode_form_ab.txt)
        d = self.args.decode
        return d == "fused" or (d == "auto" and n >= self.FUSED_DECODE_MIN
                                and self.meta_beside != "decode")

    def verify(self):
        """Every record of the batch, after the timed steps: one more pipelined
        step (same streams, slots and overlap as the timed ones) whose chunks
        are each checked once drained (_verify_chunk)."""
        torch.cuda.synchronize()
        return bool(self.step(check=self._verify_chunk))

    VERIFIED_SCOPE = ("every record of every rank: encode and decode statuses; every decoded "
                      "row byte against the source row (scalars, ULIDs, presence bits, span "
                      "lengths and span bytes, ACL entries, regions; honu_verify_decoded); "
                      "payload lengths + position-aware digests")

    def _verify_chunk(self, a, b, sl):
        """Chunk [a, b) as the pipeline left it in slot sl, on the current
        (verification) stream: encode statuses OK; honu_verify_decoded of every
        decoded row, span, ACL entry and region against the source row it was
        encoded from; every materialised payload's digest equal to its
        source's. encode_only: the chunk's records are decoded here (zero
        copy, untimed) and every Data() subslice's digest is compared."""
        L, c = self.lib, sl.codec.ctx
        n = b - a
        s = torch.cuda.current_stream(self.dev).cuda_stream
        if self.encode_only:
            _lib.check(L.honu_decode_batch(c, P(sl.out), P(sl.out_off), n, P(sl.dmeta), P(sl.dinfo),
                                           P(sl.dacl), self.acl_cap, P(sl.dreg), self.reg_cap, 0, 0,
                                           P(sl.totals), s), "decode_batch")
        st = sl.status[: 4 * n].view(torch.int32)
        info = sl.dinfo[: 32 * n].view(torch.int64).view(n, 4)
        mism = torch.empty(4 * n, dtype=torch.uint8, device=self.dev)
        _lib.check(L.honu_verify_decoded(c, P(self.meta) + 352 * a, P(self.var), P(self.acl),
                                         P(self.reg), P(self.off) + 8 * a, P(sl.out), P(sl.dmeta),
                                         P(sl.dinfo), P(sl.dacl), P(sl.dreg), n, P(mism), s),
                   "verify_decoded")
        dsrc = torch.empty(8 * n, dtype=torch.uint8, device=self.dev)
        ddst = torch.empty(8 * n, dtype=torch.uint8, device=self.dev)
        _lib.check(L.honu_digest_records(c, P(self.payload), P(self.off) + 8 * a, 0, n, P(dsrc), s),
                   "digest")
        doff, dlen = info[:, 0].contiguous(), info[:, 1].contiguous()
        _lib.check(L.honu_digest_records(c, P(sl.out if self.encode_only else sl.data), P(doff), P(dlen),
                                         n, P(ddst), s), "digest")
        ok = bool((st == 0).all()) and int(torch.count_nonzero(mism.view(torch.int32))) == 0
        ok &= torch.equal(dsrc, ddst)
        torch.cuda.current_stream(self.dev).synchronize()
        return bool(ok)

    def zero_copy_decode(self, reps=10):
        """Object.Metadata + zero-copy Object.Data (the reference's exact decode
        semantics: payloads stay in the records arena): records/s of
        honu_decode_batch with no data arena, on the chunk with the most records,
        encoded (untimed) into slot 0 first."""
        torch.cuda.synchronize()
        k = max(range(len(self.chunks)), key=lambda i: self.chunks[i][1] - self.chunks[i][0])
        a, b = self.chunks[k]
        sl = self.slots[0]
        n = b - a
        L, c = self.lib, sl.codec.ctx
        st = torch.cuda.current_stream(self.dev)
        self._sizes(sl.codec, a, b, sl.out_off, sl.status, st.cuda_stream)
        _lib.check(L.honu_encode(c, P(self.meta) + 352 * a, P(self.var), self.var_len, P(self.acl),
                                 self.acl_len, P(self.reg), self.reg_len, P(self.payload),
                                 P(self.off) + 8 * a, n, P(sl.out), self.out_cap, P(sl.out_off),
                                 P(sl.status), st.cuda_stream), "encode")
        self.zc_chunk = (a, b, sl)  # slot 0 holds this chunk's records from here on
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        # the decode runs alone here: lift the cap that keeps the metadata
        # kernels from crowding the copies in the pipelined step
        _lib.check(L.honu_ctx_set_param(c, b"lane_blocks", 0), "param")

        def once():
            _lib.check(L.honu_decode_batch(c, P(sl.out), P(sl.out_off), n, P(sl.dmeta), P(sl.dinfo),
                                           P(sl.dacl), self.acl_cap, P(sl.dreg), self.reg_cap, 0, 0,
                                           P(sl.totals), st.cuda_stream), "decode_batch")
        once()
        e0.record(st)
        for _ in range(reps):
            once()
        e1.record(st)
        # cold: before each timed decode an untimed 1 GiB write evicts the
        # chunk's tails from the 256 MB Infinity Cache (back to back, a Large
        # chunk's 66 MB of tails stay there between reps)
        scrub = torch.empty(1 << 30, dtype=torch.uint8, device=self.dev)
        cold = []
        for _ in range(reps):
            scrub.fill_(0x5A)
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record(st)
            once()
            c1.record(st)
            cold.append((c0, c1))
        torch.cuda.synchronize()
        del scrub
        ncu = torch.cuda.get_device_properties(self.dev).multi_processor_count
        _lib.check(L.honu_ctx_set_param(c, b"lane_blocks", self.lane_blocks * ncu), "param")
        t = e0.elapsed_time(e1) / 1e3 / reps
        tc = sum(x.elapsed_time(y) for x, y in cold) / 1e3 / reps
        return {"records": n, "ms": t * 1e3, "records_per_s": n / t,
                "cold_ms": tc * 1e3, "cold_records_per_s": n / tc}


    def release(self):
        """Free the payload arena, the output slots and the contexts (before a
        DecodeBench reuses the device inputs)."""
        torch.cuda.synchronize()
        self.payload = None
        for sl in getattr(self, "slots", []):
            sl.codec.close()
        self.slots = []
        self.events = None
        self.last = None
        gc.collect()
        torch.cuda.empty_cache()


def uvarint_len(x):
    """len(binary.PutUvarint(x)) of every element (numpy uint64)."""
    x = np.asarray(x, np.uint64)
    n = np.ones(x.shape, np.int64)
    for k in range(1, 10):
        n += x >= np.uint64(1 << (7 * k))
    return n


class DecodeBench:
    """configs[2]: the reference's decode over the WHOLE batch held in one
    records arena (object.go:66-99, the decode half of BenchmarkSerialization,
    object_test.go:140-159).

    Setup (untimed): every chunk's payload is generated into a scratch buffer
    and the chunk is encoded into its place in one resident records arena
    (1M Large records: ≈207 GB), with per-record digests of the source
    payloads kept for the check. Then two legs are timed:
      zero_copy      honu_decode_batch with no data arena over all records in
                     ONE call: Metadata() rows, record info (Data() subslices of
                     the arena) and the ACL / region tables;
      materialising  the same decode with Data() copied into a packed data
                     arena, chunk by chunk (the data arena of 1M Large records
                     does not fit beside the records), metadata decode of chunk
                     k+1 on one stream beside the payload copy of chunk k on
                     another, two data slots.
    Rows and record info of both legs go to whole-batch arrays; every row,
    table entry and payload is checked after the timed reps."""

    def __init__(self, bench):
        self.b = b = bench
        self.args = bench.args
        self.dev = b.dev
        self.lib = L = b.lib
        N, C = b.N, b.C
        dev = self.dev
        E = lambda nb: torch.empty(int(nb), dtype=torch.uint8, device=dev)  # noqa: E731
        self.codec = Codec(dev.index, max_records=N)
        c = self.codec.ctx
        st = torch.cuda.current_stream(dev)
        s = st.cuda_stream
        # global record offsets: sizes of every record, one scan
        self.rec_off = E(8 * (N + 1))
        self.status = E(4 * N + 16)
        _lib.check(L.honu_encode_sizes(c, P(b.meta), b.var_len, P(b.acl), b.acl_len, P(b.reg),
                                       b.reg_len, P(b.off), N, P(self.rec_off), P(self.status), s),
                   "sizes")
        _lib.check(L.honu_exclusive_scan(c, P(self.rec_off), N, P(self.rec_off), s), "scan")
        ro = self.rec_off.view(torch.int64)
        self.total = int(ro[N].item())
        self.arena = E(self.total + 16)
        self.dig_src = E(8 * N)
        scratch = E(max(b.chunk_payload) + 16)
        host_off = b.host_off
        for a, e in b.chunks:  # payload of chunk -> scratch -> encoded into the arena
            n = e - a
            base = P(scratch) - int(host_off[a])  # payload offsets are global
            _lib.check(L.honu_gen_payload(c, self.args.seed, b.first + a, n, P(b.off) + 8 * a, base,
                                          s), "gen_payload")
            _lib.check(L.honu_digest_records(c, base, P(b.off) + 8 * a, 0, n,
                                             P(self.dig_src) + 8 * a, s), "digest")
            _lib.check(L.honu_encode(c, P(b.meta) + 352 * a, P(b.var), b.var_len, P(b.acl),
                                     b.acl_len, P(b.reg), b.reg_len, base, P(b.off) + 8 * a, n,
                                     P(self.arena), self.total + 16, P(self.rec_off) + 8 * a,
                                     P(self.status) + 4 * a, s), "encode")
            st.synchronize()
        del scratch
        self.encode_ok = bool((self.status[: 4 * N].view(torch.int32) == 0).all())
        torch.cuda.empty_cache()
        # algorithmic bytes: per record the offsets pair, the
        # header, the Metadata tail; out the row, the record info, the tables
        rlen = np.diff(ro.cpu().numpy())
        plen = np.diff(host_off.astype(np.int64))
        hdr = 1 + uvarint_len(plen)
        self.tail_bytes = int((rlen - hdr - plen).sum())
        self.hdr_bytes = int(hdr.sum())
        hm = b.host_meta
        self.nacl = int(hm["acl_count"].astype(np.int64).sum())
        self.nreg = int(hm["regions_count"].astype(np.int64).sum())
        self.payload_bytes = int(plen.sum())
        # whole-batch outputs
        self.dmeta, self.dinfo = E(352 * N), E(32 * N)
        self.acl_cap, self.reg_cap = self.nacl + 1, self.nreg + 1
        self.dacl, self.dreg = E(20 * self.acl_cap), E(4 * self.reg_cap)
        self.totals = E(32)
        # table entries the default (in-place) forms write: ACL lists with a
        # nil entry only (none in the generator's records), no regions; from
        # one untimed decode
        self._zero_copy_once(s)
        st.synchronize()
        tt = self.totals[:16].view(torch.int64).tolist()
        self.acl_table_entries, self.reg_table_entries = int(tt[0]), int(tt[1])
        self.meta_bytes = self.meta_bytes_for(self.acl_table_entries, self.reg_table_entries)
        # materialising leg: two data slots of one chunk each
        self.slots = []
        for _ in range(2):
            sl = Slot.__new__(Slot)
            sl.codec = Codec(dev.index, max_records=C)
            sl.dacl, sl.dreg = E(20 * b.acl_cap), E(4 * b.reg_cap)
            sl.data, sl.totals = E(b.data_cap), E(32)
            sl.free = None
            self.slots.append(sl)
        self.sm = torch.cuda.Stream(dev)
        self.sc = torch.cuda.Stream(dev, priority=-1)
        self.sv = torch.cuda.Stream(dev)
        torch.cuda.synchronize()

    def meta_bytes_for(self, acl_table_entries, reg_table_entries):
        """Algorithmic bytes of one Metadata() + zero-copy Data() pass (SURVEY
        §8d): per record the offsets pair, the header and the Metadata tail
        read; the row, the record info, 4 per region TABLE entry and 20 per
        ACL TABLE entry written (a list returned in place writes nothing: its
        entries are read as part of the tail)."""
        N = self.b.N
        return (8 * N + self.hdr_bytes + self.tail_bytes + 352 * N + 32 * N +
                20 * acl_table_entries + 4 * reg_table_entries)

    # -- zero copy, whole batch ------------------------------------------------
    def _zero_copy_once(self, s):
        b, L = self.b, self.lib
        _lib.check(L.honu_decode_batch(self.codec.ctx, P(self.arena), P(self.rec_off), b.N,
                                       P(self.dmeta), P(self.dinfo), P(self.dacl), self.acl_cap,
                                       P(self.dreg), self.reg_cap, 0, 0, P(self.totals), s),
                   "decode_batch")

    def _zero_copy_reps(self, reps):
        st = torch.cuda.current_stream(self.dev)
        self._zero_copy_once(st.cuda_stream)
        ev = []
        for _ in range(reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            self._zero_copy_once(st.cuda_stream)
            e1.record(st)
            ev.append((e0, e1))
        torch.cuda.synchronize()
        return [x.elapsed_time(y) for x, y in ev]

    def _form_reps(self, acl, reg, reps, speculate=None):
        """reps timed calls with the context params acl_inplace / regions_inplace
        set to (acl, reg): (per-call ms, ACL table entries, region table entries)."""
        c = self.codec.ctx
        _lib.check(self.lib.honu_ctx_set_param(c, b"acl_inplace", acl), "param")
        _lib.check(self.lib.honu_ctx_set_param(c, b"regions_inplace", reg), "param")
        old = ctypes.c_int64(1)
        _lib.check(self.lib.honu_ctx_get_param(c, b"speculate", ctypes.byref(old)), "param")
        if speculate is not None:
            _lib.check(self.lib.honu_ctx_set_param(c, b"speculate", speculate), "param")
        ms = self._zero_copy_reps(reps)
        _lib.check(self.lib.honu_ctx_set_param(c, b"speculate", old.value), "param")
        tt = self.totals[:16].view(torch.int64).tolist()
        return ms, int(tt[0]), int(tt[1])

    def _form_summary(self, ms, acl_entries, reg_entries, how):
        t = sum(ms) / len(ms) / 1e3
        nb = self.meta_bytes_for(acl_entries, reg_entries)
        return {"ms": t * 1e3, "ms_min": min(ms), "records_per_s": self.b.N / t,
                "acl_table_entries": acl_entries, "region_table_entries": reg_entries,
                "algorithmic_bytes_per_launch": nb, "frac_of_spec": nb / t / 1e9 / HBM_PEAK_GBS,
                "how": how}

    def zero_copy(self, reps):
        """The default decode (ACL and region lists returned in place,
        HONU_ACL_INPLACE / HONU_REGIONS_INPLACE), then, for comparison, the
        same call with every list in its table (context params acl_inplace 0,
        regions_inplace 0: rounds 1-4) and with the ACL lists in place but the
        regions in their table (round 5's default). The forms alternate, the
        default's reps split around the others."""
        h = max(1, reps // 2)
        others = getattr(self.args, "zc_forms", "all") == "all"
        sp = getattr(self.args, "zc_speculate", -1)
        sp = None if sp < 0 else sp
        ms = self._form_reps(1, 1, h, speculate=sp)[0]
        if others:
            ms_tab, tab_acl, tab_reg = self._form_reps(0, 0, reps)
            ms_r5, r5_acl, r5_reg = self._form_reps(1, 0, reps)
            ms_sp, sp_acl, sp_reg = self._form_reps(1, 1, reps, speculate=1)
        ms2, acl_e, reg_e = self._form_reps(1, 1, reps - h, speculate=sp)
        ms = ms + ms2
        t = sum(ms) / len(ms) / 1e3
        N = self.b.N
        gbs = self.meta_bytes / t / 1e9
        return {
            "records": N,
            "reps": reps,
            "ms": t * 1e3,
            "ms_min": min(ms),
            "records_per_s": N / t,
            "list_forms": (f"in place (HONU_ACL_INPLACE, HONU_REGIONS_INPLACE): ACL lists with every "
                           f"entry present and every region list stay in the records arena; "
                           f"{acl_e} ACL and {reg_e} region table entries written"),
            "table_form": self._form_summary(
                ms_tab, tab_acl, tab_reg, "the same call with acl_inplace 0 and regions_inplace 0: "
                "every list copied into the 20-byte ACL and 4-byte region tables (rounds 1-4)")
            if others else None,
            "regions_table_form": self._form_summary(
                ms_r5, r5_acl, r5_reg, "the same call with regions_inplace 0: ACL lists in place, "
                "region lists in their table (round 5's default)") if others else None,
            "speculation": self._form_summary(
                ms_sp, sp_acl, sp_reg, "the default forms with the context param speculate 1 (the "
                "default's 2 does not speculate here): counts published before the walk ends, ACL "
                "entry flags gathered after the publish, a guarded second launch") if others else None,
            "calls": "honu_decode_batch(data arena NULL) over all records, one call",
            "roofline": {
                "bound": "hbm",
                "kernel": "k_decode_fused (no speculation: the look-back waits it would hide are "
                          "skipped by tiles with no table entries)",
                "achieved": gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": gbs / HBM_PEAK_GBS,
                # the in-place form's kernels (the PMC run also holds the
                # table form's, <..., false>, measured first)
                # <MODE, FORM, INPL>: no speculation (MODE 0) by default,
                # ticket tiles (FORM 0) at 1M records; then the forms of
                # entries measured with speculation (MODE 1)
                "traffic": (pmc_traffic(self.workload("zero_copy"), "k_decode_fused<0, 0, true>")
                            or pmc_traffic(self.workload("zero_copy"), "k_decode_fused<1, 0, true>")
                            or pmc_traffic(self.workload("zero_copy"), "k_decode_fused<1, 1, true>")),
                "traffic_commit": pmc_commit(self.workload("zero_copy")),
                "avg_launch_ms": t * 1e3,
                "algorithmic_bytes_per_launch": self.meta_bytes,
                "algorithmic_bytes": "8 (offsets) + header + Metadata tail read; 352 row + 32 info "
                                     "+ 4 per region TABLE entry + 20 per ACL TABLE entry written, "
                                     "per record (in-place lists: none)",
            },
        }

    def check_zero_copy(self):
        """Every row / table entry against its source row; every Data() subslice's
        digest against its source payload's."""
        b, L, N = self.b, self.lib, self.b.N
        torch.cuda.synchronize()
        s = torch.cuda.current_stream(self.dev).cuda_stream
        c = self.codec.ctx
        mism = torch.empty(4 * N, dtype=torch.uint8, device=self.dev)
        _lib.check(L.honu_verify_decoded(c, P(b.meta), P(b.var), P(b.acl), P(b.reg), P(b.off),
                                         P(self.arena), P(self.dmeta), P(self.dinfo), P(self.dacl),
                                         P(self.dreg), N, P(mism), s), "verify")
        info = self.dinfo.view(torch.int64).view(N, 4)
        doff, dlen = info[:, 0].contiguous(), info[:, 1].contiguous()
        dd = torch.empty(8 * N, dtype=torch.uint8, device=self.dev)
        _lib.check(L.honu_digest_records(c, P(self.arena), P(doff), P(dlen), N, P(dd), s), "digest")
        ok = int(torch.count_nonzero(mism.view(torch.int32))) == 0 and torch.equal(dd, self.dig_src)
        return bool(ok) and self.encode_ok

    # -- materialising, chunk by chunk ---------------------------------------------
    def _issue(self, k, a, e, timed):
        b, L = self.b, self.lib
        n = e - a
        sl = self.slots[k % 2]
        c = sl.codec.ctx
        sm, sc = self.sm, self.sc
        if sl.free is not None:
            sm.wait_event(sl.free)
        ms = sm.cuda_stream
        ro = P(self.rec_off) + 8 * a
        if n >= FUSED_DECODE_MIN:  # honu_decode_batch's own choice of kernels
            _lib.check(L.honu_decode_records(c, P(self.arena), ro, n, P(self.dmeta) + 352 * a,
                                             P(self.dinfo) + 32 * a, P(sl.dacl), b.acl_cap,
                                             P(sl.dreg), b.reg_cap, 1, b.data_cap, P(sl.totals), ms),
                       "decode_records")
        else:
            _lib.check(L.honu_decode_parse(c, P(self.arena), ro, n, P(self.dmeta) + 352 * a,
                                           P(self.dinfo) + 32 * a, ms), "decode_parse")
            _lib.check(L.honu_decode_tables(c, P(self.arena), n, P(self.dmeta) + 352 * a,
                                            P(self.dinfo) + 32 * a, P(sl.dacl), b.acl_cap,
                                            P(sl.dreg), b.reg_cap, P(sl.data), b.data_cap,
                                            P(sl.totals), ms), "decode_tables")
        ev = torch.cuda.Event()
        ev.record(sm)
        sc.wait_event(ev)
        e0 = torch.cuda.Event(enable_timing=True) if timed else None
        e1 = torch.cuda.Event(enable_timing=True) if timed else None
        if timed:
            e0.record(sc)
        _lib.check(L.honu_decode_payloads(c, P(self.arena), n, P(self.dinfo) + 32 * a, P(sl.data),
                                          P(sl.totals), sc.cuda_stream), "decode_payloads")
        if timed:
            e1.record(sc)
            self.events.append((a, e, e0, e1))
        sl.free = torch.cuda.Event()
        sl.free.record(sc)
        return sl

    def materialise_pass(self, timed=False, check=None):
        ok, pending = True, None
        for k, (a, e) in enumerate(self.b.chunks):
            sl = self._issue(k, a, e, timed)
            if check is not None:
                if pending is not None:
                    ok &= self._check(check, pending)
                pending = (a, e, sl)
        if pending is not None:
            ok &= self._check(check, pending)
        cur = torch.cuda.current_stream(self.dev)
        cur.wait_stream(self.sc)
        cur.wait_stream(self.sm)
        return ok

    def _check(self, check, pending):
        a, e, sl = pending
        sl.free.synchronize()
        with torch.cuda.stream(self.sv):
            return bool(check(a, e, sl))

    def _check_chunk(self, a, e, sl):
        b, L = self.b, self.lib
        n = e - a
        s = torch.cuda.current_stream(self.dev).cuda_stream
        c = sl.codec.ctx
        mism = torch.empty(4 * n, dtype=torch.uint8, device=self.dev)
        _lib.check(L.honu_verify_decoded(c, P(b.meta) + 352 * a, P(b.var), P(b.acl), P(b.reg),
                                         P(b.off) + 8 * a, P(self.arena), P(self.dmeta) + 352 * a,
                                         P(self.dinfo) + 32 * a, P(sl.dacl), P(sl.dreg), n, P(mism),
                                         s), "verify")
        info = self.dinfo[32 * a: 32 * e].view(torch.int64).view(n, 4)
        doff, dlen = info[:, 0].contiguous(), info[:, 1].contiguous()
        dd = torch.empty(8 * n, dtype=torch.uint8, device=self.dev)
        _lib.check(L.honu_digest_records(c, P(sl.data), P(doff), P(dlen), n, P(dd), s), "digest")
        ok = int(torch.count_nonzero(mism.view(torch.int32))) == 0
        ok &= torch.equal(dd, self.dig_src[8 * a: 8 * e])
        torch.cuda.current_stream(self.dev).synchronize()
        return bool(ok)

    def materialising(self, steps, warmup):
        for _ in range(warmup):
            self.materialise_pass()
        torch.cuda.synchronize()
        self.events = []
        t0 = time.perf_counter()
        for _ in range(steps):
            self.materialise_pass(timed=True)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / steps
        copy_ms = [x.elapsed_time(y) for (_, _, x, y) in self.events]
        chunk_pay = {a: p for (a, _), p in zip(self.b.chunks, self.b.chunk_payload)}
        copy_bytes = [2 * chunk_pay[a] for (a, _, _, _) in self.events]
        cg = sum(copy_bytes) / (sum(copy_ms) / 1e3) / 1e9
        step_bytes = self.meta_bytes + 2 * self.payload_bytes
        return {
            "records": self.b.N,
            "chunks": len(self.b.chunks),
            "steps": steps,
            "ms_per_pass": el * 1e3,
            "gib_s": self.total / el / 2**30,
            "records_per_s": self.b.N / el,
            "hbm_gbs_algorithmic": step_bytes / el / 1e9,
            "frac_of_spec_whole_pass": step_bytes / el / 1e9 / HBM_PEAK_GBS,
            "roofline": {
                "bound": "hbm",
                "kernel": "k_copy_segments<honu::DecodeSegments>",
                "achieved": cg,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": cg / HBM_PEAK_GBS,
                "traffic": pmc_traffic(self.workload("materialising"),
                                       "k_copy_segments<honu::DecodeSegments"),
                "traffic_commit": pmc_commit(self.workload("materialising")),
                "launches": len(copy_ms),
                "avg_launch_ms": sum(copy_ms) / len(copy_ms),
                "algorithmic_bytes_per_launch": sum(copy_bytes) / len(copy_bytes),
            },
        }

    def workload(self, leg):
        b = self.b
        return (f"{b.N} {self.args.shape} records per GPU: decode (Object.Metadata + Object.Data) "
                f"of one resident records arena, {leg}")

    def run(self, steps, warmup):
        leg = getattr(self.args, "decode_leg", "both")
        zc = mat = None
        zc_ok = mat_ok = True
        if leg in ("both", "zero_copy"):
            zc = self.zero_copy(max(3, steps))
            zc_ok = None if self.args.no_verify else self.check_zero_copy()
        if leg in ("both", "materialising"):
            mat = self.materialising(steps, warmup)
            mat_ok = None if self.args.no_verify else bool(
                self.materialise_pass(check=self._check_chunk))
        name = {"both": "zero copy (one call) + materialising (chunked)", "zero_copy": "zero_copy",
                "materialising": "materialising"}[leg]
        return {
            "workload": self.workload(name),
            "records_arena_bytes": self.total,
            "payload_bytes": self.payload_bytes,
            "metadata_tail_bytes": self.tail_bytes,
            "acl_entries": self.nacl,
            "regions": self.nreg,
            "zero_copy": zc,
            "materialising": mat,
            "verified": None if self.args.no_verify else bool(zc_ok and mat_ok),
            "verified_scope": None if self.args.no_verify else (
                "every record: encode status; both legs: every decoded row byte, span, ACL entry "
                "and region against its source row (honu_verify_decoded), every Data() subslice "
                "(zero copy) / materialised payload digest against its source's"),
        }

    def release(self):
        torch.cuda.synchronize()
        for sl in self.slots:
            sl.codec.close()
        self.codec.close()
        self.slots = []
        self.arena = None
        gc.collect()
        torch.cuda.empty_cache()


# honu_decode_batch's crossover to the single-launch decode (api.hip FUSED_DECODE_MIN_RECORDS)
FUSED_DECODE_MIN = 48 << 10


def _pmc_entry(workload):
    tpath = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(tpath):
        return {}
    return json.load(open(tpath)).get("workloads", {}).get(workload, {})


def pmc_traffic(workload, kernel_prefix):
    """HBM bytes per launch of kernel from the PMC passes of this same command
    (profiles/pmc_traffic.json, tools/pmc_traffic.py), or None."""
    pm = _pmc_entry(workload)
    for k, v in pm.get("kernels", {}).items():
        if k.startswith("void honu::" + kernel_prefix) or k.startswith("honu::" + kernel_prefix):
            return v["traffic_per_launch"]
    return None


def pmc_commit(workload):
    """The commit the PMC passes of the workload's entry were measured on
    (tools/pmc_traffic.py records it), or None."""
    return _pmc_entry(workload).get("commit")


def hbm_probe(codec, dev, nbytes=4 << 30, reps=5, modes=(0, 1, 2, 3, 4), blocks=(1, 2, 4)):
    """The part's achievable streaming rates, measured in this process with the
    library's own probe kernels (honu_hbm_probe: 16 B per lane, the layout of
    tools/hbm_probe.hip and of the guide's float4 copy): read-only, write-only
    and copy (per-wave ranges, grid-stride and per-wave ranges with
    non-temporal loads and stores, 1/2/4 workgroups per CU; the best copy is
    `copy_gbs`, the roofline's achievable denominator). Copy rates count read +
    write bytes."""
    from honu_amd import _lib
    L, c = codec.lib, codec.ctx
    s = torch.cuda.current_stream(dev).cuda_stream
    a = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    a.fill_(1)
    b.fill_(2)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def rate(mode, bpc):
        run = lambda: _lib.check(L.honu_hbm_probe(c, mode, a.data_ptr(), b.data_ptr(), nbytes, bpc, s),  # noqa: E731
                                 "hbm_probe")
        run()
        e0.record()
        for _ in range(reps):
            run()
        e1.record()
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / reps
        return (2 if mode >= 2 else 1) * nbytes / t / 1e9

    out = {"bytes": nbytes, "reps": reps}
    if 0 in modes:
        out["read_gbs"] = max(rate(0, k) for k in blocks)
    if 1 in modes:
        out["write_gbs"] = max(rate(1, k) for k in blocks)
    forms = {2: "wave ranges", 3: "grid stride", 4: "wave ranges, non-temporal"}
    best = max(((rate(m, k), m, k) for m in (2, 3, 4) if m in modes for k in blocks), key=lambda x: x[0])
    out["copy_gbs"], out["copy_form"] = best[0], f"{forms[best[1]]}, {best[2]} workgroups per CU"
    del a, b
    torch.cuda.empty_cache()
    return out


def _oracle_threads():
    """Host threads for the all-core leg: the job's CPU share (OMP_NUM_THREADS is
    the box's share; os.cpu_count() there reports the whole machine)."""
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    n = os.cpu_count() or 1
    return max(1, min(n, share) if share else min(n, 16))


def cpu_baseline(args):
    """The CPU oracle (plain-C restatement of the Go path) on a bounded sample of
    the same workload, cycled for --cpu-seconds: once on 1 thread (the README's
    single-goroutine bench) and once on all the job's cores, the sample split into
    per-thread record ranges (ctypes drops the GIL inside the C calls)."""
    import threading
    sys.path.insert(0, ROOT)
    from honu_amd.metadata import HostBatch
    from oracle import oracle

    n = args.cpu_records
    meta, var, acl, reg, off = gen_meta(args.seed, args.shape, 0, n)
    rng = np.random.default_rng(args.seed)
    payload = rng.integers(0, 256, int(off[n]) + 1, dtype=np.uint8)
    oracle.load()

    def run(ranges, seconds):
        done = [0] * len(ranges)
        nbytes = [0] * len(ranges)
        # every thread's output arrays are allocated and faulted in once, before
        # the clock starts (oracle.CycleWorkspace), so the loop times the codec
        wss = [oracle.CycleWorkspace(HostBatch(meta[a:b], var, acl, reg, payload, off[a:b + 1]))
               for a, b in ranges]
        start = threading.Barrier(len(ranges) + 1)
        stop = [0.0]

        def work(k, b_minus_a):
            ws = wss[k]
            start.wait()
            while True:
                nbytes[k] += ws.cycle()
                done[k] += b_minus_a
                if time.perf_counter() >= stop[0]:
                    break
        ths = [threading.Thread(target=work, args=(k, b - a)) for k, (a, b) in enumerate(ranges)]
        for t in ths:
            t.start()
        t0 = time.perf_counter()
        stop[0] = t0 + seconds
        start.wait()
        for t in ths:
            t.join()
        el = time.perf_counter() - t0
        return sum(nbytes) / el / 2**30, sum(done) / el, el

    T = _oracle_threads()
    one_gib, one_rps, one_s = run([(0, n)], args.cpu_seconds / 2)
    parts = [(k * n // T, (k + 1) * n // T) for k in range(T)]
    all_gib, all_rps, all_s = run([r for r in parts if r[1] > r[0]], args.cpu_seconds / 2)
    model = ""
    try:
        model = [ln.split(":", 1)[1].strip() for ln in open("/proc/cpuinfo") if "model name" in ln][0]
    except Exception:
        pass
    return {
        "value": all_gib,
        "unit": "GiB/s",
        "records_per_s": all_rps,
        "cores": T,
        "kind": "port",
        "value_1core": one_gib,
        "records_per_s_1core": one_rps,
        "sample": f"{n} {args.shape} records (seed {args.seed}) encoded + decoded (materialising) "
                  f"by the C oracle into output arrays allocated once per thread, cycled for {one_s:.1f} s on 1 thread and {all_s:.1f} s on "
                  f"{T} threads (record ranges per thread), {model}; no Go toolchain on the box, "
                  "so the Go reference itself cannot be timed",
    }


def cu_masked_stream(dev, ncu, use):
    """A torch view of a HIP stream whose kernels run only on the CUs i with
    use(i) (hipExtStreamCreateWithCUMask); the stream lives to process exit."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ncu + 31) // 32
    mask = (ctypes.c_uint32 * words)()
    for i in range(ncu):
        if use(i):
            mask[i // 32] |= 1 << (i % 32)
    h = ctypes.c_void_p()
    torch.cuda.set_device(dev)
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
    if rc != 0:
        raise RuntimeError(f"hipExtStreamCreateWithCUMask: {rc}")
    return torch.cuda.ExternalStream(h.value, device=dev)


def _free_port():
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch(args, argv):
    """--gpus N outside torchrun: start N ranks (this file again, one process
    per GPU, RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set) and return the first
    failing exit code. Nothing here touches the GPU (device_count() only
    counts), so the children own their devices from the start."""
    n = args.gpus
    if not args.dry_run and not args.shared_gpu:
        visible = torch.cuda.device_count()
        if visible < n:
            print(f"bench.py: --gpus {n} needs {n} GPUs, {visible} visible", file=sys.stderr)
            return 2
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:  # a rank that fails would leave the others blocked in a collective
        for p in list(live):
            if p.poll() is not None:
                live.remove(p)
                if p.returncode and not rc:
                    rc = p.returncode
                    for q in live:
                        q.terminate()
        time.sleep(0.2)
    return rc


def dry_run(args, world, rank):
    """The launcher's rank plumbing without device work: every rank reports
    its weak-scaling shard over a gloo group; rank 0 prints them."""
    first, n = weak_range(rank, world, args.records)
    shards = [[rank, first, n]]
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
        out = [None] * world
        dist.all_gather_object(out, [rank, first, n, os.getpid()])
        shards = out
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"dry_run": True, "ranks": world, "shards": shards}), flush=True)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse_args(argv)
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch(args, argv))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        dry_run(args, world, rank)
        return
    if args.shared_gpu:  # rehearsal: every rank on GPU 0 (gloo below)
        local = 0
    if local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} needs GPU {local}, {torch.cuda.device_count()} visible",
              file=sys.stderr)
        sys.exit(2)
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if args.shared_gpu:  # RCCL refuses two ranks on one device
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    def barrier():
        if dist is not None:
            dist.barrier()

    gather_max, all_ok = make_reducers(dist, world, torch.device("cuda", local))

    if args.mode == "decode":
        result = decode_mode(args, rank, local, world, dist, barrier, gather_max, all_ok)
    elif args.mode == "encode":
        result = encode_mode(args, rank, local, world, dist, barrier, gather_max, all_ok)
    else:
        result = encdec_mode(args, rank, local, world, dist, barrier, gather_max, all_ok)
    if result is not None and rank == 0:
        if not args.no_cpu_baseline:  # rank 0 only, after every collective leg
            result["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def make_reducers(dist, world, device):
    """(gather_max, all_ok) over the ranks of the default group (identity
    without one): gather_max(x) -> (max over ranks, every rank's x);
    all_ok(flag) -> AND over ranks (None stays None)."""
    def gather_max(x):
        if dist is None:
            return x, [x]
        t = torch.tensor([x], dtype=torch.float64, device=device)
        g = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(g, t)
        vals = [float(v.item()) for v in g]
        return max(vals), vals

    def all_ok(flag):
        if flag is None or dist is None:
            return flag
        v = torch.tensor([1 if flag else 0], device=device)
        dist.all_reduce(v, op=dist.ReduceOp.MIN)
        return bool(v.item())
    return gather_max, all_ok


def decode_legs(bench, args, world, barrier, gather_max, all_ok):
    """The whole-batch decode legs (DecodeBench) of this rank's shard, timed
    between barriers; aggregates over ranks."""
    db = DecodeBench(bench)
    barrier()
    res = db.run(args.steps, args.warmup)
    db.release()
    res["verified"] = all_ok(res["verified"])
    agg = {"ranks": world}
    if res["zero_copy"] is not None:
        zc_ms, zc_all = gather_max(res["zero_copy"]["ms"])
        agg.update(zero_copy_ms_max=zc_ms, zero_copy_records_per_s=world * bench.N / (zc_ms / 1e3),
                   per_rank_zero_copy_ms=zc_all)
    if res["materialising"] is not None:
        mat_ms, mat_all = gather_max(res["materialising"]["ms_per_pass"])
        agg.update(materialising_ms_max=mat_ms,
                   materialising_gib_s=world * db.total / (mat_ms / 1e3) / 2**30,
                   per_rank_materialising_ms=mat_all)
    res["all_ranks"] = agg
    return res


def host_path_leg(bench, args, local, world, gather_max, all_ok, measure=None):
    """SURVEY §8d/§8e host path on every rank at once: pinned H2D -> codec ->
    D2H of a ~4 GiB sample of the rank's own records (tools/host_path.py
    measure); aggregate = all ranks' bytes / the slowest rank's time. bench:
    anything with N, first and total_rec_bytes (an estimate is enough)."""
    if measure is None:
        from tools.host_path import measure
    avg = bench.total_rec_bytes / bench.N
    n = int(max(256, min(bench.N, (4 << 30) // max(1, int(avg)))))
    chunk = int(max(256, n // 16))  # 16 transfers: the pipeline fill and drain are 2 of them
    r = measure(args.shape, n, chunk, reps=2, device=local, first=bench.first)
    enc_s, _ = gather_max(r["encode_s"])
    dec_s, _ = gather_max(r["decode_s"])
    r["rows_match"] = all_ok(r["rows_match"])
    r["all_ranks"] = {
        "ranks": world,
        "encode_host_path_gbs": world * r["record_bytes"] / enc_s / 1e9,
        "decode_host_path_gbs": world * r["record_bytes"] / dec_s / 1e9,
    }
    return r


def scatter_leg(arena, off, dist, world, all_ok, decode_check, sync=None):
    """N > 1 (north_star: RCCL over xGMI only as a plain scatter of
    sub-batches): rank 0's encoded records (arena, off[n+1] int64; None on the
    other ranks) are sent as byte-balanced sub-batches to every rank in one
    group of point-to-point sends (honu_amd.shard.scatter_records: RCCL
    isend/irecv under nccl, gloo on CPU); every rank checks what arrived with
    decode_check(arena, off, n) -> bool. Outside the codec's timed region."""
    from honu_amd.shard import scatter_records
    sync = sync or (lambda: None)
    times = []
    for _ in range(2):
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        mine, moff, first, cnt, sent = scatter_records(arena, off, src=0)
        sync()
        dist.barrier()
        times.append(time.perf_counter() - t0)
    ok = all_ok(bool(decode_check(mine, moff, cnt)))
    sent_t = torch.tensor([sent], dtype=torch.int64, device=moff.device)
    dist.all_reduce(sent_t, op=dist.ReduceOp.MAX)
    sent = int(sent_t.item())
    t = min(times)
    return {"bytes_sent_by_rank0": sent, "scatter_ms": t * 1e3, "scatter_gbs": sent / t / 1e9,
            "per_link_gbs": sent / t / 1e9 / max(1, world - 1), "verified": ok,
            "how": "point-to-point sends batched in one group (batch_isend_irecv) from rank 0, "
                   "byte-balanced contiguous sub-batches, then a zero-copy parse on every rank "
                   "with every status checked"}


def gpu_parse_check(local):
    """decode_check for scatter_leg: Metadata() + Data() (zero-copy parse) of
    the received records on this rank's GPU; True when every status is OK."""
    def check(mine, moff, cnt):
        c = Codec(local, max(cnt, 1))
        dev = torch.device("cuda", local)
        mine, moff = mine.to(dev), moff.to(dev)  # (gloo: received in host memory)
        rows = torch.empty(352 * max(cnt, 1), dtype=torch.uint8, device=dev)
        info = torch.empty(32 * max(cnt, 1), dtype=torch.uint8, device=dev)
        s = torch.cuda.current_stream(dev).cuda_stream
        _lib.check(c.lib.honu_decode_parse(c.ctx, P(mine), P(moff), cnt, P(rows), P(info), s),
                   "parse")
        torch.cuda.synchronize()
        st32 = info[: 32 * cnt].view(torch.int64).view(cnt, 4)[:, 2].contiguous().view(torch.int32)
        ok = bool((st32 == 0).all())
        c.close()
        return ok
    return check


def decode_mode(args, rank, local, world, dist, barrier, gather_max, all_ok):
    """configs[2] alone: the whole-batch decode legs; the line's value is the
    materialising decode rate (records arena bytes / s, all ranks)."""
    bench = Bench(args, rank, local, pipeline=False)
    res = decode_legs(bench, args, world, barrier, gather_max, all_ok)
    if rank != 0:
        return None
    agg = res["all_ranks"]
    mat, zc = res["materialising"], res["zero_copy"]
    if mat is None:  # zero-copy leg alone: records arena bytes / s of Metadata()+Data()
        ms = agg["zero_copy_ms_max"]
        value, roof = world * res["records_arena_bytes"] / (ms / 1e3) / 2**30, zc["roofline"]
    else:
        ms = agg["materialising_ms_max"]
        value, roof = agg["materialising_gib_s"], mat["roofline"]
    return {
        "metric": METRIC,
        "value": value,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded generator mirroring object_test.go:195-386, payload bytes "
                "generated on device",
        "config": {"workload": res["workload"], "records_per_gpu": bench.N, "shape": args.shape,
                   "parallelism": f"dp{world} (records sharded, no data-path collective)"},
        "records_per_s": world * bench.N / (ms / 1e3),
        "roofline": roof,
        "decode": res,
        "verified": res["verified"],
    }


# leg -> (shape, encode only, records per GPU as a fraction of --records,
# the chunk zero-copy decode too)
LEG_SHAPES = {"small": ("small", False, 1, False), "mixed_encode": ("mixed", True, 1, False),
              "medium": ("medium", False, 1, False), "xlarge": ("xlarge", False, 1 / 16, True)}


def legs_of(args):
    """The extra legs of an encdec line (--legs): configs[1] (1M Small encode
    + decode), configs[3] (1M Mixed encode) and the README's other two shapes
    north_star names (1M Medium encode + decode; 64 K XLarge encode + decode,
    i.e. --records / 16, with its chunk zero-copy decode) ride along with the
    default 1M Large line, so that the driver's own run measures every shape."""
    if args.legs == "none":
        return []
    if args.legs == "auto":
        default = args.shape == "large" and args.records == 1 << 20 and args.mode == "encdec"
        return list(LEG_SHAPES) if default else []
    legs = [x.strip() for x in args.legs.split(",") if x.strip()]
    for x in legs:
        if x not in LEG_SHAPES:
            raise SystemExit(f"bench.py: unknown leg {x!r} (known: {', '.join(LEG_SHAPES)})")
    return legs


def pipeline_leg(args, shape, encode_only, rank, local, world, dist, barrier, gather_max, all_ok,
                 records=None, zero_copy=False):
    """One timed pipelined configuration of this rank's --records records of
    `shape` (a Bench of its own, released at the end): warmup, barrier, the
    timed steps, barrier; max over ranks. encode_only: object.Marshal only
    (configs[3]: size pass, output-offset prefix scan, headers + tails,
    payload copy), else encode + materialising decode (configs[1]). Returns
    the leg's dict (value in GiB/s of records over all ranks, the dominant
    copy kernel's roofline, the whole step's algorithmic HBM fraction).
    records: records per GPU (default --records); zero_copy: also the
    Metadata() + zero-copy Data() decode of the leg's largest chunk, alone
    (Bench.zero_copy_decode), after the check."""
    la = argparse.Namespace(**vars(args))
    la.shape = shape
    if records:
        la.records = int(records)
    bench = Bench(la, rank, local, encode_only=encode_only)
    for _ in range(la.warmup):
        bench.step()
    bench.flush()
    torch.cuda.synchronize()
    rec0 = bench.recoveries()
    bench.events = []
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(la.steps):
        bench.step(timed=True)
    bench.flush()
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    recoveries = bench.recoveries() - rec0
    elapsed, per_rank = gather_max(elapsed)
    tot = [bench.total_rec_bytes, bench.N, bench.payload_bytes]
    if dist is not None:
        tt = torch.tensor(tot, dtype=torch.int64, device=bench.dev)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        tot = [int(x) for x in tt.tolist()]
    step_s = elapsed / la.steps
    pay = [2 * bench.chunk_payload[bench.chunks.index((a, b))] for (a, b, *_) in bench.events]
    enc_ms = [x[2].elapsed_time(x[3]) for x in bench.events]
    other_ms = [x[4].elapsed_time(x[5]) for x in bench.events]  # decode copy / offsets
    enc_gbs = sum(pay) / (sum(enc_ms) / 1e3) / 1e9
    verified = None if la.no_verify else bench.verify()
    zc = bench.zero_copy_decode() if zero_copy and not encode_only else None
    bench.release()
    verified = all_ok(verified)
    what = "encode (object.Marshal)" if encode_only else \
        "encode (object.Marshal) + materialising decode (Object.Metadata + Object.Data)"
    workload = f"{bench.N} {shape} records per GPU: {what}"
    kern, kms, kgbs = "k_copy_segments<honu::EncodeSegments>", enc_ms, enc_gbs
    if not encode_only and sum(other_ms) > sum(enc_ms):
        kern, kms = "k_copy_segments<honu::DecodeSegments>", other_ms
        kgbs = sum(pay) / (sum(other_ms) / 1e3) / 1e9
    # the step's algorithmic HBM bytes: encode reads rows + inputs and writes
    # the records (~2 x record bytes), the decode reads them and writes rows +
    # payloads (~2 x record bytes again)
    step_bytes = (2 if encode_only else 4) * bench.total_rec_bytes
    out = {
        "workload": workload,
        "records_per_gpu": bench.N,
        "shape": shape,
        "chunks": len(bench.chunks),
        "steps": la.steps,
        "warmup": la.warmup,
        "ms_per_step": step_s * 1e3,
        "per_rank_ms_per_step": [x / la.steps * 1e3 for x in per_rank],
        "value": tot[0] / step_s / 2**30,
        "unit": "GiB/s",
        "records_per_s": tot[1] / step_s,
        "encoded_bytes_per_gpu": bench.total_rec_bytes,
        "payload_bytes_per_gpu": bench.payload_bytes,
        "step_hbm_gbs_algorithmic": step_bytes / step_s / 1e9,
        "step_frac_of_spec": step_bytes / step_s / 1e9 / HBM_PEAK_GBS,
        "step_bytes": f"{'2' if encode_only else '4'} x encoded record bytes per GPU",
        "roofline": {
            "bound": "hbm",
            "kernel": kern,
            "achieved": kgbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": kgbs / HBM_PEAK_GBS,
            "traffic": pmc_traffic(workload, kern.split(">")[0]),
            "traffic_commit": pmc_commit(workload),
            "launches": len(kms),
            "avg_launch_ms": sum(kms) / max(1, len(kms)),
            "algorithmic_bytes_per_launch": sum(pay) / max(1, len(pay)),
        },
        "encode_copy_gbs": enc_gbs,
        "metadata_decode": None if encode_only else ("fused" if bench.fused_decode(bench.C) else "split"),
        **bench.copy_form(),
        "decode_recoveries_in_timed_steps": None if encode_only else recoveries,
        "verified": verified,
        "verified_scope": None if verified is None else Bench.VERIFIED_SCOPE + (
            " (the records decoded untimed, zero copy, for the check)" if encode_only else ""),
    }
    if zc is not None:
        out["zero_copy_decode"] = {
            "records": zc["records"], "ms": zc["ms"], "records_per_s": zc["records_per_s"],
            "cold_ms": zc["cold_ms"], "cold_records_per_s": zc["cold_records_per_s"],
            "how": "honu_decode_batch (data arena NULL) of the leg's largest chunk, alone, 10 reps "
                   "warm and 10 after a 1 GiB scrub each (cold)"}
    if encode_only:  # configs[3] names the per-record output-offset prefix scan
        out["offsets_ms_per_step"] = sum(other_ms) / la.steps
        out["offsets"] = ("size pass (k_encode_sizes_grp) + exclusive scan (k_scan_lb) of every "
                          "chunk, on the metadata stream, events around both")
    else:
        out["decode_copy_gbs"] = sum(pay) / (sum(other_ms) / 1e3) / 1e9
    return out


def run_legs(args, rank, local, world, dist, barrier, gather_max, all_ok):
    legs = {}
    for name in legs_of(args):
        shape, enc, frac, zc = LEG_SHAPES[name]
        gc.collect()
        torch.cuda.empty_cache()
        if args.leg_pause > 0:
            torch.cuda.synchronize()
            time.sleep(args.leg_pause)
        legs[name] = pipeline_leg(args, shape, enc, rank, local, world, dist, barrier, gather_max,
                                  all_ok, records=max(1, int(args.records * frac)), zero_copy=zc)
    return legs or None


def encode_mode(args, rank, local, world, dist, barrier, gather_max, all_ok):
    """configs[3] alone: object.Marshal of this rank's records per step."""
    leg = pipeline_leg(args, args.shape, True, rank, local, world, dist, barrier, gather_max, all_ok)
    if rank != 0:
        return None
    return {
        "metric": METRIC,
        "value": leg["value"],
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": leg["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded generator mirroring object_test.go:195-386, payload bytes "
                "generated on device",
        "config": {"workload": leg["workload"], "records_per_gpu": leg["records_per_gpu"],
                   "shape": args.shape, "chunks": leg["chunks"],
                   "parallelism": f"dp{world} (records sharded, no data-path collective)"},
        "records_per_s": leg["records_per_s"],
        "roofline": leg["roofline"],
        "encode": leg,
        "verified": leg["verified"],
    }


class _Estimate:
    """N, first and an estimate of the encoded bytes of this rank's records
    (payload of a 4 K-record sample + ~1.1 KB of header and Metadata each),
    for sizing the host-path leg before the bench allocates the device."""

    def __init__(self, args, rank, world):
        from honu_amd.workload import gen_totals
        self.N = args.records
        self.first, _ = weak_range(rank, world, args.records)
        k = min(args.records, 4096)
        pay = gen_totals(args.seed, args.shape, self.first, k)[3]
        self.total_rec_bytes = int((pay / k + 1100) * self.N)


def encdec_mode(args, rank, local, world, dist, barrier, gather_max, all_ok):
    # the host-path leg first, on a device nothing else has touched yet
    # (measured after the 250 GB of bench buffers were freed it ran at 28 GB/s
    # instead of 46 for Large records)
    host_path = None if args.no_host_path or args.host_path_at != "first" else host_path_leg(
        _Estimate(args, rank, world), args, local, world, gather_max, all_ok)
    legs = None
    if args.legs_at == "first":
        legs = run_legs(args, rank, local, world, dist, barrier, gather_max, all_ok)
    gc.collect()
    torch.cuda.empty_cache()
    bench = Bench(args, rank, local)
    for _ in range(args.warmup):
        bench.step()
    bench.flush()
    torch.cuda.synchronize()
    rec0 = bench.recoveries()  # count the timed steps' only
    bench.events = []
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        bench.step(timed=True)
    bench.flush()  # (--copy-order ahead: the last decode copy)
    torch.cuda.synchronize()
    barrier()
    elapsed = time.perf_counter() - t0
    recoveries = bench.recoveries() - rec0  # before anything else decodes on the slots
    # whole-job totals: every rank encodes/decodes its own records
    per_rank_s = [elapsed]
    tot = [bench.total_rec_bytes, bench.N]
    ranks, backend = 1, None
    if dist is not None:
        ranks, backend = dist.get_world_size(), dist.get_backend()
        elapsed, per_rank_s = gather_max(elapsed)
        tt = torch.tensor(tot, dtype=torch.int64, device=bench.dev)
        dist.all_reduce(tt, op=dist.ReduceOp.SUM)
        tot = [int(x) for x in tt.tolist()]

    # per-launch kernel times of the two payload-copy kernels (the HBM-bound part)
    enc_ms = [e0.elapsed_time(e1) for (_, _, e0, e1, _, _) in bench.events]
    dec_ms = [e2.elapsed_time(e3) for (_, _, _, _, e2, e3) in bench.events]
    enc_bytes = [2 * bench.chunk_payload[i % len(bench.chunks)] for i in range(len(enc_ms))]
    enc_gbs = sum(enc_bytes) / (sum(enc_ms) / 1e3) / 1e9
    dec_gbs = sum(enc_bytes) / (sum(dec_ms) / 1e3) / 1e9
    verified = None if args.no_verify else bench.verify()
    zc = bench.zero_copy_decode()
    ok_all = all_ok(verified)
    probe = hbm_probe(bench.codec, bench.dev)
    # the legs after the timed steps: none of them changes the numbers above
    bench.payload = None  # the scatter leg keeps the output slots, nothing else
    gc.collect()
    torch.cuda.empty_cache()
    # the probe's copy forms over as many bytes as one payload copy launch
    # moves (the 4 GiB probe's best form is faster than any
    # copy of a chunk's 2 x 12 GB; profiles/r06/copy_attr/)
    probe_chunk = hbm_probe(bench.codec, bench.dev, nbytes=max(bench.chunk_payload) // 16 * 16, reps=3,
                            modes=(2, 4), blocks=(1, 2))
    scatter = None
    if dist is not None:
        arena = off = None
        if rank == 0:  # the chunk zero_copy_decode left encoded in slot 0
            a, b, sl = bench.zc_chunk
            off = sl.out_off.view(torch.int64)[: b - a + 1]
            arena = sl.out[: int(off[b - a].item())]
            if dist.get_backend() != "nccl":  # gloo moves host tensors only
                arena, off = arena.cpu(), off.cpu()
        scatter = scatter_leg(arena, off, dist, world, all_ok, gpu_parse_check(local),
                              torch.cuda.synchronize)
    bench.release()
    if args.legs_at == "after_main":
        legs = run_legs(args, rank, local, world, dist, barrier, gather_max, all_ok)
    decode = None if args.no_decode_legs else decode_legs(bench, args, world, barrier, gather_max,
                                                          all_ok)
    if args.legs_at == "end":
        legs = run_legs(args, rank, local, world, dist, barrier, gather_max, all_ok)
    if not args.no_host_path and args.host_path_at == "end":
        gc.collect()
        torch.cuda.empty_cache()
        host_path = host_path_leg(_Estimate(args, rank, world), args, local, world, gather_max, all_ok)
    if rank != 0:
        return None
    if decode is not None and decode.get("materialising") is not None:  # the copy's achievable rate too
        mr = decode["materialising"]["roofline"]
        mr["achievable"] = probe["copy_gbs"]
        mr["frac_of_achievable"] = mr["achieved"] / probe["copy_gbs"]
        mr["achievable_at_launch_bytes"] = probe_chunk["copy_gbs"]
        mr["frac_of_achievable_at_launch_bytes"] = mr["achieved"] / probe_chunk["copy_gbs"]
    step_s = elapsed / args.steps
    total_bytes, total_records = tot
    launches = len(dec_ms)
    dom_ms, dom_gbs, dom_name = (sum(dec_ms), dec_gbs, "k_copy_segments<honu::DecodeSegments>")
    if sum(enc_ms) > sum(dec_ms):
        dom_ms, dom_gbs, dom_name = (sum(enc_ms), enc_gbs, "k_copy_segments<honu::EncodeSegments>")
    workload = (f"{bench.N} {args.shape} records per GPU: encode (object.Marshal) + "
                "materialising decode (Object.Metadata + Object.Data)")
    kn = dom_name.split(">")[0]
    traffic = pmc_traffic(workload, kn)  # PMC passes of this same command (tools/pmc_traffic.py)
    result = {
        "metric": METRIC,
        "value": total_bytes / step_s / 2**30,
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": step_s * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic: seeded generator mirroring object_test.go:195-386, payload bytes "
                "generated on device",
        "config": {
            "workload": workload,
            "records_per_gpu": bench.N,
            "shape": args.shape,
            "chunks": len(bench.chunks),
            "chunk_records_max": bench.C,
            "encoded_bytes_per_gpu": bench.total_rec_bytes,
            "payload_bytes_per_gpu": bench.payload_bytes,
            "parallelism": f"dp{world} (records sharded, no data-path collective)",
            "streams": 1 if args.serial else 2,
            "meta_blocks_per_cu": 8 if (args.serial or not args.meta_blocks) else args.meta_blocks,
            "lane_blocks_per_cu": bench.lane_blocks or None,
            "copy_blocks_per_cu": args.copy_blocks or 2,
            "meta_cu_stride": args.meta_cu_stride or None,
            "metadata_beside": bench.meta_beside,
            "metadata_streams": len(bench.sms),
            "copy_streams": 1 if bench.sd is bench.sc else 2,
            "metadata_decode": "fused" if bench.fused_decode(bench.C) else "split",
            **bench.copy_form(),
            "decode_recoveries_in_timed_steps": recoveries,
        },
        "records_per_s": total_records / step_s,
        "ranks": ranks,
        "backend": backend,
        "per_rank_ms_per_step": [x / args.steps * 1e3 for x in per_rank_s],
        "encoded_bytes_all_ranks": total_bytes,
        "records_all_ranks": total_records,
        "roofline": {
            "bound": "hbm",
            "kernel": dom_name,
            "achieved": dom_gbs,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": dom_gbs / HBM_PEAK_GBS,
            "achievable": probe["copy_gbs"],
            "frac_of_achievable": dom_gbs / probe["copy_gbs"],
            "achievable_at_launch_bytes": probe_chunk["copy_gbs"],
            "frac_of_achievable_at_launch_bytes": dom_gbs / probe_chunk["copy_gbs"],
            "traffic": traffic,
            "traffic_source": "profiles/pmc_traffic.json" if traffic else None,
            "traffic_commit": pmc_commit(workload),
            "launches": launches,
            "avg_launch_ms": dom_ms / launches,
            "algorithmic_bytes_per_launch": sum(enc_bytes) / launches,
        },
        "kernels": {
            "encode_copy_gbs": enc_gbs,
            "decode_copy_gbs": dec_gbs,
            "encode_copy_ms_per_step": sum(enc_ms) / args.steps,
            "decode_copy_ms_per_step": sum(dec_ms) / args.steps,
            "step_hbm_gbs_algorithmic": 4 * bench.total_rec_bytes / step_s / 1e9,
            "hbm_probe": probe,
            "hbm_probe_at_launch_bytes": probe_chunk,
            "zero_copy_decode_records_per_s": zc["records_per_s"],
            "zero_copy_decode_ms_per_chunk": zc["ms"],
            "zero_copy_decode_chunk_records": zc["records"],
            "zero_copy_decode_cold_records_per_s": zc["cold_records_per_s"],
            "zero_copy_decode_cold_ms_per_chunk": zc["cold_ms"],
        },
        "verified": ok_all,
        "verified_scope": None if ok_all is None else Bench.VERIFIED_SCOPE,
        "decode": decode,
        "legs": legs,
        "legs_order": {"first": "before the main line", "after_main": "after the main line, before the decode legs",
                       "end": "after the main line and the decode legs"}[args.legs_at],
        "host_path_order": "before everything" if args.host_path_at == "first" else "after everything",
        "host_path": host_path,
        "scatter": scatter,
    }
    return result


if __name__ == "__main__":
    main()
