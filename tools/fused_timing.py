#!/usr/bin/env python3
"""Where the single-launch decode (k_decode_fused) spends a tile's time under
full load: the timing build (make -C honu_amd timing, -DHONU_STAGE_TIMING)
has lane 0 of every wave add the time since its previous stamp to a stage
counter at fixed points of every tile it takes (win.h WSTAMP 0..9 inside the
walk, fused.hip 10..15 after it; the ACL fill is 13 + 14 + 15: its rounds'
waits (the staging DMA and every store issued before it), its passes, the
rest). The sums are kept in LDS until the wave ends, so stamps add no waits
for outstanding stores (win.h). Sum over waves / tiles = mean stage time per
tile in microseconds (s_memrealtime, 100 MHz); the stages add up to the
launch's waves x their lifetime.

  HONU_LIB_PATH=honu_amd/libhonu_codec_timing.so python tools/fused_timing.py
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("HONU_LIB_PATH", os.path.join(ROOT, "honu_amd", "libhonu_codec_timing.so"))
from honu_amd import _lib  # noqa: E402
from honu_amd.object import Codec  # noqa: E402
from honu_amd.workload import gen_meta  # noqa: E402

STAGES = ["ticket", "rec_off", "header", "window1", "to_acl_count", "acl_flags",
          "window_after_acl", "regions_to_sig", "window_after_sig", "tail_end",
          "publish_rows_out", "lookback_wait", "info_regions", "acl_fill_rest",
          "acl_fill_wait", "acl_fill_passes"]
P = lambda t: t.data_ptr()  # noqa: E731


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="small")
    ap.add_argument("--records", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--acl-inplace", type=int, default=1, choices=[0, 1],
                    help="context param acl_inplace: 1 the in-place ACL lists (default), 0 the table")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n = a.records
    codec = Codec(0, n)
    L, c = codec.lib, codec.ctx
    _lib.check(L.honu_ctx_set_param(c, b"acl_inplace", a.acl_inplace), "param")
    meta, var, acl, reg, off = gen_meta(1, a.shape, 0, n)

    def D(x):
        x = np.ascontiguousarray(x)
        t = torch.empty(max(x.nbytes, 16), dtype=torch.uint8, device=dev)
        t[: x.nbytes].copy_(torch.from_numpy(x.view(np.uint8).reshape(-1)))
        return t
    dm, dv, da, dr, do = D(meta), D(var), D(acl), D(reg), D(off)
    s = torch.cuda.current_stream().cuda_stream
    pay = torch.empty(int(off[n]) + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_gen_payload(c, 1, 0, n, P(do), P(pay), s), "gen")
    out_off = torch.empty(8 * (n + 1), dtype=torch.uint8, device=dev)
    st = torch.empty(4 * n + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_encode_sizes(c, P(dm), len(var), P(da), len(acl), P(dr), len(reg), P(do), n,
                                   P(out_off), P(st), s), "sizes")
    _lib.check(L.honu_exclusive_scan(c, P(out_off), n, P(out_off), s), "scan")
    total = int(out_off.view(torch.int64)[n].item())
    out = torch.empty(total + 16, dtype=torch.uint8, device=dev)
    _lib.check(L.honu_encode(c, P(dm), P(dv), len(var), P(da), len(acl), P(dr), len(reg), P(pay),
                             P(do), n, P(out), total, P(out_off), P(st), s), "encode")
    del pay
    acl_cap = int(meta["acl_count"].astype(np.int64).sum()) + 1
    reg_cap = int(meta["regions_count"].astype(np.int64).sum()) + 1
    dmeta = torch.empty(352 * n, dtype=torch.uint8, device=dev)
    dinfo = torch.empty(32 * n, dtype=torch.uint8, device=dev)
    dacl = torch.empty(20 * acl_cap, dtype=torch.uint8, device=dev)
    dreg = torch.empty(4 * reg_cap, dtype=torch.uint8, device=dev)
    tot = torch.empty(32, dtype=torch.uint8, device=dev)
    fn = L.honu_debug_stage_times
    fn.restype = C.c_int32
    fn.argtypes = [C.c_void_p, C.c_uint64, C.c_int32]

    def run():
        _lib.check(L.honu_decode_records(c, P(out), P(out_off), n, P(dmeta), P(dinfo), P(dacl),
                                         acl_cap, P(dreg), reg_cap, 0, 0, P(tot), s), "decode")
    run()
    torch.cuda.synchronize()
    ms = []
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        ms.append(e0.elapsed_time(e1))
    assert fn(None, 0, 1) == 0  # zero the sums, then one stamped launch
    run()
    torch.cuda.synchronize()
    waves = 2 * 4 * torch.cuda.get_device_properties(0).multi_processor_count
    buf = np.zeros((waves, 16), np.uint64)
    assert fn(buf.ctypes.data, waves, 0) == 0
    ntiles = (n + 63) // 64
    per_tile = buf.astype(np.float64).sum(axis=0) / ntiles / 100.0  # us
    res = {"shape": a.shape, "records": n, "acl_inplace": a.acl_inplace, "tiles": ntiles, "waves": waves,
           "kernel_ms_unstamped": min(ms),
           "stage_us_per_tile": {k: round(float(per_tile[i]), 3) for i, k in enumerate(STAGES)},
           "tile_us_total": round(float(per_tile[: len(STAGES)].sum()), 3),
           "tiles_per_wave": ntiles / waves}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
