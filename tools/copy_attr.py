#!/usr/bin/env python3
"""Counter attribution of the payload copies: per
setting (a directory of rocprofv3 --pmc passes, tools/copy_attr.sh) and per
kernel of interest, every counter averaged over the kernel's launches, and
the derived rates of tools/copy_ceiling.py:

  read/write bytes per launch: 2 x FETCH_SIZE x 1024 (gfx950 correction),
    WRITE_SIZE x 1024; achieved TB/s over the launch's duration;
  rd/wr credit stall: TCC_EA0_{RD,WR}REQ_DRAM_CREDIT_STALL_sum / TCC_CYCLE_sum
    (an L2 channel's request waiting for a DRAM credit: memory queues full);
  rd/wr in flight: TCC_EA0_{RD,WR}REQ_LEVEL_sum / TCC_CYCLE_sum;
  wr stall: TCC_EA0_WRREQ_STALL_sum / TCC_CYCLE_sum; tcc busy: TCC_BUSY_sum /
    TCC_CYCLE_sum; ta busy / ta data stalled by tc: TA_BUSY_sum and
    TA_DATA_STALLED_BY_TC_CYCLES_sum over GRBM_GUI_ACTIVE x CUs.

  python tools/copy_attr.py DIR [DIR ...] > profiles/r06/copy_attr/summary.json
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = ("k_copy_segments<honu::DecodeSegments", "k_copy_segments<honu::EncodeSegments",
           "k_hbm_probe<4>", "k_hbm_probe<2>")


def summarize(root):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for f in sorted(glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True)):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                k = next((k for k in KERNELS if k in name), None)
                if k is None:
                    continue
                vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
    out = {}
    for k, cv in vals.items():
        avg = {c: sum(v) / len(v) for c, v in cv.items()}
        t = sum(durs[k]) / len(durs[k])
        res = {"launches_seen": max(len(v) for v in cv.values()), "launch_ms_mean": t * 1e3,
               "counters": {c: round(v, 1) for c, v in avg.items()}}
        rd, wr = avg.get("FETCH_SIZE", 0) * 2048, avg.get("WRITE_SIZE", 0) * 1024
        res.update(bytes_read=rd, bytes_written=wr, achieved_tbs=(rd + wr) / t / 1e12 if t else None)
        cyc = avg.get("TCC_CYCLE_sum")
        if cyc:
            for c, nm in (("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "rd_credit_stall"),
                          ("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "wr_credit_stall"),
                          ("TCC_EA0_RDREQ_LEVEL_sum", "rd_in_flight"),
                          ("TCC_EA0_WRREQ_LEVEL_sum", "wr_in_flight"),
                          ("TCC_EA0_WRREQ_STALL_sum", "wr_stall"),
                          ("TCC_BUSY_sum", "tcc_busy")):
                if c in avg:
                    res[nm] = round(avg[c] / cyc, 4)
        gui = avg.get("GRBM_GUI_ACTIVE")
        if gui:
            for c, nm in (("TA_BUSY_sum", "ta_busy_per_cu"),
                          ("TA_DATA_STALLED_BY_TC_CYCLES_sum", "ta_data_stalled_by_tc_per_cu")):
                if c in avg:
                    res[nm] = round(avg[c] / gui / 256, 4)
        out[k] = res
    return out


def main():
    print(json.dumps({os.path.basename(os.path.normpath(d)): summarize(d) for d in sys.argv[1:]}, indent=1))


if __name__ == "__main__":
    main()
