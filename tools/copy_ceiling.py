#!/usr/bin/env python3
"""The box's streaming ceiling from the copy-sweep counter passes (VERDICT
r04 item 3): rocprofv3 --pmc passes of tools/copy_sweep in its one-form modes
(read, write, copy; tools/tmp scripts), one directory per (mode, pass) named
pmc_<mode>_<first counter>/ with run_counter_collection.csv inside. For every
mode it averages each counter over the form's launches (the k_read / k_write
/ k_copy kernels, the fill launches excluded) and derives:

  bytes_read / bytes_written per launch: FETCH_SIZE x 2 x 1024 (the gfx950
    correction, MI355X_MICROARCH.md "HBM") and WRITE_SIZE x 1024;
  achieved TB/s: those bytes / the launch's duration;
  rd/wr DRAM credit stall: TCC_EA0_{RD,WR}REQ_DRAM_CREDIT_STALL_sum / TCC_CYCLE_sum,
    the share of L2-channel cycles a request waited for a DRAM credit
    (the memory controllers' queues full);
  rd/wr in flight: TCC_EA0_{RD,WR}REQ_LEVEL_sum / TCC_CYCLE_sum, the mean
    number of outstanding DRAM requests per L2 channel.

  python tools/copy_ceiling.py gpurun_out/r05c > profiles/r05/copy_ceiling.json
"""
import collections
import csv
import glob
import json
import os
import sys

KERNELS = {"read": "k_read", "write": "k_write", "copy": "k_copy"}


def main():
    root = sys.argv[1]
    out = {}
    for mode, kern in KERNELS.items():
        vals = collections.defaultdict(list)
        durs = []
        for d in sorted(glob.glob(os.path.join(root, f"pmc_{mode}_*"))):
            f = os.path.join(d, "run_counter_collection.csv")
            if not os.path.isdir(d) or not os.path.exists(f):
                continue
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    if kern not in r["Kernel_Name"]:
                        continue
                    vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
                    durs.append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e9)
        if not vals:
            continue
        avg = {k: sum(v) / len(v) for k, v in vals.items()}
        t = sum(durs) / len(durs)
        res = {"counters": {k: round(v, 1) for k, v in avg.items()}, "launch_s_mean": t}
        rd = avg.get("FETCH_SIZE", 0) * 2 * 1024
        wr = avg.get("WRITE_SIZE", 0) * 1024
        res["bytes_read"], res["bytes_written"] = rd, wr
        res["achieved_tbs"] = (rd + wr) / t / 1e12
        cyc = avg.get("TCC_CYCLE_sum")
        if cyc:
            for k, name in (("TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum", "rd_credit_stall"),
                            ("TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum", "wr_credit_stall"),
                            ("TCC_EA0_RDREQ_LEVEL_sum", "rd_in_flight"),
                            ("TCC_EA0_WRREQ_LEVEL_sum", "wr_in_flight"),
                            ("TCC_BUSY_sum", "tcc_busy")):
                if k in avg:
                    res[name] = round(avg[k] / cyc, 3)
        out[mode] = res
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
