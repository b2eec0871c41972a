"""tools/timed_stats.py cuts a bench run's timed steps out of its rocprofv3
kernel trace: a synthetic trace with a warmup step, timed steps and a slow
verification step must give the timed launches only."""
import csv
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import timed_stats  # noqa: E402

ENC = "void honu::k_copy_segments<honu::EncodeSegments, 4, 0>(...)"
DEC = "void honu::k_copy_segments<honu::DecodeSegments, 4, 0>(...)"
META = "honu::k_decode_fused(...)"


def _trace(path, warmup, steps, chunks, timed_ns, slow_ns):
    rows, t = [], 1000
    for step in range(warmup + steps + 1):  # + the verification step
        d = slow_ns if step == warmup + steps else timed_ns
        for _ in range(chunks):
            rows.append((META, t, t + 50))
            rows.append((ENC, t + 10, t + 10 + d))
            rows.append((DEC, t + 20 + d, t + 20 + 2 * d))
            t += 30 + 2 * d
        t += 100  # barrier / synchronize between steps
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writerows(rows)


def test_timed_window(tmp_path):
    warmup, steps, chunks = 1, 3, 4
    tr = tmp_path / "kernel_trace.csv"
    _trace(tr, warmup, steps, chunks, timed_ns=4000, slow_ns=5500)
    ks = timed_stats.load(tr)
    t0, t1 = timed_stats.window(ks, warmup, steps, chunks)
    st = {r["Name"]: r for r in timed_stats.stats(ks, t0, t1)}
    assert st[ENC]["Calls"] == steps * chunks and st[DEC]["Calls"] == steps * chunks
    assert st[ENC]["AverageNs"] == 4000 and st[DEC]["MaxNs"] == 4000  # no verification launch
    assert st[META]["Calls"] == steps * chunks
    # the whole CLI: bench line in, stats file out
    bench = tmp_path / "bench.json"
    bench.write_text(json.dumps({"warmup": warmup, "steps": steps, "ms_per_step": 0.0,
                                 "config": {"chunks": chunks},
                                 "roofline": {"algorithmic_bytes_per_launch": 8e6, "peak": 8000.0}}))
    out = tmp_path / "timed.csv"
    timed_stats.main([str(tr), str(bench), str(out)])
    with open(out) as f:
        got = {r["Name"]: r for r in csv.DictReader(f)}
    assert int(got[ENC]["Calls"]) == steps * chunks


def test_window_needs_enough_launches(tmp_path):
    tr = tmp_path / "kernel_trace.csv"
    _trace(tr, 1, 1, 2, timed_ns=100, slow_ns=100)
    ks = timed_stats.load(tr)
    try:
        timed_stats.window(ks, 1, 5, 2)
    except SystemExit as e:
        assert "decode copies" in str(e)
    else:
        raise AssertionError("window() accepted a trace shorter than the run")
