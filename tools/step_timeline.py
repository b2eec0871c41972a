"""Timeline of a bench run's timed steps from its rocprofv3 kernel trace:
for each timed step, every kernel's start and end relative to the end of the
previous step's decode copy, and the time the copy engine spent idle (no
payload copy running) with what was running meanwhile.

A pipelined step's kernels overlap, so the per-kernel averages of
tools/timed_stats.py cannot tell which chain sets the step time; the idle gaps
between consecutive payload copies can: a gap is time the bandwidth-bound
copies wait for a metadata kernel.

usage: python tools/step_timeline.py KERNEL_TRACE.csv[.gz] BENCH.json [STEPS_SHOWN]
"""
import csv
import gzip
import io
import json
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from timed_stats import DEC, ENC, window  # noqa: E402

SHORT = [("k_encode_meta_lane", "lane"), ("k_encode_acl_grp", "acl"), ("k_encode_sizes_grp", "sizes"),
         ("k_scan_lb", "scan"), ("k_decode_fused", "decode"), ("k_decode_guard", "guard"),
         ("k_decode_parse_win", "parse"), ("k_decode_fill_grp", "fill"), (ENC, "ENC_COPY"),
         (DEC, "DEC_COPY")]


def short(name):
    for k, s in SHORT:
        if k in name:
            return s
    return name.split("(")[0][-24:]


def load(path):
    raw = gzip.open(path, "rt") if path.endswith(".gz") else open(path, newline="")
    rows = list(csv.DictReader(io.StringIO(raw.read())))
    ks = [(r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
    ks.sort(key=lambda k: k[1])
    return ks


def main(argv):
    trace, bench_json = argv[0], argv[1]
    shown = int(argv[2]) if len(argv) > 2 else 3
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    chunks, steps = b["config"]["chunks"], b["steps"]
    ks = load(trace)
    t0, t1 = window(ks, b["warmup"], steps, chunks)
    inw = [k for k in ks if k[1] >= t0 and k[2] <= t1 + 1]
    copies = sorted([k for k in inw if DEC in k[0] or ENC in k[0]], key=lambda k: k[1])
    idle, busy = 0, 0
    gaps = []
    prev_end = t0
    for name, s, e in copies:
        if s > prev_end:
            gap = s - prev_end
            idle += gap
            running = sorted({short(n) for n, a, z in inw if a < s and z > prev_end and n not in (DEC, ENC)
                              and DEC not in n and ENC not in n})
            gaps.append((prev_end - t0, gap, short(name), running))
        busy += e - max(s, prev_end)
        prev_end = max(prev_end, e)
    span = t1 - t0
    print(f"timed window {span / 1e6:.3f} ms over {steps} steps = {span / 1e6 / steps:.3f} ms/step")
    print(f"payload copies busy {busy / 1e6:.3f} ms ({100.0 * busy / span:.1f} %), "
          f"idle {idle / 1e6:.3f} ms = {idle / 1e6 / steps:.3f} ms/step")
    by = {}
    for at, gap, nxt, running in gaps:
        key = (nxt, tuple(running))
        by.setdefault(key, [0, 0])
        by[key][0] += 1
        by[key][1] += gap
    print("copy-engine idle gaps by the copy that ends them and the kernels running in them:")
    for (nxt, running), (n, g) in sorted(by.items(), key=lambda kv: -kv[1][1]):
        print(f"  before {nxt:9s} {n:4d} gaps {g / 1e6:8.3f} ms  beside: {', '.join(running) or '-'}")
    step_len = span / steps
    for i in range(min(shown, steps)):
        a = t0 + i * step_len
        z = a + step_len
        print(f"step {i} (window {a - t0:.0f}..{z - t0:.0f} ns)")
        for name, s, e in inw:
            if e > a and s < z:
                print(f"  {short(name):9s} {(s - a) / 1e3:9.1f} .. {(e - a) / 1e3:9.1f} us  ({(e - s) / 1e3:7.1f})")


if __name__ == "__main__":
    main(sys.argv[1:])
