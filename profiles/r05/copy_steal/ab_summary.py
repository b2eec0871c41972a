"""Per-variant summary of interleaved bench A/B runs: tags <shape>_s<variant>_r<round>.json."""
import collections
import glob
import json
import statistics
import sys

d = collections.defaultdict(list)
for f in sorted(glob.glob(sys.argv[1] + "/*_r*.json")):
    txt = open(f).read().strip()
    if not txt:
        print("empty", f)
        continue
    j = json.loads(txt)
    tag = f.split("/")[-1][:-5]
    k, r = tag.rsplit("_r", 1)
    d[k].append((int(r), j["ms_per_step"], j.get("verified")))
for k, v in sorted(d.items()):
    v.sort()
    ms = [x[1] for x in v]
    print(f"{k:16s} median {statistics.median(ms):8.3f}  min {min(ms):8.3f}  all verified {all(x[2] for x in v)}  "
          + " ".join(f"{x:.2f}" for x in ms))
