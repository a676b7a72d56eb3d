"""Summarise scripts/fetch_calib.sh: per kernel, the rocprofv3 counters per dispatch
against the known byte count, i.e. the factor that turns FETCH_SIZE / WRITE_SIZE (KiB)
into bytes at that access width.  Writes <out>/fetch_calib.json (and, with --commit,
profiles/<round>/fetch_calib.json)."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/fcal"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
timing = {}
for line in open(os.path.join(out, "timing.log")):
    m = re.match(r"(\w+) bytes=(\S+) ms_mean=(\S+) ms_best=(\S+) GBps_mean=(\S+)", line)
    if m:
        timing[m.group(1)] = {"bytes": float(m.group(2)), "ms_mean": float(m.group(3)),
                              "GBps": float(m.group(5))}
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(out, "p*", "**", "*counter_collection.csv"), recursive=True):
    per = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(f)):
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"].split("(")[0]
    for (d, c), v in per.items():
        vals[names[d]][c].append(v)
res = {}
for k, t in timing.items():
    cs = {c: sum(v) / len(v) for c, v in vals.get(k, {}).items()}
    e = {"known_bytes": t["bytes"], "ms_mean": t["ms_mean"], "GBps_mean": t["GBps"], "counters": cs}
    if "FETCH_SIZE" in cs and cs["FETCH_SIZE"] > 0:
        e["fetch_factor"] = t["bytes"] / (cs["FETCH_SIZE"] * 1024.0)   # bytes = factor x FETCH_SIZE(KiB) x 1024
    if "WRITE_SIZE" in cs and cs["WRITE_SIZE"] > 0:
        e["write_factor"] = t["bytes"] / (cs["WRITE_SIZE"] * 1024.0)
    res[k] = e
doc = {"what": "rocprofv3 FETCH_SIZE / WRITE_SIZE vs a known byte count on a 2 GiB array (8x the Infinity "
               "Cache), gfx950; factor = known bytes / (counter KiB x 1024)",
       "source": "scripts/fetch_calib.hip, scripts/fetch_calib.sh", "kernels": res}
json.dump(doc, open(os.path.join(out, "fetch_calib.json"), "w"), indent=1)
print(json.dumps(doc, indent=1))
if "--commit" in sys.argv:
    dst = sys.argv[sys.argv.index("--commit") + 1]
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump(doc, open(dst, "w"), indent=1)
