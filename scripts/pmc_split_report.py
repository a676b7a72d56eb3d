"""Report for scripts/pmc_split.py: counters per PGD evaluation per wave."""
import csv, glob, json, sys
from collections import defaultdict
d = sys.argv[1]
ev = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "rl_optimize_kernel" in r["Kernel_Name"]:
            per[int(r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
ids = sorted(per)
a, b = per[ids[0]], per[ids[1]]
dev = ev["evals"][0] - ev["evals"][1]
waves = ev["waves"]
out = {"evals": ev["evals"], "per_eval_per_wave": {c: (a[c] - b[c]) / dev * 1024 / waves for c in a},
       "rest_per_wave": {c: b[c] / waves for c in b}, "full_per_wave": {c: a[c] / waves for c in a}}
print(json.dumps(out, indent=1))
