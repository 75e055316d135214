"""Per-kernel averages of every counter in rocprofv3 --pmc output dirs.

  python tools/summ_pmc.py <dir> [<dir> ...]
"""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].replace("(anonymous namespace)", "anon").split("(")[0]
            k = k.replace("void ", "").split("::")[-1]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        if k.startswith("__amd"):
            continue
        print(f"{d}  {k}: " + ", ".join(f"{c}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))
