"""Summarise gpurun_out/split/: per variant, the bench call time and each kernel's average."""
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/split"
for d in sorted(glob.glob(os.path.join(root, "*/"))):
    name = os.path.basename(d.rstrip("/"))
    line = ""
    log = os.path.join(root, name + ".log")
    if os.path.exists(log):
        for x in open(log):
            if x.startswith("{"):
                r = json.loads(x)
                line = f"{r['value']:.1f} {r['unit']}  call {r['roofline'].get('call_us', 0):.1f} us"
    ks = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rocclr" in r["Name"]:
                continue
            short = r["Name"].split("::")[-1].split("(")[0]
            ks.append(f"{short} {float(r['AverageNs']) / 1e3:.1f}")
    print(f"{name:12s} {line} | " + "; ".join(ks))
