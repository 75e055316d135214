"""Summarise A/B profile output (tools/gpu.sh senv steps): bench ms/step and per-kernel totals per call."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/abp"
for log in sorted(glob.glob(os.path.join(d, "bench_*.log"))):
    tag = os.path.basename(log)[6:-4]
    line = [ln for ln in open(log) if ln.startswith("{")]
    if not line:
        print(tag, "no result")
        continue
    r = json.loads(line[-1])
    st = glob.glob(os.path.join(d, tag, "**", "*kernel_stats.csv"), recursive=True)
    ks = {}
    if st:
        for row in csv.DictReader(open(st[0])):
            name = row["Name"].replace("(anonymous namespace)", "anon").split("(")[0].split("<")[0].split("::")[-1].replace("void ", "")
            ks[name] = ks.get(name, 0.0) + float(row["TotalDurationNs"]) / 1e3
    calls = r["steps"] + r["warmup"] + max(r["steps"], 10)
    print(f"{tag:24s} {r['ms_per_step'] * 1e3:7.1f} us  " +
          "  ".join(f"{k} {v / calls:6.1f}" for k, v in sorted(ks.items()) if k.startswith("k_")))
