"""Summarise a tools/gpu.sh session: per bench step the JSON line's value /
ms_per_step / roofline frac and the rocprof averages of the XTILE kernels.
Usage: python tools/summ_r6.py gpurun_out/<session> [step ...]"""
import csv
import json
import os
import sys

d = sys.argv[1]
steps = sys.argv[2:] or sorted(f[:-5] for f in os.listdir(d) if f.endswith(".json"))
for st in steps:
    j = json.load(open(os.path.join(d, st + ".json")))
    line = f"{st:14s} {j.get('value', 0):8.1f} {j.get('unit', '')} ms {j.get('ms_per_step', 0):.4f}"
    if "roofline" in j:
        line += f" frac {j['roofline']['frac']:.4f}"
    ks = os.path.join(d, st, "run_kernel_stats.csv")
    if os.path.exists(ks):
        for r in csv.DictReader(open(ks)):
            n = r["Name"]
            for tag in ("k_xtile_reduce", "k_xtile_gather", "k_xtile_fixup", "k_stencil7", "k_spmv_sell", "k_radix"):
                if tag in n:
                    line += f" | {n.split('(')[0].split('::')[-1][:24]} {float(r['AverageNs']) / 1e3:.1f}us x{r['Calls']}"
                    break
    print(line)
