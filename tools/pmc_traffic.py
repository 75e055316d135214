"""Turn rocprofv3 FETCH_SIZE / WRITE_SIZE passes into per-launch byte counts.

  python tools/pmc_traffic.py <tag> <fetch_dir> <write_dir> [calib_dir] [--out profiles/traffic.json]
                             [--per-call KERNEL=N ...]

--per-call k_xtile_gather=3 says a call launches that kernel 3 times (XTILE
cache-sized ranges): its per-dispatch average is multiplied by 3 in
bytes_per_call.  --exclude k_a,k_b leaves set-up kernels (run once per solve,
not per step) out of bytes_per_call; --fetch-factor F applies F instead of a
calibration pass (the gfx950 factor the calibration passes measured: 2.0).

Counters are in KiB per dispatch (FETCH_SIZE = TCC_EA0_RDREQ-based, so
Infinity-Cache hits are included).  Per MI355X_MICROARCH.md §HBM, FETCH_SIZE
reads 1/2 of a 16 B/lane stream on gfx950; other widths are uncalibrated, so
the calibration pass (tools/pmc_calibrate.py) measures the factor for the
4 B/lane loads these kernels issue, and that factor is applied.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


# kernels of the device-input plan build (bench.py times it once per run)
PLAN_BUILD = {"k_validate_device_csr", "k_xt_counts", "k_xt_scatter", "k_xt_permute_blocks"}


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != counter:
                continue
            name = row["Kernel_Name"].replace("(anonymous namespace)", "anon")
            short = name.split("(")[0].split("<")[0].split("::")[-1].replace("void ", "")
            vals[short].append(float(row["Counter_Value"]) * 1024.0)
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out = "profiles/traffic.json"
    if "--out" in sys.argv:
        out = sys.argv[sys.argv.index("--out") + 1]
        args = [a for a in args if a != out]
    per_call = {}
    exclude, fixed_factor = set(), None
    for i, a in enumerate(sys.argv):
        if a == "--per-call":
            k, v = sys.argv[i + 1].split("=")
            per_call[k] = int(v)
            args = [b for b in args if b != sys.argv[i + 1]]
        if a == "--exclude":
            exclude = set(sys.argv[i + 1].split(","))
            args = [b for b in args if b != sys.argv[i + 1]]
        if a == "--fetch-factor":
            fixed_factor = float(sys.argv[i + 1])
            args = [b for b in args if b != sys.argv[i + 1]]
    tag, fdir, wdir = args[:3]
    cal = {"k_read16": 1 << 30, "k_read4": 1 << 30}
    factor4 = None
    factor16 = None
    if len(args) > 3:
        cf, _ = per_kernel(args[3], "FETCH_SIZE")
        for k, v in cf.items():
            if k.startswith("k_read16"):
                factor16 = cal["k_read16"] / v
            if k.startswith("k_read4"):
                factor4 = cal["k_read4"] / v
    fetch, n = per_kernel(fdir, "FETCH_SIZE")
    write, _ = per_kernel(wdir, "WRITE_SIZE")
    db = json.load(open(out)) if os.path.exists(out) else {}
    if fixed_factor:
        factor4 = factor16 = fixed_factor
    f4 = factor4 if factor4 else 1.0
    ent = {"kernels": {}, "fetch_factor_4B": factor4, "fetch_factor_16B": factor16,
           "note": "FETCH_SIZE*1024*fetch_factor_4B + WRITE_SIZE*1024, averaged over dispatches; "
                   "fabric-side bytes (Infinity-Cache hits included)"}
    tot = 0.0
    for k in fetch:
        if not k.startswith("k_"):
            continue
        rb = fetch[k] * f4
        wb = write.get(k, 0.0)
        ent["kernels"][k] = {"read_bytes": rb, "write_bytes": wb, "dispatches": n[k],
                             "raw_fetch_bytes": fetch[k], "launches_per_call": per_call.get(k, 1)}
        if k.startswith("k_copy"):  # bench.py copy / read ceiling probes, not part of the workload
            ent["kernels"][k]["probe"] = True
            continue
        if k in PLAN_BUILD:  # device-side plan build (once per plan, not per call)
            ent["kernels"][k]["plan_build"] = True
            continue
        if k in exclude:  # set-up kernels of an iterative workload
            ent["kernels"][k]["setup"] = True
            continue
        tot += (rb + wb) * per_call.get(k, 1)
    ent["bytes_per_call"] = tot
    db[tag] = ent
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(db, open(out, "w"), indent=1)
    print(json.dumps({tag: ent}, indent=1))


if __name__ == "__main__":
    main()
