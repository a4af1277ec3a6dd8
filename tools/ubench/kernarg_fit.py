"""Per-workgroup and fixed FETCH_SIZE / WRITE_SIZE (calibrated bytes) of the kernels of a ubench that runs
each at 1024 and 4096 workgroups, three times (tools/ubench/kernarg_fetch, code_fetch).
    python tools/ubench/kernarg_fit.py <fetch_dir> <write_dir> <calib.json> <out.json> [name,name,...]"""
import csv
import glob
import json
import os
import sys

import numpy as np

GRIDS, REPS = (1024, 4096), 3
NAMES = ("karg_byval", "karg_byptr", "wr_packed", "wr_aligned")


def per_kernel(d, counter, names):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        name = next((n for n in names if n in r["Kernel_Name"]), None)
        if name:
            key = (name, int(r["Dispatch_Id"]))
            per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for n in names:
        v = [per[k] for k in sorted(per) if k[0] == n]
        out[n] = v
    return out


def main(fdir, wdir, calib, path, names=",".join(NAMES)):
    names = names.split(",")
    cal = json.load(open(calib))
    res = {}
    for ctr, d, unit in (("FETCH_SIZE", fdir, cal["fetch_units_per_byte_read8"]),
                         ("WRITE_SIZE", wdir, cal["write_units_per_byte_write8"])):
        for n, v in per_kernel(d, ctr, names).items():
            b = np.array(v) / unit
            g = np.repeat(GRIDS, REPS)[:len(b)]
            med = [float(np.median(b[g == x])) for x in GRIDS]
            slope = (med[1] - med[0]) / (GRIDS[1] - GRIDS[0])
            res.setdefault(n, {})[ctr] = {"median_bytes": med, "bytes_per_workgroup": slope,
                                          "fixed_bytes": med[0] - slope * GRIDS[0]}
            print(f"{n:12s} {ctr:10s} per workgroup {slope:8.1f} B   fixed {med[0] - slope * GRIDS[0]:10.0f} B   "
                  f"medians {med[0]:.0f} / {med[1]:.0f}")
    json.dump(res, open(path, "w"), indent=1)


if __name__ == "__main__":
    main(*sys.argv[1:6])
