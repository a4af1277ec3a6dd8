"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) of the solve
kernel into a per-launch HBM traffic figure that bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <agents> <out.json> [kernel]

FETCH_SIZE and WRITE_SIZE are in KiB per dispatch (rocprofv3).  No gfx950 x2 correction is
applied to FETCH_SIZE: that correction is calibrated for 16-B/lane streaming reads
(MI355X_MICROARCH.md, HBM section) and this kernel's fetches are instruction fetches and
8-B/lane loads, so the raw value is reported and labelled as such.
"""
import csv
import glob
import json
import os
import statistics
import sys


def per_launch(d, counter, kernel="srb_nmpc_kernel"):
    """median over dispatches of the counter summed over its rows (per-XCD rows, if any)"""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            per[r["Dispatch_Id"]] = per.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    vals = list(per.values())
    return statistics.median(vals), len(vals)


def main():
    fdir, wdir, cfg, agents, out = sys.argv[1:6]
    kernel = sys.argv[6] if len(sys.argv) > 6 else "srb_nmpc_kernel"
    fk, nf = per_launch(fdir, "FETCH_SIZE", kernel)
    wk, nw = per_launch(wdir, "WRITE_SIZE", kernel)
    d = {"kernel": kernel, "config": cfg if not cfg.lstrip("-").isdigit() else int(cfg), "agents": int(agents), "fetch_kib_per_launch": fk, "write_kib_per_launch": wk,
         "hbm_bytes_per_launch": (fk + wk) * 1024.0, "dispatches": [nf, nw],
         "note": "raw FETCH_SIZE + WRITE_SIZE (KiB, median over dispatches), separate rocprofv3 --pmc passes; "
                 "no x2 FETCH correction (reads are not 16-B/lane streams)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
