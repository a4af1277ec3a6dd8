"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs) of the solve
kernel into a per-launch HBM traffic figure that bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <agents> <out.json>

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


def per_launch(d, counter):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(f))
            if "srb_nmpc_kernel" in r["Kernel_Name"] and r["Counter_Name"] == counter]
    return statistics.median(vals), len(vals)


def main():
    fdir, wdir, cfg, agents, out = sys.argv[1:6]
    fk, nf = per_launch(fdir, "FETCH_SIZE")
    wk, nw = per_launch(wdir, "WRITE_SIZE")
    d = {"config": int(cfg), "agents": int(agents), "fetch_kib_per_launch": fk, "write_kib_per_launch": wk,
         "hbm_bytes_per_launch": (fk + wk) * 1024.0, "dispatches": [nf, nw],
         "note": "raw FETCH_SIZE + WRITE_SIZE (KiB, median over dispatches), separate rocprofv3 --pmc passes; "
                 "no x2 FETCH correction (reads are not 16-B/lane streams)"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


if __name__ == "__main__":
    main()
