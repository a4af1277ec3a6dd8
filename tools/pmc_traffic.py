"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (separate runs, MI355X_MICROARCH.md
HBM section) into per-launch HBM traffic figures that bench.py reports as roofline.traffic.

    python tools/pmc_traffic.py calib <fetch_dir> <write_dir> <out.json>
        the counters of tools/ubench/fetch_calib (1 GiB touched once per dispatch by 8-B/lane
        reads, 16-B/lane reads and 8-B/lane writes) -> counter units per true byte for each
        access width (the guide calibrates only 16-B/lane streams; our kernels load and store
        8 B per lane, so the factor is measured, not assumed)
    python tools/pmc_traffic.py <fetch_dir> <write_dir> <config> <agents> <out.json> [calib.json] [polish_fused]
        per-launch FETCH / WRITE of every srb_* kernel of a bench run (median over dispatches),
        raw and divided by the measured 8-B/lane factors of calib.json

Counter rows are summed per dispatch (one row per XCD / instance where rocprofv3 splits them).
"""
import csv
import glob
import json
import os
import statistics
import sys

KERNELS = ("srb_nmpc_kernel", "srb_polish_kernel", "srb12_kernel", "srb12_pos_kernel", "srb_knn_kernel", "srb_grid_build_kernel", "srb_ll_kernel",
           "calib_read8", "calib_read16", "calib_write8")


def per_dispatch(d, counter):
    """{kernel family: [per-dispatch counter sums]}"""
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    per = {}
    for r in csv.DictReader(open(f)):
        if r["Counter_Name"] != counter:
            continue
        fam = next((k for k in KERNELS if k in r["Kernel_Name"]), None)
        if fam is None:
            continue
        key = (fam, r["Dispatch_Id"])
        per[key] = per.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (fam, _), v in per.items():
        out.setdefault(fam, []).append(v)
    return out


def calib(fdir, wdir, out):
    f, w = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    true_bytes = float(1 << 30)
    d = {"bytes_per_dispatch": true_bytes,
         "fetch_units_per_byte_read8": statistics.median(f["calib_read8"]) / true_bytes,
         "fetch_units_per_byte_read16": statistics.median(f["calib_read16"]) / true_bytes,
         "write_units_per_byte_write8": statistics.median(w["calib_write8"]) / true_bytes,
         "raw": {"FETCH_SIZE": {k: v for k, v in f.items() if k.startswith("calib")},
                 "WRITE_SIZE": {k: v for k, v in w.items() if k.startswith("calib")}},
         "note": "tools/ubench/fetch_calib: 1 GiB (4x the Infinity Cache) touched once per dispatch; counter value "
                 "per true byte for each access width, median over dispatches"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in d.items() if k != "raw"}))


def traffic(fdir, wdir, cfg, agents, out, calib_json=None, polish_fused=0):
    f, w = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    cal = json.load(open(calib_json)) if calib_json else None
    kern = {}
    for fam in sorted(set(f) | set(w)):
        fv = statistics.median(f[fam]) if fam in f else 0.0
        wv = statistics.median(w[fam]) if fam in w else 0.0
        e = {"fetch_raw": fv, "write_raw": wv, "dispatches": [len(f.get(fam, [])), len(w.get(fam, []))]}
        if cal:
            e["fetch_bytes"] = fv / cal["fetch_units_per_byte_read8"]
            e["write_bytes"] = wv / cal["write_units_per_byte_write8"]
            e["hbm_bytes"] = e["fetch_bytes"] + e["write_bytes"]
        kern[fam] = e
    solve = kern.get("srb_nmpc_kernel", kern.get("srb12_kernel", kern.get("srb_ll_kernel", {})))
    d = {"config": int(cfg) if cfg.lstrip("-").isdigit() else cfg, "agents": int(agents), "kernels": kern,
         "hbm_bytes_per_launch": solve.get("hbm_bytes"),
         "calibration": calib_json, "polish_fused": int(polish_fused),
         "note": "FETCH_SIZE / WRITE_SIZE from separate rocprofv3 --pmc passes, median over dispatches, divided by "
                 "the 8-B/lane factors measured by tools/ubench/fetch_calib (calibration file); "
                 "hbm_bytes_per_launch = the solve kernel's"}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps(d))


def main():
    if sys.argv[1] == "calib":
        calib(*sys.argv[2:5])
    else:
        fdir, wdir, cfg, agents, out = sys.argv[1:6]
        traffic(fdir, wdir, cfg, agents, out, sys.argv[6] if len(sys.argv) > 6 else None,
                int(sys.argv[7]) if len(sys.argv) > 7 else 0)


if __name__ == "__main__":
    main()
