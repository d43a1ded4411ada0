"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs (separate passes) for
one kernel into profiles/pmc_<tag>.json, the `roofline.traffic` source of
bench.py.

usage: python tools/pmc_summary.py <fetch_dir> <write_dir> <kernel> <out.json> [command]

FETCH_SIZE / WRITE_SIZE are KB (x1024).  Per MI355X_MICROARCH.md (HBM
section), gfx950 FETCH_SIZE reports half the bytes of wide (16 B/lane)
coalesced streaming reads; the search kernels read their weight images with
16 B/lane loads and everything else with 4 B/lane, so the read side is
reported both raw and with the x2 correction applied to the weight-image share
(`hbm_bytes_per_launch` uses the corrected value).
"""
import csv
import glob
import json
import os
import statistics
import sys


def counter_values(d, counter, kernel):
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == counter and row["Kernel_Name"].startswith(kernel):
                    vals.append(float(row["Counter_Value"]))
    return vals


def main():
    fetch_dir, write_dir, kernel, out = sys.argv[1:5]
    command = sys.argv[5] if len(sys.argv) > 5 else ""
    fv = counter_values(fetch_dir, "FETCH_SIZE", kernel)
    wv = counter_values(write_dir, "WRITE_SIZE", kernel)
    if not fv or not wv:
        raise SystemExit(f"no {kernel} dispatches in {fetch_dir} / {write_dir}")
    f_kb, w_kb = statistics.median(fv), statistics.median(wv)
    res = {
        "kernel": kernel,
        "command": command,
        "fetch_size_kb_per_launch": f_kb,
        "write_size_kb_per_launch": w_kb,
        "hbm_bytes_per_launch_raw": (f_kb + w_kb) * 1024.0,
        "hbm_bytes_per_launch": (2.0 * f_kb + w_kb) * 1024.0,
        "note": "median over dispatches; FETCH_SIZE doubled (gfx950 reports half of 16 B/lane "
                "streaming reads; the dominant read is the 16 B/lane weight image), WRITE_SIZE as read",
        "raw": {"FETCH_SIZE_kb": fv, "WRITE_SIZE_kb": wv},
    }
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "raw"}))


if __name__ == "__main__":
    main()
