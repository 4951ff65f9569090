"""Summarise rocprofv3 PMC passes into per-launch HBM bytes for the bench's kernels."""
import csv
import glob
import json
import os
import sys


def rows(pattern):
    out = []
    for f in glob.glob(pattern, recursive=True):
        with open(f) as fh:
            out += list(csv.DictReader(fh))
    return out


def main(d):
    res = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        per = {}
        for r in rows(os.path.join(d, c, "**", "*counter_collection.csv")):
            name = r.get("Kernel_Name", "")
            if "qppvm" not in name:
                continue
            k = "fast" if "fast" in name else "active"
            per.setdefault(k, []).append(float(r["Counter_Value"]))
        res[c] = {k: sum(v) / len(v) for k, v in per.items()}  # KB per dispatch
    stats = {}
    for r in rows(os.path.join(d, "trace", "**", "*kernel_stats.csv")):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"])}
    fetch = sum(res["FETCH_SIZE"].values())
    write = sum(res["WRITE_SIZE"].values())
    out = {
        "fetch_kb_per_solve_raw": fetch,
        "write_kb_per_solve_raw": write,
        # MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half the bytes of wide coalesced
        # streaming reads; our reads are 8-B-per-lane buffer loads (uncalibrated width), so
        # both the raw and the x2-corrected read bytes are reported.
        "hbm_bytes_per_solve_raw": (fetch + write) * 1024,
        "hbm_bytes_per_solve_fetch_x2": (2 * fetch + write) * 1024,
        "per_kernel": res,
        "kernel_stats": stats,
    }
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
