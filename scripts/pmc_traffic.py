#!/usr/bin/env python3
"""Turn rocprofv3 --pmc CSVs (FETCH_SIZE pass + WRITE_SIZE pass) into HBM bytes per launch of
the lift kernel, with the gfx950 correction of MI355X_MICROARCH.md §HBM: FETCH_SIZE reads half
the bytes of a wide coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B
stores.  Both counters are in KiB.

usage: pmc_traffic.py <fetch_counter_collection.csv> <write_counter_collection.csv> <config> <records> <out.json> [kernel]
"""
import csv
import json
import statistics
import sys


def per_dispatch(path, counter, name_sub):
    """Per-dispatch totals of the workload's full-size lift launches (bench.py's clock spin-up
    lifts a smaller record set)."""
    vals, names = {}, {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if counter not in row.get("Counter_Name", "") or name_sub not in row.get("Kernel_Name", ""):
                continue
            d = row.get("Dispatch_Id") or row.get("Correlation_Id")
            names[d] = row["Kernel_Name"]
            vals[d] = vals.get(d, 0.0) + float(row["Counter_Value"])
    if not vals:
        return []
    top = max(vals.values())  # the workload's full-size launches
    return [v for v in vals.values() if v >= 0.9 * top]


def main():
    fetch_csv, write_csv, config, records, out = sys.argv[1:6]
    kernel = sys.argv[6] if len(sys.argv) > 6 else "k_lift"
    fetch = per_dispatch(fetch_csv, "FETCH_SIZE", kernel)
    write = per_dispatch(write_csv, "WRITE_SIZE", kernel)
    if not fetch or not write:
        raise SystemExit(f"no {kernel} dispatches found in the PMC CSVs")
    f_kib, w_kib = statistics.median(fetch), statistics.median(write)
    doc = {
        "config": config, "records": int(records), "kernel": kernel,
        "fetch_size_kib_raw": f_kib, "write_size_kib": w_kib,
        "hbm_read_bytes_per_launch": 2 * f_kib * 1024,
        "hbm_write_bytes_per_launch": w_kib * 1024,
        "hbm_bytes_per_launch": 2 * f_kib * 1024 + w_kib * 1024,
        "correction": "FETCH_SIZE x2 (gfx950 half-count of wide streaming reads, MI355X_MICROARCH.md §HBM)",
        "dispatches": {"fetch": len(fetch), "write": len(write)},
    }
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
