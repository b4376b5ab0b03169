#!/usr/bin/env python3
"""Per-launch read-request mix of the lift kernel from two rocprofv3 --pmc passes (pmc_reqsize.sh).

usage: pmc_reqsize.py <req_counter_collection.csv> <hit_counter_collection.csv> <config> <records> <out.json>
"""
import csv
import json
import statistics
import sys


def per_dispatch(path):
    per, waves = {}, {}
    for row in csv.DictReader(open(path)):
        if "k_lift" not in row.get("Kernel_Name", ""):
            continue
        d = row.get("Dispatch_Id") or row.get("Correlation_Id")
        per.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
        per[d][row["Counter_Name"]] += float(row["Counter_Value"])
        waves[d] = row.get("Grid_Size") or row.get("Grid_Size_X") or "0"
    # the workload's full-size launches: the largest grids (the clock spin-up lifts a smaller set)
    top = max(float(w) for w in waves.values())
    return [v for d, v in per.items() if float(waves[d]) >= 0.99 * top]


def med(rows, name):
    vals = [r[k] for r in rows for k in r if k.startswith(name) and k[len(name):] in ("", "_sum")]
    return statistics.median(vals) if vals else None


def main():
    req, hit, config, records, out = sys.argv[1:6]
    a, b = per_dispatch(req), per_dispatch(hit)
    dram32 = med(a, "TCC_EA0_RDREQ_DRAM_32B")
    r128, r64, r32 = med(a, "TCC_EA0_RDREQ_128B"), med(a, "TCC_EA0_RDREQ_64B"), med(a, "TCC_EA0_RDREQ_32B")
    h, m, rq = med(b, "TCC_HIT"), med(b, "TCC_MISS"), med(b, "TCC_EA0_RDREQ")
    doc = {"config": config, "records": int(records), "dispatches": [len(a), len(b)],
           "dram_read_bytes": dram32 * 32 if dram32 is not None else None,
           "ea_read_requests": {"128B": r128, "64B": r64, "32B": r32, "all": rq},
           "ea_read_bytes_by_width": (r128 or 0) * 128 + (r64 or 0) * 64 + (r32 or 0) * 32,
           "fetch_size_equiv_bytes": rq * 64 if rq is not None else None,
           "l2_hit_rate": h / (h + m) if h is not None and m else None, "tcc_hit": h, "tcc_miss": m}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
