#!/usr/bin/env python3
"""Per-kernel DRAM bytes and instruction mix of config5's batch kernels from scripts/pmc_c5.sh's
three rocprofv3 --pmc passes, with the average duration of each kernel from a kernel-stats CSV of
the same workload: DRAM read bytes = TCC_EA0_RDREQ_DRAM_32B x 32; write bytes = 64-B write
requests x 64 + the other write requests x 32.

usage: pmc_c5_summary.py <gpurun_out dir> <kernel_stats.csv> <out.json>"""
import csv
import json
import os
import statistics
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].replace("void ", "").replace("rh::", "")


def main():
    root, stats, out = sys.argv[1:4]
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> counter -> value
    for i in (1, 2, 3):
        path = os.path.join(root, f"pmc_c5_{i}", "run_counter_collection.csv")
        for r in csv.DictReader(open(path)):
            d = (i, r.get("Dispatch_Id") or r.get("Correlation_Id"))
            k = short(r["Kernel_Name"])
            per[k][d][r["Counter_Name"]] = per[k][d].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    dur = {}
    for r in csv.DictReader(open(stats)):
        dur[short(r["Name"])] = float(r["AverageNs"])
    res = {}
    for k, ds in sorted(per.items()):
        def med(c):
            v = [x[c] for x in ds.values() if c in x]
            return statistics.median(v) if v else None
        rd = med("TCC_EA0_RDREQ_DRAM_32B_sum")
        w64, wall = med("TCC_EA0_WRREQ_64B_sum"), med("TCC_EA0_WRREQ_sum")
        row = {"dram_read_bytes": rd * 32 if rd is not None else None,
               "dram_write_bytes": (w64 * 64 + (wall - w64) * 32) if (w64 is not None and wall is not None) else None,
               "l2_hit_rate": (lambda h, m: h / (h + m) if h is not None and m else None)(med("TCC_HIT_sum"), med("TCC_MISS_sum")),
               "valu_per_wave": (lambda v, w: v / w if v is not None and w else None)(med("SQ_INSTS_VALU"), med("SQ_WAVES")),
               "vmem_rd_per_wave": (lambda v, w: v / w if v is not None and w else None)(med("SQ_INSTS_VMEM_RD"), med("SQ_WAVES")),
               "lds_bank_conflict_cycles": med("SQ_LDS_BANK_CONFLICT"),
               "avg_ns": dur.get(k)}
        if row["avg_ns"] and row["dram_read_bytes"] is not None and row["dram_write_bytes"] is not None:
            row["dram_gb_per_s"] = round((row["dram_read_bytes"] + row["dram_write_bytes"]) / row["avg_ns"], 1)
        res[k] = row
    json.dump({"workload": "config5: 1 M random inserts per batch into 100 M (bench.py --config config5 --steps 6)",
               "counters": "median per dispatch over the passes of scripts/pmc_c5.sh", "kernels": res},
              open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
