#!/usr/bin/env python3
"""VALU roofline inputs for the lift kernel from a rocprofv3 --pmc pass (SQ_INSTS_VALU,
SQ_WAVES, GRBM_GUI_ACTIVE) and the kernel-trace stats of the same command.

SQ_INSTS_VALU counts wave-level VALU instructions (summed over the chip).  Peak issue:
1024 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction (the full-rate 2-operand ops; the
measured rate of the 3-operand / shift-rotate forms BLAKE3 needs is ~4 cycles, see
profiles/r01_micro_valu_*.log).

usage: pmc_valu.py <counter_collection.csv> <kernel_stats.csv> <config> <records> <out.json> [kernel]
"""
import csv
import json
import statistics
import sys


def main():
    pmc, stats, config, records, out = sys.argv[1:6]
    kernel = sys.argv[6] if len(sys.argv) > 6 else "k_lift"
    per, names = {}, {}
    for row in csv.DictReader(open(pmc)):
        if kernel not in row.get("Kernel_Name", ""):
            continue
        d = row.get("Dispatch_Id") or row.get("Correlation_Id")
        names[d] = row["Kernel_Name"]
        per.setdefault(d, {}).setdefault(row["Counter_Name"], 0.0)
        per[d][row["Counter_Name"]] += float(row["Counter_Value"])
    # the workload's full-size lift launches: the most waves per launch (bench.py's clock
    # spin-up lifts another, smaller record set)
    top = max(v.get("SQ_WAVES", 0) for v in per.values())
    per = {d: v for d, v in per.items() if v.get("SQ_WAVES", 0) >= 0.99 * top}
    name = names[next(iter(per))]
    insts = statistics.median(v.get("SQ_INSTS_VALU", 0) for v in per.values())
    waves = statistics.median(v.get("SQ_WAVES", 0) for v in per.values())
    gui = statistics.median(v.get("GRBM_GUI_ACTIVE", 0) for v in per.values())
    avg_ns = None
    for row in csv.DictReader(open(stats)):
        if row["Name"] == name:
            avg_ns = float(row["AverageNs"])
            break
    peak = 1024 * 2.4e9 / 2.0
    doc = {"config": config, "records": int(records), "kernel": name, "valu_wave_instructions_per_launch": insts,
           "waves_per_launch": waves, "valu_per_wave": insts / waves if waves else None,
           "kernel_avg_ns": avg_ns, "grbm_gui_active": gui,
           "effective_clock_ghz": (gui / 8 / avg_ns) if avg_ns else None,
           "achieved_wave_instr_per_s": insts / (avg_ns * 1e-9) if avg_ns else None,
           "peak_wave_instr_per_s": peak}
    if avg_ns:
        doc["frac_of_full_rate_peak"] = doc["achieved_wave_instr_per_s"] / peak
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
