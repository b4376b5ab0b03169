"""Kernel time inside each drive of a tier_interleave run (TIER_INTERLEAVE_CYCLES=1 prints every
cycle's write / drive start, CLOCK_MONOTONIC, the clock of rocprofv3's timestamps).

  python scripts/drive_kernels.py <trace dir with *_kernel_trace.csv> <the run's log>"""
import collections
import csv
import glob
import os
import re
import sys


def main():
    d, log = sys.argv[1], sys.argv[2]
    ks = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        ks += list(csv.DictReader(open(f)))
    cyc = []
    for line in open(log):
        m = re.match(r"cycle (\d+): write ([\d.]+) us, drive ([\d.]+) us.*drive at ([\d.]+) ms", line)
        if m:
            cyc.append((int(m.group(1)), float(m.group(3)), float(m.group(4))))
    for c, dur_us, start_ms in cyc:
        a, b = start_ms * 1e6, start_ms * 1e6 + dur_us * 1e3
        agg = collections.defaultdict(lambda: [0, 0.0])
        busy = 0.0
        for k in ks:
            s, e = int(k["Start_Timestamp"]), int(k["End_Timestamp"])
            if a <= s <= b:
                n = k["Kernel_Name"].split("(")[0][:70]
                agg[n][0] += 1
                agg[n][1] += (e - s) / 1e3
                busy += (e - s) / 1e3
        print("cycle %d: drive %.1f us, kernels %.1f us" % (c, dur_us, busy))
        for n, (cnt, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:10]:
            print("  %4d %9.1f us  %s" % (cnt, t, n))


if __name__ == "__main__":
    main()
