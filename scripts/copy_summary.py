"""Large copies and kernel totals from a rocprofv3 kernel + memory-copy trace (csv): every copy of at
least 1 MiB with its duration and rate, the gaps in them, and the kernels' time by name -- to see
what the host tier's background refresh costs beside the store's own work (scripts/gpu_session.sh).

  python scripts/copy_summary.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv>"""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    copies, kern = [], collections.defaultdict(lambda: [0, 0.0])
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            b = int(r.get("Bytes", r.get("Size", "0")) or 0)
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), b,
                           r.get("Direction", r.get("Operation", "?"))))
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = kern[r["Kernel_Name"].split("(")[0][:70]]
            k[0] += 1
            k[1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    copies.sort()
    # the copy trace may carry no byte count: a copy of >= 1 MiB or of >= 1 ms counts as large
    big = [c for c in copies if c[2] >= 1 << 20 or c[1] - c[0] >= 1_000_000]
    t0 = copies[0][0] if copies else 0
    print("copies: %d in all, %d of >= 1 MiB or >= 1 ms" % (len(copies), len(big)))
    for s, e, b, dr in big:
        us = (e - s) / 1e3
        print("  at %10.1f ms  %-14s %10.1f MB  %9.1f us  %6.1f GB/s" % ((s - t0) / 1e6, dr, b / 1e6, us,
                                                                       b / us / 1e3 if us > 0 else 0))
    small = [c for c in copies if c not in big]
    if small:
        durs = sorted((e - s) / 1e3 for s, e, _, _ in small)
        print("small copies: %d, median %.1f us, p99 %.1f us, max %.1f us" %
              (len(durs), durs[len(durs) // 2], durs[int(0.99 * (len(durs) - 1))], durs[-1]))
    print("kernels by total time:")
    for name, (n, us) in sorted(kern.items(), key=lambda kv: -kv[1][1])[:25]:
        print("  %8.1f us  %6d x  %8.1f avg  %s" % (us, n, us / n, name))


if __name__ == "__main__":
    main()
