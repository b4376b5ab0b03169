"""Device timeline of single-row writes from a rocprofv3 kernel + memory-copy trace
(scripts/gpu_session.sh): every kernel and copy between two consecutive occurrences of a marker kernel,
with the idle gap before each and the span per write.

  python scripts/write_timeline.py <dir with *_kernel_trace.csv and *_memory_copy_trace.csv> <marker> [k ...]

marker: a substring of the kernel that opens one write (e.g. k_lift_search or k_small_front);
k: which occurrences to print (default: the last three full ones).  Prints a summary line with
the median span and command count over every occurrence."""
import csv
import glob
import os
import statistics
import sys


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:80]))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = "copy " + r.get("Direction", r.get("Operation", "?")) + " " + r.get("Bytes", r.get("Size", ""))
            ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name))
    return sorted(ev)


def main():
    d, mark = sys.argv[1], sys.argv[2]
    ev = load(d)
    starts = [i for i, e in enumerate(ev) if mark in e[2]]
    if len(starts) < 2:
        print("marker %r seen %d times" % (mark, len(starts)))
        return
    spans, cmds = [], []
    for a, b in zip(starts, starts[1:]):
        spans.append((ev[b][0] - ev[a][0]) / 1e3)
        cmds.append(b - a)
    want = [int(x) for x in sys.argv[3:]] or list(range(max(0, len(starts) - 4), len(starts) - 1))
    for k in want:
        i0, i1 = starts[k], starts[k + 1]
        t0, prev = ev[i0][0], ev[i0][0]
        print("--- occurrence %d: span %.1f us to the next, %d commands" % (k, (ev[i1][0] - t0) / 1e3, i1 - i0))
        for s, e, name in ev[i0:i1]:
            print("%8.1f gap %6.1f dur %7.1f  %s" % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, name))
            prev = max(prev, e)
    print("summary: %d occurrences, median span %.1f us, median commands %d" %
          (len(spans), statistics.median(spans), int(statistics.median(cmds))))


if __name__ == "__main__":
    main()
