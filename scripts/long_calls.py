"""The longest HIP API calls, kernels and copies of a rocprofv3 trace (csv), in time order: where a
host thread waited (hipEventSynchronize, hipStreamSynchronize, hipHostMalloc, ...) and what the
device ran meanwhile (scripts/gpu_session.sh).

  python scripts/long_calls.py <dir with *_hip_api_trace.csv [*_kernel_trace.csv]> [min_us]"""
import csv
import glob
import os
import sys


def rows(d, pat):
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        yield from csv.DictReader(open(f))


def main():
    d = sys.argv[1]
    min_us = float(sys.argv[2]) if len(sys.argv) > 2 else 2000.0
    ev = []
    for r in rows(d, "*hip_api_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "api", r.get("Function", r.get("Operation", "?"))))
    for r in rows(d, "*kernel_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "kernel", r["Kernel_Name"].split("(")[0][:60]))
    for r in rows(d, "*memory_copy_trace.csv"):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy", r.get("Direction", "?")))
    if not ev:
        print("no trace rows")
        return
    t0 = min(e[0] for e in ev)
    long_ = sorted(e for e in ev if (e[1] - e[0]) / 1e3 >= min_us)
    print("%d events, %d of >= %.0f us" % (len(ev), len(long_), min_us))
    for s, e, kind, name in long_:
        print("%12.1f ms %10.1f us  %-6s %s" % ((s - t0) / 1e6, (e - s) / 1e3, kind, name))


if __name__ == "__main__":
    main()
