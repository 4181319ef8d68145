#!/usr/bin/env python3
"""GPU idle gaps of a traced bench run and the host API calls inside them.

    python tools/trace_gaps.py gpurun_out/<tag>/trace_<name> [--min-gap-ms 0.5] [--kernel irls_]

Reads the csv files of `rocprofv3 --runtime-trace --kernel-trace --output-format
csv` (tools/gpu.sh `trace:` step): the kernel trace and the HIP API trace.
Prints the launch-ordered kernels whose name contains --kernel, with each
one's duration and the GPU idle time before it, and for every idle gap above
--min-gap-ms the HIP runtime calls that overlap it (the host work that kept
the GPU waiting), longest first.
"""

import argparse
import csv
import glob
import os


def load(pattern_dir, suffix):
    rows = []
    for f in glob.glob(os.path.join(pattern_dir, "**", f"*{suffix}"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    return rows


def col(row, *names):
    for n in names:
        if n in row:
            return row[n]
    raise KeyError(names)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--min-gap-ms", type=float, default=0.5)
    ap.add_argument("--kernel", default="")
    a = ap.parse_args()
    ks = load(a.dir, "kernel_trace.csv")
    api = load(a.dir, "hip_api_trace.csv")
    kern = sorted(((int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")),
                    col(r, "Kernel_Name")) for r in ks))
    calls = sorted(((int(col(r, "Start_Timestamp")), int(col(r, "End_Timestamp")),
                     col(r, "Function", "Operation", "Name")) for r in api))
    if not kern:
        raise SystemExit("no kernel trace under " + a.dir)
    t0 = kern[0][0]
    prev_end = kern[0][0]
    for s, e, name in kern:
        gap = (s - prev_end) / 1e6
        if a.kernel in name:
            print(f"{(s - t0) / 1e6:10.3f} ms  {(e - s) / 1e6:8.3f} ms  idle before {gap:7.3f} ms  "
                  f"{name[:70]}")
        if gap > a.min_gap_ms:
            inside = [(min(ce, s) - max(cs, prev_end), n) for cs, ce, n in calls
                      if ce > prev_end and cs < s]
            inside.sort(reverse=True)
            top = ", ".join(f"{n} {d / 1e6:.3f}" for d, n in inside[:6])
            print(f"    gap {gap:.3f} ms before {name[:40]}: {top}")
        prev_end = max(prev_end, e)


if __name__ == "__main__":
    main()
