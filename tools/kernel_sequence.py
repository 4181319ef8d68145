#!/usr/bin/env python3
"""Launch-ordered durations of the kernels whose name contains a substring,
from a rocprofv3 rocpd SQLite database (per-launch A/B, e.g. the first full
bf16 pass against the later ones).

    python tools/kernel_sequence.py gpurun_out/<tag>/prof/run_results.db irls_coop
"""

import re
import sqlite3
import sys


def short(name):
    m = re.match(r"(?:void )?(?:dlsa::)?(\w+)(<[^>(]*>)?", name)
    return (m.group(1) + (m.group(2) or "")) if m else name[:60]


def main(path, pat):
    con = sqlite3.connect(path)
    rows = con.execute("select name, start, end, grid_x from kernels order by start").fetchall()
    t0 = None
    for name, start, end, gx in rows:
        if pat not in name:
            continue
        t0 = start if t0 is None else t0
        print(f"{(start - t0) / 1e6:10.3f} ms  {(end - start) / 1e6:8.3f} ms  grid {gx:>9}  {short(name)}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "dlsa::")
