"""Synthetic airline-like CSV for the dummy-level selection fixtures: the
rows and the exact text (a fixed formatter, so the reference run in
make_golden.py and the tests read byte-identical files)."""

import numpy as np

CARRIERS = np.array(["AA", "DL", "UA", "WN", "B6", "NK", "F9", "AS", "HA", "G4"])
ORIGINS = np.array(["ATL", "ORD", "DFW", "DEN", "LAX", "SEA", "SFO", "BOS", "JFK", "MIA",
                    "PHX", "IAH"])


def rows(n=70000, seed=5):
    """Columns of the file; level frequencies drift along the file so the
    first buffer's value_counts order differs from the global order."""
    rs = np.random.RandomState(seed)
    t = np.arange(n) / n
    month = (rs.randint(1, 13, size=n)).astype(np.int64)
    u = rs.rand(n)
    carrier = CARRIERS[np.minimum((10 * u ** (2.0 - 1.5 * t)).astype(int), 9)]
    v = rs.rand(n)
    origin = ORIGINS[np.minimum((12 * v ** (1.0 + t)).astype(int), 11)]
    dist = np.round(rs.exponential(800.0, size=n) + 100.0, 1)
    label = (rs.rand(n) < 0.4).astype(np.int64)
    return {"Month": month, "UniqueCarrier": carrier, "Origin": origin, "Distance": dist,
            "ArrDelay": label}


def text(cols):
    """CSV text: header + one line per row, fixed formatting."""
    names = list(cols)
    n = len(cols[names[0]])
    out = [",".join(names)]
    for i in range(n):
        out.append(f"{cols['Month'][i]},{cols['UniqueCarrier'][i]},{cols['Origin'][i]},"
                   f"{cols['Distance'][i]:.1f},{cols['ArrDelay'][i]}")
    return "\n".join(out) + "\n"
