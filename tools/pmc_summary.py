"""Summarise a tools/pmc.sh run into profiles/.

Reads gpurun_out/<tag>/p{1..4}/run_counter_collection.csv, writes
profiles/<out>_pmc.csv (per-dispatch counters of the IRLS pass kernels) and
updates profiles/pmc_traffic.json, the file bench.py reads for
roofline.traffic.  HBM bytes = 2 x FETCH_SIZE (gfx950 reports half the bytes
of a 16 B/lane streaming read, MI355X_MICROARCH.md "HBM / rocprofv3") +
WRITE_SIZE, both in KB (x1024).

Usage: python tools/pmc_summary.py <tag> <out-prefix> <config> <n> <p> <kernel-label> [regex]

<regex> selects the dispatches of the roofline kernel (default: the config-2
bf16 cooperative pass, irls_coop_kernel<.., 0, false, ..>).
"""
import csv
import json
import os
import re
import sys

tag, prefix, config, n, p, label = sys.argv[1:7]
pattern = re.compile(sys.argv[7] if len(sys.argv) > 7 else r"irls_coop_kernel<.*, 0, false")
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
base = os.path.join(root, "gpurun_out", tag)
rows = []
for i in range(1, 5):
    f = os.path.join(base, f"p{i}", "run_counter_collection.csv")
    if not os.path.exists(f):
        continue
    for r in csv.DictReader(open(f)):
        if any(t in r["Kernel_Name"] for t in ("irls_", "wide_", "cat_", "part_")):
            rows.append({"pass": i, "dispatch": r["Dispatch_Id"], "kernel": r["Kernel_Name"][:120],
                         "grid": r["Grid_Size"], "counter": r["Counter_Name"],
                         "value": r["Counter_Value"],
                         "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
out_csv = os.path.join(root, "profiles", f"{prefix}_pmc.csv")
with open(out_csv, "w", newline="") as fh:
    w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)

# bf16 (approximate) pass dispatches: the kernel template with HMODE 0
def pick(counter):
    return [float(r["value"]) for r in rows
            if r["counter"] == counter and pattern.search(r["kernel"])]
fetch, write = pick("FETCH_SIZE"), pick("WRITE_SIZE")
assert fetch and len(fetch) == len(write), (len(fetch), len(write))
per_launch = (2 * sum(fetch) + sum(write)) * 1024 / len(fetch)
tf = os.path.join(root, "profiles", "pmc_traffic.json")
d = json.load(open(tf)) if os.path.exists(tf) else {}
d[f"config{config}"] = {
    "n": int(n), "p": int(p), "kernel": label, "launches": len(fetch),
    "hbm_bytes_per_launch": per_launch,
    "fetch_size_kb_per_launch": sum(fetch) / len(fetch),
    "write_size_kb_per_launch": sum(write) / len(write),
    "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KB x 1024",
    "source": f"profiles/{prefix}_pmc.csv (tools/pmc.sh, rocprofv3 --pmc, one counter group per run)",
}
json.dump(d, open(tf, "w"), indent=1)
print(json.dumps(d, indent=1))
