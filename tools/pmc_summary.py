"""Summarise a tools/pmc.sh run into profiles/.

Reads gpurun_out/<tag>/<run>/**/*counter_collection.csv (one counter
group per run directory), writes
profiles/<prefix>_pmc.csv (per-dispatch counters of the pass kernels) and
updates profiles/pmc_traffic.json, the file bench.py reads for
roofline.traffic.  HBM bytes of a dispatch = 2 x FETCH_SIZE (gfx950 reports
half the bytes of a 16 B/lane streaming read, MI355X_MICROARCH.md "HBM /
rocprofv3") + WRITE_SIZE, both in KB (x1024).  The record is bytes PER ROW of
a full-data launch (the dispatches of the selected kernel with the largest
grid stream all n rows), so bench.py can scale it to the rows per launch of
whatever launch mix it measured -- traffic and the algorithmic bytes then
describe the same launches.

Usage: python tools/pmc_summary.py <tag> <out-prefix> <config> <n> <p> <kernel-key> <regex> [<run-prefix>]

<run-prefix> keeps only the run directories whose name starts with it (a
tools/gpu.sh / closing_run.sh tag holds every config's passes: pmc_c2_p1,
pmc_c2_p2, pmc_c3_p1, ...; use e.g. "pmc_c2_").
"""
import csv
import glob
import json
import os
import re
import sys

tag, prefix, config, n, p, key, rx = sys.argv[1:8]
run_prefix = sys.argv[8] if len(sys.argv) > 8 else ""
pattern = re.compile(rx)
root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
base = os.path.join(root, "gpurun_out", tag)
rows = []
for f in sorted(glob.glob(os.path.join(base, "**", "*counter_collection.csv"), recursive=True)):
    i = os.path.relpath(f, base).split(os.sep)[0]  # one counter group per run directory
    if not i.startswith(run_prefix):
        continue
    for r in csv.DictReader(open(f)):
        if any(t in r["Kernel_Name"] for t in ("irls_", "wide_", "cat_", "part_", "ols_")):
            rows.append({"pass": i, "dispatch": r["Dispatch_Id"],
                         "kernel": r["Kernel_Name"][:120], "grid": int(r["Grid_Size"]),
                         "counter": r["Counter_Name"], "value": float(r["Counter_Value"]),
                         "ms": (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6})
out_csv = os.path.join(root, "profiles", f"{prefix}_pmc.csv")
with open(out_csv, "w", newline="") as fh:
    w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
    w.writeheader()
    w.writerows(rows)

sel = [r for r in rows if pattern.search(r["kernel"])]
# the full-data launches: the largest grid and, among those, the long
# dispatches (a warm-start level can keep the grid but stream 1/16 of the rows)
gmax = max(r["grid"] for r in sel)
tmax = max(r["ms"] for r in sel if r["grid"] == gmax)
full = [r for r in sel if r["grid"] == gmax and r["ms"] >= 0.7 * tmax]
fetch = [r["value"] for r in full if r["counter"] == "FETCH_SIZE"]
write = [r["value"] for r in full if r["counter"] == "WRITE_SIZE"]
assert fetch and write, (len(fetch), len(write))
per_launch = (2 * sum(fetch) / len(fetch) + sum(write) / len(write)) * 1024
tf = os.path.join(root, "profiles", "pmc_traffic.json")
d = json.load(open(tf)) if os.path.exists(tf) else {}
rec_key = os.environ.get("PMC_RECORD_KEY", f"config{config}")
d[rec_key] = {
    "n": int(n), "p": int(p), "kernel_key": key, "kernel": full[0]["kernel"],
    "full_pass_launches": len(fetch),
    "hbm_bytes_per_full_launch": per_launch,
    "hbm_bytes_per_row": per_launch / int(n),
    "fetch_size_kb_per_launch": sum(fetch) / len(fetch),
    "write_size_kb_per_launch": sum(write) / len(write),
    "correction": "2 x FETCH_SIZE (gfx950 half-count) + WRITE_SIZE, KB x 1024; full-data "
                  "dispatches only (largest grid, >= 0.7 x the longest)",
    "source": f"profiles/{prefix}_pmc.csv (rocprofv3 --pmc, one counter group per run: "
              "tools/closing_run.sh / tools/pmc.sh)",
}
json.dump(d, open(tf, "w"), indent=1)
print(json.dumps(d[rec_key], indent=1))
