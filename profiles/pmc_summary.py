"""Per-kernel HBM traffic from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE), gfx950-corrected.

    python profiles/pmc_summary.py --fetch DIR_OR_CSV --write DIR_OR_CSV [--out traffic.json]

Each pass is a separate ``rocprofv3 --pmc <counter>`` run of the same bench command
(MI355X_MICROARCH.md §rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE do not fit one pass).
Both counters are in KiB per dispatch.  Correction (MI355X_MICROARCH.md §HBM): on gfx950
FETCH_SIZE reports half the bytes of a wide coalesced streaming read, so fetched bytes =
2 × FETCH_SIZE; WRITE_SIZE is taken as is.  Dispatches are grouped by (kernel name, grid
size), so one template launched with different shapes gives separate rows.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def _csvs(path: str):
    if os.path.isfile(path):
        return [path]
    return sorted(glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True))


def _short(name: str) -> str:
    name = re.sub(r"\(.*$", "", name.replace("gnnmp::(anonymous namespace)::", ""))
    return name.strip()


def read_counter(path: str, counter: str):
    """{(kernel, grid): [value per dispatch]} for one counter."""
    per_dispatch = defaultdict(float)
    key_of = {}
    for f in _csvs(path):
        with open(f, newline="") as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                d = (f, row["Dispatch_Id"])
                per_dispatch[d] += float(row["Counter_Value"])
                key_of[d] = (_short(row["Kernel_Name"]), int(row["Grid_Size"]))
    out = defaultdict(list)
    for d, v in per_dispatch.items():
        out[key_of[d]].append(v)
    return out


def summarise(fetch_path: str, write_path: str):
    fetch = read_counter(fetch_path, "FETCH_SIZE")
    write = read_counter(write_path, "WRITE_SIZE")
    rows = []
    for key in sorted(set(fetch) | set(write)):
        fr = fetch.get(key, [])
        wr = write.get(key, [])
        f_kib = sum(fr) / len(fr) if fr else None
        w_kib = sum(wr) / len(wr) if wr else None
        fetch_b = 2 * 1024 * f_kib if f_kib is not None else None
        write_b = 1024 * w_kib if w_kib is not None else None
        rows.append({
            "kernel": key[0], "grid_threads": key[1], "dispatches": max(len(fr), len(wr)),
            "fetch_size_kib_raw": f_kib, "write_size_kib_raw": w_kib,
            "fetch_bytes": fetch_b, "write_bytes": write_b,
            "traffic_bytes": (fetch_b or 0) + (write_b or 0) if fetch_b is not None and write_b is not None else None,
        })
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--out")
    a = ap.parse_args()
    rows = summarise(a.fetch, a.write)
    for r in sorted(rows, key=lambda r: -(r["traffic_bytes"] or 0)):
        tb = r["traffic_bytes"]
        print(f"{r['kernel'][:90]:90s} grid={r['grid_threads']:>9d} n={r['dispatches']:>4d} "
              f"traffic={tb / 1e6 if tb else float('nan'):9.1f} MB")
    if a.out:
        with open(a.out, "w") as fh:
            json.dump({"correction": "fetch_bytes = 2 x FETCH_SIZE KiB x 1024 (gfx950 half-count of wide reads); "
                                     "write_bytes = WRITE_SIZE KiB x 1024",
                       "kernels": rows}, fh, indent=1)


if __name__ == "__main__":
    main()
