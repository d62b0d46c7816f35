"""Summarise rocprofv3 PMC passes into profiles/<round>_c4_pmc_traffic.json.

Input: the ``*_counter_collection.csv`` files of separate counter passes over
the same command (``--pmc FETCH_SIZE``, ``--pmc WRITE_SIZE``, optionally
``--pmc TCC_HIT_sum TCC_MISS_sum``), one pass per directory.

HBM bytes per launch follow MI355X_MICROARCH.md's HBM/rocprofv3 section:
read = 2 x FETCH_SIZE (gfx950: FETCH_SIZE counts half of a wide coalesced
stream), write = WRITE_SIZE, both in KiB.  "first" values are from the first
dispatch of each kernel (tools/kbench.py runs the bench configuration first).

Diagnostic tooling only; not imported by the package or the tests.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def short_name(full: str) -> str:
    """Kernel name up to its argument list (template arguments kept)."""
    full = full.replace("void ", "", 1).replace("(anonymous namespace)::", "")
    depth = 0
    for i, ch in enumerate(full):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return full[:i]
    return full


def load_pass(directory: str) -> dict:
    """{kernel: {dispatch_id: {counter: value}}} for one counter pass."""
    out: dict = defaultdict(lambda: defaultdict(dict))
    files = glob.glob(os.path.join(directory, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no *counter_collection.csv under {directory}")
    for path in files:
        with open(path, newline="") as fh:
            for row in csv.DictReader(fh):
                k = short_name(row["Kernel_Name"])
                d = int(row["Dispatch_Id"])
                c = row["Counter_Name"]
                out[k][d][c] = out[k][d].get(c, 0.0) + float(row["Counter_Value"])
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--hit", default=None)
    ap.add_argument("--source", default="")
    ap.add_argument("--gather-alg-bytes", type=float, default=None,
                    help="algorithmic bytes of one C4 forward gather launch")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()

    fetch, write = load_pass(a.fetch), load_pass(a.write)
    hit = load_pass(a.hit) if a.hit else {}
    kernels = {}
    for k in sorted(set(fetch) & set(write)):
        if not (k.startswith("gather") or k.startswith("gemm") or k.startswith("post")
                or k.startswith("ws_") or k.startswith("slab") or k.startswith("colsum")
                or "narrow" in k or "rowptr" in k):
            continue
        f0 = fetch[k][min(fetch[k])].get("FETCH_SIZE", 0.0)
        w0 = write[k][min(write[k])].get("WRITE_SIZE", 0.0)
        ent = {"launches": len(fetch[k]), "fetch_size_kb_first": f0, "write_size_kb_first": w0,
               "hbm_bytes_per_launch_first": 2 * f0 * 1024 + w0 * 1024}
        if k in hit:
            d = hit[k][min(hit[k])]
            h, m = d.get("TCC_HIT_sum", 0.0), d.get("TCC_MISS_sum", 0.0)
            if h + m > 0:
                ent["l2_hit_rate"] = h / (h + m)
        kernels[k] = ent
    res = {"source": a.source,
           "correction": "hbm_read_bytes = 2 * FETCH_SIZE * 1024 (gfx950), "
                         "hbm_write_bytes = WRITE_SIZE * 1024",
           "kernels": kernels}
    # the forward mean gather: <TI, TO, V, NCH, MEAN=true, ADD=false[, NT]>
    gk = [k for k in kernels if k.startswith("gather_rows_kernel")
          and re.search(r"true, false(, \w+)?>$", k)]
    if gk and a.gather_alg_bytes:
        res["gather_fwd_c4"] = {"kernel": gk[0],
                                "hbm_bytes_per_launch": kernels[gk[0]]["hbm_bytes_per_launch_first"],
                                "algorithmic_bytes_per_launch": a.gather_alg_bytes}
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, v in kernels.items():
        print(f"{k[:70]:70s} {v['hbm_bytes_per_launch_first'] / 1e9:8.2f} GB/launch")


if __name__ == "__main__":
    main()
