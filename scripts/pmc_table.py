#!/usr/bin/env python
"""Summarise rocprofv3 --pmc runs: for every <dir>/<job>_<i>/run_counter_collection.csv, average
each counter per dispatch over the dispatches of kernels whose name matches --kernel, and print
one table per job plus derived ratios (MFMA busy, LDS conflict share, waits)."""
import argparse
import collections
import csv
import glob
import os
import re


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--kernel", default="dna|gemm|attn")
    ap.add_argument("--per-kernel", action="store_true",
                    help="one table per (job, kernel name) instead of one per job")
    a = ap.parse_args()
    pat = re.compile(a.kernel)
    jobs = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(a.root, "*", "run_counter_collection.csv"))):
        job0 = os.path.basename(os.path.dirname(f)).rsplit("_", 1)[0]
        per = collections.defaultdict(lambda: collections.defaultdict(float))
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if not pat.search(row["Kernel_Name"]):
                    continue
                key = row["Kernel_Name"].split("(")[0][:60] if a.per_kernel else ""
                per[(key, row["Counter_Name"])][row["Dispatch_Id"]] += float(row["Counter_Value"])
        for (key, c), d in per.items():
            job = f"{key}" if a.per_kernel else job0
            jobs[job][c] = sum(d.values()) / len(d)
            jobs[job]["dispatches"] = max(jobs[job].get("dispatches", 0), len(d))
    for job, cs in jobs.items():
        print(f"== {job}")
        for c in sorted(cs):
            print(f"  {c:28s} {cs[c]:16.4g}")
        g = cs.get("GRBM_GUI_ACTIVE")
        if g and "SQ_VALU_MFMA_BUSY_CYCLES" in cs:
            # MFMA busy is summed over SIMDs (4 per CU, 256 CUs); GRBM_GUI_ACTIVE over the 8 XCDs
            # (the forward GEMM's ratio x 8 matches its HIP-event TF/s at the measured clock)
            print(f"  -> MFMA busy frac          {cs['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.3f}")
        if cs.get("SQ_LDS_IDX_ACTIVE"):
            print(f"  -> LDS bank-conflict share {cs.get('SQ_LDS_BANK_CONFLICT', 0) / cs['SQ_LDS_IDX_ACTIVE']:.3f}")
        if cs.get("SQ_WAVE_CYCLES"):
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS",
                      "SQ_ACTIVE_INST_MFMA", "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VALU"):
                if k in cs:
                    print(f"  -> {k}/WAVE_CYCLES {cs[k] / cs['SQ_WAVE_CYCLES']:.3f}")


if __name__ == "__main__":
    main()
