#!/usr/bin/env python
"""Cross-check bench.py's HIP-event op averages against a rocprofv3 --stats CSV of the same command.

    python scripts/roofline_agree.py STATS_CSV BENCH_JSON [TRACED_STEPS]
Per family: kernel-time sum / op launches (rocprof) vs kernels[f].avg_ms (bench, HIP events).
With TRACED_STEPS (steps + warm-up of the profiled run) the op launches are bench's
launches_per_step x TRACED_STEPS, so a row-blocked GEMM call (two kernel launches) counts once."""
import csv
import json
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from traffic_from_pmc import FAMILIES  # noqa: E402


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    b = json.load(open(sys.argv[2]))
    print("| op family | rocprof avg us / launch | bench HIP-event avg us | launches (rocprof) |")
    print("|---|---:|---:|---:|")
    for fam, (sel, one) in FAMILIES.items():
        tot = sum(float(r["TotalDurationNs"]) for r in rows if re.search(sel, r["Name"]))
        n = sum(int(r["Calls"]) for r in rows if re.search(one, r["Name"]))
        if not n or fam not in b.get("kernels", {}):
            continue
        if len(sys.argv) > 3:
            n = int(round(b["kernels"][fam]["launches_per_step"] * int(sys.argv[3])))
        print(f"| {fam} | {tot / n / 1e3:.1f} | {b['kernels'][fam]['avg_ms'] * 1e3:.1f} | {n} |")


if __name__ == "__main__":
    main()
