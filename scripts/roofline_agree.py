#!/usr/bin/env python
"""Cross-check bench.py's HIP-event op averages against a rocprofv3 --stats CSV of the same command.

    python scripts/roofline_agree.py STATS_CSV BENCH_JSON
Per family: kernel-time sum / op launches (rocprof) vs kernels[f].avg_ms (bench, HIP events)."""
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
        print(f"| {fam} | {tot / n / 1e3:.1f} | {b['kernels'][fam]['avg_ms'] * 1e3:.1f} | {n} |")


if __name__ == "__main__":
    main()
