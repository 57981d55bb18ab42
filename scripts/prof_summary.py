#!/usr/bin/env python
"""Summarise a rocprofv3 --kernel-trace --stats CSV into a markdown table for profiles/.

    python scripts/prof_summary.py gpurun_out/prof1/run_kernel_stats.csv [--steps N] > profiles/x.md
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("stats_csv")
    ap.add_argument("--steps", type=int, default=0, help="steps traced (for per-step columns)")
    ap.add_argument("--top", type=int, default=40)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.stats_csv)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"Source: `{a.stats_csv}` (rocprofv3 --kernel-trace --stats); total kernel time "
          f"{tot / 1e6:.1f} ms" + (f" over {a.steps} traced steps" if a.steps else "") + "\n")
    print("| share | calls | avg us | min us | max us | kernel |")
    print("|---:|---:|---:|---:|---:|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: a.top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 120:
            name = name[:117] + "..."
        print(f"| {float(r['TotalDurationNs']) / tot * 100:.2f}% | {r['Calls']} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | {float(r['MinNs']) / 1e3:.1f} | "
              f"{float(r['MaxNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main()
