#!/usr/bin/env python
"""Per-kernel HBM traffic and GB/s of the FFT long-conv kernels from separate FETCH_SIZE /
WRITE_SIZE --pmc passes (FETCH_SIZE doubled: gfx950 correction; KiB -> bytes), divided by the
kernel's average duration from the --stats pass.  usage: fft_traffic.py FETCH_DIR WRITE_DIR STATS_CSV"""
import collections
import csv
import os
import sys


def per_kernel(d, counter, scale):
    acc = collections.defaultdict(lambda: [0.0, set()])
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter or "fftc" not in r["Kernel_Name"]:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[name][0] += float(r["Counter_Value"]) * scale
            acc[name][1].add(r["Dispatch_Id"])
    return {k: v[0] / len(v[1]) for k, v in acc.items()}


def main():
    fd, wd, stats = sys.argv[1:4]
    fe = per_kernel(fd, "FETCH_SIZE", 2048.0)
    wr = per_kernel(wd, "WRITE_SIZE", 1024.0)
    dur = {}
    with open(stats) as f:
        for r in csv.DictReader(f):
            dur[r["Name"].split("(")[0].replace("void ", "")] = float(r["AverageNs"])
    print("| kernel (avg over launches) | read MB | write MB | avg us | HBM GB/s | frac of 8 TB/s |")
    print("|---|---:|---:|---:|---:|---:|")
    for k in sorted(fe, key=lambda k: -(fe[k] + wr.get(k, 0))):
        b = fe[k] + wr.get(k, 0.0)
        t = dur.get(k)
        gbs = b / (t * 1e-9) / 1e9 if t else float("nan")
        print(f"| `{k}` | {fe[k] / 1e6:.1f} | {wr.get(k, 0) / 1e6:.1f} | {t / 1e3 if t else float('nan'):.1f} | "
              f"{gbs:.0f} | {gbs / 8000:.3f} |")


if __name__ == "__main__":
    main()
