#!/usr/bin/env python
"""HBM traffic per op launch from two rocprofv3 --pmc passes over the same bench command.
Usage: traffic_from_pmc.py FETCH_DIR WRITE_DIR OUT.json [BATCH [PASS_BENCH.json]]

    python scripts/traffic_from_pmc.py FETCH_DIR WRITE_DIR OUT.json [BATCH]

FETCH_SIZE / WRITE_SIZE are rocprofv3 derived counters in KiB per dispatch. Per
MI355X_MICROARCH.md (HBM section) FETCH_SIZE reports exactly half the bytes of 16-B/lane
streaming reads on gfx950, so it is doubled; WRITE_SIZE is taken as is. Both count
Infinity-Cache (MALL) hits as well as HBM. Kernels are grouped into the op families bench.py
times (dna_amd.functional._timed names); bytes_per_launch = family bytes / op launches."""
import collections
import csv
import json
import os
import re
import sys

# family -> (regex selecting its kernels, regex selecting the one kernel counted per op launch)
FAMILIES = {
    # csrc/gemm.hip: EPI 0 = bf16 epilogue (forward / data gradient), EPI 2 = the GeGLU epilogue
    # of the fused gated_layers GEMM (its own op family, gemm_geglu), EPI 3 = gemm_geglu_bwd
    "gemm_hip": (r"gemmp_kernel<0|gemm_kernel<(true|false), (true|false), 0|gemmp_kernelILi0|gemm_kernelILb[01]ELb[01]ELi0",
                 r"gemmp_kernel<0|gemm_kernel<(true|false), (true|false), 0|gemmp_kernelILi0|gemm_kernelILb[01]ELb[01]ELi0"),
    "gemm_geglu": (r"gemmp_kernel<2|gemmp_kernelILi2|gemm_kernel<true, true, 2|gemm_kernelILb1ELb1ELi2",
                   r"gemmp_kernel<2|gemmp_kernelILi2|gemm_kernel<true, true, 2|gemm_kernelILb1ELb1ELi2"),
    # EPI 3: wo's data gradient with the GeGLU backward in the epilogue (GeGLUOut)
    "gemm_geglu_bwd": (r"gemmp_kernel<3|gemmp_kernelILi3", r"gemmp_kernel<3|gemmp_kernelILi3"),
    "gemm_wgrad": (r"Cijk_|sum_slices_kernel|wgradp_kernel", r"Cijk_|wgradp_kernel"),
    "attn_fwd": (r"attn::fwd2?_bf16_kernel|attn4fwd_bf16|attn16fwd2_bf16",
                 r"attn::fwd2?_bf16_kernel|attn4fwd_bf16|attn16fwd2_bf16"),
    # the fused backward (bwd3) is one launch per op; the two-kernel pair counts its dQ kernel
    "attn_bwd": (r"attn::(dq|dkdv)2?_bf16_kernel|attn(2dq|4dkdv)_bf16|dq2_bf16|dkdv2_bf16|bwd3_bf16_kernel",
                 r"attn::dq2?_bf16_kernel|attn2dq_bf16|dq2_bf16|bwd3_bf16_kernel"),
    "geglu_fwd": (r"geglu10fwd_kernel|geglu::fwd_kernel", r"geglu10fwd_kernel|geglu::fwd_kernel"),
    "geglu_bwd": (r"geglu10bwd_kernel|geglu::bwd_kernel", r"geglu10bwd_kernel|geglu::bwd_kernel"),
    "ln_fwd": (r"2ln10fwd_kernel|ln::fwd_kernel", r"2ln10fwd_kernel|ln::fwd_kernel"),
    "ln_bwd": (r"2ln10bwd_kernel|ln::bwd_kernel|ln::reduce_partials|2ln15reduce_partials",
               r"2ln10bwd_kernel|ln::bwd_kernel"),
}


def per_dispatch(path, counter):
    """{dispatch_id: (kernel_name, value)} summed over the rows of one dispatch."""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            if row["Counter_Name"] != counter:
                continue
            d = row["Dispatch_Id"]
            name, v = out.get(d, (row["Kernel_Name"], 0.0))
            out[d] = (name, v + float(row["Counter_Value"]))
    return out


def families(disp, scale):
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    for name, v in disp.values():
        for fam, (sel, one) in FAMILIES.items():
            if re.search(sel, name):
                tot[fam] += v * scale
                if re.search(one, name):
                    cnt[fam] += 1
    return tot, cnt


def main():
    fdir, wdir, out = sys.argv[1:4]
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else None
    # optional: the bench JSON line each pass printed -- op launches = launches_per_step x
    # (steps + warmup), so a row-blocked GEMM call (two kernel launches, csrc/gemm.hip) counts once
    ops = {}
    if len(sys.argv) > 5 and os.path.exists(sys.argv[5]):
        with open(sys.argv[5]) as f:
            line = [l for l in f.read().splitlines() if l.startswith("{")][-1]
        bj = json.loads(line)
        for fam, k in bj.get("kernels", {}).items():
            ops[fam] = k["launches_per_step"] * (bj["steps"] + bj["warmup"])
    fetch = per_dispatch(os.path.join(fdir, "run_counter_collection.csv"), "FETCH_SIZE")
    write = per_dispatch(os.path.join(wdir, "run_counter_collection.csv"), "WRITE_SIZE")
    ft, fc = families(fetch, 2 * 1024.0)   # KiB, x2 gfx950 FETCH_SIZE correction
    wt, wc = families(write, 1024.0)
    res = {}
    for fam in FAMILIES:
        n = fc.get(fam) or wc.get(fam)
        if not n:
            continue
        if fam in ops:
            fc[fam] = wc[fam] = n = ops[fam]
        res[fam] = {"bytes_per_launch": int((ft[fam] / fc[fam] if fc.get(fam) else 0)
                                            + (wt[fam] / wc[fam] if wc.get(fam) else 0)),
                    "read_bytes_per_launch": int(ft[fam] / fc[fam]) if fc.get(fam) else None,
                    "write_bytes_per_launch": int(wt[fam] / wc[fam]) if wc.get(fam) else None,
                    "launches_profiled": int(n)}
    doc = {"method": "rocprofv3 --kernel-trace --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate "
                     "passes) over `python bench.py --steps 6 --warmup 2 --no-cpu-baseline --batch B`; "
                     "FETCH_SIZE x2 (gfx950 correction), KiB->bytes; includes Infinity-Cache hits",
           "batch": batch, "families": res}
    with open(out, "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
