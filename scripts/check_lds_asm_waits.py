#!/usr/bin/env python
"""Build-time ISA check of the inline-asm transposed LDS reads in gemm.hip.

gemm.hip issues `ds_read_b64_tr_b16` through inline asm (the builtin made hipcc drain the
LDS-DMA pipeline with vmcnt(0) at every phase). SIInsertWaitcnts does not count asm as an LDS
op, so nothing but the kernels' own explicit `s_waitcnt lgkmcnt(0)` makes the destination
VGPRs valid -- and CDNA has no scoreboard for LDS results. This check disassembles the gfx950
code object of a built object file and walks every function linearly: from each asm
`ds_read_b64_tr_b16` until the next `s_waitcnt ... lgkmcnt(0)`, NO other instruction may name
one of its destination VGPRs (a read would see stale data, a write would be clobbered by the
landing load). A register-allocation change that puts a copy or a consumer between a read and
its wait fails the build check instead of silently corrupting a GEMM.

    python scripts/check_lds_asm_waits.py [build/native/gemm.hip.o]   # exit 1 on a violation
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
_VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def disassemble(obj):
    """gfx950 disassembly of the device code bundled in a hipcc object file."""
    with tempfile.TemporaryDirectory() as d:
        fat, co = os.path.join(d, "fat.bin"), os.path.join(d, "dev.co")
        subprocess.run(["objcopy", "--dump-section", f".hip_fatbin={fat}", obj,
                        os.path.join(d, "host.o")], check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o",
                        f"--targets={TARGET}", f"--input={fat}", f"--output={co}"],
                       check=True, capture_output=True)
        r = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                           check=True, capture_output=True, text=True)
    return r.stdout


def vregs(text):
    out = set()
    for m in _VREG.finditer(text):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def check(dis):
    """Returns (number of asm tr reads seen, [violation strings])."""
    func, pending, n_reads, bad = None, {}, 0, []
    for line in dis.splitlines():
        if line.endswith(">:"):  # function label
            func, pending = line.split("<", 1)[1][:-2], {}
            continue
        s = line.strip()
        if not s or s.startswith(("//", "Disassembly")) or ":" in s.split("//")[0].split()[0]:
            continue
        code = s.split("//")[0].strip()
        if not code:
            continue
        mnem, _, ops = code.partition(" ")
        if mnem == "ds_read_b64_tr_b16":
            dst, _, addr = ops.partition(",")
            hit = vregs(addr) & set(pending)
            if hit:
                bad.append(f"{func}: address of `{code}` is an unsettled read result v{sorted(hit)}")
            n_reads += 1
            for r in vregs(dst):
                pending[r] = code
            continue
        if mnem.startswith("s_waitcnt") and "lgkmcnt(0)" in ops:
            pending = {}
            continue
        hit = vregs(ops) & set(pending)
        if hit:
            bad.append(f"{func}: `{code}` names v{sorted(hit)} before the lgkmcnt(0) that "
                       f"settles `{pending[min(hit)]}`")
            for r in hit:
                pending.pop(r, None)
    return n_reads, bad


def main(argv):
    obj = argv[1] if len(argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "build", "native", "gemm.hip.o")
    n, bad = check(disassemble(obj))
    for b in bad[:50]:
        print(b)
    print(f"{os.path.basename(obj)}: {n} asm ds_read_b64_tr_b16, {len(bad)} violations")
    return 1 if bad or n == 0 else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv))
