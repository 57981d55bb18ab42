"""Build the native library dna_amd/lib/libdna_amd.so (HIP kernels for gfx950 + host C++).

    python -m dna_amd.build            # incremental
    python -m dna_amd.build --clean

Device code: hipcc --offload-arch=gfx950 (cross-compiles without a GPU). Host-only sources
(BPE tokenizer, masking, FASTA) build with g++. The .so is built in-tree so it travels with the
repo snapshot to the GPU box; it is git-ignored.
"""
import argparse
import concurrent.futures as cf
import glob
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
BUILD = os.path.join(ROOT, "build", "native")
LIB = os.path.join(HERE, "lib", "libdna_amd.so")
ARCH = os.environ.get("DNA_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

HIP_FLAGS = ["--offload-arch=" + ARCH, "-O3", "-fPIC", "-std=c++17", "-I", INCLUDE, "-I", CSRC,
             "-mllvm", "-amdgpu-mfma-vgpr-form",
             "-Wno-unused-result"]
# per-file extra device flags. attention.hip: scores are never NaN, and without -fno-honor-nans
# every fmaxf of an MFMA result gets a canonicalising v_max in front of it; the SLP vectoriser
# turns the per-score multiplies into v_pk_mul_f32 on odd register pairs (v_mov/v_alignbit
# shuffles around every pair, and packed f32 beside MFMAs is slower anyway)
FILE_FLAGS = {"attention.hip": ["-fno-honor-nans", "-fno-slp-vectorize"]}
# experiment hook: DNA_AMD_FILE_FLAGS="gemm.hip:-fno-slp-vectorize -DX=1;other.hip:..." adds flags
# per file (the object is rebuilt whenever its command line changes)
for _item in filter(None, os.environ.get("DNA_AMD_FILE_FLAGS", "").split(";")):
    _f, _, _fl = _item.partition(":")
    FILE_FLAGS[_f.strip()] = FILE_FLAGS.get(_f.strip(), []) + _fl.split()
CXX_FLAGS = ["-O3", "-fPIC", "-std=c++17", "-pthread", "-I", INCLUDE, "-I", CSRC, "-Wall",
             "-Wno-unused-function"]


def _headers_mtime():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(INCLUDE, "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0)


def _compile(src):
    obj = os.path.join(BUILD, os.path.basename(src) + ".o")
    if src.endswith(".hip"):
        cmd = [HIPCC] + HIP_FLAGS + FILE_FLAGS.get(os.path.basename(src), []) + ["-c", src, "-o", obj]
    else:
        cmd = ["g++"] + CXX_FLAGS + ["-c", src, "-o", obj]
    stamp = obj + ".cmd"
    line = " ".join(cmd)
    prev = open(stamp).read() if os.path.exists(stamp) else None
    if (os.path.exists(obj) and (prev == line or (prev is None and not os.environ.get("DNA_AMD_FILE_FLAGS")))
            and os.path.getmtime(obj) >= max(os.path.getmtime(src), _headers_mtime())):
        return obj, None
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        return obj, f"$ {line}\n{r.stdout}\n{r.stderr}"
    with open(stamp, "w") as f:
        f.write(line)
    return obj, None


def _check_asm_lds_waits():
    """gemm.hip's inline-asm ds_read_b64_tr_b16 results are settled only by explicit
    lgkmcnt(0) waits the compiler does not know about: fail the build if any instruction names a
    destination VGPR between such a read and its wait (scripts/check_lds_asm_waits.py). Run
    once per rebuilt object (a stamp file next to it)."""
    obj = os.path.join(BUILD, "gemm.hip.o")
    stamp = obj + ".ldscheck"
    if not os.path.exists(obj) or (os.path.exists(stamp) and
                                   os.path.getmtime(stamp) >= os.path.getmtime(obj)):
        return
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    try:
        import check_lds_asm_waits as chk
    finally:
        sys.path.pop(0)
    n, bad = chk.check(chk.disassemble(obj))
    if bad or n == 0:
        os.remove(obj)
        raise RuntimeError(f"gemm.hip: {len(bad)} instructions touch an inline-asm LDS read's "
                           f"destination before its lgkmcnt(0) ({n} reads):\n" + "\n".join(bad[:20]))
    open(stamp, "w").close()


def build(verbose=False, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    srcs = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))
    jobs = jobs or min(8, os.cpu_count() or 4)
    errors, objs = [], []
    with cf.ThreadPoolExecutor(jobs) as ex:
        for obj, err in ex.map(_compile, srcs):
            objs.append(obj)
            if err:
                errors.append(err)
    if errors:
        raise RuntimeError("native build failed:\n" + "\n".join(errors))
    _check_asm_lds_waits()
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(o) for o in objs):
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-pthread", "-o", LIB] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n$ {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        # a kernel template whose host-side instantiation failed silently leaves its launch stub
        # undefined (hipcc emits no diagnostic for it); the library would then fail at dlopen
        r = subprocess.run(["nm", "-D", "--undefined-only", LIB], capture_output=True, text=True)
        missing = [l.split()[-1] for l in r.stdout.splitlines() if "_ZN3dna" in l]
        if missing:
            os.remove(LIB)
            raise RuntimeError(f"libdna_amd.so has undefined own symbols: {missing}")
    if verbose:
        print(f"built {LIB}")
    return LIB


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    args = ap.parse_args()
    if args.clean:
        shutil.rmtree(BUILD, ignore_errors=True)
        if os.path.exists(LIB):
            os.remove(LIB)
    build(verbose=True, jobs=args.j)


if __name__ == "__main__":
    sys.exit(main())
