"""AddressSanitizer + UBSan build of the native host code (csrc/bpe.cpp, csrc/data.cpp, capi.cpp:
the BPE tokenizer, masking and FASTA reader that run inside forked DataLoader workers, SURVEY
§5), compiled with g++ and driven through the C ABI over the golden fixtures by
tests/asan/asan_driver.cpp. CPU only."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from tests.conftest import BPE_JSON, GOLDEN

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(ROOT, "dna_amd", "csrc")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_cpp_under_asan_ubsan(tmp_path):
    exe = tmp_path / "asan_driver"
    cmd = ["g++", "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-pthread",
           "-I", os.path.join(ROOT, "include"), "-I", CSRC,
           os.path.join(HERE, "asan", "asan_driver.cpp"), os.path.join(CSRC, "bpe.cpp"),
           os.path.join(CSRC, "data.cpp"), os.path.join(CSRC, "capi.cpp"), "-o", str(exe)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]

    z = np.load(os.path.join(GOLDEN, "tok_golden.npz"))
    data, off = z["seq_data"].tobytes(), z["seq_off"]
    fo, fd, ds = z["full_off"], z["full_data"], z["ds130"]
    lines = []
    for i in range(len(off) - 1):
        w = data[off[i]:off[i + 1]].decode()
        if any(c.isspace() for c in w):
            continue
        full = fd[fo[i]:fo[i + 1]].astype(np.int64).tolist()
        lines.append(f"B {w or '-'} | " + " ".join(map(str, full)))
        lines.append("D 130 " + " ".join(map(str, ds[i].astype(np.int64).tolist())))
    g = json.load(open(os.path.join(GOLDEN, "fasta_golden.json")))
    fa = tmp_path / "g.fa"
    with open(fa, "w") as f:
        for name, seq in g["chroms"].items():
            f.write(f">{name}\n")
            for k in range(0, len(seq), 60):
                f.write(seq[k:k + 60] + "\n")
    for c in g["cases"]:
        lines.append(f"F {c['chr']} {c['start']} {c['end']} {c['max_length']} "
                     f"{int(c['pad_interval'])} {c['out'] or '-'}")
    cases = tmp_path / "cases.txt"
    cases.write_text("\n".join(lines) + "\n")
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:verify_asan_link_order=0:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([str(exe), BPE_JSON, str(cases), str(fa)], capture_output=True, text=True,
                       timeout=600, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-6000:]
    assert "0 failures" in r.stdout
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr
