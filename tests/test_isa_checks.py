"""Build-time ISA checks of hand-scheduled device code (CPU: disassembles the built objects)."""
import os
import sys

import pytest

from tests.conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))
import check_lds_asm_waits as chk  # noqa: E402

OBJ = os.path.join(ROOT, "build", "native", "gemm.hip.o")


@pytest.mark.skipif(not os.path.exists(OBJ), reason="native build absent")
def test_gemm_asm_tr_reads_settled_before_use():
    """Every inline-asm ds_read_b64_tr_b16 of the built gemm.hip is followed by an explicit
    lgkmcnt(0) before any instruction names its destination VGPRs."""
    n, bad = chk.check(chk.disassemble(OBJ))
    assert n > 100 and not bad, bad[:10]


def test_checker_flags_early_use_and_accepts_settled_use():
    ok = """
0000000000000000 <k>:
\tds_read_b64_tr_b16 v[10:11], v2 offset:1024   // 000000: 00
\tv_add_u32_e32 v3, v4, v5                        // 000008: 00
\ts_waitcnt lgkmcnt(0)                            // 000010: 00
\tv_mfma_f32_16x16x32_bf16 v[20:23], v[10:13], v[14:17], 0 // 000018: 00
"""
    assert chk.check(ok) == (1, [])
    early_copy = ok.replace("v_add_u32_e32 v3, v4, v5", "v_mov_b32_e32 v30, v11")
    n, bad = chk.check(early_copy)
    assert n == 1 and len(bad) == 1 and "v[11]" in bad[0]
    partial_wait = ok.replace("lgkmcnt(0)", "lgkmcnt(1)")
    assert len(chk.check(partial_wait)[1]) == 1
    clobber = ok.replace("v_add_u32_e32 v3, v4, v5", "v_add_u32_e32 v10, v4, v5")
    assert len(chk.check(clobber)[1]) == 1
