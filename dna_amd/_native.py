"""ctypes binding of libdna_amd.so (the C ABI declared in include/dna_amd.h).

The product path has no fallback: if the library is missing or fails to load, every op raises.
torch is imported first so that the library's libamdhip64.so.7 dependency resolves (by SONAME) to
the HIP runtime torch already loaded -- one runtime per process, so torch's hipStream_t handles
and device pointers are valid in our kernels.
"""
import ctypes
import os
import re

import torch  # noqa: F401  (must precede the dlopen below, see module docstring)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DNA_AMD_LIB", os.path.join(_HERE, "lib", "libdna_amd.so"))
HEADER = os.path.join(os.path.dirname(_HERE), "include", "dna_amd.h")

F32, BF16, F16 = 0, 1, 2
ACT_NONE, ACT_GELU = 0, 1

_vp, _i, _u64, _f, _sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_uint64, ctypes.c_float, ctypes.c_size_t
_i64 = ctypes.c_int64

_SIGS = {
    "dna_abi_version": (_i, []),
    "dna_last_error": (ctypes.c_char_p, []),
    "dna_attn_fwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp]),
    "dna_attn_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp]),
    "dna_attn_bwd_ex": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp, _vp]),
    "dna_attn_dbias_part_rows": (_i, [_i, _i]),
    "dna_flash_lse_rows": (_i, [_i]),
    "dna_flash_fwd": (_i, [_vp, _i, _vp, _i, _i, _i64, _i64, _i64, _i, _i, _i, _i, _i, _f, _vp, _vp, _vp]),
    "dna_flash_bwd": (_i, [_vp, _i, _vp, _i, _i, _i64, _i64, _i64, _vp, _vp, _vp, _i, _i, _i, _i, _i,
                           _f, _vp, _vp, _vp]),
    "dna_colsum_f32": (_i, [_vp, _i, _i, _vp, _i, _vp]),
    "dna_colsum_bf16_workspace": (_sz, [_i, _i]),
    "dna_colsum_bf16": (_i, [_vp, _i, _i, _vp, _i, _vp, _sz, _vp]),
    "dna_flip_rows": (_i, [_vp, _i, _i, _sz, _vp, _vp]),
    "dna_causal_conv1d_fwd": (_i, [_vp, _sz, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "dna_causal_conv1d_part_rows": (_sz, [_i, _i]),
    "dna_causal_conv1d_bwd": (_i, [_vp, _sz, _i, _vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _sz, _vp, _vp]),
    "dna_hyena_shortconv_fwd": (_i, [_vp, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp]),
    "dna_hyena_shortconv_part_elems": (_sz, [_i, _i, _i, _i, _i]),
    "dna_hyena_shortconv_bwd": (_i, [_vp, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _vp]),
    "dna_hyena_gate_out_fwd": (_i, [_vp, _vp, _i, _i, _i, _i, _sz, _vp, _vp]),
    "dna_hyena_gate_out_bwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _sz, _vp, _vp, _vp]),
    "dna_hyena_modulate_t_fwd": (_i, [_vp, _i, _vp, _vp, _f, _i, _i, _i, _vp, _vp]),
    "dna_hyena_modulate_t_bwd": (_i, [_vp, _vp, _vp, _f, _i, _i, _i, _vp, _i, _vp]),
    "dna_hyena_filter_part_elems": (_i, [_i, _i, _i, _i]),
    "dna_hyena_filter_part_stride": (_i, [_i, _i, _i]),
    "dna_hyena_filter_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _f, _i, _i, _i, _i,
                                  _vp, _vp]),
    "dna_hyena_filter_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _f, _i, _i, _i, _i,
                                  _vp, _vp, _vp, _vp]),
    "dna_hyena_filter_finish": (_i, [_vp, _i, _i, _i, _vp, _vp]),
    "dna_ln_fwd": (_i, [_vp, _i, _vp, _i, _f, _u64, _u64, _vp, _vp, _vp, _i, _i, _f, _vp, _vp,
                        _vp, _vp, _vp]),
    "dna_ln_bwd_workspace": (_sz, [_i, _i]),
    "dna_ln_bwd": (_i, [_vp, _vp, _vp, _i, _vp, _i, _f, _u64, _u64, _vp, _vp, _vp, _vp, _i, _i,
                        _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dna_ln_bwd_from_y": (_i, [_vp, _vp, _vp, _i, _f, _u64, _u64, _vp, _vp, _vp, _i, _i, _vp,
                               _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dna_ln_bwd_from_y_acc": (_i, [_vp, _vp, _vp, _i, _f, _u64, _u64, _vp, _vp, _vp, _i, _i, _vp,
                                   _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dna_add_ln_fwd": (_i, [_vp, _i, _vp, _vp, _vp, _i, _i, _f, _i, _vp, _vp, _vp, _vp, _vp, _vp]),
    "dna_add_ln_bwd": (_i, [_vp, _vp, _vp, _vp, _i, _vp, _vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp,
                            _vp, _vp, _sz, _vp]),
    "dna_rms_fwd": (_i, [_vp, _i, _vp, _i, _i, _f, _vp, _vp, _vp, _vp]),
    "dna_rms_bwd": (_i, [_vp, _vp, _vp, _i, _vp, _vp, _i, _i, _vp, _vp, _vp, _sz, _vp]),
    "dna_embed_ln_fwd": (_i, [_vp, _vp, _vp, _vp, _vp, _i, _i, _i, _f, _f, _u64, _u64, _vp, _vp,
                              _vp, _vp, _vp]),
    "dna_embed_ln_bwd": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _i, _f, _u64,
                              _u64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dna_embed_ln_bwd_rows": (_i, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _i, _i, _i, _f, _u64,
                                   _u64, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dna_embed_grad_segsum_workspace": (_sz, [_i, _i]),
    "dna_embed_grad_segsum": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "dna_sum_slices_accum": (_i, [_vp, _i, _sz, _vp, _vp]),
    "dna_sum_slices": (_i, [_vp, _i, _sz, _vp, _vp]),
    "dna_geglu_fwd": (_i, [_vp, _i, _i, _i, _f, _u64, _u64, _vp, _vp, _vp]),
    "dna_geglu_bwd": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_linear_fwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_linear_gelu_fwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _vp]),
    "dna_linear_dgrad": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_linear_wgrad": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "dna_transpose_bf16": (_i, [_vp, _i, _i, _vp, _vp]),
    "dna_linear_wgrad_p_splits": (_i, [_i, _i, _i]),
    "dna_linear_fwd_f32": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_linear_dgrad_f32": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_linear_wgrad_f32_splits": (_i, [_i, _i, _i]),
    "dna_linear_wgrad_f32": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "dna_gemm_strided_splits": (_i, [_i, _i, _i, _i]),
    "dna_gemm_bf16_strided": (_i, [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _i64,
                                   _i, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "dna_proj_cm_bf16": (_i, [_vp, _vp, _vp, _i, _i, _i, _i, _i, _vp, _vp]),
    "dna_gemm_bf16_strided_cat": (_i, [_vp, _vp, _i, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _vp,
                                       _i64, _i64, _i, _vp, _vp, _i, _i, _i, _i, _i, _vp]),
    "dna_gemm_f32_strided": (_i, [_vp, _i64, _i64, _i64, _vp, _i64, _i64, _i64, _vp, _i64, _i64,
                                  _vp, _i, _i, _i, _i, _i, _vp]),
    "dna_linear_wgrad_p": (_i, [_vp, _vp, _i, _i, _i, _i, _vp, _vp]),
    "dna_geglu_linear_fwd": (_i, [_vp, _vp, _vp, _i, _i, _i, _f, _u64, _u64, _vp, _vp, _vp]),
    "dna_geglu_linear_dgrad": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_geglu_linear_dgrad_p": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_gelu_linear_dgrad_p": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp]),
    "dna_fftconv_workspace": (_sz, [_i, _i, _i]),
    "dna_fftconv_kspec_elems": (_sz, [_i]),
    "dna_fftconv_filter": (_i, [_vp, _vp, _i, _i, _i, _vp, _vp, _sz, _vp]),
    "dna_fftconv_fwd": (_i, [_vp, _i, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _sz, _vp]),
    "dna_fftconv_bwd": (_i, [_vp, _vp, _i, _vp, _vp, _i, _i, _i, _i, _vp, _vp, _vp, _vp, _sz, _vp]),
    "dna_selective_scan_states": (_sz, [_i, _i, _i, _i]),
    "dna_selective_scan_fwd": (_i, [_vp] * 8 + [_i] * 6 + [_vp] * 4),
    "dna_selective_scan_bwd": (_i, [_vp] * 8 + [_i] * 6 + [_vp] * 11),
    "dna_xent_fwd": (_i, [_vp, _i, _vp, _i, _i, _vp, _vp, _vp]),
    "dna_xent_bwd": (_i, [_vp, _i, _vp, _vp, _vp, _f, _i, _i, _vp, _vp]),
    "dna_sumsq_workspace": (_sz, [_sz]),
    "dna_sumsq": (_i, [_vp, _sz, _vp, _vp, _sz, _vp]),
    "dna_adamw_step": (_i, [_vp, _vp, _vp, _vp, _vp, _sz, _f, _f, _f, _f, _f, _i, _vp, _f, _f,
                            _vp]),
    "dna_bpe_create": (_vp, [ctypes.c_char_p]),
    "dna_bpe_destroy": (None, [_vp]),
    "dna_bpe_vocab_size": (_i, [_vp]),
    "dna_bpe_encode": (_i, [_vp, ctypes.c_char_p, _i, _vp, _i]),
    "dna_bpe_encode_batch": (_i, [_vp, _vp, _vp, _i, _i, _i, _vp, _vp, _i]),
    "dna_bert_mask_from_draws": (_i, [_vp, _i, _vp, _vp, _vp, _i, _i, _f, _f, _f, _vp, _vp, _vp]),
    "dna_bert_mask": (_i, [_vp, _i, _i, _vp, _i, _i, _i, _f, _f, _f, _u64, _u64, _vp, _vp, _vp]),
    "dna_fasta_open": (_vp, [ctypes.c_char_p]),
    "dna_fasta_close": (None, [_vp]),
    "dna_fasta_num_records": (_i, [_vp]),
    "dna_fasta_record_name": (ctypes.c_char_p, [_vp, _i]),
    "dna_fasta_record_length": (_i64, [_vp, ctypes.c_char_p]),
    "dna_fasta_interval": (_i, [_vp, ctypes.c_char_p, _i64, _i64, _i64, _i, _i, ctypes.c_char_p,
                                _i64, _vp]),
}


class NativeError(RuntimeError):
    pass


_lib = None


def lib():
    """The loaded library; raises (never falls back) when it is missing."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(
                f"dna_amd native library not found at {LIB_PATH}; build it with "
                "`python -m dna_amd.build` (hipcc, gfx950). There is no CPU fallback.")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.dna_abi_version() != 1:
            raise NativeError("dna_amd ABI version mismatch")
        _lib = L
    return _lib


def last_error():
    return lib().dna_last_error().decode(errors="replace")


def check(status, name):
    if status != 0:
        raise NativeError(f"{name} failed ({status}): {last_error()}")


def call(name, *args):
    check(getattr(lib(), name)(*args), name)


def declared_symbols():
    """Function names declared in include/dna_amd.h (for the export test)."""
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dna_[a-z0-9_]+)\s*\(", src)))


def stream_ptr(device=None):
    return torch.cuda.current_stream(device).cuda_stream


def ptr(t):
    return None if t is None else t.data_ptr()
