"""dna_amd -- MI355X-native DNABERT-2 masked-LM pretraining hot path.

Product path: hand-written HIP kernels for gfx950 behind a C ABI (include/dna_amd.h,
dna_amd/csrc/, built into dna_amd/lib/libdna_amd.so), bound by ctypes. Host side mirrors the
reference's plugin interfaces: registry model "dnabert2" (bert_layers.BertForMaskedLM), dataset
"bert_hg38" (hg38), task "hg38" + loss "bert_cross_entropy" (tasks), train.py entry point.
"""
__version__ = "0.1.0"
