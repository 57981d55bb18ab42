"""CPU oracle for the DNABERT-2 MLM pretraining hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may import anything in
this package, and only as the checker / the timed CPU baseline. The product path (`dna_amd`)
never imports it and fails loudly when its HIP library is missing.

Parity pins: tests/golden/*.npz|json, produced by tests/golden/make_golden.py, which runs the
reference (/root/reference, imported by path in the build container) -- see DESIGN.md §Oracle.
"""
