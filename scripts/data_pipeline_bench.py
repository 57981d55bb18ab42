#!/usr/bin/env python
"""Host data path of train.py at the bench shape: the registry dataset "bert_hg38" (BertHG38 ->
BertHG38Dataset over synthetic hg38 FASTA/BED, 4096-bp windows, BPE pad_max_length 514) through
its torch DataLoader (batched __getitems__: FASTA -> native multithreaded BPE -> native masking;
worker processes, pinned memory) and DeviceBatch.from_host (host row bookkeeping + H2D copy),
exactly as train.py consumes it. Reports sequences/s per worker layout on this host's cores.

    python scripts/data_pipeline_bench.py [--workers 4,8,16] [--batches 30]
"""
import argparse
import json
import os
import sys
import tempfile
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def measure(root, workers, batch=256, batches=60, warmup=None, device=None):
    """Steady-state seq/s of DataLoader iteration + DeviceBatch.from_host over `batches` batches:
    the timer starts after 2 x workers x prefetch_factor(2) batches, i.e. once the batches the
    workers prefetched at start-up have been consumed."""
    warmup = 4 * max(1, workers) + 1 if warmup is None else warmup
    from dna_amd.hg38 import BertHG38
    from dna_amd.trainer import DeviceBatch
    os.environ["DATA_PATH"] = root
    dm = BertHG38(tokenizer_name="bpe", max_length=4096, pad_max_length=514, add_eos=False,
                  batch_size=batch, num_workers=workers, shuffle=True, pin_memory=True,
                  drop_last=True)
    dm.setup()
    loader = dm.train_dataloader()
    it = iter(loader)
    dev = device or (torch.device("cuda", 0) if torch.cuda.is_available() else torch.device("cpu"))
    n = 0
    t0 = None
    for i in range(warmup + batches):
        if i == warmup:
            if dev.type == "cuda":
                torch.cuda.synchronize()
            t0 = time.perf_counter()
        try:
            (masked, mask, labels), target = next(it)
        except StopIteration:  # dataset smaller than warm-up + timed batches: next epoch
            it = iter(loader)
            (masked, mask, labels), target = next(it)
        DeviceBatch.from_host(masked, mask, labels, target, dev)
        if i >= warmup:
            n += masked.shape[0]
    if dev.type == "cuda":
        torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    del it, loader
    return n / dt


def synthetic_root(n_chroms=8, chrom_len=33_554_432):
    from dna_amd.synthetic import write_hg38
    root = tempfile.mkdtemp(prefix="dna_hg38_")
    write_hg38(root, n_chroms=n_chroms, chrom_len=chrom_len, max_length=4096)
    return root


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workers", default="4,8,16")
    ap.add_argument("--batches", type=int, default=60)
    ap.add_argument("--batch", type=int, default=256)
    a = ap.parse_args()
    from dna_amd.hg38 import host_threads
    cores = host_threads()
    root = synthetic_root()
    res = {}
    for w in (int(x) for x in a.workers.split(",")):
        res[w] = round(measure(root, w, a.batch, a.batches), 1)
        print(json.dumps({"workers": w, "seq_per_s": res[w], "host_threads": cores}), flush=True)


if __name__ == "__main__":
    main()
