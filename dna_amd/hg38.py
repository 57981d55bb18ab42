"""hg38 window dataset for DNABERT-2 MLM pretraining (registry dataset "bert_hg38").

Mirrors src/dataloaders/datasets/hg38_dataset.py (FastaInterval :40-124, bert_mask :238-286,
BertHG38Dataset :289-399) and the data module BertHG38 (src/dataloaders/genomics.py:1059-1254).
FASTA access goes through the native mmap reader (dna_fasta_*, replacing pyfaidx); tokenisation
through the native BPE. `bert_mask` keeps the reference's torch RNG draw order, so with the same
torch seed it yields the reference's exact masks; `bert_mask_fast` draws with Philox in C++ for
the high-throughput batch pipeline.
"""
import ctypes
import os
from random import random, randrange

import numpy as np
import torch

from . import _native as N
from .tokenizer import DNABertTokenizer

_COMP = {"A": "T", "C": "G", "G": "C", "T": "A", "a": "t", "c": "g", "g": "c", "t": "a"}


def string_reverse_complement(seq):
    return "".join(_COMP.get(b, b) for b in reversed(seq))


def coin_flip():
    return random() > 0.5


class FastaInterval:
    def __init__(self, *, fasta_file, return_seq_indices=False, shift_augs=None, rc_aug=False,
                 pad_interval=False):
        fasta_file = str(fasta_file)
        assert os.path.exists(fasta_file), "path to fasta file must exist"
        self.fasta_file = fasta_file
        self.return_seq_indices = return_seq_indices
        self.shift_augs = shift_augs
        self.rc_aug = rc_aug
        self.pad_interval = pad_interval
        self._open()

    def _open(self):
        L = N.lib()
        self._h = L.dna_fasta_open(self.fasta_file.encode())
        if not self._h:
            raise N.NativeError(f"dna_fasta_open: {N.last_error()}")
        self.chr_lens = {}
        for i in range(L.dna_fasta_num_records(self._h)):
            name = L.dna_fasta_record_name(self._h, i).decode()
            self.chr_lens[name] = L.dna_fasta_record_length(self._h, name.encode())

    def __getstate__(self):
        st = dict(self.__dict__)
        st.pop("_h", None)
        return st

    def __setstate__(self, st):
        self.__dict__.update(st)
        self._open()

    def close(self):
        if getattr(self, "_h", None):
            N.lib().dna_fasta_close(self._h)
            self._h = None

    def __call__(self, chr_name, start, end, max_length, return_augs=False):
        start, end = int(start), int(end)
        if self.shift_augs is not None:  # hg38_dataset.py:82-91
            min_shift, max_shift = self.shift_augs
            max_shift += 1
            L = self.chr_lens[chr_name]
            min_shift = max(start + min_shift, 0) - start
            max_shift = min(end + max_shift, L) - end
            rand_shift = randrange(min_shift, max_shift)
            start += rand_shift
            end += rand_shift
        rc = 1 if (self.rc_aug and coin_flip()) else 0
        cap = max(int(max_length), end - start) + 16
        if self.pad_interval:
            cap += int(max_length)
        buf = ctypes.create_string_buffer(cap)
        n = ctypes.c_int64(0)
        N.call("dna_fasta_interval", self._h, chr_name.encode(), start, end, int(max_length),
               int(self.pad_interval), rc, buf, cap, ctypes.addressof(n))
        return buf.raw[: n.value].decode()


def bert_mask(seq, mask_token_id, pad_token_id, vocab_size, mask_prob=0.15, random_token_prob=0.1,
              unchanged_token_prob=0.1, special_token_ids=None):
    """Reference masking with the reference's torch RNG draw order (hg38_dataset.py:238-286):
    rand(shape), rand(shape), randint(0, V, shape), then re-draws of special ids."""
    u1 = torch.rand(seq.shape)
    u2 = torch.rand(seq.shape)
    rt = torch.randint(0, vocab_size, seq.shape, dtype=torch.long)
    sp = torch.tensor(special_token_ids if special_token_ids is not None else [])
    while torch.isin(rt, sp).any():
        bad = torch.isin(rt, sp)
        rt[bad] = torch.randint(0, vocab_size, (int(bad.sum()),), dtype=torch.long)
    return bert_mask_from_draws(seq, u1, u2, rt, mask_token_id, pad_token_id, mask_prob,
                                random_token_prob, unchanged_token_prob)


def bert_mask_from_draws(seq, u1, u2, rand_tok, mask_token_id=4, pad_token_id=3, mask_prob=0.15,
                         random_token_prob=0.1, unchanged_token_prob=0.1):
    seq = torch.as_tensor(seq, dtype=torch.long).contiguous()
    u1 = torch.as_tensor(u1, dtype=torch.float32).contiguous()
    u2 = torch.as_tensor(u2, dtype=torch.float32).contiguous()
    rt = torch.as_tensor(rand_tok, dtype=torch.long).contiguous()
    n = seq.numel()
    out = torch.empty_like(seq)
    mask = torch.empty(seq.shape, dtype=torch.bool)
    labels = torch.empty_like(seq)
    N.call("dna_bert_mask_from_draws", seq.data_ptr(), n, u1.data_ptr(), u2.data_ptr(),
           rt.data_ptr(), mask_token_id, pad_token_id, mask_prob, random_token_prob,
           unchanged_token_prob, out.data_ptr(), mask.data_ptr(), labels.data_ptr())
    return out, mask, labels


def bert_mask_fast(seq, mask_token_id, pad_token_id, vocab_size, special_token_ids, seed,
                   sample_id, mask_prob=0.15, random_token_prob=0.1, unchanged_token_prob=0.1):
    """Same semantics, Philox4x32-10 draws keyed by (seed, sample_id) in C++ (no torch RNG)."""
    seq = torch.as_tensor(seq, dtype=torch.long).contiguous()
    sp = torch.as_tensor(list(special_token_ids), dtype=torch.long)
    out = torch.empty_like(seq)
    mask = torch.empty(seq.shape, dtype=torch.bool)
    labels = torch.empty_like(seq)
    N.call("dna_bert_mask", seq.data_ptr(), seq.numel(), vocab_size, sp.data_ptr(), sp.numel(),
           mask_token_id, pad_token_id, mask_prob, random_token_prob, unchanged_token_prob,
           seed, sample_id, out.data_ptr(), mask.data_ptr(), labels.data_ptr())
    return out, mask, labels


def random_mask(seq, mask_token_id, mask_prob=0.15):
    """hg38_dataset.py:228-236 (objective != stdmlm)."""
    mask = torch.rand(seq.shape) < mask_prob
    masked = seq.clone()
    masked[mask] = mask_token_id
    return masked, mask


class BertHG38Dataset(torch.utils.data.Dataset):
    """BED rows of one split -> ((masked_ids, mask, labels), target)  (hg38_dataset.py:289-399)."""

    def __init__(self, split, bed_file, fasta_file, max_length, pad_max_length=None, tokenizer=None,
                 tokenizer_name=None, add_eos=False, return_seq_indices=False, shift_augs=None,
                 rc_aug=False, return_augs=False, replace_N_token=False, pad_interval=False,
                 use_tokenizer=True, objective="stdmlm"):
        import pandas as pd
        self.max_length = max_length
        self.pad_max_length = pad_max_length if pad_max_length is not None else max_length
        self.tokenizer_name = tokenizer_name
        self.tokenizer = tokenizer
        self.return_augs = return_augs
        self.add_eos = add_eos
        self.replace_N_token = replace_N_token
        self.pad_interval = pad_interval
        self.use_tokenizer = use_tokenizer
        self.objective = objective
        assert os.path.exists(str(bed_file)), "path to .bed file must exist"
        df = pd.read_csv(str(bed_file), sep="\t", names=["chr_name", "start", "end", "split"])
        df = df[df["split"] == split]
        self.rows = list(zip(df["chr_name"].tolist(), df["start"].tolist(), df["end"].tolist()))
        self.fasta = FastaInterval(fasta_file=fasta_file, return_seq_indices=return_seq_indices,
                                   shift_augs=shift_augs, rc_aug=rc_aug, pad_interval=pad_interval)

    def __len__(self):
        return len(self.rows)

    def _ids(self, seq):
        if self.tokenizer_name == "bpe":
            ids = self.tokenizer(seq, padding="max_length", max_length=self.pad_max_length,
                                 truncation=True)["input_ids"]
            ids = ids[1:] if self.add_eos else ids[1:-1]
        elif self.tokenizer_name == "char":
            ids = self.tokenizer(seq, add_special_tokens=bool(self.add_eos), padding="max_length",
                                 max_length=self.max_length, truncation=True)["input_ids"]
        else:  # the reference's __getitem__ has no kmer branch either (hg38_dataset.py:357-380)
            raise NotImplementedError(f"items for tokenizer {self.tokenizer_name!r}: the reference "
                                      "dataset tokenises bpe / char only (kmer: tokenizer only)")
        return torch.LongTensor(ids)

    # ---- batched fetch (torch DataLoader calls __getitems__ with a whole batch of indices):
    # FASTA windows -> one multithreaded native BPE call for the batch -> native BERT masking with
    # Philox draws keyed by (mask_seed, dataset index) -- reproducible for any worker layout, the
    # same mask statistics as the reference's torch-RNG draws; __getitem__ keeps the
    # reference's exact torch draw order for the parity tests. bpe + stdmlm only; any other
    # configuration falls back to per-item __getitem__.
    # Indices may arrive epoch-tagged (EpochSampler: epoch * len + i), so a window draws a fresh
    # mask every epoch as the reference's per-__getitem__ torch draws do; mask_seed is set from
    # train.seed by the data module's owner.
    mask_seed = 2222
    bpe_threads = 0  # 0: all cores (set per worker by BertHG38 when it starts several workers)

    def __getitems__(self, indices):
        if not (self.tokenizer_name == "bpe" and self.objective == "stdmlm" and self.use_tokenizer
                and not self.replace_N_token and hasattr(self.tokenizer, "encode_windows")):
            return [self[i] for i in indices]
        wins = []
        n = len(self.rows)
        for i in indices:
            chr_name, start, end = self.rows[int(i) % n]
            wins.append(self.fasta(chr_name, start, end, max_length=self.max_length,
                                   return_augs=self.return_augs))
        tok = self.tokenizer
        ids = torch.from_numpy(tok.encode_windows(wins, self.pad_max_length, add_eos=self.add_eos,
                                                  nthreads=self.bpe_threads))
        out = []
        for j, i in enumerate(indices):
            target = ids[j]
            data = bert_mask_fast(target, tok.mask_token_id, tok.pad_token_id, tok.vocab_size,
                                  tok.all_special_ids, seed=self.mask_seed, sample_id=int(i))
            out.append((data, target))
        return out

    def __getitem__(self, idx):
        chr_name, start, end = self.rows[int(idx) % len(self.rows)]
        seq = self.fasta(chr_name, start, end, max_length=self.max_length,
                         return_augs=self.return_augs)
        seq = self._ids(seq)
        if not self.use_tokenizer:  # hg38_dataset.py:383-386
            seq = seq - 7
            m = (seq >= 4) | (seq < 0)
            seq[m] = 4
        if self.replace_N_token:  # hg38_dataset.py:388-390 (needs the char vocab)
            vocab = getattr(self.tokenizer, "_vocab_str_to_int", None)
            if vocab is None:
                raise AttributeError("replace_N_token needs the char tokenizer (_vocab_str_to_int)")
            seq = torch.where(seq == vocab["N"], torch.full_like(seq, self.tokenizer.pad_token_id), seq)
        data, target = seq.clone(), seq.clone()
        tok = self.tokenizer
        if self.objective == "stdmlm":
            return bert_mask(data, tok.mask_token_id, tok.pad_token_id, tok.vocab_size,
                             special_token_ids=tok.all_special_ids), target
        return random_mask(data, tok.mask_token_id), target


class EpochSampler(torch.utils.data.Sampler):
    """Wraps the loader's index sampler and tags every index with the epoch (epoch * len + i):
    the indices travel to the (persistent) worker processes with each batch, so the dataset's
    masking key changes per epoch without any state in the workers. set_epoch is forwarded to a
    wrapped DistributedSampler (permutation = randperm(seed + epoch), as torch DDP)."""

    def __init__(self, base, n):
        self.base, self.n, self.epoch = base, int(n), 0

    def set_epoch(self, epoch):
        self.epoch = int(epoch)
        if hasattr(self.base, "set_epoch"):
            self.base.set_epoch(epoch)

    def __iter__(self):
        off = self.epoch * self.n
        return (off + int(i) for i in self.base)

    def __len__(self):
        return len(self.base)


class FaultTolerantDistributedSampler(torch.utils.data.distributed.DistributedSampler):
    """The reference's resumable sampler (fault_tolerant_sampler.py:64-122): a DistributedSampler
    (permutation randperm(seed + epoch), padded / trimmed to whole shards, rank-strided) that
    counts the indices it has yielded; state_dict() = {epoch, counter}; after load_state_dict the
    next iteration starts `counter` indices into this rank's shard, once. Used for every world
    size when the data module has fault_tolerant=True (the reference's one-process
    RandomFaultTolerantSampler draws its permutation from an unseeded generator; here one
    process is the world-1 case of the same seeded sampler)."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        self.counter = 0
        self.restarting = False

    def state_dict(self):
        return {"epoch": self.epoch, "counter": self.counter}

    def load_state_dict(self, state):
        self.epoch = int(state["epoch"])
        self.counter = int(state["counter"])
        self.restarting = True

    def __iter__(self):
        shard = list(super().__iter__())
        if self.restarting:
            shard = shard[self.counter:]
            self.restarting = False
        else:
            self.counter = 0
        for i in shard:
            self.counter += 1
            yield i
        self.counter = 0


def check_fault_tolerant_args(shuffle, fault_tolerant, ddp, fast_forward_epochs,
                              fast_forward_batches):
    """The reference data modules' argument checks (genomics.py:1117-1126)."""
    if fault_tolerant and not shuffle:
        raise ValueError("fault_tolerant=True needs shuffle=True (genomics.py:1117-1118)")
    if ddp and not fault_tolerant:
        raise ValueError("ddp=True needs fault_tolerant=True (genomics.py:1120-1121)")
    if (fast_forward_epochs is not None or fast_forward_batches is not None) and \
            not (ddp and fault_tolerant):
        raise ValueError("fast_forward_epochs / fast_forward_batches need ddp=True and "
                         "fault_tolerant=True (genomics.py:1125-1126)")


class FaultTolerantMixin:
    """fault_tolerant / ddp / fast_forward_* of the reference's data modules: train.py reads
    them and, on a resume, fast-forwards the FaultTolerantDistributedSampler instead of reading
    and discarding the consumed batches."""

    def _init_fault_tolerant(self, shuffle, fault_tolerant, ddp, fast_forward_epochs,
                             fast_forward_batches):
        check_fault_tolerant_args(shuffle, fault_tolerant, ddp, fast_forward_epochs,
                                  fast_forward_batches)
        self.fault_tolerant = bool(fault_tolerant)
        self.ddp = bool(ddp)
        self.fast_forward_epochs = fast_forward_epochs
        self.fast_forward_batches = fast_forward_batches

    def load_state_dict(self, checkpoint):
        """genomics.py:1249-1253: the fit loop's completed epochs / batches of a checkpoint."""
        if self.fault_tolerant:
            loops = checkpoint["loops"]["fit_loop"]
            self.fast_forward_epochs = loops["epoch_progress"]["current"]["completed"]
            self.fast_forward_batches = loops["epoch_loop.batch_progress"]["current"]["completed"]


def _profiler_attached():
    """rocprofv3 preloads its tool library, which brings the HSA runtime up before main()."""
    pre = os.environ.get("LD_PRELOAD", "")
    return "rocprof" in pre or any(k.startswith(("ROCPROF", "ROCP_")) for k in os.environ)


def worker_context(num_workers):
    """DataLoader workers are never forked from a process whose HIP runtime is up (train.py builds
    its loader after the model is on the GPU; under rocprofv3 the tool library has brought HSA up
    before main): a forked child inherits the parent's HIP/HSA state -- queues, doorbells, the
    profiler's interception of them -- and can fault in it (round 2's "workers crash under the
    profiler"). Such a process gets spawned workers (the native FASTA and BPE handles re-open on
    unpickle); before any GPU init the default fork stays (bench.py measures its data path
    there)."""
    if num_workers > 0 and (_profiler_attached() or
                            (torch.cuda.is_available() and torch.cuda.is_initialized())):
        return "spawn"
    return None


def host_threads():
    """CPU threads this process may use: the affinity set, capped by OMP_NUM_THREADS when the
    launcher sets it (a GPU host shares its cores among the GPUs' processes)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return n


class SequenceDataset:
    """`_name_` registry populated by subclasses (src/dataloaders/base.py:169-183)."""
    registry = {}

    def __init_subclass__(cls, **kw):
        super().__init_subclass__(**kw)
        if getattr(cls, "_name_", None):
            SequenceDataset.registry[cls._name_] = cls


class BertHG38(FaultTolerantMixin, SequenceDataset):
    """Data module "bert_hg38" (genomics.py:1059-1254)."""
    _name_ = "bert_hg38"

    def __init__(self, bed_file=None, fasta_file=None, tokenizer_name=None, dataset_config_name=None,
                 max_length=1024, d_output=2, rc_aug=False, max_length_val=None,
                 max_length_test=None, val_ratio=0.0005, val_split_seed=2357,
                 use_fixed_len_val=False, add_eos=True, detokenize=False, val_only=False,
                 batch_size=32, batch_size_eval=None, num_workers=1, shuffle=False,
                 pin_memory=False, drop_last=False, fault_tolerant=False, ddp=False,
                 fast_forward_epochs=None, fast_forward_batches=None, replace_N_token=False,
                 pad_interval=False, use_tokenizer=True, pad_max_length=None, objective="stdmlm",
                 tokenizer_path=None, **kwargs):
        data_root = os.environ.get("DATA_PATH", os.path.join(os.getcwd(), "data"))
        self.bed_file = bed_file or os.path.join(data_root, self._name_, "human-sequences.bed")
        self.fasta_file = fasta_file or os.path.join(data_root, self._name_, "hg38.ml.fa")
        self.tokenizer_name = tokenizer_name
        self.tokenizer_path = tokenizer_path
        self.max_length = max_length
        self.max_length_val = max_length_val if max_length_val is not None else max_length
        self.max_length_test = max_length_test if max_length_test is not None else max_length
        self.add_eos = add_eos
        self.rc_aug = rc_aug
        self.batch_size = batch_size
        self.batch_size_eval = batch_size_eval if batch_size_eval is not None else batch_size
        self.num_workers = num_workers
        self.shuffle = shuffle
        self.pin_memory = pin_memory
        self.drop_last = drop_last
        self.replace_N_token = replace_N_token
        self.pad_interval = pad_interval
        self.use_tokenizer = use_tokenizer
        self.pad_max_length = pad_max_length
        self.objective = objective
        self._init_fault_tolerant(shuffle, fault_tolerant, ddp, fast_forward_epochs,
                                  fast_forward_batches)
        if use_fixed_len_val:
            raise NotImplementedError("use_fixed_len_val (BertHG38FixedDataset) is out of scope")

    def setup(self, stage=None):
        if self.tokenizer_name == "bpe":
            self.tokenizer = DNABertTokenizer(self.tokenizer_path)
        elif self.tokenizer_name == "char":  # genomics.py:1132-1138
            from .tokenizer import CharacterTokenizer
            self.tokenizer = CharacterTokenizer(characters=["A", "C", "G", "T", "N"],
                                                model_max_length=self.max_length + 2)
        elif self.tokenizer_name == "kmer":  # genomics.py:1142-1144 (NT-v2 6-mer EsmTokenizer)
            from .tokenizer import KmerTokenizer
            self.tokenizer = KmerTokenizer(model_max_length=2048)
        else:
            raise NotImplementedError(f"tokenizer_name={self.tokenizer_name!r}: bpe / char / kmer")
        self.vocab_size = len(self.tokenizer)
        self.init_datasets()

    def init_datasets(self):
        self.dataset_train, self.dataset_val, self.dataset_test = [
            BertHG38Dataset(split=split, bed_file=self.bed_file, fasta_file=self.fasta_file,
                            max_length=ml, tokenizer=self.tokenizer,
                            tokenizer_name=self.tokenizer_name, add_eos=self.add_eos,
                            rc_aug=self.rc_aug, replace_N_token=self.replace_N_token,
                            pad_interval=self.pad_interval, use_tokenizer=self.use_tokenizer,
                            pad_max_length=self.pad_max_length, objective=self.objective)
            for split, ml in zip(["train", "valid", "test"],
                                 [self.max_length, self.max_length_val, self.max_length_test])]

    def _data_loader(self, dataset, batch_size, shuffle=False, sampler=None):
        # each worker tokenises whole batches with the native multithreaded BPE: split the cores
        cores = host_threads()
        dataset.bpe_threads = max(1, cores // max(1, self.num_workers)) if self.num_workers else 0
        if sampler is None:
            sampler = (torch.utils.data.RandomSampler(dataset) if shuffle
                       else torch.utils.data.SequentialSampler(dataset))
        return torch.utils.data.DataLoader(dataset, batch_size=batch_size,
                                           num_workers=self.num_workers,
                                           sampler=EpochSampler(sampler, len(dataset)),
                                           drop_last=self.drop_last, pin_memory=self.pin_memory,
                                           persistent_workers=self.num_workers > 0,
                                           multiprocessing_context=worker_context(self.num_workers))

    def train_dataloader(self, sampler=None, **kwargs):
        return self._data_loader(self.dataset_train, self.batch_size,
                                 shuffle=self.shuffle and sampler is None, sampler=sampler)

    def val_dataloader(self, sampler=None, **kwargs):
        return self._data_loader(self.dataset_val, self.batch_size_eval, sampler=sampler)

    def test_dataloader(self, sampler=None, **kwargs):
        return self._data_loader(self.dataset_test, self.batch_size_eval, sampler=sampler)
