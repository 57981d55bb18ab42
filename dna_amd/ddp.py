"""Data-parallel gradient exchange: bucketed RCCL all-reduce overlapped with backward.

Replaces the reference's PyTorch-Lightning DDP (strategy: ddp, dnabert2_hg38_pretrain.yaml:53;
torch DDP reducer with 25 MB buckets and NCCL_P2P_DISABLE=1 from train.py:3). Design for MI355X:
  * gradients already live in ONE flat fp32 buffer (dna_amd.flat), laid out in backward order,
    so a bucket is a contiguous slice: no pack/unpack copies, one all-reduce per bucket;
  * a bucket fires as soon as every parameter in it has received all of its gradient
    contributions (post-accumulate-grad hooks; the tied embedding/decoder weight gets two);
    the collective runs on RCCL's stream, overlapping the rest of the backward on the compute
    stream; RCCL P2P over xGMI stays enabled;
  * SUM all-reduce; the 1/world_size averaging is folded into the fused AdamW kernel
    (grad_scale), saving a pass over 468 MB.
The expected contribution count per parameter is discovered on the first backward (which
reduces everything at the end, unoverlapped) -- robust to unused / shared parameters like DDP's
find_unused_parameters=True (train.py:630-639).
"""
import os

import torch
import torch.distributed as dist


def _host_staged(t, group=None):
    """gloo (the one-GPU multi-rank rehearsal) reduces CUDA tensors through its CUDA algorithms,
    which deadlocked with more than two ranks sharing one GPU (round 6: every rank parked in the
    first bucket's wait at 4 ranks, fine at 2): its collectives go through a host copy instead.
    RCCL (the real multi-GPU path) reduces device buffers in place."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def all_reduce_(t, op=dist.ReduceOp.SUM, group=None):
    """In-place all-reduce of `t` (blocking), host-staged under gloo (a bf16 tensor is summed in
    fp32 there and rounded once; RCCL's ring rounds every hop -- scripts/wire_error.py emulates
    that order)."""
    if _host_staged(t, group):
        torch.cuda.current_stream(t.device).synchronize()
        c = t.float().cpu() if t.dtype == torch.bfloat16 else t.cpu()
        dist.all_reduce(c, op=op, group=group)
        t.copy_(c)
    else:
        dist.all_reduce(t, op=op, group=group)
    return t


def broadcast_(t, src=0, group=None):
    """In-place broadcast of `t` from rank `src` (blocking), host-staged under gloo."""
    if _host_staged(t, group):
        torch.cuda.current_stream(t.device).synchronize()
        c = t.cpu()
        dist.broadcast(c, src=src, group=group)
        t.copy_(c)
    else:
        dist.broadcast(t, src=src, group=group)
    return t


class _Done:
    """A finished collective (the host-staged gloo path is synchronous)."""

    def wait(self):
        return True


class GradBucketReducer:
    """wire_dtype "fp32" (default) all-reduces the fp32 gradient buckets in place; "bf16" halves
    the bytes on the wire (234 MB instead of 468 MB for DNABERT-2): each bucket is
    cast to a persistent bf16 staging slice when it fires, all-reduced (SUM) there, and cast back
    into the fp32 flat gradient in finish(), after its collective. The 1/world average stays in
    the AdamW kernel either way (grad_scale)."""

    def __init__(self, flat, bucket_mb: float = 25.0, group=None, wire_dtype="fp32", force=None):
        """force=True (or DNA_DDP_FORCE=1) runs the bucketed collectives even at world size 1,
        over an initialised process group: on a one-GPU box that is the only way the RCCL leg
        (per-bucket async all-reduce on RCCL's stream, finish()'s waits, the bf16 wire cast-back)
        executes on hardware before a multi-GPU run (tests/test_gpu_rccl.py)."""
        self.flat = flat
        self.group = group
        if wire_dtype not in ("fp32", "bf16"):
            raise ValueError(f"wire_dtype {wire_dtype!r}: fp32 or bf16")
        self.wire_dtype = wire_dtype
        self._wire = None  # bf16 staging buffer (allocated on first use)
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        cap = int(bucket_mb * 1024 * 1024 / 4)
        # contiguous buckets of whole parameters, in flat (= backward) order
        self.buckets = []  # [start, end, [param ids]]
        cur = None
        for p, (o, n, _) in sorted(zip(flat.params, flat.slices), key=lambda t: t[1][0]):
            if cur is None or (o + n - cur[0] > cap and cur[2]):
                cur = [o, o + n, []]
                self.buckets.append(cur)
            cur[1] = o + n
            cur[2].append(id(p))
        self.bucket_of = {pid: bi for bi, b in enumerate(self.buckets) for pid in b[2]}
        self.expected = None  # per-param contribution counts, learned on the first backward
        self._seen = {}
        self._pending = [0] * len(self.buckets)
        self._works = []
        self._fired = [False] * len(self.buckets)
        self._sync = True
        self.fired_in_backward = 0
        self._handles = [p.register_post_accumulate_grad_hook(self._hook) for p in flat.params]
        for p in flat.params:  # contributions written directly by fused kernels report here
            p._dna_notify = self._hook
        if force is None:
            force = os.environ.get("DNA_DDP_FORCE", "0") == "1"
        if force and not dist.is_initialized():
            raise RuntimeError("GradBucketReducer(force=True) needs an initialised process group "
                               "(DNA_DDP_FORCE=1 with WORLD_SIZE=1: bench.py / train.py create it)")
        self.enabled = self.world > 1 or bool(force)

    def _hook(self, p):
        if not self.enabled or not self._sync:
            return
        pid = id(p)
        self._seen[pid] = self._seen.get(pid, 0) + 1
        if self.expected is None:
            return
        if self._seen[pid] == self.expected.get(pid, 0):
            bi = self.bucket_of[pid]
            self._pending[bi] -= 1
            if self._pending[bi] == 0:
                self._launch(bi)

    def _launch(self, bi):
        s, e, _ = self.buckets[bi]
        self._fired[bi] = True
        # weight gradients may still be in flight on the side stream (functional.Linear)
        from .functional import join_side_stream
        if self.flat.grad.is_cuda:
            join_side_stream()
        if self.wire_dtype == "bf16":
            if self._wire is None:
                self._wire = torch.empty(self.flat.grad.numel(), dtype=torch.bfloat16,
                                         device=self.flat.grad.device)
            buf = self._wire[s:e]
            buf.copy_(self.flat.grad[s:e])
        else:
            buf = self.flat.grad[s:e]
        if _host_staged(buf, self.group):  # rehearsal backend: synchronous, through the host
            all_reduce_(buf, group=self.group)
            self._works.append((_Done(), s, e))
        else:
            self._works.append((dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group,
                                                async_op=True), s, e))

    def prepare(self, sync=True):
        """Call before each backward; sync=False for accumulation micro-batches (no collective,
        gradients keep accumulating locally, like DDP's no_sync())."""
        self._sync = sync
        if not sync or not self.enabled:
            return
        self._seen = {}
        self._works = []
        self._fired = [False] * len(self.buckets)
        if self.expected is not None:
            self._pending = [sum(1 for pid in b[2] if self.expected.get(pid, 0) > 0)
                             for b in self.buckets]
            for bi, n in enumerate(self._pending):
                if n == 0:
                    self._launch(bi)  # bucket of parameters that never get gradients

    def finish(self):
        """Call after backward: launch what did not fire, wait for all collectives."""
        if not self.enabled or not self._sync:
            return
        # how many buckets the backward itself launched (overlap evidence; tests read it)
        self.fired_in_backward = sum(self._fired)
        if self.expected is None:
            self.expected = dict(self._seen)
        for bi in range(len(self.buckets)):
            if not self._fired[bi]:
                self._launch(bi)
        for w, s, e in self._works:
            w.wait()
            if self.wire_dtype == "bf16":
                self.flat.grad[s:e].copy_(self._wire[s:e])
        self._works = []

    @property
    def grad_scale(self):
        return 1.0 / self.world


def reduce_metrics(loss, num_tokens, group=None, extra=None):
    """Rank-mean of the step loss and the global token count as ONE small all-reduce (SURVEY
    §8(e): DDP loss semantics = mean of per-rank masked-token means; scalar metrics packed into
    one collective at the logging interval). Returns (mean_loss, total_tokens) as Python numbers;
    without a process group, the local values. With `extra` (a list of scalar tensors or numbers:
    torchmetric states whose dist_reduce_fx is "sum"), returns (mean_loss, [their global sums])
    in place of the token count, still one collective."""
    lv = loss.detach().reshape(()).to(torch.float64)
    grouped = dist.is_available() and dist.is_initialized()
    if grouped and dist.get_backend(group) == "nccl" and not lv.is_cuda:
        # RCCL reduces device buffers only (evaluate() passes a CPU placeholder loss)
        lv = lv.to(torch.device("cuda", torch.cuda.current_device()))
    vals = [num_tokens] if extra is None else list(extra)
    t = torch.stack([lv] + [torch.as_tensor(v).detach().to(device=lv.device, dtype=torch.float64)
                            .reshape(()) for v in vals])
    if grouped:
        all_reduce_(t, group=group)
        world = dist.get_world_size(group)
    else:
        world = 1
    out = t.cpu().tolist()
    if extra is None:
        return out[0] / world, int(round(out[1]))
    return out[0] / world, out[1:]
