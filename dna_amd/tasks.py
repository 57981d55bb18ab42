"""Task / loss / metric glue of the MLM path (reference src/tasks/*).

  bert_cross_entropy   src/tasks/metrics.py:268-273  (registered as output_metric_fns name)
  LMTask / HG38Task    src/tasks/tasks.py:169-191, :254-339 (identity encoder/decoder,
                       flatten logits, loss by name); registry "lm", "hg38"
  Perplexity, NumTokens  src/tasks/torchmetrics.py:24-115 (state kept as tensors; the
                       distributed reduction is a SUM all-reduce, like dist_reduce_fx="sum")
"""
import math

import torch
import torch.nn.functional as F


def bert_cross_entropy(x, y):
    """CE over the masked positions: x = (logits [(b*S), V], mask [b, S]), y = target ids."""
    logits = x[0]
    mask = x[1].reshape(y.shape)
    return F.cross_entropy(logits[mask], y[mask])


def cross_entropy(logits, y, ignore_index=-100):
    logits = logits.view(-1, logits.shape[-1])
    return F.cross_entropy(logits, y.view(-1), ignore_index=ignore_index)


output_metric_fns = {"bert_cross_entropy": bert_cross_entropy, "cross_entropy": cross_entropy}


class Perplexity:
    """exp(sum(loss * count) / sum(count)) accumulated in float64 (torchmetrics.py:24-73)."""

    def __init__(self):
        self.reset()

    def reset(self):
        self.total_log_probs = torch.zeros((), dtype=torch.float64)
        self.count = torch.zeros((), dtype=torch.int64)

    def update(self, preds, target, loss):
        self.update_count(loss, target.numel())

    def update_count(self, loss, count):
        """update() given target.numel() instead of the target tensor (no device sync)."""
        self.total_log_probs = self.total_log_probs.to(loss.device) + loss.detach().double() * count
        self.count = self.count.to(loss.device) + count

    def compute(self):
        return torch.exp(self.total_log_probs / self.count)


class NumTokens:
    """Running count of target tokens, never reset between epochs (torchmetrics.py:75-115)."""

    def __init__(self):
        self.count = torch.zeros((), dtype=torch.int64)

    def reset(self):
        pass

    def update(self, preds, target, loss=None):
        self.count = self.count + target.numel()

    def compute(self):
        return self.count


torchmetric_fns = {"perplexity": Perplexity, "num_tokens": NumTokens}


class LMTask:
    """forward(batch, model) -> (x, y, w) exactly like LMTask.forward (tasks.py:169-191) with
    identity encoder/decoder (encoder: null, decoder: null in configs/pipeline/bert_hg38.yaml)."""

    def __init__(self, dataset=None, model=None, loss="cross_entropy", torchmetrics=None,
                 metrics=None, **unused):
        name = loss if isinstance(loss, str) else loss["_name_"]
        self.loss_name = name
        self.loss = output_metric_fns[name]
        self.torchmetric_names = list(torchmetrics or [])
        self.train_torchmetrics = {n: torchmetric_fns[n]() for n in self.torchmetric_names}

    def forward(self, batch, model, state=None):
        x, y = batch[0], batch[1]
        out, state = model(x, state=state)
        logits = out.logits
        if isinstance(logits, tuple):
            logits = list(logits)
            logits[0] = logits[0].reshape(-1, logits[0].shape[-1])
        else:
            logits = logits.reshape(-1, logits.shape[-1])
        return logits, y.reshape(-1), {}


class HG38Task(LMTask):
    pass


registry = {"lm": LMTask, "hg38": HG38Task}
