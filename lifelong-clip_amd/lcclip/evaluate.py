"""Online evaluation and the continual-learning summary metrics of qcNPU/LifeLong-CLIP
(methods/adapter_clip.py:132-175, methods/_trainer.py:359-378, 519-534), over the HIP forward.

* interpret_pred    _trainer.py:519-534: per-bucket sample / correct counts with bucket =
                    y // n_tasks in a fixed table of 10 (the reference's torch.zeros(10)); a
                    label whose bucket is >= 10 raises IndexError as it does there (e.g. 200
                    classes over 5 tasks). n_buckets=None sizes the table to fit instead.
* online_evaluate   adapter_clip.py:132-175: argmax of the model's first output over a loader,
                    avg_acc, per-bucket accuracies (`cls_acc` and `task_acc` are the same list),
                    avg_loss (0: the reference never accumulates a loss), confusion matrix.
* summarize         _trainer.py:367-378: A_auc = mean of the periodic test accuracies,
                    A_avg = mean task accuracy, A_last = last task's, F_last = mean over buckets
                    of (best earlier accuracy - last accuracy) where the best is > 0. The
                    reference never fills its eval_results (A_auc is NaN there):
                    AUCTracker records (samples seen, test accuracy) every eval_period samples,
                    which is the anytime-accuracy curve A_auc averages.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def interpret_pred(y, pred, n_tasks: int, n_buckets: int | None = 10):
    y = y.long()
    b = torch.div(y, n_tasks, rounding_mode="floor")
    size = n_buckets
    if size is None:
        size = int(b.max().item()) + 1 if b.numel() else 1
    elif b.numel() and int(b.max().item()) >= size:
        raise IndexError(f"label bucket {int(b.max().item())} out of range for {size} buckets "
                         "(_trainer.py:521 allocates torch.zeros(10))")
    num = torch.bincount(b, minlength=size).float().cpu()
    corr = torch.bincount(b[y == pred.long()], minlength=size).float().cpu()
    return num, corr


def confusion_matrix(labels, preds):
    """sklearn.metrics.confusion_matrix(labels, preds): rows = true, cols = predicted, over the
    sorted union of the values present."""
    labels = np.asarray(labels, dtype=np.int64)
    preds = np.asarray(preds, dtype=np.int64)
    vals = np.unique(np.concatenate([labels, preds]))
    idx = {v: i for i, v in enumerate(vals.tolist())}
    cm = np.zeros((len(vals), len(vals)), dtype=np.int64)
    np.add.at(cm, ([idx[v] for v in labels.tolist()], [idx[v] for v in preds.tolist()]), 1)
    return cm


@torch.no_grad()
def online_evaluate(model, loader, n_tasks: int, device=None, n_buckets: int | None = 10):
    """model(x) -> (logits or probs, ...) as AdapterCLIP.forward; loader yields (x, y)."""
    was_training = model.training
    model.eval()
    correct_l = num_l = None
    label, pred_list = [], []
    for x, y in loader:
        if device is not None:
            x, y = x.to(device), y.to(device)
        out = model(x)
        logit = out[0] if isinstance(out, (tuple, list)) else out
        pred = torch.argmax(logit, dim=-1)
        num, corr = interpret_pred(y, pred, n_tasks, n_buckets)
        if num_l is None:
            num_l, correct_l = num, corr
        else:
            if num.numel() > num_l.numel():  # n_buckets=None: grow the table
                num_l = torch.nn.functional.pad(num_l, (0, num.numel() - num_l.numel()))
                correct_l = torch.nn.functional.pad(correct_l, (0, num.numel() - correct_l.numel()))
            num_l[:num.numel()] += num
            correct_l[:corr.numel()] += corr
        label += y.tolist()
        pred_list += pred.tolist()
    model.train(was_training)
    total = num_l.sum()
    task_acc = (correct_l / (num_l + 1e-5)).tolist()
    return {"avg_loss": 0.0 / total.item() if total.item() else 0.0,
            "avg_acc": (correct_l.sum() / total).item(),
            "cls_acc": task_acc, "task_acc": task_acc,
            "confusion_matrix": confusion_matrix(label, pred_list).tolist()}


class AUCTracker:
    """Anytime accuracy: evaluate every `eval_period` training samples (the reference's
    eval_period / data_cnt bookkeeping, _trainer.py:359-364) and keep the curve."""

    def __init__(self, eval_period: int):
        self.eval_period = int(eval_period)
        self.test_acc, self.data_cnt = [], []
        self._next = self.eval_period

    def due(self, samples_seen: int) -> bool:
        return samples_seen >= self._next

    def record(self, samples_seen: int, acc: float):
        self.test_acc.append(float(acc))
        self.data_cnt.append(int(samples_seen))
        while self._next <= samples_seen:
            self._next += self.eval_period

    def results(self):
        return {"test_acc": list(self.test_acc), "data_cnt": list(self.data_cnt)}


def summarize(task_records, eval_results, n_tasks: int):
    """_trainer.py:367-378 -> {A_auc, A_avg, A_last, F_last}."""
    ta = eval_results.get("test_acc", []) if eval_results else []
    a_auc = float(np.mean(ta)) if len(ta) else math.nan
    a_avg = float(np.mean(task_records["task_acc"]))
    a_last = float(task_records["task_acc"][n_tasks - 1])
    cls_acc = np.array(task_records["cls_acc"])
    diffs = []
    for j in range(n_tasks):
        best = np.max(cls_acc[:-1, j]) if cls_acc.shape[0] > 1 else 0.0
        if best > 0:
            diffs.append(best - cls_acc[-1, j])
    f_last = float(np.mean(diffs)) if diffs else math.nan
    return {"A_auc": a_auc, "A_avg": a_avg, "A_last": a_last, "F_last": f_last}
