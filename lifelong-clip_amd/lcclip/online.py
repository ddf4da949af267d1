"""The online continual-learning loop of qcNPU/LifeLong-CLIP's AdapterCLIP trainer, composed from
this package's pieces (VERDICT r1 "the online loop itself").

Reference loop (methods/_trainer.py:320-357, methods/adapter_clip.py:34-176):

    for task in tasks:                                   _trainer.py:320
        total_classes = known + disjoint_class_num[task] _trainer.py:322
        sampler.set_task(task); online_before_task       :332-334  (freeze + reset AdamW, Q14)
        for epoch in range(epochNum):                    :336
            for images, labels in loader(batch_size):    :342
                online_step:                             adapter_clip.py:34-47
                    add_new_class(labels)                (exposed / batch-visible class lists)
                    online_iter x online_train(x.clone(), y.clone())
        online_after_task: set_token(class_names[:total_classes])   adapter_clip.py:129-130
        online_evaluate on the test samples of the exposed classes  _trainer.py:431-449
    A_auc / A_avg / A_last / F_last                      _trainer.py:367-378

online_train (adapter_clip.py:49-107): remap y into the batch's class list, GPU train
transform, tokens of the class list, fwd + CE-on-probs + bwd + AdamW (OnlineTrainer.step).

Pieces: SiBlurryStream / ClassBook (stream.py), TrainTransform (transforms.py), OnlineTrainer
(trainer.py), online_evaluate / AUCTracker / summarize (evaluate.py). The scheduler is the
reference's 'default' (constant LambdaLR, utils/train_utils.py:57-58), i.e. no-op. The replay
memory is disabled on this path (memory_batchsize = 0). A_auc: the reference
never fills eval_results (NaN); here every `eval_period` training samples the model
is evaluated on the test samples of the classes exposed so far, with the tokens of
class_names[:classes of the tasks so far] (class ids index the logit columns, as in the
reference's end-of-task evaluation), and A_auc is the mean of that curve.
"""
from __future__ import annotations

import torch

from .evaluate import AUCTracker, online_evaluate, summarize


class OnlineLoop:
    """trainer: OnlineTrainer over an AdapterCLIP wrapper; stream: SiBlurryStream over the
    training targets; book: ClassBook(class_names); train_x / test_x: f32 [n, 3, H, W] in [0, 1]
    (ToTensor values) when a transform is given, else already-normalised model inputs;
    tokenize(names) -> int64 [C, 77] token ids; transform: TrainTransform or None."""

    def __init__(self, trainer, stream, book, train_x, train_y, test_x, test_y, tokenize,
                 transform=None, batch_size=16, online_iter=3, epochs=1, eval_period=None,
                 test_batch=256, n_buckets=10, on_step=None):
        self.trainer = trainer
        self.wrapper = trainer.wrapper
        self.stream = stream
        self.book = book
        self.train_x, self.train_y = train_x, torch.as_tensor(train_y).long()
        self.test_x, self.test_y = test_x, torch.as_tensor(test_y).long()
        self.tokenize = tokenize
        self.transform = transform
        self.batch_size = int(batch_size)
        self.online_iter = int(online_iter)
        self.epochs = int(epochs)
        self.auc = AUCTracker(eval_period) if eval_period else None
        self.test_batch = int(test_batch)
        self.n_buckets = n_buckets
        self.on_step = on_step  # callback(step_index, loss, acc) after every optimizer step
        self.device = trainer.flat_p.device
        self.samples_seen = 0
        self.steps = 0
        self.log = []

    # ------------------------------------------------------------------ the step
    def online_train(self, x, y):
        """methods/adapter_clip.py:49-107 -> (loss, acc)."""
        ids, names = self.book.train_classes()
        y = self.book.remap(y)                                   # :75-76
        x = x.to(self.device, non_blocking=True)
        y = y.to(self.device, non_blocking=True)
        if self.transform is not None:
            x = self.transform(x, layout="patches")              # :81 (one draw per call)
        tokens = self.tokenize(names)                            # :84 set_token(names)
        if isinstance(tokens, torch.Tensor):
            tokens = tokens.to(self.device)
        loss, probs = self.trainer.step(x, y, tokens)            # :86-96
        acc = (probs.argmax(-1) == y).float().mean()
        loss_v, acc_v = float(loss.item()), float(acc.item())    # :103-104 (host sync)
        self.steps += 1
        if self.on_step is not None:
            self.on_step(self.steps, loss_v, acc_v)
        return loss_v, acc_v

    def online_step(self, images, labels):
        """methods/adapter_clip.py:34-47."""
        self.book.add_new_class(labels)
        tot_l = tot_a = 0.0
        for _ in range(self.online_iter):
            l, a = self.online_train(images.clone(), labels.clone())
            tot_l += l
            tot_a += a
        return tot_l / self.online_iter, tot_a / self.online_iter

    # ------------------------------------------------------------------ evaluation
    def _test_batches(self, classes):
        keep = torch.isin(self.test_y, torch.as_tensor(sorted(classes), dtype=torch.long))
        idx = keep.nonzero().flatten()                           # OnlineTestSampler
        for s in range(0, len(idx), self.test_batch):
            b = idx[s:s + self.test_batch]
            yield self.test_x[b], self.test_y[b]

    def evaluate(self, n_classes):
        """online_evaluate with the tokens of class_names[:n_classes] (online_after_task)."""
        self.wrapper.set_token(self.tokenize(self.book.class_names[:n_classes]))
        return online_evaluate(self.wrapper, self._test_batches(self.book.exposed_classes),
                               self.stream.num_tasks, device=self.device, n_buckets=self.n_buckets)

    # ------------------------------------------------------------------ the loop
    def run(self):
        task_records = {"task_acc": [], "cls_acc": []}
        known = 0
        for task in range(self.stream.num_tasks):
            total = known + self.stream.disjoint_class_num[task]   # _trainer.py:322
            self.stream.set_task(task)
            self.trainer.reset_optimizer()                          # online_before_task
            for epoch in range(self.epochs):
                idx = self.stream.task_indices()
                tl = ta = 0.0
                nb = 0
                for s in range(0, len(idx), self.batch_size):
                    b = torch.as_tensor(idx[s:s + self.batch_size], dtype=torch.long)
                    l, a = self.online_step(self.train_x[b], self.train_y[b])
                    tl, ta, nb = tl + l, ta + a, nb + 1
                    self.samples_seen += len(b)
                    if self.auc is not None and self.auc.due(self.samples_seen):
                        acc = self.evaluate(total)["avg_acc"]
                        self.auc.record(self.samples_seen, acc)
                self.log.append({"task": task, "epoch": epoch, "train_loss": tl / max(nb, 1),
                                 "train_acc": ta / max(nb, 1)})
            ev = self.evaluate(total)                               # online_after_task + eval
            task_records["task_acc"].append(ev["avg_acc"])
            task_records["cls_acc"].append(ev["cls_acc"])
            known = total
        eval_results = self.auc.results() if self.auc is not None else {}
        return {"task_records": task_records, "eval_results": eval_results,
                "summary": summarize(task_records, eval_results, self.stream.num_tasks),
                "log": self.log, "steps": self.steps, "samples_seen": self.samples_seen}
