"""Si-Blurry online stream and the class bookkeeping around the online step.

CPU producers of the two inputs the MI355X step consumes besides the pixels: which samples form
each task's stream (SiBlurryStream, restating utils/online_sampler.py:9-249 OnlineSampler) and
which class list / label indices a batch trains against (ClassBook, restating
methods/_trainer.py:404-413 add_new_class and methods/adapter_clip.py:49-76, 263-283).

Same torch.Generator call sequence as the reference for a given seed, so the streams are
identical. Kept quirks: N% disjoint / M% blurry split rounded down to multiples of the task
count; blurred samples redistributed evenly with the remainder dropped (non-varying mode);
disjoint_class_num = classes per task of the WHOLE class list (online_sampler.py:60-62).
Deviation: the varying-N/M mode (rnd_NM) also defines disjoint_class_num (the
reference leaves it unset there and _trainer.py:320 fails); it counts the task's disjoint +
blurry classes, which is what the non-varying mode's value equals.

class_order: 'sequential' follows HEAD (torch.arange, online_sampler.py:57-58); 'random' is the
torch.randperm the reference's own logged run used (nohup.out:10 matches it for seed 0).
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch


class SiBlurryStream:
    def __init__(self, targets: Sequence[int], num_classes: int, num_tasks: int, m: int, n: int,
                 rnd_seed: int, varing_NM: bool = False, class_order: str = "sequential",
                 num_replicas: int = 1, rank: int = 0, cur_task: int = 0):
        if class_order not in ("sequential", "random"):
            raise ValueError("class_order must be 'sequential' or 'random'")
        if not (0 <= rank < num_replicas):
            raise ValueError("rank out of range")
        self.targets = torch.as_tensor(list(targets), dtype=torch.long)
        self.num_classes = int(num_classes)
        self.num_tasks = int(num_tasks)
        self.m, self.n = int(m), int(n)
        self.varing_NM = bool(varing_NM)
        self.num_replicas, self.rank = int(num_replicas), int(rank)
        self.generator = torch.Generator().manual_seed(rnd_seed)
        T = self.num_tasks
        C = self.num_classes

        disjoint_num = (C * self.n // 100) // T * T
        blurry_num = (C - disjoint_num) // T * T
        self.disjoint_num, self.blurry_num = disjoint_num, blurry_num
        g = self.generator

        if not self.varing_NM:
            if class_order == "random":
                order = torch.randperm(C, generator=g)
            else:
                order = torch.arange(C)
            if C % T:
                raise ValueError("the class list must split evenly over the tasks")
            self.disjoint_classes = order[:disjoint_num].reshape(T, -1).tolist()
            self.blurry_classes = order[disjoint_num:disjoint_num + blurry_num].reshape(T, -1).tolist()
            self.disjoint_class_num = [C // T] * T
            disj_idx, blur_idx, _ = self._split_indices()
            blurred = []
            for t in range(T):
                k = len(blur_idx[t]) * self.m // 100
                blurred += blur_idx[t][:k]
                blur_idx[t] = blur_idx[t][k:]
            blurred = torch.tensor(blurred, dtype=torch.long)
            blurred = blurred[torch.randperm(len(blurred), generator=g)].tolist()
            per = len(blurred) // T
            for t in range(T):
                blur_idx[t] += blurred[:per]
                blurred = blurred[per:]
        else:
            order = torch.randperm(C, generator=g)
            disj = order[:disjoint_num].tolist()
            if disjoint_num > 0:
                cut = [0] + torch.randint(0, disjoint_num, (T - 1,), generator=g).sort().values.tolist() + [disjoint_num]
                self.disjoint_classes = [disj[cut[t]:cut[t + 1]] for t in range(T)]
            else:
                self.disjoint_classes = [[] for _ in range(T)]
            if blurry_num > 0:
                cut = [0] + torch.randint(0, blurry_num, (T - 1,), generator=g).sort().values.tolist() + [blurry_num]
                self.blurry_classes = [order[disjoint_num + cut[t]:disjoint_num + cut[t + 1]].tolist()
                                       for t in range(T)]
            else:
                self.blurry_classes = [[] for _ in range(T)]
            self.disjoint_class_num = [len(self.disjoint_classes[t]) + len(self.blurry_classes[t])
                                       for t in range(T)]
            disj_idx, blur_idx, n_blur = self._split_indices()
            n_blur = n_blur * self.m // 100
            if n_blur > 0:
                cut = [0] + torch.randint(0, n_blur, (T - 1,), generator=g).sort().values.tolist() + [n_blur]
                blurred = []
                for t in range(T):
                    k = cut[t + 1] - cut[t]
                    blurred += blur_idx[t][:k]
                    blur_idx[t] = blur_idx[t][k:]
                blurred = torch.tensor(blurred, dtype=torch.long)
                blurred = blurred[torch.randperm(len(blurred), generator=g)].tolist()
                for t in range(T):
                    k = cut[t + 1] - cut[t]
                    blur_idx[t] += blurred[:k]
                    blurred = blurred[k:]

        self.disjoint_indices, self.blurry_indices = disj_idx, blur_idx
        self.indices = []
        for t in range(T):
            idx = torch.tensor(disj_idx[t] + blur_idx[t], dtype=torch.long)
            self.indices.append(idx[torch.randperm(len(idx), generator=g)].tolist())
        self.set_task(cur_task)

    def _split_indices(self):
        """Sample indices of each task's disjoint and blurry classes, in sample order."""
        T = self.num_tasks
        owner = torch.full((self.num_classes,), -1, dtype=torch.long)
        kind = torch.zeros(self.num_classes, dtype=torch.long)
        for t in range(T):
            for c in self.disjoint_classes[t]:
                owner[c], kind[c] = t, 0
            for c in self.blurry_classes[t]:
                owner[c], kind[c] = t, 1
        disj = [[] for _ in range(T)]
        blur = [[] for _ in range(T)]
        n_blur = 0
        for i, y in enumerate(self.targets.tolist()):
            t = int(owner[y])
            if t < 0:
                continue
            if kind[y] == 0:
                disj[t].append(i)
            else:
                blur[t].append(i)
                n_blur += 1
        return disj, blur, n_blur

    # ------------------------------------------------------------------ Sampler interface
    def set_task(self, task: int) -> None:
        if not (0 <= task < len(self.indices)):
            raise ValueError("task out of range")
        self.task = task
        self.num_samples = len(self.indices[task]) // self.num_replicas
        self.total_size = self.num_samples * self.num_replicas

    def task_indices(self, task: Optional[int] = None) -> List[int]:
        t = self.task if task is None else task
        n = len(self.indices[t]) // self.num_replicas
        return self.indices[t][self.rank:n * self.num_replicas:self.num_replicas]

    def __iter__(self):
        return iter(self.task_indices())

    def __len__(self) -> int:
        return self.num_samples


class ClassBook:
    """Exposed classes and the per-batch training class list (visible_classes = 'batch' | 'all').

    add_new_class(labels): every label not seen yet joins exposed_classes in first-seen order
    (_trainer.py:404-413); the batch list is exposed_classes itself when a memory buffer exists,
    else the batch's distinct labels in first-seen order (adapter_clip.py:263-283).
    train_classes() / remap(labels) give the logit columns and label indices of online_train
    (adapter_clip.py:52-76)."""

    def __init__(self, class_names: Sequence[str], memory_size: int = 0, visible: str = "batch"):
        if visible not in ("batch", "all"):
            raise ValueError("visible must be 'batch' or 'all'")
        self.class_names = list(class_names)
        self.memory_size = int(memory_size)
        self.visible = visible
        self.exposed_classes: List[int] = []
        self.batch_exposed_classes: List[int] = []

    @property
    def exposed_classes_names(self):
        return [self.class_names[i] for i in self.exposed_classes]

    def add_new_class(self, labels) -> None:
        ys = [int(v) for v in torch.as_tensor(labels).reshape(-1).tolist()]
        for y in ys:
            if y not in self.exposed_classes:
                self.exposed_classes.append(y)
        if self.memory_size > 0:
            self.batch_exposed_classes = self.exposed_classes
        else:
            self.batch_exposed_classes = []
            for y in ys:
                if y not in self.batch_exposed_classes:
                    self.batch_exposed_classes.append(y)

    def train_classes(self):
        ids = self.batch_exposed_classes if self.visible == "batch" else self.exposed_classes
        return list(ids), [self.class_names[i] for i in ids]

    def remap(self, labels) -> torch.Tensor:
        ids, _ = self.train_classes()
        pos = {c: i for i, c in enumerate(ids)}
        return torch.tensor([pos[int(v)] for v in torch.as_tensor(labels).reshape(-1).tolist()],
                            dtype=torch.long)
