"""Si-Blurry stream + class bookkeeping (lcclip/stream.py), CPU.

Pinned by the reference's own logged run (tests/golden/siblurry_cifar100_seed0.json, extracted
from nohup.out by tests/golden/make_stream_golden.py): CIFAR-100, 10 tasks, N = 100, M = 0,
seed 0, random class order -> the logged per-task class lists and 5000 samples per task.
The other cases check the stream's defining properties."""
import json
import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "lifelong-clip_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

from lcclip.stream import ClassBook, SiBlurryStream  # noqa: E402

GOLD = os.path.join(ROOT, "tests", "golden", "siblurry_cifar100_seed0.json")


def cifar_like_targets(num_classes=100, per_class=500, seed=5):
    """CIFAR-100's train split has 500 images per class (in a shuffled order)."""
    t = torch.arange(num_classes).repeat_interleave(per_class)
    return t[torch.randperm(len(t), generator=torch.Generator().manual_seed(seed))].tolist()


def test_matches_reference_logged_run():
    gold = json.load(open(GOLD))
    cfg = gold["config"]
    s = SiBlurryStream(cifar_like_targets(), 100, cfg["n_tasks"], cfg["m"], cfg["n"],
                       cfg["rnd_seed"], varing_NM=cfg["rnd_NM"], class_order="random")
    assert s.disjoint_classes == gold["disjoint_classes"]
    assert s.blurry_classes == gold["blurry_classes"]
    sizes = [[len(s.disjoint_indices[t]), len(s.blurry_indices[t])] for t in range(cfg["n_tasks"])]
    assert sizes == gold["task_sizes_disjoint_blurry"]
    assert s.disjoint_class_num == [10] * 10


def _check_partition(s, targets, T):
    seen = []
    for t in range(T):
        seen += s.indices[t]
    # every sample of an assigned class appears at most once; none is invented
    assert len(seen) == len(set(seen))
    assert set(seen) <= set(range(len(targets)))
    for t in range(T):
        for i in s.disjoint_indices[t]:
            assert targets[i] in s.disjoint_classes[t]


@pytest.mark.parametrize("n,m", [(50, 10), (0, 100), (100, 0), (70, 30)])
def test_sequential_blurry_properties(n, m):
    targets = cifar_like_targets(20, 30)
    T = 5
    s = SiBlurryStream(targets, 20, T, m, n, rnd_seed=3)
    _check_partition(s, targets, T)
    assert s.disjoint_num == 20 * n // 100 // T * T
    # disjoint classes are exclusive to their task's stream
    for t in range(T):
        cls_t = {targets[i] for i in s.indices[t]}
        for u in range(T):
            if u != t:
                assert not (set(s.disjoint_classes[u]) & cls_t)
    # the M% blurred samples moved: each task keeps (1 - M%) of its own blurry samples
    own_blurry = sum(len(s.blurry_indices[t]) for t in range(T))
    total_blurry = sum(1 for y in targets if any(y in b for b in s.blurry_classes))
    moved = total_blurry * 0 + sum(len(b) for b in s.blurry_classes)  # classes count, sanity
    assert own_blurry <= total_blurry and moved == s.blurry_num


def test_deterministic_and_seed_dependent():
    targets = cifar_like_targets(20, 30)
    a = SiBlurryStream(targets, 20, 4, 10, 50, rnd_seed=1)
    b = SiBlurryStream(targets, 20, 4, 10, 50, rnd_seed=1)
    c = SiBlurryStream(targets, 20, 4, 10, 50, rnd_seed=2)
    assert a.indices == b.indices
    assert a.indices != c.indices


@pytest.mark.parametrize("n,m", [(50, 10), (100, 0), (0, 50)])
def test_varying_nm_defines_class_counts(n, m):
    targets = cifar_like_targets(20, 30)
    T = 4
    s = SiBlurryStream(targets, 20, T, m, n, rnd_seed=7, varing_NM=True)
    _check_partition(s, targets, T)
    assert len(s.disjoint_class_num) == T
    assert sum(s.disjoint_class_num) == s.disjoint_num + s.blurry_num
    for t in range(T):
        assert s.disjoint_class_num[t] == len(s.disjoint_classes[t]) + len(s.blurry_classes[t])


def test_distributed_ranks_split_the_task():
    targets = cifar_like_targets(10, 21)
    full = SiBlurryStream(targets, 10, 2, 0, 100, rnd_seed=0)
    parts = [SiBlurryStream(targets, 10, 2, 0, 100, rnd_seed=0, num_replicas=3, rank=r) for r in range(3)]
    for t in range(2):
        for p in parts:
            p.set_task(t)
        got = [list(p) for p in parts]
        n = len(full.indices[t]) // 3
        assert all(len(g) == n == len(p) for g, p in zip(got, parts))
        merged = sorted(sum(got, []))
        assert merged == sorted(full.indices[t][:n * 3])
    with pytest.raises(ValueError):
        full.set_task(2)


def test_classbook_batch_and_all():
    names = [f"c{i}" for i in range(10)]
    cb = ClassBook(names, memory_size=0, visible="batch")
    cb.add_new_class(torch.tensor([7, 3, 7, 1]))
    assert cb.exposed_classes == [7, 3, 1]
    ids, nm = cb.train_classes()
    assert ids == [7, 3, 1] and nm == ["c7", "c3", "c1"]
    assert cb.remap(torch.tensor([7, 3, 7, 1])).tolist() == [0, 1, 0, 2]
    cb.add_new_class(torch.tensor([3, 5]))
    assert cb.exposed_classes == [7, 3, 1, 5]
    assert cb.train_classes()[0] == [3, 5]          # batch-visible: this batch's classes only
    assert cb.remap(torch.tensor([5, 3])).tolist() == [1, 0]
    ca = ClassBook(names, memory_size=0, visible="all")
    ca.add_new_class(torch.tensor([2, 4]))
    ca.add_new_class(torch.tensor([4, 9]))
    assert ca.train_classes()[0] == [2, 4, 9]
    assert ca.remap(torch.tensor([9, 2])).tolist() == [2, 0]
    cm = ClassBook(names, memory_size=100, visible="batch")
    cm.add_new_class(torch.tensor([1]))
    cm.add_new_class(torch.tensor([6]))
    assert cm.train_classes()[0] == [1, 6]          # with memory: every exposed class
