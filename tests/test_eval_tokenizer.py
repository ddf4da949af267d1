"""SURVEY §8(f) f4 on the CPU: the evaluation bookkeeping (interpret_pred with the reference's
10-bucket table, the confusion matrix, the summary metrics) against direct restatements of
methods/_trainer.py:367-378, 519-534 and sklearn; the BPE tokenizer's structural pins (vocab
layout, special ids, ids of the byte symbols derived from the byte table, round trip). The
tokenizer tests need the merges file: /root/reference's copy when present (skipped otherwise —
it is data the build does not ship)."""
import math
import os

import numpy as np
import pytest
import torch

from lcclip import evaluate as ev

BPE = "/root/reference/models/clip/bpe_simple_vocab_16e6.txt.gz"


def interpret_ref(y, pred, n_tasks):
    """_trainer.py:519-534, loop for loop."""
    num, corr = torch.zeros(10), torch.zeros(10)
    cls = y // n_tasks
    for c, n in zip(*cls.unique(return_counts=True)):
        num[c] = n
    ok = y.masked_select(y == pred) // n_tasks
    for c, n in zip(*ok.unique(return_counts=True)):
        corr[c] = n
    return num, corr


def test_interpret_pred_matches_reference_loop():
    g = torch.Generator().manual_seed(0)
    for n_tasks in (10, 20):
        y = torch.randint(0, 100, (257,), generator=g)
        pred = torch.where(torch.rand(257, generator=g) < 0.6, y,
                           torch.randint(0, 100, (257,), generator=g))
        a = ev.interpret_pred(y, pred, n_tasks)
        b = interpret_ref(y, pred, n_tasks)
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])


def test_interpret_pred_bucket_quirk():
    y = torch.tensor([0, 199])
    with pytest.raises(IndexError):       # 200 classes / 5 tasks: bucket 39 >= 10
        ev.interpret_pred(y, y, 5)
    num, corr = ev.interpret_pred(y, y, 5, n_buckets=None)
    assert num.numel() == 40 and num[39] == 1 and corr.sum() == 2


def test_confusion_matrix_matches_sklearn():
    from sklearn.metrics import confusion_matrix
    rng = np.random.default_rng(1)
    y = rng.integers(0, 7, 500)
    p = np.where(rng.random(500) < 0.5, y, rng.integers(2, 9, 500))
    assert np.array_equal(ev.confusion_matrix(y, p), confusion_matrix(y, p))


def test_summarize_matches_trainer_formulas():
    rec = {"task_acc": [0.9, 0.8, 0.7],
           "cls_acc": [[0.9, 0.0, 0.0], [0.85, 0.75, 0.0], [0.6, 0.7, 0.8]]}
    s = ev.summarize(rec, {"test_acc": [0.5, 0.7, 0.9]}, 3)
    assert math.isclose(s["A_auc"], 0.7) and math.isclose(s["A_avg"], 0.8)
    assert math.isclose(s["A_last"], 0.7)
    assert math.isclose(s["F_last"], ((0.9 - 0.6) + (0.75 - 0.7)) / 2)  # bucket 2 never > 0
    assert math.isnan(ev.summarize(rec, {}, 3)["A_auc"])  # the reference's empty eval_results


def test_auc_tracker_periods():
    t = ev.AUCTracker(100)
    seen = 0
    for step in range(1, 31):
        seen += 16
        if t.due(seen):
            t.record(seen, step / 30)
    assert t.data_cnt == [112, 208, 304, 400]
    assert t.results()["test_acc"] == [7 / 30, 13 / 30, 19 / 30, 25 / 30]


@pytest.mark.skipif(not os.path.isfile(BPE), reason="BPE merges file not available")
def test_tokenizer_structure():
    from lcclip.tokenizer import BPETokenizer, byte_table
    t = BPETokenizer(BPE)
    assert t.vocab_size == 49408 and (t.sot, t.eot) == (49406, 49407)
    # a single printable byte b is symbol index (b - 33) among the 188 kept bytes, and the
    # word-final form is 256 further: 'a' -> 256 + 64 = 320
    assert t.encode("a") == [256 + ord("a") - ord("!")]
    assert byte_table()[32] == chr(256 + 32)  # space is a moved byte (the 33rd: 0..32)
    for s in ["a bad photo of a cat.", "it's 42 Golden retrievers!", "ünïcödé 日本"]:
        ids = t.encode(s)
        assert all(0 <= i < 49406 for i in ids)
        assert "".join(t.decode(ids).split()) == "".join(t.clean(s).split())
    # every merge id decodes to the concatenation of its two parts
    assert t.decoder[t.encoder["a</w>"]] == "a</w>"


@pytest.mark.skipif(not os.path.isfile(BPE), reason="BPE merges file not available")
def test_labels_tokenize_with_bpe():
    from lcclip import AdapterCLIP
    from lcclip.tokenizer import BPETokenizer
    from tests.test_surface import TINY_ARCH
    m = AdapterCLIP("tiny", peft_method="adapter", peft_encoder="both", arch_overrides=TINY_ARCH,
                    tokenizer=BPETokenizer(BPE))
    tok = m.labels_tokenize(["cat", "golden retriever"])
    assert tok.shape == (2, 77) and (tok[:, 0] == 49406).all()
    assert (tok.argmax(1) == torch.tensor([8, 9])).all()  # SOT + 6 template ids + name + '.'


TOKEN_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                            "clip_tokens_cifar100.json")


def _token_golden():
    import json
    with open(TOKEN_GOLDEN) as f:
        return json.load(f)


def test_token_fixture_known_ids():
    """Runs without /root/reference: the committed CIFAR-100 prompt rows carry the public CLIP
    ids of the template words ("a"=320, "bad"=2103, "photo"=1125, "of"=539, "."=269, SOT 49406,
    EOT 49407), every row fits 77 tokens, and the class-name part differs between classes."""
    d = _token_golden()
    rows = d["ids"]
    assert len(rows) == 100 and d["template"] == "a bad photo of a {}."
    for name, ids in rows.items():
        assert ids[:6] == [49406, 320, 2103, 1125, 539, 320], name
        assert ids[-2:] == [269, 49407], name
        assert len(ids) <= 77 and all(0 <= i < 49406 for i in ids[1:-1])
    assert len({tuple(v[6:-2]) for v in rows.values()}) == 100


def test_labels_tokenize_matches_fixture_rows():
    """AdapterCLIP.labels_tokenize (models/adapter_clip.py:43-74: SOT + ids + EOT, zero padded to
    77) over a tokenizer that replays the fixture's ids: the wrapper's row layout, no BPE file."""
    from lcclip import AdapterCLIP
    from tests.test_surface import TINY_ARCH
    d = _token_golden()
    table = {d["template"].format(n): ids[1:-1] for n, ids in d["ids"].items()}
    m = AdapterCLIP("tiny", peft_method="adapter", peft_encoder="both", arch_overrides=TINY_ARCH,
                    tokenizer=lambda text: table[text])
    names = ["apple", "aquarium_fish", "wolf"]
    tok = m.labels_tokenize(names)
    assert tok.shape == (3, 77) and tok.dtype == torch.int64
    for i, n in enumerate(names):
        ids = d["ids"][n]
        assert tok[i, :len(ids)].tolist() == ids and (tok[i, len(ids):] == 0).all()


@pytest.mark.skipif(not os.path.isfile(BPE), reason="BPE merges file not available")
def test_tokenizer_reproduces_token_fixture():
    from lcclip.tokenizer import BPETokenizer
    t = BPETokenizer(BPE)
    d = _token_golden()
    for name, ids in d["ids"].items():
        assert [t.sot] + t.encode(d["template"].format(name)) + [t.eot] == ids, name


TOKEN_GOLDEN_HF = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden",
                               "clip_tokens_cifar100_hf.json")


def test_token_fixture_matches_independent_tokenizer():
    """Runs without /root/reference: every CIFAR-100 prompt row of the build's fixture equals the
    ids of an independent CLIP BPE implementation (transformers' CLIPTokenizer over the same
    merges file, tests/golden/make_token_golden_hf.py), so the class-name ids are pinned by more
    than the build's own tokenizer."""
    import json
    d = _token_golden()
    with open(TOKEN_GOLDEN_HF) as f:
        hf = json.load(f)["ids"]
    for name, ids in d["ids"].items():
        assert hf[d["template"].format(name)] == ids, name


@pytest.mark.skipif(not os.path.isfile(BPE), reason="BPE merges file not available")
def test_tokenizer_matches_independent_tokenizer_free_text():
    """Free text (punctuation, digits, case, underscores, contractions) through lcclip's BPE vs the
    independent implementation's committed ids."""
    import json
    from lcclip.tokenizer import BPETokenizer
    t = BPETokenizer(BPE)
    with open(TOKEN_GOLDEN_HF) as f:
        hf = json.load(f)["ids"]
    for text, ids in hf.items():
        assert [t.sot] + t.encode(text) + [t.eot] == ids, text
