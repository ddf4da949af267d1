"""Generates tests/golden/clip_tokens_cifar100.json: the 77-wide token rows AdapterCLIP.labels_tokenize
(models/adapter_clip.py:41-74: template "a bad photo of a {}.", SOT/EOT, zero padding) produces
for the 100 CIFAR-100 class names, with this build's BPE tokenizer (lcclip/tokenizer.py) over the
reference's own merges file and class-name list (data files read here; neither ships).

    python tests/golden/make_token_golden.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "lifelong-clip_amd"))

BPE = "/root/reference/models/clip/bpe_simple_vocab_16e6.txt.gz"
NAMES = "/root/reference/datasets/gpt/gpt_data/classname/cifar100.txt"
TEMPLATE = "a bad photo of a {}."


def main():
    from lcclip.tokenizer import BPETokenizer
    t = BPETokenizer(BPE)
    names = [ln.strip() for ln in open(NAMES) if ln.strip()]
    rows = {}
    for n in names:
        ids = [t.sot] + t.encode(TEMPLATE.format(n)) + [t.eot]
        rows[n] = ids
    out = {"template": TEMPLATE, "context_length": 77, "sot": t.sot, "eot": t.eot,
           "source": "lcclip.tokenizer.BPETokenizer over the reference's bpe_simple_vocab_16e6.txt.gz "
                     "and datasets/gpt/gpt_data/classname/cifar100.txt",
           "ids": rows}
    path = os.path.join(ROOT, "tests", "golden", "clip_tokens_cifar100.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {len(rows)} class rows to {path}")


if __name__ == "__main__":
    main()
