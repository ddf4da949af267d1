"""Generates tests/golden/clip_tokens_cifar100_hf.json: the CIFAR-100 prompt token ids produced by
an INDEPENDENT CLIP BPE implementation — Hugging Face transformers' CLIPTokenizer (slow, pure
Python; transformers 4.x/5.x as installed here) — over vocab/merges files derived from the
reference's own merges file (models/clip/bpe_simple_vocab_16e6.txt.gz) and class-name list
(datasets/gpt/gpt_data/classname/cifar100.txt). tests/test_eval_tokenizer.py pins the build's
tokenizer fixture (clip_tokens_cifar100.json, made by lcclip.tokenizer) against it, so the
class-name ids are no longer checked only against the build's own BPE.

The vocab / merges derivation restates CLIP's SimpleTokenizer construction (the reference's
models/clip/simple_tokenizer.py, read as text): merges = lines 1 .. 49152 - 256 - 2 of the file;
vocab = the 256 byte symbols, the same with '</w>', every merge's concatenation, then
'<|startoftext|>', '<|endoftext|>' (ids 49406, 49407).

    python tests/golden/make_token_golden_hf.py
"""
import gzip
import json
import os
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
BPE = "/root/reference/models/clip/bpe_simple_vocab_16e6.txt.gz"
NAMES = "/root/reference/datasets/gpt/gpt_data/classname/cifar100.txt"
TEMPLATE = "a bad photo of a {}."
EXTRA = ["it's 42 Golden retrievers!", "a photo of a maple_tree.", "Sweet pepper, lawn-mower"]


def byte_symbols():
    """GPT-2 / CLIP byte -> printable unicode table (the published bytes_to_unicode rule)."""
    keep = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + \
        list(range(ord("®"), ord("ÿ") + 1))
    cs = keep[:]
    n = 0
    for b in range(256):
        if b not in keep:
            keep.append(b)
            cs.append(256 + n)
            n += 1
    return [chr(c) for c in cs]  # in the order of `keep`, as the vocab lists them


def main():
    from transformers import CLIPTokenizer
    lines = gzip.open(BPE).read().decode("utf-8").split("\n")
    merges = [tuple(m.split()) for m in lines[1:49152 - 256 - 2 + 1]]
    syms = byte_symbols()
    vocab = syms + [s + "</w>" for s in syms] + ["".join(m) for m in merges]
    vocab += ["<|startoftext|>", "<|endoftext|>"]
    assert len(vocab) == 49408
    with tempfile.TemporaryDirectory() as d:
        vf, mf = os.path.join(d, "vocab.json"), os.path.join(d, "merges.txt")
        with open(vf, "w") as f:
            json.dump({t: i for i, t in enumerate(vocab)}, f)
        with open(mf, "w") as f:
            f.write("#version: 0.2\n" + "\n".join(" ".join(m) for m in merges) + "\n")
        tok = CLIPTokenizer(vf, mf)
        names = [ln.strip() for ln in open(NAMES) if ln.strip()]
        texts = [TEMPLATE.format(n) for n in names] + EXTRA
        ids = {t: tok(t)["input_ids"] for t in texts}
    out = {"template": TEMPLATE, "sot": 49406, "eot": 49407,
           "source": "transformers.CLIPTokenizer (slow) over vocab/merges derived from the "
                     "reference's bpe_simple_vocab_16e6.txt.gz; class names from "
                     "datasets/gpt/gpt_data/classname/cifar100.txt",
           "ids": ids}
    path = os.path.join(ROOT, "tests", "golden", "clip_tokens_cifar100_hf.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print(f"wrote {len(ids)} rows to {path}")


if __name__ == "__main__":
    main()
