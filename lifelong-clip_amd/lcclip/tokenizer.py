"""CLIP byte-level BPE tokenizer (the scheme models/clip/tokenizer.py:62-139 implements),
written for this build: text -> token ids without SOT/EOT, as AdapterCLIP / CLIP_MVP / MaPLe take
through their `tokenizer=` argument.

Vocabulary layout (49 408 ids): the 256 byte symbols in byte-table order, the same 256 with the
end-of-word marker '</w>', the 48 894 merges of the BPE file in rank order, then
'<start_of_text>' (49406) and '<end_of_text>' (49407). The merges file (OpenAI's
bpe_simple_vocab_16e6.txt.gz) is data, not shipped here: pass its path or set LCCLIP_BPE_PATH.

Cleaning: HTML entities unescaped (twice), whitespace collapsed, lower-cased. The reference also
runs ftfy.fix_text (not installed in this image); it only changes mis-decoded Unicode, so class
names in plain text tokenize identically.
"""
from __future__ import annotations

import gzip
import html
import os
from functools import lru_cache

import regex

SOT, EOT = "<start_of_text>", "<end_of_text>"
N_MERGES = 49152 - 256 - 2
# contractions | letter runs | single digits | runs of other non-space characters
_SPLIT = regex.compile(r"<start_of_text>|<end_of_text>|'s|'t|'re|'ve|'m|'ll|'d|[\p{L}]+|[\p{N}]"
                       r"|[^\s\p{L}\p{N}]+", regex.IGNORECASE)


@lru_cache(maxsize=1)
def byte_table():
    """byte -> printable unicode symbol: bytes that are printable Latin-1 keep their own code
    point, the other 68 are moved to 256, 257, ... in byte order."""
    keep = set(range(ord("!"), ord("~") + 1)) | set(range(ord("¡"), ord("¬") + 1)) | \
        set(range(ord("®"), ord("ÿ") + 1))
    table, extra = {}, 0
    for b in range(256):
        if b in keep:
            table[b] = chr(b)
        else:
            table[b] = chr(256 + extra)
            extra += 1
    return table


def _byte_symbols():
    """The 256 byte symbols in vocabulary order: printable ones first (by byte), then the moved."""
    t = byte_table()
    return [t[b] for b in range(256) if ord(t[b]) < 256] + \
        [t[b] for b in range(256) if ord(t[b]) >= 256]


class BPETokenizer:
    def __init__(self, bpe_path: str | None = None):
        bpe_path = bpe_path or os.environ.get("LCCLIP_BPE_PATH")
        if not bpe_path or not os.path.isfile(bpe_path):
            raise FileNotFoundError("CLIP BPE merges file not found: pass bpe_path or set "
                                    "LCCLIP_BPE_PATH (bpe_simple_vocab_16e6.txt.gz)")
        with gzip.open(bpe_path, "rt", encoding="utf-8") as f:
            lines = f.read().split("\n")
        merges = [tuple(ln.split()) for ln in lines[1:1 + N_MERGES]]
        syms = _byte_symbols()
        vocab = syms + [s + "</w>" for s in syms] + [a + b for a, b in merges] + [SOT, EOT]
        self.encoder = {tok: i for i, tok in enumerate(vocab)}
        self.decoder = vocab
        self.rank = {m: r for r, m in enumerate(merges)}
        self.bytes = byte_table()
        self.unbytes = {c: b for b, c in self.bytes.items()}
        self.sot, self.eot = self.encoder[SOT], self.encoder[EOT]
        self.vocab_size = len(vocab)
        self._memo = {SOT: [SOT], EOT: [EOT]}

    @staticmethod
    def clean(text: str) -> str:
        text = html.unescape(html.unescape(text)).strip()
        return " ".join(text.split()).lower()

    def _merge_word(self, word: str):
        """Greedy BPE: repeatedly fuse every occurrence of the lowest-ranked adjacent pair."""
        got = self._memo.get(word)
        if got is not None:
            return got
        parts = list(word[:-1]) + [word[-1] + "</w>"]
        while len(parts) > 1:
            best, best_rank = None, None
            for pair in zip(parts, parts[1:]):
                r = self.rank.get(pair)
                if r is not None and (best_rank is None or r < best_rank):
                    best, best_rank = pair, r
            if best is None:
                break
            fused, i = [], 0
            while i < len(parts):
                if i + 1 < len(parts) and (parts[i], parts[i + 1]) == best:
                    fused.append(parts[i] + parts[i + 1])
                    i += 2
                else:
                    fused.append(parts[i])
                    i += 1
            parts = fused
        self._memo[word] = parts
        return parts

    def encode(self, text: str):
        ids = []
        for piece in _SPLIT.findall(self.clean(text)):
            word = "".join(self.bytes[b] for b in piece.encode("utf-8"))
            ids.extend(self.encoder[p] for p in self._merge_word(word))
        return ids

    __call__ = encode

    def decode(self, ids):
        raw = bytearray()
        for i in ids:
            tok = self.decoder[i]
            if tok in (SOT, EOT):
                raw += tok.encode("utf-8")
                continue
            end = tok.endswith("</w>")
            raw += bytes(self.unbytes[c] for c in (tok[:-4] if end else tok))
            if end:
                raw += b" "
        return raw.decode("utf-8", errors="replace")
