"""Frozen-text-feature cache.

With a frozen text tower (peft_encoder 'image' / 'none', MVP-CLIP) the text features depend only
on the prompt token ids and the text weights, so they are computed once per token CONTENT
instead of every step (methods/adapter_clip.py:84 re-encodes them at every online_train call).

The cache keeps the token tensor itself, so its storage cannot be freed and reused by another
tensor that would then look identical by (data_ptr, _version). The same tensor object at the
same version is a hit without touching the device; any other tensor is compared by content (one
device compare and a host sync). The hit decision is thus a function of the token values and
the weights' versions only: under data parallelism every rank passes the same global prompt
list, so all ranks decide alike and issue the same collectives.
"""
from __future__ import annotations

import torch


class TokenFeatureCache:
    def __init__(self):
        self._entry = None  # (tokens, version, weights_key, features)

    def clear(self):
        self._entry = None

    def get(self, tokens, weights_key):
        e = self._entry
        if e is None:
            return None
        tok, ver, wkey, feats = e
        if wkey != weights_key:
            return None
        if tokens is tok and tokens._version == ver:
            return feats
        if tokens.shape != tok.shape or tokens.device != tok.device or tokens.dtype != tok.dtype:
            return None
        if tokens is tok:  # modified in place since: compare with what was encoded
            return None
        if not torch.equal(tokens, tok):
            return None
        # follow the caller's tensor (the next call with it is a device-free hit)
        self._entry = (tokens, tokens._version, wkey, feats)
        return feats

    def put(self, tokens, weights_key, feats):
        # a private copy: an in-place edit of the caller's tensor must not alias the key
        tok = tokens.clone()
        self._entry = (tok, tok._version, weights_key, feats)

    def __bool__(self):
        return self._entry is not None
