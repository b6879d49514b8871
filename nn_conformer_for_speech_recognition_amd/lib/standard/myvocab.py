"""Vocab — the reference's word vocabulary surface (lib/standard/myvocab.py) without torchtext.

The reference builds a torchtext ``vocab`` (absent from this image) and uses three of its
behaviours on the hot path's boundary:

  parse(sentence)   whitespace split, token -> id                           (myvocab.py:199-210)
  decode(batch)     ids (B, T) -> one string per row: tokens looked up, <pad> and <blank> dropped,
                    NO repeat collapse, joined by single spaces              (myvocab.py:211-231)
  pad / blank ids   the dataset's HParams setters (speechcommands.py:39-46)

Here the vocabulary is a plain token list (index = id).  ``decode`` accepts the reference's input (an
id tensor, e.g. ASRNN.predict's argmax) and, as a fast path, the compact device output of
``ctc.greedy_decode`` (pad/blank already removed on the GPU, rows padded with -1 plus lengths), so a
pseudo-label pass moves only the surviving ids to the host.
"""
from __future__ import annotations

import torch


class Vocab:
    def __init__(self, tokens, pad_token="<pad>", blank_token="<blank>", unk_token="<unk>"):
        self.itos = list(tokens)
        for t in (pad_token, blank_token):
            if t not in self.itos:
                raise ValueError(f"vocabulary lacks the special token {t!r}")
        self.stoi = {t: i for i, t in enumerate(self.itos)}
        if len(self.stoi) != len(self.itos):
            raise ValueError("duplicate tokens in the vocabulary")
        self.pad_token, self.blank_token, self.unk_token = pad_token, blank_token, unk_token
        self.pad_idx = self.stoi[pad_token]
        self.blank_idx = self.stoi[blank_token]

    @classmethod
    def from_file(cls, path, ntokens=None, **kw):
        """myVocab.read_vocab (myvocab.py:163-176): one token per line in id order (the file save_vocab
        writes), the first `ntokens` kept."""
        with open(path, "r", encoding="utf-8") as f:
            toks = f.read().split("\n")
        return cls(toks[:ntokens], **kw)

    def __len__(self):
        return len(self.itos)

    def lookup_tokens(self, ids):
        return [self.itos[i] for i in ids]

    def parse(self, sentence):
        """myvocab.py:199-210: whitespace-split words -> ids (unknown words -> <unk> if present)."""
        unk = self.stoi.get(self.unk_token)
        out = []
        for w in sentence.strip().split():
            if w in self.stoi:
                out.append(self.stoi[w])
            elif unk is not None:
                out.append(unk)
            else:
                raise KeyError(f"word {w!r} not in the vocabulary")
        return out

    def decode(self, batch, lengths=None):
        """myvocab.py:211-231.  batch: (B, T) ids (tensor / nested lists) -> list of B strings with
        <pad>/<blank> tokens removed (no repeat collapse).  With `lengths` the rows are the compact
        device output of ctc.greedy_decode (ids already filtered; entries >= lengths[b] ignored)."""
        if torch.is_tensor(batch):
            batch = batch.cpu().tolist()
        if lengths is not None:
            lengths = lengths.cpu().tolist() if torch.is_tensor(lengths) else list(lengths)
            return [" ".join(self.itos[i] for i in row[:n]) for row, n in zip(batch, lengths)]
        drop = {self.pad_idx, self.blank_idx}
        return [" ".join(self.itos[i] for i in row if i not in drop) for row in batch]


def wer(reference, hypothesis):
    """jiwer.wer (runner.py:160,230) for lists of sentences: total word-level edit distance over the
    total number of reference words.  Inputs: a string or a list of strings (one sentence each)."""
    if isinstance(reference, str):
        reference = [reference]
    if isinstance(hypothesis, str):
        hypothesis = [hypothesis]
    if len(reference) != len(hypothesis):
        raise ValueError("reference and hypothesis must hold the same number of sentences")
    errors = words = 0
    for r, h in zip(reference, hypothesis):
        rw, hw = r.split(), h.split()
        words += len(rw)
        prev = list(range(len(hw) + 1))
        for i, a in enumerate(rw, 1):
            cur = [i] + [0] * len(hw)
            for j, b in enumerate(hw, 1):
                cur[j] = min(prev[j] + 1, cur[j - 1] + 1, prev[j - 1] + (a != b))
            prev = cur
        errors += prev[-1]
    if words == 0:
        raise ValueError("reference has no words")
    return errors / words


def build_vocab(sentences, ntokens=None, tokens=None):
    """myVocab.build_vocab (myvocab.py:61-96) without torchtext: words by descending frequency (ties in
    first-seen order, as Counter + a stable sort), the first `ntokens` kept, then <unk>, <pad>, <blank>
    each inserted at index 0 -> ids 0 = <blank>, 1 = <pad>, 2 = <unk>, words from 3."""
    from collections import Counter
    words = [w for s in sentences for w in s.strip().split()]
    if tokens is not None:
        words = [w for w in words if w in tokens]
    ranked = sorted(Counter(words).items(), key=lambda kv: kv[1], reverse=True)
    if ntokens is not None:
        ranked = ranked[:ntokens]
    itos = [w for w, _ in ranked]
    for special in ("<unk>", "<pad>", "<blank>"):
        if special not in itos:
            itos.insert(0, special)
    return Vocab(itos)


myVocab = Vocab   # the reference's class name (its constructor reads/writes vocab files; build_vocab here)
