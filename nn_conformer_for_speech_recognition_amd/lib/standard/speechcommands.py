"""MelDataset — the batch / shuffle / mix surface of the reference's SpeechCommands dataset
(lib/standard/speechcommands.py:150-226) over in-memory log-mel clips.

The reference reads Speech Commands wav files with librosa (absent here, and no network for the
data): the log-mels come from the caller — e.g. ``melspec.LogMel`` (the on-GPU log-mel front-end) or
synthetic arrays.  What the Runner's hot path depends on is kept:

  data[type] / idxes[type]          'train', 'validation', 'test', 'pretrain' (unlabelled U), 'mix'
  get_batch(i, type)                the reference's batch dict: input.mels (B, F, max_len) padded
                                    with zeros up to hp.batch_size rows, input.tau, target.transcripts
                                    (B, max_target_len), target.lens, unpadded_len  (:176-198)
  shuffle(type)                     python random, in place (:156-165)
  mix_datasets(U, targets)          NST: labelled train set + U with generated labels (empty label ->
                                    [0]), dropping labels longer than max_target_len (:211-226)
"""
from __future__ import annotations

import copy
from random import shuffle as _shuffle

import numpy as np
import torch


class MelDataset:
    def __init__(self, hp, vocab, splits):
        """splits: {type: [(mel (F, tau) array, transcript str or None), ...]}."""
        self.hp = hp
        self.vocab = vocab
        self.data, self.idxes = {}, {}
        self.max_len = 0
        self.max_target_len = 0
        for kind, items in splits.items():
            rows = []
            for mel, text in items:
                mel = np.asarray(mel, dtype=np.float32)
                tgt = vocab.parse(text) if text else [0]
                rows.append({"input": {"mels": mel.tolist(), "tau": int(mel.shape[1])},
                             "target": {"transcripts": tgt, "lens": len(tgt) if text else 0}})
                self.max_len = max(self.max_len, mel.shape[1])
                self.max_target_len = max(self.max_target_len, len(tgt))
            self.data[kind] = rows
            self.idxes[kind] = list(range(len(rows)))
        first = next(iter(splits.values()))
        n_mels = np.asarray(first[0][0]).shape[0] if first else hp.n_mels
        hp.set_max_len(self.max_len)
        hp.set_target_max_len(self.max_target_len)
        hp.set_input_dim(n_mels, self.max_len)
        hp.set_vocab_len(len(vocab))
        hp.set_ntokens(len(vocab))
        hp.set_blank_index(vocab.blank_idx)
        for kind in self.data:
            for r in self.data[kind]:
                t = r["target"]["transcripts"]
                r["target"]["transcripts"] = t + [vocab.pad_idx] * (self.max_target_len - len(t))

    def shuffle(self, dataset_type="train"):
        _shuffle(self.data[dataset_type])

    def get_item(self, i, dataset_type="train"):
        return self.data[dataset_type][i]

    @staticmethod
    def padding(rows, left, shape):
        return rows + [np.zeros(shape, dtype=np.float32)] * left

    def get_batch(self, i, dataset_type="train"):
        B = self.hp.batch_size
        rows = self.data[dataset_type][i * B:(i + 1) * B]
        F = self.hp.input_rows
        mels = []
        for r in rows:
            m = np.asarray(r["input"]["mels"], dtype=np.float32)
            mels.append(np.pad(m, ((0, 0), (0, self.max_len - m.shape[1]))))
        mels = self.padding(mels, B - len(rows), (F, self.max_len))
        tau = [r["input"]["tau"] for r in rows] + [0] * (B - len(rows))
        tr = [r["target"]["transcripts"] for r in rows] + [[0] * self.max_target_len] * (B - len(rows))
        tl = [r["target"]["lens"] for r in rows] + [0] * (B - len(rows))
        dev = self.hp.device
        return {"input": {"mels": torch.from_numpy(np.stack(mels)).to(dev), "tau": torch.LongTensor(tau).to(dev)},
                "target": {"transcripts": torch.LongTensor(tr).to(dev), "lens": torch.LongTensor(tl).to(dev)},
                "unpadded_len": len(rows)}

    def mix_datasets(self, U, targets):
        """speechcommands.py:211-226: train + U's clips with the generated labels."""
        enc = [self.vocab.parse(t) if len(t) > 0 else [0] for t in targets]
        n = min(len(U.data["pretrain"]), len(enc))
        u = []
        for i in range(n):
            if len(enc[i]) > self.max_target_len:
                continue
            t = enc[i] + [self.vocab.pad_idx] * (self.max_target_len - len(enc[i]))
            u.append({"input": {"mels": U.data["pretrain"][i]["input"]["mels"],
                                "tau": U.data["pretrain"][i]["input"]["tau"]},
                      "target": {"transcripts": t, "lens": len(enc[i])}})
        self.data["mix"] = copy.deepcopy(self.data["train"]) + u
        self.idxes["mix"] = self.idxes["train"] + list(range(len(u)))
        _shuffle(self.data["mix"])
