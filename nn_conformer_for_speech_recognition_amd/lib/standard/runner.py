"""Runner — the reference's training / evaluation / pseudo-labelling driver (lib/standard/runner.py:17-282)
over the MI355X hot path.

Same constructor, methods and control flow as the reference; what runs underneath:

  loss         ctc.CTCLoss(blank=hp.blank_idx, zero_infinity=True)  (runner.py:35; libcfm CTC kernels)
  optimizer    optim.Adafactor(lr=hp.lr, beta1, scale_parameter, relative_step)  (runner.py:36; one
               multi-tensor HIP step)
  predict      ASRNN.predict -> cfm_ctc_greedy_decode (device argmax, torch.argmax tie rule)
  labels       generate_labels (runner.py:253-281): eval-mode forward (BatchNorm running stats, no
               dropout) -> device greedy decode with <pad>/<blank> stripped ON the device (no repeat
               collapse, the reference's Vocab.decode rule) -> only surviving ids go to the host.
               Under torch.distributed (world > 1) the batches are sharded round-robin over the ranks
               and the label lists are all-gathered back into batch order.
  WER          myvocab.wer (jiwer's sentence-list WER; jiwer is not in this image)

Dropped (outside the hot path): tqdm colours, Evals plots (losses / WER are kept on
the Runner as .history and written to hp.plots_dir/history.json), the language-model fusion.
"""
from __future__ import annotations

import json
import os
from functools import reduce
from math import ceil, isnan
from statistics import mean

import torch
import torch.nn as nn

from ...ctc import CTCLoss, greedy_decode
from ...optim import Adafactor
from .myvocab import wer


def _word_lists(target_strs, predicted_strs):
    """The reference's WER preparation (runner.py:151-160): drop empty targets, split predictions into
    words ('_' for empty), pad each target with '_' to its prediction's length, flatten both."""
    predicted = [predicted_strs[i] for i in range(min(len(target_strs), len(predicted_strs))) if target_strs[i] != ""]
    target = [x for x in target_strs if x != ""]
    predicted = [x.strip().split() if len(x.strip()) > 0 else ["_"] for x in predicted]
    target = [[x] for x in target]
    target = [target[i] + ["_"] * (len(predicted[i]) - len(target[i])) for i in range(len(predicted))]
    if not predicted:
        return [], []
    return reduce(lambda a, b: a + b, target), reduce(lambda a, b: a + b, predicted)


class Runner:
    def __init__(self, model, hp, lr=None, lm=False):
        self.model = model
        self.hp = hp
        self.lm = lm
        if lr is None:
            lr = hp.lr
        self.lr = lr
        self.model.to(hp.device)
        self.loss = CTCLoss(blank=hp.blank_idx, zero_infinity=True)
        # runner.py:36 builds the optimizer with hp.lr (its `lr` argument is unused there); same here
        self.optimizer = Adafactor(model.parameters(), lr=hp.lr, beta1=hp.beta1, scale_parameter=hp.scale_parameter,
                                   relative_step=hp.relative_step)
        self.history = {"loss": [], "metric": [], "val_loss": [], "val_metric": []}

    def set_model(self, model):
        self.__init__(model, self.hp)

    def save_model(self, finetuning=False):
        """runner.py:48-60."""
        path = self.hp.finetuning_model_path if finetuning else (
            self.hp.standard_model_path if not self.lm else self.hp.lm_model_path)
        torch.save(self.model.state_dict(), path)

    def load_model(self, model_path):
        """runner.py:61-77: keep the checkpoint's keys that exist in the model AND contain 'conformer';
        every other entry keeps the current model's value."""
        pretrained = torch.load(model_path, map_location="cpu", weights_only=True)
        self.model.cpu()
        cur = self.model.state_dict()
        keep = {k: v for k, v in pretrained.items() if k in cur and "conformer" in k}
        keep.update({k: v for k, v in cur.items() if k not in keep})
        self.model.load_state_dict(keep)
        self.model.to(self.hp.device)

    def fuse_models(self, lm_path):
        raise NotImplementedError("language-model fusion (runner.py:78-101) is outside the MI355X hot path")

    # ----------------------------------------------------------------------------- train / test
    def _metric(self, dataset, logits, target):
        predicted = self.model.predict(logits)
        t_strs = dataset.vocab.decode(target)
        p_strs = dataset.vocab.decode(predicted)
        tw, pw = _word_lists(t_strs, p_strs)
        return wer(tw, pw) * 100 if tw else 0.0

    def train(self, train_set, epochs, SpecAugment=False, use_mix=False, finetuning=False):
        """runner.py:102-182."""
        dataset_type = "mix" if use_mix else "train"
        train_size = ceil(len(train_set.idxes[dataset_type]) / self.hp.batch_size)
        want_wer = getattr(self.hp, "train_wer", True)     # WER forces a host sync per step
        for _ in range(epochs):
            self.model.train()
            train_set.shuffle(dataset_type)
            eloss, emetric = [], []
            for i in range(train_size):
                batch = train_set.get_batch(i, dataset_type)
                inbatch, input_lens = batch["input"]["mels"], batch["input"]["tau"]
                target, target_lens = batch["target"]["transcripts"], batch["target"]["lens"]
                self.optimizer.zero_grad()
                logits, output_lengths = self.model(inbatch, input_lens, SpecAugment, finetuning=finetuning)
                output_lengths = nn.functional.pad(output_lengths, (0, self.hp.batch_size - output_lengths.shape[0]))
                output_lengths = output_lengths.clamp(max=logits.shape[1])
                loss = self.loss(logits.transpose(0, 1), target, output_lengths, target_lens)
                cur = loss.item()
                loss.backward()
                self.optimizer.step()
                eloss.append(cur)
                if want_wer:
                    emetric.append(self._metric(train_set, logits.detach(), target))
            self._check_device_errors()
            self.history["loss"].append(mean([100 if isnan(x) else x for x in eloss]))
            self.history["metric"].append(mean(emetric) if emetric else float("nan"))
            if "validation" in train_set.idxes:
                vl, vm = self.test(train_set, "validation", finetuning=finetuning)
                self.history["val_loss"].append(vl)
                self.history["val_metric"].append(vm)
        self._write_history()
        if getattr(self.hp, "base_dir", None) is not None:
            self.save_model(finetuning)

    def test(self, test_set, dataset_type="test", heatmap=False, finetuning=False):
        """runner.py:183-252 -> (mean loss, mean WER %)."""
        self.model.eval()
        n = ceil(len(test_set.idxes[dataset_type]) / self.hp.batch_size)
        eloss, emetric = [], []
        with torch.no_grad():
            for i in range(n):
                batch = test_set.get_batch(i, dataset_type)
                inbatch, input_lens = batch["input"]["mels"], batch["input"]["tau"]
                target, target_lens = batch["target"]["transcripts"], batch["target"]["lens"]
                logits, output_lens = self.model(inbatch, input_lens, finetuning=finetuning)
                output_lens = nn.functional.pad(output_lens, (0, self.hp.batch_size - output_lens.shape[0]))
                output_lens = output_lens.clamp(max=logits.shape[1])
                loss = self.loss(logits.transpose(0, 1), target, output_lens, target_lens)
                eloss.append(loss.item())
                emetric.append(self._metric(test_set, logits, target))
        self._check_device_errors()
        eloss = mean([100 if isnan(x) else x for x in eloss])
        return eloss, mean(emetric)

    # ----------------------------------------------------------------------------- NST labels
    def generate_labels(self, dataset):
        """runner.py:253-281: pseudo-labels for every clip of dataset's 'pretrain' split, in order."""
        self.model.eval()
        n = ceil(len(dataset.idxes["pretrain"]) / self.hp.batch_size)
        voc = dataset.vocab
        world, rank = 1, 0
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            world, rank = torch.distributed.get_world_size(), torch.distributed.get_rank()
        mine = {}
        with torch.no_grad():
            for i in range(rank, n, world):
                batch = dataset.get_batch(i, "pretrain")["input"]
                logits, _ = self.model(batch["mels"], batch["tau"])
                # ASRNN.predict + Vocab.decode in one device pass: argmax, <pad>/<blank> removed, no collapse
                _, toks, cnt = greedy_decode(logits, None, blank=voc.blank_idx, pad=voc.pad_idx, collapse=False)
                mine[i] = voc.decode(toks, cnt)
        self._check_device_errors()
        if world > 1:
            parts = [None] * world
            torch.distributed.all_gather_object(parts, mine)
            for p in parts:
                mine.update(p)
        targets = []
        for i in range(n):
            targets += mine[i]
        return targets

    def _check_device_errors(self):
        """End-of-pass synchronising check of the BiLSTM recurrences' wait-limit flags: each forward only polls
        the flags of EARLIER passes (no host sync per launch), so a failure in the last pass of an epoch / test /
        label pass would otherwise go unreported."""
        from ...lstm import LSTM
        if any(isinstance(m, LSTM) for m in self.model.modules()):
            LSTM.check_errors()

    def _write_history(self):
        d = getattr(self.hp, "plots_dir", None)
        if d:
            with open(os.path.join(d, "history.json"), "w") as f:
                json.dump(self.history, f)
