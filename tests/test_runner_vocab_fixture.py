"""The Runner / vocabulary surface pinned to the reference itself.

tests/golden/runner_vocab.json was produced by tests/golden/make_golden.py::gen_runner_vocab, which imports
the reference's lib/standard/myvocab.py and lib/standard/runner.py (recording stubs for jiwer / tqdm /
colorama, torchtext's published vocab semantics, a stub model returning fixed logits) and records:
  * the vocabulary read from the reference's shipped vocabs/myvocab.txt (myvocab.py:163-176) and one built
    from sentences (myvocab.py:61-96), parse() of two sentences (myvocab.py:199-210);
  * myVocab.decode on fixed id rows (myvocab.py:211-231: <pad>/<blank> dropped, no repeat collapse);
  * the (target, predicted) word lists Runner.train / Runner.test hand to jiwer.wer (runner.py:149-160,
    :219-230) for two training batches and one validation batch;
  * Runner.generate_labels' strings for two pretrain batches (runner.py:253-281).
CPU tests check the host logic (lib/standard/runner.py::_word_lists, Vocab.decode / parse / build_vocab);
the -m gpu test drives this build's Runner.train / test / generate_labels (device argmax / greedy decode,
libcfm CTC, Adafactor) on the same stub model and compares what reaches its WER and its labels."""
import json
import os

import pytest
import torch

from nn_conformer_for_speech_recognition_amd.lib.standard import runner as runner_mod
from nn_conformer_for_speech_recognition_amd.lib.standard.myvocab import Vocab, build_vocab
from nn_conformer_for_speech_recognition_amd.lib.standard.runner import _word_lists

FX = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "runner_vocab.json")


@pytest.fixture(scope="module")
def fx():
    with open(FX) as f:
        return json.load(f)


def _tensors(fx):
    return (torch.tensor(fx["logits"], dtype=torch.float32), torch.tensor(fx["out_lens"]),
            torch.tensor(fx["targets"]), torch.tensor(fx["target_lens"]))


def test_vocab_read_decode_parse_build(fx, tmp_path):
    p = tmp_path / "myvocab.txt"
    p.write_text("\n".join(fx["itos"]), encoding="utf-8")          # the format save_vocab writes
    v = Vocab.from_file(str(p))
    assert v.itos == fx["itos"]
    assert v.decode(torch.tensor(fx["decode_rows"])) == fx["decoded"]
    assert [v.parse(s) for s in ["yes no", "up unknownword down"]] == fx["parsed"]
    assert build_vocab(fx["built_from"]).itos == fx["built_itos"]


def test_wer_word_lists_match_reference(fx):
    v = Vocab(fx["itos"])
    logits, _, tgts, _ = _tensors(fx)
    got = []
    for k, j in ((0, 0), (1, 1), (2, 2)):            # train batch 0, train batch 1, validation
        pred = torch.argmax(torch.log_softmax(logits[k], -1), dim=-1)
        got.append(list(_word_lists(v.decode(tgts[j]), v.decode(pred))))
    assert got == fx["wer_calls"]


def test_generate_labels_rule_matches_reference(fx):
    v = Vocab(fx["itos"])
    logits = _tensors(fx)[0]
    labels = []
    for k in (3, 4):
        labels += v.decode(torch.argmax(logits[k], dim=-1))
    assert labels == fx["labels"]


class _StubModel(torch.nn.Module):
    """Returns the fixture's fixed logits (the reference run used the same), predicts on the device with the
    build's greedy decode (ASRNN.predict's path)."""

    def __init__(self, logits, out_lens):
        super().__init__()
        self.w = torch.nn.Parameter(torch.zeros(1))
        self.logits, self.out_lens = logits, out_lens

    def forward(self, x, input_lens, SpecAugment=False, lm=None, finetuning=False):
        k = int(x.reshape(-1)[0].item())
        return torch.log_softmax(self.logits[k].to(self.w.device) + self.w, -1), self.out_lens.to(self.w.device)

    def predict(self, lg):
        from nn_conformer_for_speech_recognition_amd.lib.standard.asrnn import ASRNN
        return ASRNN.predict(self, lg)


@pytest.mark.gpu
def test_runner_on_gpu_matches_reference(fx, tmp_path, monkeypatch):
    from nn_conformer_for_speech_recognition_amd.lib.hparams import HParams
    v = Vocab(fx["itos"])
    logits, out_lens, tgts, tlens = _tensors(fx)
    B, T = fx["batch"], fx["T"]
    hp = HParams(None)
    hp.device = torch.device("cuda")
    hp.batch_size = B
    hp.set_blank_index(v.blank_idx)
    hp.plots_dir = str(tmp_path)

    class Data:
        idxes = {"train": list(range(8)), "validation": list(range(4)), "pretrain": list(range(8))}
        vocab = v

        def shuffle(self, kind):
            pass

        def get_batch(self, i, kind):
            k = {"train": i, "validation": 2, "pretrain": 3 + i}[kind]
            j = min(k, 2)
            return {"input": {"mels": torch.full((B, 1, 4, 4), float(k), device="cuda"),
                              "tau": torch.full((B,), T, device="cuda")},
                    "target": {"transcripts": tgts[j].cuda(), "lens": tlens[j].cuda()}, "unpadded_len": B}

    calls = []

    def rec(t, p):
        calls.append((list(t), list(p)))
        return 0.25
    monkeypatch.setattr(runner_mod, "wer", rec)
    r = runner_mod.Runner(_StubModel(logits, out_lens).cuda(), hp)
    r.train(Data(), 1)
    assert [list(c) for c in calls] == fx["wer_calls"]
    assert r.generate_labels(Data()) == fx["labels"]
