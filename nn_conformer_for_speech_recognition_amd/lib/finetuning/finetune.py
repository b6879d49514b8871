"""FineTune — noisy-student training (lib/finetuning/finetune.py:6-35) over the MI355X Runner.

fine_tuning(model, S, U): train on the labelled set S with SpecAugment, then for hp.ft_epochs rounds
(if hp.nst) pseudo-label the unlabelled set U with the current model (Runner.generate_labels: device
forward + greedy decode), mix the labels into S (S.mix_datasets) and train on the mix.
"""
from __future__ import annotations

from ..standard.runner import Runner


class FineTune:
    def __init__(self, hp):
        self.hp = hp

    def fine_tuning(self, model, S, U):
        runner = Runner(model, self.hp, lr=self.hp.ft_lr)
        runner.train(S, self.hp.ft_train_epochs, SpecAugment=True, finetuning=True)
        for _ in range(self.hp.ft_epochs):
            if self.hp.nst:
                labels = runner.generate_labels(U)
                S.mix_datasets(U, labels)
            runner.train(S, self.hp.ft_train_epochs, SpecAugment=True, use_mix=self.hp.nst, finetuning=True)
        return runner
