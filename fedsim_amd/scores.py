"""Stateful scores used as the local criterion and as round metrics
(reference: fedsim/scores.py:10-346).  Outside the accelerated path; restated
with the reference's arithmetic so that local training and the round reports
come out bit-identical: each loss is taken with ``reduction="sum"`` and the
batch value returned is ``sum / batch`` (a tensor divide), micro = as if the
batches were concatenated, macro = mean of per-batch values."""
from __future__ import annotations

import torch


class Score(object):
    """Base class (scores.py:10-94)."""

    def __init__(self, log_freq: int = 1, split="test", score_name="", reduction="micro"):
        if log_freq < 1:
            raise Exception(f"invalid log_freq ({log_freq}) given to {score_name}")
        self.log_freq = log_freq
        self.split = split
        self.score_name = score_name
        self.reduction = reduction
        self._sum = 0
        self._weight = 0

    def get_name(self) -> str:
        return self.score_name

    def __call__(self, input, target):
        raise NotImplementedError

    def _update(self, cur_sum, n):
        if self.reduction == "micro":
            self._sum += cur_sum.item()
            self._weight += n
        elif self.reduction == "macro":
            self._sum += cur_sum.item() / n
            self._weight += 1
        return cur_sum / n

    @staticmethod
    def _check(input, target):
        if not (target.shape[0] == input.shape[0]):
            raise Exception(f"size mismatch between input {input.shape[0]} and{target.shape[0]}")

    def get_score(self) -> float:
        if self._weight < 1:
            return 0
        return self._sum / self._weight

    def reset(self) -> None:
        self._sum = 0
        self._weight = 0

    def is_differentiable(self) -> bool:
        raise NotImplementedError


class Accuracy(Score):
    """scores.py:97-177: argmax hits over the batch."""

    def __init__(self, log_freq: int = 1, split="test", score_name="accuracy",
                 reduction: str = "micro"):
        super().__init__(log_freq, split, score_name, reduction)

    def __call__(self, input, target):
        self._check(input, target)
        return self._update((input.argmax(dim=1) == target).sum(), input.shape[0])

    def is_differentiable(self) -> bool:
        return False


class CrossEntropyScore(Score):
    """scores.py:180-267: CrossEntropyLoss(reduction="sum") / batch."""

    def __init__(self, log_freq: int = 1, split="test", score_name="cross_entropy_score",
                 weight=None, reduction: str = "micro", label_smoothing: float = 0.0):
        super().__init__(log_freq, split, score_name, reduction)
        self._base_class = torch.nn.CrossEntropyLoss(weight=weight,
                                                     label_smoothing=label_smoothing,
                                                     reduction="sum")

    def __call__(self, input, target):
        self._check(input, target)
        return self._update(self._base_class(input, target), input.shape[0])

    def is_differentiable(self) -> bool:
        return True


class KLDivScore(Score):
    """scores.py:270-346: KLDivLoss(reduction="sum") / batch (FedDF's
    distillation criterion, feddf.py:132)."""

    def __init__(self, log_freq: int = 1, split="test", score_name="kl_dic_score",
                 reduction: str = "micro", log_target=False):
        super().__init__(log_freq, split, score_name, reduction)
        self._base_class = torch.nn.KLDivLoss(log_target=log_target, reduction="sum")

    def __call__(self, input, target):
        self._check(input, target)
        return self._update(self._base_class(input, target), input.shape[0])

    def is_differentiable(self) -> bool:
        return True
