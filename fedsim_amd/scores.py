"""Minimal stateful scores (reference: fedsim/scores.py:10-346), enough for the
round loop's criterion / metric plumbing.  Outside the accelerated path."""
from __future__ import annotations

import torch
import torch.nn.functional as F


class Score(object):
    def __init__(self, log_freq: int = 1, split="test", score_name="", reduction="micro"):
        self.log_freq = log_freq
        self.split = split
        self.score_name = score_name
        self.reduction = reduction
        self.reset()

    def get_name(self) -> str:
        return self.score_name

    def reset(self) -> None:
        self._sum = 0
        self._weight = 0

    def get_score(self) -> float:
        if self._weight < 1:
            return 0
        return self._sum / self._weight


class CrossEntropyScore(Score):
    def __init__(self, log_freq: int = 1, split="test", score_name="cross_entropy_score",
                 reduction="micro"):
        super().__init__(log_freq, split, score_name, reduction)

    def __call__(self, input, target):
        loss = F.cross_entropy(input, target, reduction="mean")
        n = target.shape[0]
        self._sum += float(loss.detach()) * n
        self._weight += n
        return loss

    def is_differentiable(self) -> bool:
        return True


class Accuracy(Score):
    def __init__(self, log_freq: int = 1, split="test", score_name="accuracy",
                 reduction="micro"):
        super().__init__(log_freq, split, score_name, reduction)

    def __call__(self, input, target):
        correct = (input.argmax(dim=-1) == target).sum().item()
        self._sum += correct
        self._weight += target.shape[0]
        return torch.tensor(correct / max(1, target.shape[0]))

    def is_differentiable(self) -> bool:
        return False
