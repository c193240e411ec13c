"""torch-CPU restatement of the reference's per-client aggregation loop.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).  This is what bench.py's
``cpu_baseline`` leg times: the same ATen CPU operations, in the same order and
with the same allocations, that one FedSim round performs on the server:

  serial_aggregation   fedsim/distributed/centralized/training/utils.py:34
      params = local_params.clone().detach().data        (one [P] copy)
  SerialAggregator.add fedsim/utils/aggregators.py:21,37-40
      new_v = params * weight                             (fresh [P])
      sum_v = sum_v + new_v  (first time: 0 + tensor)     (fresh [P])
      cur_w = cur_w + weight                              (Python scalar)
  SerialAggregator.pop fedsim/utils/aggregators.py:118-122
      v / w                                               (fresh [P])
"""
from __future__ import annotations

from typing import Sequence

import torch


def aggregate_round(rows: Sequence[torch.Tensor], weights: Sequence, ret_sum: bool = False):
    sum_v, cur_w = 0, 0
    for x, w in zip(rows, weights):
        params = x.clone().detach().data
        if w > 0:
            new_v = params * w
            sum_v = sum_v + new_v
            cur_w = cur_w + w
    if ret_sum:
        return sum_v, cur_w
    if cur_w == 0:
        return sum_v
    return sum_v / cur_w
