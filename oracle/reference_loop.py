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


class ReferenceSerialAggregator(object):
    """The reference's SerialAggregator restated on torch CPU
    (fedsim/utils/aggregators.py:11-144): per key, ``value * weight`` added to
    the running sum (first add: ``0 + tensor``), the Python weight sum, and
    ``sum / weight`` on get / pop (the raw sum for a zero / None weight).
    Any value type torch arithmetic accepts (fp64 / bf16 / integer tensors,
    Python numbers).  TEST / MEASUREMENT INFRASTRUCTURE: the reference leg of
    tools/bench_host_rounds.py and the checker of the dtype-generic keys
    (tests/test_generic_keys.py, pinned to tests/golden/generic_keys.*)."""

    def __init__(self) -> None:
        self._members = dict()

    def add(self, key, value, weight=None):
        # aggregators.py:17-21 (_get_pair) and :35-40, in the reference's order
        new_v, new_w = (value, None) if weight is None else (value * weight, weight)
        sum_v, cur_w = self._members.get(key, (0, 0))
        if (sum_v is None) or (new_v is None):
            self._members[key] = (sum_v + new_v, None)
        else:
            self._members[key] = (sum_v + new_v, cur_w + new_w)

    def get(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")
        v, w = self._members[key]
        if w is None or w == 0:
            return v
        return v / w

    def get_sum(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")
        return self._members[key][0]

    def get_weight(self, key):
        if key not in self._members:
            raise Exception(f"{key} is not in the aggregator")
        return self._members[key][1]

    def keys(self):
        return self._members.keys()

    def pop(self, key):
        v = self.get(key)
        del self._members[key]
        return v

    def items(self):
        return {k: self.get(k) for k in self._members}.items()

    def pop_all(self):
        return {k: self.pop(k) for k in list(self._members)}

    def __contains__(self, key):
        return key in self._members
