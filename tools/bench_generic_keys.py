"""The dtype-generic keys of SerialAggregator in HBM: a round of K client
vectors of a bf16 / fp16 / fp64 model, ``add`` x K then ``pop``, through

  kernel  fedsim_amd's SerialAggregator: fedagg_reduce_rows_ref, borrowed
          (handed-over) or snapshotted rows
  torch   the reference's own expression on the same HIP tensors (value *
          weight, sum + new_v: two torch launches and three passes per
          client) -- what the keys ran as before the kernel

timed with HIP events; client bytes reduced per second.  The two sums are
compared bit for bit (the quotient differs by design: torch's HIP division
multiplies by the reciprocal, the drop-in divides as ATen's CPU does).

python tools/bench_generic_keys.py [--P 25000000] [--K 200] [--reps 3]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd.utils import SerialAggregator  # noqa: E402


class TorchExpression(object):
    """The timed baseline leg: the reference's add / get_sum expression
    (aggregators.py:17-40) written out on the same HIP tensors -- value *
    weight, then sum + new_v, two torch launches and three passes per
    client -- what the keys ran as before the kernel."""

    def __init__(self):
        self.sum_v, self.cur_w = 0, 0

    def add(self, key, value, weight):
        new_v = value * weight
        self.sum_v, self.cur_w = self.sum_v + new_v, self.cur_w + weight

    def get_sum(self, key):
        return self.sum_v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=25_000_000)
    ap.add_argument("--K", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for dt in (torch.bfloat16, torch.float16, torch.float64):
        P = a.P if dt != torch.float64 else a.P // 4
        g = torch.Generator(device=dev).manual_seed(7)
        base = torch.empty(P, device=dev, dtype=torch.float32).normal_(0, 0.05, generator=g)
        rows = [(base + torch.empty_like(base).normal_(0, 1e-3, generator=g)).to(dt)
                for _ in range(a.K)]
        del base
        w = [int(v) for v in torch.randint(50, 601, (a.K,))]
        nbytes = a.K * P * rows[0].element_size()
        sums = {}
        for mode in ("kernel_borrow", "kernel_snapshot", "torch"):
            best = None
            for _ in range(a.reps):
                agg = (TorchExpression() if mode == "torch" else
                       SerialAggregator(borrow=mode == "kernel_borrow"))
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for k in range(a.K):
                    agg.add("p", rows[k], w[k])
                s = agg.get_sum("p")
                e1.record()
                torch.cuda.synchronize()
                ms = e0.elapsed_time(e1)
                best = ms if best is None else min(best, ms)
                sums[mode] = s
                del agg
            print(json.dumps(dict(dtype=str(dt).replace("torch.", ""), mode=mode, K=a.K, P=P,
                                  ms=round(best, 3), gbps=round(nbytes / best / 1e6, 1))),
                  flush=True)
        same = all(torch.equal(sums[m].view(-1).view(torch.uint8),
                               sums["torch"].view(-1).view(torch.uint8))
                   for m in ("kernel_borrow", "kernel_snapshot"))
        print(json.dumps(dict(dtype=str(dt).replace("torch.", ""), sums_bitwise_equal=same)),
              flush=True)
        del rows, sums
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
