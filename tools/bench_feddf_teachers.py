"""FedDF's teacher forwards per distillation batch: the traced replay with
the Linear layers on the matrix cores (teacher_program.py) against the
whole-model torch.vmap over the teacher slab, for the reference's model
shapes (SimpleMLP 784-200-200-10 and SimpleCNN on MNIST, SimpleCNN2 on
CIFAR-100; fedsim_amd.models, each with the reference's Resize leaf), B = 64
(the server's test_batch_size), K teachers.  Kernel time from HIP events,
median of repeated calls.

python tools/bench_feddf_teachers.py [--K 10,100,1000]
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd.distributed.centralized.training.feddf import TeacherEnsemble  # noqa: E402


from fedsim_amd.models import SimpleCNN, SimpleCNN2, SimpleMLP  # noqa: E402  (the reference's
# classes restated, Resize leaf included: fedsim/models/simple_models.py:23-256)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    ms = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ms.append(e0.elapsed_time(e1))
    return float(np.median(ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--K", default="10,100,1000")
    ap.add_argument("--models", default="SimpleMLP,SimpleCNN,SimpleCNN2")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--no-vmap", action="store_true", help="time the replay only")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    for name, cls, shape in (("SimpleMLP", SimpleMLP, (64, 1, 28, 28)),
                             ("SimpleCNN", SimpleCNN, (64, 1, 28, 28)),
                             ("SimpleCNN2", lambda: SimpleCNN2(num_classes=100), (64, 3, 24, 24))):
        if name not in a.models.split(","):
            continue
        torch.manual_seed(0)
        model = cls().to(dev)
        P = sum(p.numel() for p in model.parameters())
        x = torch.randn(*shape, device=dev)
        for K in [int(v) for v in a.K.split(",")]:
            base = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
            teachers = [base + 0.05 * torch.randn_like(base) for _ in range(K)]
            ens = TeacherEnsemble(model, teachers, dev)
            ens.mean_logits(x)  # first-batch check
            kept = ens.program is not None
            t_prog = timed(lambda: ens.mean_logits(x), a.reps) if kept else None
            t_vmap = None
            if not a.no_vmap:
                vm = TeacherEnsemble(model, teachers, dev, program=False)
                t_vmap = timed(lambda: vm.mean_logits(x), a.reps)
                del vm
            st = ens.stats()
            print(json.dumps(dict(model=name, P=P, K=K, B=shape[0], program_kept=kept,
                                  fallback=st["reason"], fused_pools=st["fused_pools"],
                                  matrix_core_ms=t_prog, vmap_ms=t_vmap,
                                  speedup=(t_vmap / t_prog) if t_prog and t_vmap else None)),
                  flush=True)
            del ens, teachers
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
