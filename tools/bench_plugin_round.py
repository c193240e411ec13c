"""End-to-end server round through the plugin surface, as a FedSim run drives
it: ``FedAvg.receive_from_client`` x K (serial_aggregation -> SerialAggregator
.add, plus the per-split scalar metrics) and ``FedAvg.optimize`` (pop + server
SGD step, fused into the round's last reduction).  Wall clock per round, split
into the host-side receive loop and the rest, for client vectors that are

  device_borrow   HBM-resident tensors handed over (the round driver's default)
  device_snap     HBM-resident tensors snapshotted at add (borrow=False)
  host_pinned     pinned host tensors (CPU-side local trainers)
  host_pageable   pageable host tensors (what vectorize_module returns on CPU)
  cpu_run         pageable host tensors AND the cloud on the host: FedSim's
                  device="cpu" run (config 1), aggregation on the MI355X; timed
                  beside the reference's own CPU arithmetic for the same round
                  (oracle/reference_loop.py: clone + mul + add per client,
                  divide, then cloud - avg and the SGD step, torch CPU)

and, for reference, the device-resident kernel time of the same reduce + step
(tools/bench_configs.py).

python tools/bench_plugin_round.py [--only cfg2_K1000] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedsim_amd.distributed.centralized.training import FedAvg  # noqa: E402
from fedsim_amd.utils import SerialAggregator, Storage  # noqa: E402
from fedsim_amd.utils.handover import hand_over, handover_round  # noqa: E402

CONFIGS = {
    "cfg1": (5, 199_210),
    "cfg2_K10": (10, 1_085_668),
    "cfg2_K1000": (1000, 1_085_668),
}


def messages(K, P, where, dev, seed=11):
    weights = [int(v) for v in np.random.default_rng(seed).integers(50, 601, size=K)]
    g = torch.Generator(device=dev).manual_seed(seed)
    msgs = []
    for k in range(K):
        t = torch.empty(P, device=dev).normal_(0.0, 0.05, generator=g)
        if where == "host_pinned":
            t = t.cpu().pin_memory()
        elif where in ("host_pageable", "cpu_run"):
            t = t.cpu()
        msgs.append(dict(local_params=t, num_steps=1, diverged=False,
                         num_samples={"train": weights[k]},
                         metrics={"train": {"cross_entropy_score": 1.0 + 1e-3 * k}}))
    return msgs


def one_round(msgs, cloud, borrow):
    """``msgs`` is consumed: each message is handed over as the round driver
    hands it (a ``handover_round`` with the client's ``hand_over`` of its
    vector, utils/handover.py; the aggregator borrows it only then and only
    if nothing else holds it, training/utils.py _handed_over)."""
    st = Storage()
    st.write("cloud_params", cloud)
    st.write("optimizer", torch.optim.SGD(params=[cloud], lr=1.0))
    st.write("lr_scheduler", None)
    agg = SerialAggregator(expected_rows=len(msgs), borrow=borrow)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    with handover_round():
        for k in range(len(msgs)):
            msg, msgs[k] = msgs[k], None
            hand_over(msg["local_params"])  # the client's send_to_server does this
            FedAvg.receive_from_client(st, k, msg, "train", agg, None)
            del msg
    t1 = time.perf_counter()
    FedAvg.optimize(st, agg, None)
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    return t1 - t0, t2 - t0


def reference_round(msgs, P, reps=3):
    """The reference's arithmetic for the same round on the host (oracle leg):
    serial_aggregation's clone + SerialAggregator's mul/add per client, the
    divide, then FedAvg.optimize's cloud - avg and SGD(lr=1) step."""
    from oracle.reference_loop import aggregate_round

    rows = [m["local_params"] for m in msgs]
    weights = [m["num_samples"]["train"] for m in msgs]
    best = None
    for _ in range(reps):
        cloud = torch.zeros(P, requires_grad=True)
        opt = torch.optim.SGD(params=[cloud], lr=1.0)
        t0 = time.perf_counter()
        avg = aggregate_round(rows, weights)
        opt.zero_grad()
        cloud.grad = cloud.data - avg
        opt.step()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best


class _Flat(torch.nn.Module):
    """A GPU model of P fp32 parameters in a few ragged tensors (the client
    side of the headline round; only the parameter layout matters here)."""

    def __init__(self, P):
        super().__init__()
        sizes = [P // 2 + 3, P // 4 - 1, P // 8 + 5]
        sizes.append(P - sum(sizes))
        self.ps = torch.nn.ParameterList(
            torch.nn.Parameter(torch.empty(n).normal_(0.0, 0.05)) for n in sizes)


def headline_round(K, P, dev, mode, reps, ragged=False):
    """One FedAvg round of K GPU-trained clients at the headline size, the
    clients' vectorize included (the loop), optimize timed on its own after
    the clients' kernels have finished:

      slab_rows       vectorize_module(model, out=reserved row of the round's
                      slab): one pack launch per client, reduce + step from the
                      column-blocked slab (the bench kernel)
      borrow_vector   vectorize_module(model) (torch.cat, a fresh tensor) handed
                      over and borrowed: reduce + step over the row pointers
    """
    from fedsim_amd.utils import initialize_module, slab_rows, vectorize_module

    model = _Flat(P).to(dev)
    if not ragged:
        # as in a round: send_to_client's initialize_module makes the client
        # model's parameters views of one vector (one segment to pack)
        initialize_module(model, vectorize_module(model))
    w = [int(v) for v in np.random.default_rng(11).integers(50, 601, size=K)]
    res = []
    for rep in range(reps + 1):
        cloud = torch.zeros(P, device=dev, requires_grad=True)
        st = Storage()
        st.write("cloud_params", cloud)
        st.write("optimizer", torch.optim.SGD(params=[cloud], lr=1.0))
        st.write("lr_scheduler", None)
        C = 4096
        # room for K + 1 rows: the ring never drains before optimize
        agg = SerialAggregator(expected_rows=K, borrow=True,
                               slab_bytes=4 * (K + 1) * ((P + C - 1) // C) * C)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with slab_rows.round_aggregator(agg), handover_round():
            for k in range(K):
                row = slab_rows.reserve_round_row("local_params", model) \
                    if mode == "slab_rows" else None
                msg = dict(local_params=hand_over(vectorize_module(model, out=row)), num_steps=1,
                           diverged=False, num_samples={"train": w[k]},
                           metrics={"train": {"cross_entropy_score": 1.0}})
                del row
                FedAvg.receive_from_client(st, k, msg, "train", agg, None)
                del msg
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        FedAvg.optimize(st, agg, None)
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        del agg
        torch.cuda.empty_cache()
        if rep:  # the first is a warm-up
            res.append((t1 - t0, t2 - t1))
    loop = min(r[0] for r in res)
    opt = min(r[1] for r in res)
    return dict(clients_loop_ms=loop * 1e3, optimize_ms=opt * 1e3,
                optimize_client_GBps=4.0 * K * P / opt / 1e9,
                pack_GBps_per_client_byte=4.0 * K * P / loop / 1e9)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--headline", action="store_true",
                    help="also K=1000 x P=25M with GPU clients (slab rows vs borrowed vectors)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if a.headline:
        K, P = 1000, 25_000_000
        res = dict(K=K, P=P)
        for mode, ragged in (("slab_rows", False), ("borrow_vector", False),
                             ("slab_rows", True)):
            name = mode + ("_ragged_params" if ragged else "")
            res[name] = headline_round(K, P, dev, mode, a.reps, ragged)
            print(json.dumps({"headline_" + name: res[name]}), flush=True)
        print(json.dumps({"headline": res}), flush=True)
        # the reference's own model sizes through the same GPU-client round
        for name, (K, P) in CONFIGS.items():
            res = dict(K=K, P=P)
            for mode in ("slab_rows", "borrow_vector"):
                res[mode] = headline_round(K, P, dev, mode, max(a.reps, 5))
            print(json.dumps({"gpu_clients_" + name: res}), flush=True)
        if a.only == "headline":
            return
    names = [n for n in CONFIGS if not a.only or n in a.only.split(",")]
    out = {}
    for name in names:
        K, P = CONFIGS[name]
        res = dict(K=K, P=P)
        for where, borrow in (("device_borrow", True), ("device_snap", False),
                              ("host_pinned", False), ("host_pageable", False),
                              ("cpu_run", False)):
            cloud = torch.zeros(P, device="cpu" if where == "cpu_run" else dev,
                                requires_grad=True)
            one_round(messages(K, P, where, dev), cloud, borrow)  # warm-up
            runs = [one_round(messages(K, P, where, dev), cloud, borrow)
                    for _ in range(a.reps)]
            msgs = messages(K, P, where, dev)
            recv, total = min(r[0] for r in runs), min(r[1] for r in runs)
            res[where] = dict(round_ms=total * 1e3, receive_loop_ms=recv * 1e3,
                              per_client_us=recv / K * 1e6,
                              client_GBps=4.0 * K * P / total / 1e9)
            if where == "cpu_run":
                res["reference_cpu_round_ms"] = reference_round(msgs, P) * 1e3
                res["cpu_threads"] = torch.get_num_threads()
            del msgs, cloud
            torch.cuda.empty_cache()
        out[name] = res
        print(json.dumps({name: res}), flush=True)
    print(json.dumps({"all": out}), flush=True)


if __name__ == "__main__":
    main()
