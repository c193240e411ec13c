"""serial_aggregation and the fused server step.

``serial_aggregation`` keeps the reference contract
(fedsim/distributed/centralized/training/utils.py:7-57): divergence -> False,
weight = ``train_weight`` or ``num_samples[train_split_name]``, skip when the
weight is <= 0, per-split scalar metrics added with the (sticky) other_weight.
The reference's defensive ``clone()`` (utils.py:34) is kept only where it
changes anything.  ``SerialAggregator.add`` snapshots host vectors (into the
pinned staging ring) and, by default, HBM vectors (into the ring slab); the
round driver's aggregator instead *borrows* HBM-resident vectors and reads
them when the round is reduced.  Borrowing is only sound when the client gave
the vector away: a client that reuses one output buffer, or keeps the tensor
or a view of it, could otherwise change it before the round is reduced.  In
the round driver that is declared, not inferred: the producer's hand-over
token (utils/handover.py; the library's clients set it, local_updates.py)
plus no alias of the storage.  The vector is cloned here -- the reference's
own copy -- whenever the aggregator would borrow it and that ownership is not
shown (``_handed_over``); a tensor modified in place after all is caught by
its version counter at the drain.

``fused_server_step`` runs the FedAvg / AdaBest / FedDyn ``optimize`` epilogues
(fedavg.py:193-208, adabest.py:172-189, feddyn.py:169-194) together with the
server optimizer's update as ONE libfedagg kernel whenever the optimizer is a
``torch.optim.SGD`` over exactly ``[cloud_params]`` (any momentum / dampening /
nesterov / weight decay / maximize).  It reproduces torch CPU SGD.step bit for
bit, including the momentum buffer it leaves in ``optimizer.state``.  Any other
optimizer takes the reference's torch.optim route on the averaged vector (the
aggregation itself is still the HIP kernel).
"""
from __future__ import annotations

import os
from typing import Optional

import torch

from .... import ops
from ....local import local_inference
from ....utils import initialize_module, vectorize_module
from ....utils.aggregators import SerialAggregator as _DeviceSerialAggregator
from ....utils.handover import take_token, unaliased
from ....utils.slab_rows import SlabRow


def serial_aggregation(
    server_storage,
    client_id,
    client_msg,
    train_split_name,
    aggregator,
    train_weight=None,
    other_weight=None,
    purge_msg=True,
):
    params = client_msg["local_params"]
    if _would_borrow(aggregator, params) and not _handed_over(params):
        params = params.clone()  # the reference's snapshot (utils.py:34)
    if params.requires_grad:  # detach only when needed: it allocates a tensor object
        params = params.detach()
    diverged = client_msg["diverged"]
    metrics = client_msg["metrics"]
    n_samples = client_msg["num_samples"]

    if diverged:
        return False

    if train_weight is None:
        train_weight = n_samples[train_split_name]

    if train_weight > 0:
        aggregator.add("local_params", params, train_weight)
        for split_name, split_metrics in metrics.items():
            if other_weight is None:
                other_weight = n_samples[split_name]
            for key, metric in split_metrics.items():
                aggregator.add(f"clients.{split_name}.{key}", metric, other_weight)

    if purge_msg:
        del client_msg
    return True


def _handed_over(t: torch.Tensor) -> bool:
    """Whether ``t`` was given away by its client, so the aggregator may read
    it after add returns: an explicit hand-over token of the open
    ``handover_round`` (utils/handover.py) and no alias of its storage.
    Ownership is never inferred: outside a hand-over round (user code calling
    receive_from_client on its own) no vector is handed over, and a borrowing
    aggregator gets the reference's clone -- user code that wants the borrow
    opens ``handover_round()`` and calls ``hand_over`` as the driver does."""
    if isinstance(t, SlabRow) and t.in_slab and not t._committed:
        # a row the client reserved in the round's slab (reserve_round_row):
        # handed over by that protocol -- it is the aggregator's own memory,
        # and torch ops on the SlabRow afterwards act on a private copy
        take_token(t)
        return True
    return bool(take_token(t)) and unaliased(t)


def _would_borrow(aggregator, t) -> bool:
    """The aggregator reads ``t`` after add returns: an HBM vector borrowed
    in place, or a host vector staged by the ingest worker while the next
    client trains (aggregators._Ingest.put_async)."""
    opts = getattr(aggregator, "_opts", None)
    if not (isinstance(aggregator, _DeviceSerialAggregator) and opts is not None
            and isinstance(t, torch.Tensor)):
        return False
    return opts.borrow if t.device.type == "cuda" else opts.borrow_host


def pop_average(aggregator, key="local_params") -> torch.Tensor:
    """Pop the averaged vector, keeping it in HBM when the aggregator is ours."""
    if isinstance(aggregator, _DeviceSerialAggregator):
        return aggregator.pop_device(key)
    return aggregator.pop(key)


def _scalar(x) -> Optional[float]:
    if isinstance(x, torch.Tensor):
        return float(x.item()) if x.numel() == 1 else None
    return float(x)


def sgd_config(optimizer, param) -> Optional[dict]:
    """The SGD hyper-parameters if ``optimizer`` is torch.optim.SGD over
    exactly ``[param]`` (fp32, contiguous), else None."""
    if type(optimizer) is not torch.optim.SGD or len(optimizer.param_groups) != 1:
        return None
    g = optimizer.param_groups[0]
    if len(g["params"]) != 1 or g["params"][0] is not param:
        return None
    if param.dtype != torch.float32 or not param.is_contiguous():
        return None
    cfg = dict(lr=_scalar(g["lr"]), momentum=_scalar(g.get("momentum", 0)),
               dampening=_scalar(g.get("dampening", 0)),
               weight_decay=_scalar(g.get("weight_decay", 0)),
               nesterov=bool(g.get("nesterov", False)), maximize=bool(g.get("maximize", False)))
    if any(v is None for v in cfg.values()):
        return None
    return cfg


def plain_sgd_lr(optimizer, param) -> Optional[float]:
    """lr if ``optimizer`` is a momentum-free, decay-free SGD over ``[param]``."""
    cfg = sgd_config(optimizer, param)
    if cfg is None or cfg["momentum"] or cfg["weight_decay"] or cfg["nesterov"] or \
            cfg["maximize"]:
        return None
    return cfg["lr"]


def _hip_device_for(*tensors) -> torch.device:
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.device.type == "cuda":
            return t.device
    return torch.device("cuda", torch.cuda.current_device())


def _work_copy(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    """Flat contiguous copy on ``dev`` (always a fresh copy)."""
    return t.detach().reshape(-1).to(dev, copy=True).contiguous()


def fused_server_step(algo: str, cloud: torch.Tensor, avg, optimizer,
                      cfg: dict, coef: float = 0.0, aux: Optional[torch.Tensor] = None,
                      want_avg_prev: bool = False):
    """One kernel: algorithm pseudo-gradient + SGD update of ``cloud``.

    ``avg`` is the averaged tensor, or ``(aggregator, key)``: then the key is
    popped and, when the aggregator is ours, the step runs fused into the
    round's last reduction pass (the average is never stored).

    Leaves ``cloud.grad`` = pseudo-gradient and the momentum buffer in
    ``optimizer.state[cloud]`` exactly as ``optimizer.step()`` would, and marks
    the optimizer as stepped for LR schedulers.  Returns ``(aux', avg_prev')``
    on the devices of ``aux`` / ``cloud`` (None where not requested)."""
    source = None
    if isinstance(avg, tuple):
        source, avg = avg, None
        agg, key = source
        dev = agg.device_of(key) if isinstance(agg, _DeviceSerialAggregator) else None
        if dev is None:
            avg, source = agg.pop(key), None
    if source is None:
        dev = _hip_device_for(avg, cloud)
    state = optimizer.state[cloud]
    prev = state.get("momentum_buffer") if cfg["momentum"] != 0 else None
    if _host_state(cloud, aux, prev, dev):
        return _fused_server_step_host(algo, cloud, avg, source, optimizer, cfg, coef, aux,
                                       want_avg_prev, dev, prev)
    c = cloud.data if cloud.device == dev else cloud.data.to(dev)
    x = _work_copy(aux, dev) if aux is not None else None
    ap = torch.empty_like(c) if want_avg_prev else None
    g = torch.empty_like(c)
    buf, init = None, False
    if cfg["momentum"] != 0:
        init = prev is None
        buf = torch.empty_like(c) if init else _work_copy(prev, dev)
    step = ops.ServerStep(algo, c.view(-1), lr=cfg["lr"], momentum=cfg["momentum"],
                          dampening=cfg["dampening"], weight_decay=cfg["weight_decay"],
                          nesterov=cfg["nesterov"], maximize=cfg["maximize"], coef=coef,
                          aux=x, avg_prev=ap, momentum_buf=buf, momentum_init=init, grad_out=g)
    if source is not None:
        agg.pop_step(key, step)
    else:
        step.apply((avg if avg.device == dev else avg.to(dev)).reshape(-1).contiguous())
    if c is not cloud.data:
        cloud.data.copy_(c)
    optimizer.zero_grad()
    cloud.grad = g if g.device == cloud.device else g.to(cloud.device)
    if buf is not None:
        state["momentum_buffer"] = buf.view_as(cloud).to(cloud.device)
    # The kernel replaced optimizer.step(); LR schedulers check this flag
    # (torch/optim/lr_scheduler.py) to detect a step.
    optimizer._opt_called = True
    x_out = None if x is None else x.view_as(aux).to(aux.device)
    ap_out = None if ap is None else ap.view_as(cloud).to(cloud.device)
    return x_out, ap_out


def _host_state(cloud, aux, prev, dev) -> bool:
    """The cloud (and the aux vector and momentum buffer, when present) in
    host memory, fp32, while the step runs on the GPU: FedSim's device="cpu"
    runs (BASELINE config 1)."""
    if dev.type != "cuda" or cloud.device.type != "cpu":
        return False
    return all(t is None or (t.device.type == "cpu" and t.dtype == torch.float32)
               for t in (aux, prev))


# How host-resident server state reaches the step kernel: "zero_copy", the
# kernel reading and writing one page-locked buffer in place over PCIe (no
# DMA to issue either way), or "dma", one pinned DMA each way (round 5).
_HOST_STEP = os.environ.get("FEDSIM_AMD_HOST_STEP", "zero_copy")


def _fused_server_step_host(algo, cloud, avg, source, optimizer, cfg, coef, aux, want_avg_prev,
                            dev, prev):
    """fused_server_step for host-resident server state (FedSim's
    device="cpu" runs): the cloud -- and the aux vector, momentum buffer and
    previous average when the algorithm has them -- are copied into ONE
    page-locked buffer whose rows the step kernel reads and writes in place
    over PCIe (ops.host_mapped), instead of a pageable copy per tensor each
    way; its rows become ``cloud.grad``, the momentum buffer and the returned
    vectors (fresh tensors each round, as the reference's step leaves them).
    With ``_HOST_STEP = "dma"``, or a sharded aggregator (whose collectives
    need the operands in HBM), the buffer crosses PCIe as one pinned DMA each
    way instead.  Same kernel, same bits."""
    P = cloud.numel()
    rows = ["c", "g"] + (["x"] if aux is not None else []) + \
        (["ap"] if want_avg_prev else []) + (["buf"] if cfg["momentum"] != 0 else [])
    at = {name: i for i, name in enumerate(rows)}
    ins = [("c", cloud.data)] + ([("x", aux)] if aux is not None else []) + \
        ([("buf", prev)] if prev is not None else [])
    if _HOST_STEP == "zero_copy" and (source is None or
                                      type(source[0]) is _DeviceSerialAggregator):
        # rows padded to 16 bytes: the fused reduce + step entries take them
        H = torch.empty(len(rows), -(-P // 4) * 4, dtype=torch.float32, pin_memory=True)
        if ops.host_mapped(H):
            row = {name: H[i, :P] for i, name in enumerate(rows)}
            for name, t in ins:
                t = t.detach().reshape(-1)
                if name in ("c", "buf") and t.data_ptr() % 16 == 0 and ops.host_mapped(t):
                    # page-locked already (init_cloud pins the cloud; the
                    # momentum buffer is last round's row): updated in place,
                    # as optimizer.step() updates the parameter and its buffer
                    row[name] = t
                else:
                    row[name].copy_(t)
            step = ops.ServerStep(
                algo, row["c"], lr=cfg["lr"], momentum=cfg["momentum"],
                dampening=cfg["dampening"], weight_decay=cfg["weight_decay"],
                nesterov=cfg["nesterov"], maximize=cfg["maximize"], coef=coef,
                aux=row.get("x"), avg_prev=row.get("ap"), momentum_buf=row.get("buf"),
                momentum_init=cfg["momentum"] != 0 and prev is None, grad_out=row["g"],
                device=dev)
            if source is not None:
                source[0].pop_step(source[1], step)
            else:
                step.apply((avg if avg.device == dev else avg.to(dev)).reshape(-1).contiguous())
            torch.cuda.current_stream(dev).synchronize()
            return _host_step_results(cloud, optimizer, aux, want_avg_prev, row)
    D = torch.empty(len(rows), P, dtype=torch.float32, device=dev)
    hin = torch.empty(len(ins), P, dtype=torch.float32, pin_memory=True)
    for j, (name, t) in enumerate(ins):
        hin[j].copy_(t.detach().reshape(-1))
    cur = torch.cuda.current_stream(dev)
    if [at[name] for name, _ in ins] == list(range(len(ins))):
        D[:len(ins)].copy_(hin, non_blocking=True)  # one DMA (inputs are the leading rows)
    else:
        for j, (name, _) in enumerate(ins):
            D[at[name]].copy_(hin[j], non_blocking=True)
    row = {name: D[i] for i, name in enumerate(rows)}
    step = ops.ServerStep(algo, row["c"], lr=cfg["lr"], momentum=cfg["momentum"],
                          dampening=cfg["dampening"], weight_decay=cfg["weight_decay"],
                          nesterov=cfg["nesterov"], maximize=cfg["maximize"], coef=coef,
                          aux=row.get("x"), avg_prev=row.get("ap"), momentum_buf=row.get("buf"),
                          momentum_init=cfg["momentum"] != 0 and prev is None,
                          grad_out=row["g"])
    if source is not None:
        agg, key = source
        agg.pop_step(key, step)
    else:
        step.apply((avg if avg.device == dev else avg.to(dev)).reshape(-1).contiguous())
    hout = torch.empty(len(rows), P, dtype=torch.float32, pin_memory=True)
    hout.copy_(D, non_blocking=True)
    done = torch.cuda.Event()
    done.record(cur)
    done.synchronize()
    return _host_step_results(cloud, optimizer, aux, want_avg_prev,
                              {name: hout[i] for i, name in enumerate(rows)})


def _host_step_results(cloud, optimizer, aux, want_avg_prev, out):
    """The host step's rows handed back as optimizer.step() leaves them."""
    cloud.data.copy_(out["c"].view_as(cloud))
    optimizer.zero_grad()
    cloud.grad = out["g"].view_as(cloud)
    if "buf" in out:
        optimizer.state[cloud]["momentum_buffer"] = out["buf"].view_as(cloud)
    # The kernel replaced optimizer.step(); LR schedulers check this flag
    # (torch/optim/lr_scheduler.py) to detect a step.
    optimizer._opt_called = True
    x_out = out["x"].view_as(aux) if aux is not None else None
    ap_out = out["ap"].view_as(cloud) if want_avg_prev else None
    return x_out, ap_out


# ---------------------------------------------------------------------------
# Server-side state shared by the FedAvg family (fedavg.py:70-85, 210-256)
# ---------------------------------------------------------------------------
def init_cloud(server_storage):
    """Build the cloud model on the server device and its flat parameter
    vector (the tensor the fused server step updates in place), plus the
    server optimizer / LR scheduler over ``[cloud_params]``."""
    model = server_storage.read("model_def")().to(server_storage.read("device"))
    cloud = vectorize_module(model, clone=True, detach=True)
    if cloud.device.type == "cpu" and torch.cuda.is_available():
        # device="cpu" with the aggregation on the GPU: a page-locked cloud
        # is stepped in place over PCIe (_fused_server_step_host)
        cloud = cloud.pin_memory()
    cloud.requires_grad = True
    opt = server_storage.read("optimizer_def")(params=[cloud])
    sched_def = server_storage.read("lr_scheduler_def")
    for key, obj in (("model", model), ("cloud_params", cloud), ("optimizer", opt),
                     ("lr_scheduler", None if sched_def is None else sched_def(optimizer=opt))):
        server_storage.write(key, obj)
    return cloud


def init_drift_state(server_storage):
    """``avg_params`` (last round's average) and the zero ``h`` vector that
    AdaBest and FedDyn keep next to the cloud vector."""
    cloud = server_storage.read("cloud_params")
    server_storage.write("avg_params", cloud.clone().detach())
    server_storage.write("h", torch.zeros_like(cloud))


def cloud_model_message(server_storage):
    """The cloud vector unflattened into the server's model (views of one
    device-resident vector, see utils/convert_parameters.py)."""
    model = server_storage.read("model")
    initialize_module(model, server_storage.read("cloud_params"), clone=True, detach=True)
    return dict(model=model)


NORM_REPORT_FREQ = 50


def deployment_report(server_storage, dataloaders, rounds, scores, device, optimize_reports,
                      deployment_points=None):
    """Scores of every deployment point on every scored server split, plus the
    point's parameter norm every NORM_REPORT_FREQ rounds."""
    model = server_storage.read("model")
    out, norms = dict(), dict()
    for point_name, point in (deployment_points or dict()).items():
        initialize_module(model, point, clone=True, detach=True)
        for split_name, loader in dataloaders.items():
            if split_name in scores:
                local_inference(model, loader, scores=scores[split_name], device=device)
                for score_name, score in scores[split_name].items():
                    out[f"server.{point_name}.{split_name}.{score_name}"] = score.get_score()
            if rounds % NORM_REPORT_FREQ == 0:
                norms[f"server.{point_name}.param.norm"] = point.norm().item()
    return {**out, **optimize_reports, **norms}
