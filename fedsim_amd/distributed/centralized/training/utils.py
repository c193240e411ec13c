"""serial_aggregation and the fused server-step helpers.

``serial_aggregation`` keeps the reference contract
(fedsim/distributed/centralized/training/utils.py:7-57): divergence -> False,
weight = ``train_weight`` or ``num_samples[train_split_name]``, skip when the
weight is <= 0, per-split scalar metrics added with the (sticky) other_weight.
The reference's defensive ``clone()`` (utils.py:34) is dropped: the aggregator's
``add`` already snapshots the vector into HBM, so the copy bought nothing.

The server-step helpers run the FedAvg / AdaBest epilogues
(fedavg.py:193-208, adabest.py:172-189) as one fused libfedagg kernel when the
server optimizer is plain SGD, reproducing torch CPU SGD.step bit for bit
(``param.add_(grad, alpha=-lr)`` = fma(-lr, g, p), torch/optim/sgd.py).
Any other optimizer takes the reference's torch.optim route on the averaged
vector (the aggregation itself is still the HIP kernel).
"""
from __future__ import annotations

from typing import Optional

import torch

from .... import ops
from ....utils.aggregators import SerialAggregator as _DeviceSerialAggregator


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
    params = client_msg["local_params"].detach()
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


def pop_average(aggregator, key="local_params") -> torch.Tensor:
    """Pop the averaged vector, keeping it in HBM when the aggregator is ours."""
    if isinstance(aggregator, _DeviceSerialAggregator):
        return aggregator.pop_device(key)
    return aggregator.pop(key)


def plain_sgd_lr(optimizer, param) -> Optional[float]:
    """lr if ``optimizer`` is torch.optim.SGD over exactly ``[param]`` with no
    momentum / weight decay / nesterov / maximize, else None."""
    if type(optimizer) is not torch.optim.SGD or len(optimizer.param_groups) != 1:
        return None
    g = optimizer.param_groups[0]
    if len(g["params"]) != 1 or g["params"][0] is not param:
        return None
    if g.get("momentum", 0) or g.get("weight_decay", 0) or g.get("nesterov", False) or g.get(
        "maximize", False
    ):
        return None
    if param.dtype != torch.float32 or not param.is_contiguous():
        return None
    lr = g["lr"]
    return float(lr.item()) if isinstance(lr, torch.Tensor) else float(lr)


def _hip_device_for(*tensors) -> torch.device:
    for t in tensors:
        if isinstance(t, torch.Tensor) and t.device.type == "cuda":
            return t.device
    return torch.device("cuda", torch.cuda.current_device())


def _mark_stepped(optimizer) -> None:
    # The fused kernel replaces optimizer.step(); tell LR schedulers a step
    # happened (torch/optim/lr_scheduler.py checks optimizer._opt_called).
    optimizer._opt_called = True


def fused_fedavg_step(cloud: torch.Tensor, avg: torch.Tensor, lr: float, optimizer) -> None:
    """cloud.grad = cloud - avg ; cloud <- fma(-lr, grad, cloud), one kernel."""
    dev = _hip_device_for(avg, cloud)
    c = cloud.data if cloud.device == dev else cloud.data.to(dev)
    a = (avg if avg.device == dev else avg.to(dev)).reshape(-1)
    g = torch.empty_like(c)
    ops.fedavg_sgd(a, c, lr, grad_out=g)
    if c is not cloud.data:
        cloud.data.copy_(c)
    optimizer.zero_grad()
    cloud.grad = g if g.device == cloud.device else g.to(cloud.device)
    _mark_stepped(optimizer)


def _to_dev(t: torch.Tensor, dev: torch.device) -> torch.Tensor:
    """Working copy on ``dev`` (a fresh copy even if already there)."""
    return t.detach().reshape(-1).to(dev, copy=True).contiguous()


def fused_feddyn_step(cloud: torch.Tensor, avg: torch.Tensor, h: torch.Tensor, ratio: float,
                      lr: float, optimizer):
    """FedDyn epilogue in one kernel.  Returns (new_h, new_avg_params), each on
    the device of the tensor it replaces."""
    dev = _hip_device_for(avg, cloud)
    c = cloud.data if cloud.device == dev else cloud.data.to(dev)
    a = (avg if avg.device == dev else avg.to(dev)).reshape(-1)
    hh = _to_dev(h, dev)
    ap = torch.empty_like(c)
    g = torch.empty_like(c)
    ops.feddyn_sgd(a, c, hh, ratio, lr, avg_prev=ap, grad_out=g)
    if c is not cloud.data:
        cloud.data.copy_(c)
    optimizer.zero_grad()
    cloud.grad = g if g.device == cloud.device else g.to(cloud.device)
    _mark_stepped(optimizer)
    return hh.view_as(h).to(h.device), ap.view_as(cloud).to(cloud.device)


def fused_adabest_step(cloud: torch.Tensor, avg: torch.Tensor, avg_prev: torch.Tensor,
                       beta: float, lr: float, optimizer) -> torch.Tensor:
    """h = beta*(avg_prev - avg); new = avg - h; cloud.grad = cloud - new;
    cloud <- fma(-lr, grad, cloud); avg_prev <- avg.  Returns the new
    avg_params tensor (on avg_prev's device)."""
    dev = _hip_device_for(avg, cloud)
    c = cloud.data if cloud.device == dev else cloud.data.to(dev)
    a = (avg if avg.device == dev else avg.to(dev)).reshape(-1)
    ap = avg_prev.detach().clone() if avg_prev.device == dev else avg_prev.to(dev)
    ap = ap.reshape(-1).contiguous()
    g = torch.empty_like(c)
    ops.adabest_sgd(a, c, ap, beta, lr, grad_out=g)
    if c is not cloud.data:
        cloud.data.copy_(c)
    optimizer.zero_grad()
    cloud.grad = g if g.device == cloud.device else g.to(cloud.device)
    _mark_stepped(optimizer)
    return ap.view_as(avg_prev) if ap.device == avg_prev.device else ap.to(avg_prev.device)
