"""Client-side local training / inference — PRODUCERS of the client updates.

Outside the accelerated path: a compact restatement of the
reference's fedsim/local/training/{training.py:12-112, step_closures.py:9-76,
inference.py:11-51} so that FedAvg.send_to_server runs end to end.  Plain torch
autograd; nothing here is a HIP kernel of this project.
"""
from __future__ import annotations

import inspect

import torch
from torch.nn.utils import clip_grad_norm_


def default_step_closure(x, y, model, criterion, optimizer, scores, max_grad_norm=1000,
                         device="cpu", transform_grads=None, transform_y=None, **kwargs):
    if transform_y is not None:
        y = transform_y(y)
    x = x.to(device)
    y = y.reshape(-1).long().to(device)
    model.train()
    outputs = model(x)
    loss = criterion(outputs, y)
    if loss.isnan() or loss.isinf():
        return loss
    loss.backward()
    if transform_grads is not None:
        transform_grads(model)
    clip_grad_norm_(parameters=model.parameters(), max_norm=max_grad_norm)
    optimizer.step()
    optimizer.zero_grad()
    if scores is not None:
        for score in scores.values():
            score(outputs, y)
    return loss


def _scheduler_step(lr_scheduler, scores, criterion):
    """training.py:90-105: a scheduler whose step takes ``metrics`` (e.g.
    ReduceLROnPlateau) is fed the score named by its ``trigger_metric``."""
    if "metrics" in inspect.signature(lr_scheduler.step).parameters:
        comb_scores = {**scores, **{criterion.get_name(): criterion}}
        trigger_metric = lr_scheduler.trigger_metric
        if trigger_metric not in comb_scores:
            raise Exception(f"{trigger_metric} not in local scores. "
                            f"Possible options are {comb_scores.keys()}")
        lr_scheduler.step(comb_scores[trigger_metric].get_score())
    else:
        lr_scheduler.step()


def local_train(model, train_data_loader, epochs, steps, criterion, optimizer,
                lr_scheduler=None, device="cpu", step_closure=default_step_closure,
                scores=None, max_grad_norm=1000, **step_ctx):
    """Returns (num_train_samples, num_steps, diverged)."""
    if steps > 0:
        epochs += 1
    num_steps, num_train_samples, diverged = 0, 0, False
    if train_data_loader is not None:
        for _ in range(epochs):
            if diverged:
                break
            for x, y in train_data_loader:
                loss = step_closure(x, y, model, criterion, optimizer, scores, max_grad_norm,
                                    device=device, **step_ctx)
                if loss.isnan() or loss.isinf():
                    diverged = True
                    break
                num_steps += 1
                num_train_samples += y.shape[0]
                if lr_scheduler is not None:
                    _scheduler_step(lr_scheduler, scores, criterion)
    return num_train_samples, num_steps, diverged


def local_inference(model, data_loader, scores, device="cpu", transform_y=None):
    num_samples = 0
    was_training = model.training
    model.eval()
    with torch.no_grad():
        for X, y in data_loader:
            if transform_y is not None:
                y = transform_y(y)
            y = y.reshape(-1).long().to(device)
            outputs = model(X.to(device))
            num_samples += len(y)
            for score in scores.values():
                score(outputs, y)
    if was_training:
        model.train()
    return num_samples
