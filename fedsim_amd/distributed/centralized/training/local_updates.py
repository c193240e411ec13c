"""Client-side updates of the centralized algorithms — the PRODUCERS of the
vectors the accelerated server path reduces.

Outside the HIP path (SURVEY §8a row a2 is where it ends: one flat fp32
vector per client).  The plugin classes' static ``send_to_server`` methods
delegate here so that their files hold only the plugin surface and the
server side.  Each function restates the reference's client arithmetic
operation for operation (same RNG consumption, same tensor op order), which
is what tests/test_client_cpu.py checks bit for bit on CPU:

  sgd_update         fedavg.py:87-179   local SGD, per-split scores, message
  proximal_update    fedprox.py:79-127  + mu/2 (params - params_init) on grads
  drift_update       adabest.py:97-148  + mu_adaptive * -h on grads; h update
  dynamic_reg_update feddyn.py:104-155  + alpha_adaptive (0.5 (p - p0) - h)

Every function returns the client message dict the server's
``receive_from_client`` consumes: ``local_params``, ``num_steps``,
``diverged``, ``num_samples``, ``metrics``.
"""
from __future__ import annotations

import math
from functools import partial

from torch.nn.utils import parameters_to_vector
from torch.utils.data import DataLoader, RandomSampler

from ....local import default_step_closure, local_inference, local_train
from ....utils import vector_to_parameters_like, vectorize_module
from ....utils.handover import hand_over
from ....utils.slab_rows import reserve_round_row


def _grad_hook(coef_vec_fn):
    """A ``transform_grads`` callback adding ``coef_vec_fn(model)`` (a flat
    vector, or None for no-op) to the parameters' gradients, parameter by
    parameter in registration order."""

    def transform(model):
        extra = coef_vec_fn(model)
        if extra is None:
            return
        for p, g in zip(model.parameters(), vector_to_parameters_like(extra, model.parameters())):
            p.grad += g

    return transform


def _split_scores(scores, split):
    return {n: s.get_score() for n, s in scores.get(split, dict()).items()}


def sgd_update(rounds, datasets, train_split_name, scores, epochs, criterion, train_batch_size,
               inference_batch_size, optimizer_def, lr_scheduler_def, device, ctx,
               step_closure=None):
    """Local SGD on the client's train split (sampled with replacement, a
    whole number of batches), then inference on every other scored split."""
    train_set = datasets[train_split_name]
    n_draw = math.ceil(len(train_set) / train_batch_size) * train_batch_size
    loader = DataLoader(train_set, batch_size=train_batch_size,
                        sampler=RandomSampler(train_set, replacement=True, num_samples=n_draw))
    model = ctx["model"]
    opt = optimizer_def(model.parameters())
    sched = None if lr_scheduler_def is None else lr_scheduler_def(optimizer=opt)
    train_scores = scores.get(train_split_name, dict())
    n_train, n_steps, diverged = local_train(
        model, loader, epochs, 0, criterion, opt, sched, device,
        default_step_closure if step_closure is None else step_closure, scores=train_scores,
    )
    metrics = {train_split_name: _split_scores(scores, train_split_name)}
    if rounds % getattr(criterion, "log_freq", 1) == 0 and hasattr(criterion, "get_name"):
        metrics[train_split_name][criterion.get_name()] = criterion.get_score()
    counts = {train_split_name: n_train}
    for name, split in datasets.items():
        if name == train_split_name or name not in scores:
            continue
        counts[name] = local_inference(
            model, DataLoader(split, batch_size=inference_batch_size, shuffle=False),
            scores[name], device=device)
        metrics[name] = _split_scores(scores, name)
    # on the GPU the update is written straight into the round's HBM slab;
    # the vector is fresh and kept nowhere: handed over to the server
    row = reserve_round_row("local_params", model)
    return dict(local_params=hand_over(vectorize_module(model, out=row)), num_steps=n_steps,
                diverged=diverged, num_samples=counts, metrics=metrics)


def proximal_update(rounds, datasets, train_split_name, scores, epochs, criterion,
                    train_batch_size, inference_batch_size, optimizer_def, lr_scheduler_def,
                    device, ctx):
    """FedProx client: gradient += mu * 0.5 * (params - params_init)."""
    mu = ctx["mu"]
    p0 = vectorize_module(ctx["model"], clone=True, detach=True)
    hook = _grad_hook(lambda m: mu * (0.5 * (parameters_to_vector(m.parameters()) - p0)))
    return sgd_update(rounds, datasets, train_split_name, scores, epochs, criterion,
                      train_batch_size, inference_batch_size, optimizer_def, lr_scheduler_def,
                      device, ctx, step_closure=partial(default_step_closure,
                                                        transform_grads=hook))


def drift_update(rounds, storage, datasets, train_split_name, scores, epochs, criterion,
                 train_batch_size, inference_batch_size, optimizer_def, lr_scheduler_def,
                 device, ctx):
    """AdaBest client: gradient += mu_adaptive * -h, then the client's drift
    estimate h <- h / (rounds - last_round) + (params_init - params)."""
    model = ctx["model"]
    p0 = vectorize_module(model, clone=True, detach=True)
    h = storage.read("h")
    mu_adaptive = ctx["mu"] / len(datasets[train_split_name]) * ctx["average_sample"] * epochs
    hook = _grad_hook(lambda m: None if h is None else mu_adaptive * -h)
    msg = sgd_update(rounds, datasets, train_split_name, scores, epochs, criterion,
                     train_batch_size, inference_batch_size, optimizer_def, lr_scheduler_def,
                     device, ctx, step_closure=partial(default_step_closure,
                                                       transform_grads=hook))
    delta = p0 - vectorize_module(model, clone=True, detach=True)
    if h is None:
        storage.write("h", delta)
    else:
        last = storage.read("last_round")
        gap = rounds - (rounds - 1 if last is None else last)
        storage.write("h", 1 / gap * h + delta)
    storage.write("last_round", rounds)
    return msg


def dynamic_reg_update(rounds, storage, datasets, train_split_name, scores, epochs, criterion,
                       train_batch_size, inference_batch_size, optimizer_def, lr_scheduler_def,
                       device, ctx):
    """FedDyn client: gradient += alpha_adaptive * (0.5 (params - params_init)
    - h), then h <- h + (params_init - params)."""
    model = ctx["model"]
    p0 = vectorize_module(model, clone=True, detach=True)
    h = storage.read("h")
    alpha_adaptive = ctx["alpha"] / len(datasets[train_split_name]) * ctx["average_sample"]

    def extra(m):
        v = 0.5 * (vectorize_module(m) - p0)
        if h is not None:
            v -= h
        return alpha_adaptive * v

    msg = sgd_update(rounds, datasets, train_split_name, scores, epochs, criterion,
                     train_batch_size, inference_batch_size, optimizer_def, lr_scheduler_def,
                     device, ctx, step_closure=partial(default_step_closure,
                                                       transform_grads=_grad_hook(extra)))
    delta = p0 - vectorize_module(model, clone=True, detach=True)
    storage.write("h", delta if h is None else delta + h)
    return msg
