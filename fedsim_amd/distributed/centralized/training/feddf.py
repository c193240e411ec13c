"""FedDF (ensemble distillation) on the MI355X aggregation path.

Reference: fedsim/distributed/centralized/training/feddf.py:19-142.  Per round:
the client vectors are averaged like FedAvg (``pop``, here the exact HIP
reduction) and the average becomes the cloud model (feddf.py:97-99); then, for
every batch of the server's distillation split, the K client models are run
as teachers, their logits averaged through a SerialAggregator with weight 1
(feddf.py:117-122), and the cloud model takes one server-optimizer step on the
KL divergence to that average (feddf.py:124-140).

MI355X-first differences:

* The reference re-copies every teacher into the model for every batch
  (``initialize_module``, K x P bytes per batch).  Here the K teacher vectors
  are stacked once per round into one [K, P] HBM slab.
* On a HIP device, and for models without buffers, the K teacher forwards run
  as ONE batched forward into a [K, B*C] logits slab: the model's traced graph
  replayed over all K teachers (teacher_program.py) -- every ``nn.Linear``
  (``fedagg_teacher_linear_f32``, v_mfma_f32_16x16x4_f32) and ``nn.Conv2d``
  (``fedagg_teacher_conv2d_f32``, v_mfma_f32_32x32x2_f32 implicit GEMM) on
  the matrix cores with a following ReLU fused, every zero-pad / LRN /
  max-pool chain as one pass (``fedagg_pad_lrn_maxpool_f32``), the remaining
  nodes under ``torch.vmap`` and parameterless foreign leaves (the reference
  models' ``Resize``) once per batch.  The teacher average is one launch of
  the exact-mode reduce kernel (``fedagg_reduce_f32``, weights 1, divide by
  fl32(K)): the reference's ``add(target, 1)`` x K + ``get`` arithmetic and
  order on the same logits.
* Parity is normwise, not bitwise, on this path: the matrix-core layers sum
  each output as one fmaf chain (not the CPU GEMM's order) and the LRN power
  is exp2/log2, a few ulps from powf.  The replay is checked against the
  whole-model ``vmap`` on its first batch (normwise 1e-4; on the first and
  last 32 teachers when there are more than 64) and pinned to the
  reference's own SimpleCNN2 / SimpleCNN FedDF rounds
  (tests/golden/feddf_cnn.*, tests/test_gpu_feddf_cnn.py).
* Whenever the replay is not used -- the forward does not trace, a kernel
  raises, or the first-batch check fails -- the ensemble falls back to the
  whole-model ``vmap`` (and, when that raises too, e.g. on random ops, to
  the reference's one-teacher-at-a-time loop), warns once with the reason and
  counts it: ``TeacherEnsemble.fallbacks`` / ``fallback_reason``, and per
  round in the server storage entry ``"teacher_replay"`` (with the kernel
  launch counts).
* The teachers are fixed for the whole distillation (they are this round's
  client models), so when the loader does not shuffle and the forward is a
  pure function of (teacher, input) -- no buffers, no dropout, no random
  op in the traced graph -- the ensemble's mean logits of each batch are
  computed in the first epoch and reused by the later ones (``global_epochs``
  > 1), after checking that the batch's input is the same tensor value
  (``torch.equal``; a dataset with random transforms recomputes).
* Elsewhere (host-resident model, or a model with buffers such as BatchNorm,
  whose running statistics cannot be updated under vmap) the teachers run one
  after another, as in the reference, and their logits go through the
  device-backed SerialAggregator.  With ``device="cpu"`` every forward is
  then the reference's own CPU arithmetic and the whole round is bitwise
  equal to it (tests/test_gpu_roundloop.py).
"""
from __future__ import annotations

import warnings

import torch
from torch.func import functional_call
from torch.nn.functional import log_softmax

from .... import ops
from ....scores import KLDivScore
from ....utils import SerialAggregator, initialize_module, vector_to_named_parameters_like
from . import teacher_program
from .fedavg import FedAvg
from .utils import serial_aggregation

_TEACHER_CHUNK = 64  # teachers per batched forward (bounds activation memory)
# teachers the replay is checked on against the whole-model vmap (first
# batch of a round): all of them up to this many, else the first and the last
# half of it -- the replay runs every teacher through the same kernels, and
# the ends cover the first and last teacher chunk and slab rows; the check
# then costs a 64-teacher vmap instead of a K-teacher one (131 ms at K=1000
# for SimpleCNN2, more than five replayed batches)
_CHECK_TEACHERS = 64


def _in_order(loader) -> bool:
    """Whether iterating ``loader`` yields the same batches every time (no
    shuffling or random sampling): then per-sample targets can be reused."""
    from torch.utils.data import BatchSampler, SequentialSampler

    bs = getattr(loader, "batch_sampler", None)
    return isinstance(bs, BatchSampler) and isinstance(bs.sampler, SequentialSampler)


def _pure_forward(model) -> bool:
    """A forward with no side effects and no randomness: no buffers (e.g.
    BatchNorm running statistics, updated by every reference forward in train
    mode) and no dropout in train mode.  Only then may a teacher's output be
    reused instead of recomputed as the reference does."""
    if any(True for _ in model.buffers()):
        return False
    return not any(isinstance(m, torch.nn.modules.dropout._DropoutNd) and m.training
                   for m in model.modules())


def _stack_rows(vectors, device) -> torch.Tensor:
    """The teachers' flat vectors as the rows of a [K, P] view whose row pitch
    is padded to 16 bytes, so every teacher's layer weights start where the
    matrix-core kernels can stage them with 16-byte loads (an odd-P model,
    e.g. SimpleMLP's 199 210, would otherwise misalign every other row)."""
    K = len(vectors)
    P = vectors[0].numel() if K else 0
    buf = torch.empty((K, (P + 3) // 4 * 4), dtype=torch.float32, device=device)
    slab = buf[:, :P]
    for k, t in enumerate(vectors):
        slab[k].copy_(t.reshape(-1))
    return slab


class TeacherEnsemble(object):
    """K teacher parameter vectors stacked in one slab; ``mean_logits(x)`` is
    the reference's weight-1 SerialAggregator average of their outputs."""

    def __init__(self, model, teacher_vectors, device, program=True):
        self.model = model
        self.named = list(model.named_parameters())
        self.slab = _stack_rows(teacher_vectors, device)
        self.K = self.slab.shape[0]
        self.batched = (self.slab.device.type == "cuda"
                        and len(list(model.buffers())) == 0)
        self._w32 = None
        self.fallbacks = 0
        self.fallback_reason = None
        self.program = None
        # the traced forward with its layers on the matrix cores
        # (teacher_program.py); checked against the vmap path on first use
        if program and self.batched:
            self.program, why = teacher_program.build_or_reason(model, self.named, self.slab)
            if self.program is None:
                self._fall_back(why)
        self._checked = False

    def _fall_back(self, reason: str) -> None:
        """The replay (or the batched path) is not used: count it, warn once."""
        self.fallbacks += 1
        self.fallback_reason = reason
        warnings.warn(f"FedDF teacher replay not used, {reason}; the teachers run under "
                      f"{'torch.vmap' if self.batched else 'a per-teacher loop'}",
                      RuntimeWarning, stacklevel=3)

    @property
    def deterministic(self) -> bool:
        """Whether the teachers' outputs are a pure function of the input on
        the path in use (no random op in the traced graph; a vmap'd forward
        with one raises, and the per-teacher loop is not trusted)."""
        if not self.batched:
            return False
        return self.program is None or not self.program.has_random_ops

    def stats(self) -> dict:
        p = self.program
        return dict(replayed=p is not None, batched=self.batched, fallbacks=self.fallbacks,
                    reason=self.fallback_reason,
                    linear_launches=p.linear_launches if p else 0,
                    conv_launches=p.conv_launches if p else 0,
                    pool_launches=p.pool_launches if p else 0,
                    fused_pools=p.fused_pools if p else 0)

    def _forward(self, flat, x):
        return functional_call(self.model, vector_to_named_parameters_like(flat, self.named), (x,))

    def _vmap_logits(self, x, rows=None):
        slab = self.slab if rows is None else self.slab[rows]
        chunks = []
        for k0 in range(0, slab.shape[0], _TEACHER_CHUNK):
            part = slab[k0:k0 + _TEACHER_CHUNK]
            chunks.append(torch.vmap(self._forward, in_dims=(0, None))(part, x))
        return torch.cat(chunks) if len(chunks) > 1 else chunks[0]

    def _check_rows(self):
        """The teachers the first-batch check compares (None: all)."""
        if self.K <= _CHECK_TEACHERS:
            return None
        h = _CHECK_TEACHERS // 2
        return torch.cat([torch.arange(h), torch.arange(self.K - h, self.K)]).to(self.slab.device)

    def teacher_logits(self, x):
        """[K, ...] outputs of every teacher on ``x`` (batched path)."""
        if self.program is None:
            return self._vmap_logits(x)
        if self._checked:
            try:
                return self.program(x)
            except Exception as e:  # noqa: BLE001 - e.g. a later batch's shape
                self.program = None
                self._fall_back(f"the replay raised {type(e).__name__} on a later batch: {e}")
                return self._vmap_logits(x)
        # first use: the program must reproduce the vmap'd forward (same
        # graph, f32 matrix-core arithmetic: normwise) on the checked
        # teachers, else it is dropped
        rows = self._check_rows()
        ref = self._vmap_logits(x, rows)
        try:
            got = self.program(x)
            cmp = got if rows is None else got[rows]
            why = None
            if got.shape[0] != self.K or cmp.shape != ref.shape:
                why = (f"its output shape {tuple(got.shape)} is not "
                       f"{(self.K,) + tuple(ref.shape[1:])}")
            elif not bool((torch.isfinite(cmp) == torch.isfinite(ref)).all()):
                why = "its first batch has non-finite values where the vmap'd forward has not"
            else:
                err = float(torch.linalg.vector_norm((cmp - ref).double().nan_to_num()))
                ref_n = float(torch.linalg.vector_norm(ref.double().nan_to_num()))
                if err > 1e-4 * ref_n + 1e-30:
                    why = (f"its first batch differs from the vmap'd forward (normwise "
                           f"{err / max(ref_n, 1e-30):.3g} > 1e-4)")
        except Exception as e:  # noqa: BLE001 - a graph the replay cannot run: keep vmap
            got, why = None, f"the replay raised {type(e).__name__}: {e}"
        self._checked = True
        if why is not None:
            self.program = None
            self._fall_back(why)
            return ref if rows is None else self._vmap_logits(x)
        return got

    def _sequential_mean(self, x):
        agg = SerialAggregator()
        for k in range(self.K):
            agg.add("target", self._forward(self.slab[k], x).clone(), 1)
        return agg.get("target")

    def _batched_logits(self, x):
        """[K, ...] teacher outputs on the batched path, or None when it
        raised (counted; the per-teacher path takes over)."""
        try:
            return self.teacher_logits(x)
        except Exception as e:  # noqa: BLE001 - e.g. random ops under vmap
            self.batched, self.program = False, None
            self._fall_back(f"the vmap'd forward raised {type(e).__name__}: {e}")
            return None

    @torch.no_grad()
    def logit_rows(self, x):
        """Every teacher's output on ``x`` as the rows of a [K, n] fp32 slab,
        and the output shape: what a client-sharded round sums across ranks."""
        logits = self._batched_logits(x) if self.batched else None
        if logits is None:
            logits = torch.stack([self._forward(self.slab[k], x).clone() for k in range(self.K)])
        K, shape = logits.shape[0], logits.shape[1:]
        return logits.reshape(K, -1).float().contiguous(), shape

    @torch.no_grad()
    def mean_logits(self, x):
        if not self.batched:
            return self._sequential_mean(x)
        logits = self._batched_logits(x)
        if logits is None:
            return self._sequential_mean(x)
        K, shape = logits.shape[0], logits.shape[1:]
        rows = logits.reshape(K, -1).float().contiguous()
        if self._w32 is None:
            self._w32 = torch.ones(K, dtype=torch.float32, device=rows.device)
        out = torch.empty(rows.shape[1], dtype=torch.float32, device=rows.device)
        ops.reduce_slab(rows, self._w32, out, W=K)
        return out.view(shape)

    def load_last(self):
        """Leave the model holding the last teacher, as the reference's
        per-teacher initialize_module does (feddf.py:119)."""
        initialize_module(self.model, self.slab[-1])


class ShardedTeachers(object):
    """FedDF's teachers in a client-sharded round
    (``CentralFLAlgorithm(..., shard_clients=...)``): each rank holds the
    vectors of the clients it trained (the others are RemoteRow stand-ins in
    the appendix aggregator), replays its own teachers -- the same
    TeacherEnsemble kernels, K/N teachers per GPU -- and the per-rank logit
    sums are combined by the round's ClientShardedSerialAggregator:
    ``chain`` adds rank after rank in arrival order, the reference's
    ``target_agg.add(target, 1)`` x K order bit for bit (feddf.py:120-126);
    ``allreduce`` sums from +0 per rank and all-reduces (normwise).  Then
    the divide by fl32(K) (``get``, feddf.py:126) and the same student step
    on every rank."""

    def __init__(self, model, values, agg, device):
        from ....sharding import RemoteRow

        me = agg.rank
        self.agg = agg
        self.model = model
        self.K = len(values)
        seq = [v.owner if isinstance(v, RemoteRow) else me for v in values]
        self.owners = [r for i, r in enumerate(seq) if i == 0 or seq[i - 1] != r]
        self.last_owner = seq[-1]
        local = [v for v in values if not isinstance(v, RemoteRow)]
        self.local = TeacherEnsemble(model, local, device) if local else None

    @property
    def deterministic(self) -> bool:
        # agreed by every rank: a batch's targets are reused on all or none
        return self.agg._all_true(self.local is None or self.local.deterministic)

    def stats(self) -> dict:
        st = self.local.stats() if self.local is not None else dict(
            replayed=False, batched=False, fallbacks=0, reason=None, linear_launches=0,
            conv_launches=0, pool_launches=0, fused_pools=0)
        return dict(st, teachers_total=self.K,
                    teachers_local=0 if self.local is None else self.local.K,
                    rank=self.agg.rank, client_reduction=self.agg.mode)

    @torch.no_grad()
    def mean_logits(self, x):
        if self.local is not None:
            rows, shape = self.local.logit_rows(x)
        else:  # no teacher on this rank: only the output's shape is needed
            rows, shape = None, self.model(x).shape
        n = 1
        for d in shape:
            n *= d
        s = self.agg.ordered_rows_sum(rows, self.owners, n)
        return self.agg.divide(s, self.K).view(shape).to(x.device)

    def sync_student(self, cloud, optimizer) -> None:
        """Every rank distilled the same student from the same targets, but
        the student's GPU backward (MIOpen / rocBLAS) need not give the same
        bits twice: rank 0's cloud and the optimizer state of it are
        broadcast, so every rank starts the next round from one model."""
        self.agg.broadcast_from(cloud.data, 0)
        for t in optimizer.state.get(cloud, {}).values():
            if isinstance(t, torch.Tensor) and t.dim() > 0:
                self.agg.broadcast_from(t, 0)

    def load_last(self):
        """The model holds the last teacher afterwards, as after the
        reference's loop (feddf.py:122): broadcast from the rank holding it."""
        dev = self.agg._reduce_device()
        P = sum(p.numel() for p in self.model.parameters())
        if self.agg.rank == self.last_owner:
            vec = self.local.slab[-1].to(dev).contiguous().clone()
        else:
            vec = torch.empty(P, dtype=torch.float32, device=dev)
        self.agg.broadcast_from(vec, self.last_owner)
        initialize_module(self.model, vec.to(next(self.model.parameters()).device))


def _teachers(model, values, serial_aggregator, device):
    """The round's teacher ensemble: split over the ranks of a
    client-sharded round (decided alike on every rank), else one slab."""
    if getattr(serial_aggregator, "collective", False):
        return ShardedTeachers(model, values, serial_aggregator, device)
    return TeacherEnsemble(model, values, device)


class FedDF(FedAvg):
    def init(server_storage, *args, **kwrag):
        default_global_train_split = "valid"
        default_global_epochs = 1
        FedAvg.init(server_storage)
        server_storage.write("global_train_split",
                             kwrag.get("global_train_split", default_global_train_split))
        server_storage.write("global_epochs", kwrag.get("global_epochs", default_global_epochs))

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator):
        params = client_msg["local_params"].clone().detach().data
        appendix_aggregator.append("local_params", params)
        return serial_aggregation(server_storage, client_id, client_msg, train_split_name,
                                  serial_aggregator)

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        if "local_params" in serial_aggregator:
            param_avg = serial_aggregator.pop("local_params")
            cloud_params = server_storage.read("cloud_params")
            cloud_params.data = param_avg.data

            model = server_storage.read("model")
            global_train_split = server_storage.read("global_train_split")
            train_data_loader = server_storage.read("global_dataloaders").get(global_train_split)
            if train_data_loader is None:
                raise Exception(f"no dataloader made for split {global_train_split} on the server!")
            global_epochs = server_storage.read("global_epochs")
            optimizer = server_storage.read("optimizer")
            lr_scheduler = server_storage.read("lr_scheduler")
            device = server_storage.read("device")

            teachers = _teachers(model, appendix_aggregator.get_values("local_params"),
                                 serial_aggregator, device)
            # the same batches every epoch: mean logits computed once, reused
            # for a batch whose input is the same value again
            cache = [] if (global_epochs > 1 and _in_order(train_data_loader)
                           and _pure_forward(model)) else None
            ran = False
            for _ in range(global_epochs):
                for j, (x, _) in enumerate(train_data_loader):
                    x = x.to(device)
                    if cache is not None and not teachers.deterministic:
                        cache = None
                    if cache is not None and j < len(cache) and torch.equal(cache[j][0], x):
                        logits = cache[j][1]
                    else:
                        logits = teachers.mean_logits(x)
                        if cache is not None:
                            if j < len(cache):
                                cache[j] = (x, logits)
                            else:
                                cache.append((x, logits))
                    target_out = log_softmax(logits, 1)
                    criterion = KLDivScore(log_target=True)
                    param_dict = vector_to_named_parameters_like(cloud_params,
                                                                 model.named_parameters())
                    pred = functional_call(model, param_dict, x)
                    pred_out = log_softmax(pred, 1)
                    loss = criterion(pred_out, target_out.data)
                    optimizer.zero_grad()
                    loss.backward()
                    optimizer.step()
                    if lr_scheduler is not None:
                        lr_scheduler.step()
                    ran = True
            if ran:
                if isinstance(teachers, ShardedTeachers):
                    teachers.sync_student(cloud_params, optimizer)
                teachers.load_last()
            server_storage.write("teacher_replay", teachers.stats())
        return serial_aggregator.pop_all()
