"""CentralFLAlgorithm — the round driver and the static user-method plugin contract.

Same constructor, storage entries, user-method table and round loop as the
reference (fedsim/distributed/centralized/centralized_fl_algorithm.py:30-828).
The one change on the hot path: the per-round aggregator created at :417 is
the device-backed ``fedsim_amd.utils.SerialAggregator``, so every
``receive_from_client`` streams its client vector into HBM and ``optimize``
pops a kernel-reduced average.  ``aggregator_factory`` lets a caller pass slab
/ device / tuning options for that aggregator.
"""
from __future__ import annotations

import inspect
import random
from functools import partial
from typing import Any, Dict, Optional

import torch
from torch import nn
from torch.utils.data import DataLoader

from ... import scores as _scores
from ...utils import AppendixAggregator, SerialAggregator, Storage, apply_on_dict
from ...utils.handover import handover_round
from ...utils.slab_rows import round_aggregator

try:  # progress bar is cosmetic
    from tqdm import trange as _trange
except Exception:  # pragma: no cover
    _trange = range


def _distributed_world() -> int:
    d = torch.distributed
    return d.get_world_size() if d.is_available() and d.is_initialized() else 1


def _to_host(obj):
    """A client-storage value made picklable across ranks: tensors to host
    memory, tagged with where they lived."""
    if isinstance(obj, torch.Tensor):
        return ("__fedsim_tensor__", obj.detach().cpu(), obj.device.type, obj.requires_grad)
    return obj


def _from_host(obj, device):
    if isinstance(obj, tuple) and len(obj) == 4 and obj[0] == "__fedsim_tensor__":
        _, t, kind, rg = obj
        if kind == "cuda" and device.type == "cuda":
            # detached first: the host copy may already require grad, and a
            # copy of it would be a non-leaf (no .grad, refused by optimizers)
            t = t.detach().to(device)
        return t.requires_grad_(rg) if rg else t
    return obj


_SKIP = object()


def _plain(v):
    """A picklable, exactly comparable image of a plain-data value (floats by
    their hex form, small tensors by value); _SKIP for anything else (models,
    large tensors, objects)."""
    if v is None or isinstance(v, (bool, int, str)):
        return v
    if isinstance(v, float):
        return ("f", v.hex())
    if type(v).__module__ == "numpy" and hasattr(v, "item") and getattr(v, "ndim", 1) == 0:
        return _plain(v.item())
    if isinstance(v, (list, tuple)):
        items = tuple(_plain(x) for x in v)
        return _SKIP if any(x is _SKIP for x in items) else (type(v).__name__, items)
    if isinstance(v, torch.Tensor) and v.numel() <= 16 and v.device.type != "meta":
        vals = v.detach().cpu().reshape(-1).double().tolist()
        return ("t", str(v.dtype), tuple(v.shape), tuple(float(x).hex() for x in vals))
    return _SKIP


def _context_fingerprint(ctx) -> Optional[dict]:
    """The plain-data entries of a send_to_client message (e.g. AdaBest's
    ``average_sample``): what a client-sharded round compares to find clients
    whose context depends on earlier clients' receive_from_client."""
    if not isinstance(ctx, dict):
        return None
    out = {}
    for k, v in ctx.items():
        fp = _plain(v)
        if fp is not _SKIP:
            out[k] = fp
    return out


def _storage_state(st: Storage):
    """What a client storage holds now: its entries by reference, plus the
    version counter of each tensor (an in-place change shows there)."""
    items = dict(st._storage)
    versions = {k: obj._version for k, (obj, _, _) in items.items()
                if isinstance(obj, torch.Tensor)}
    return items, versions


def _changed_keys(st: Storage, state) -> list:
    items, versions = state
    out = []
    for k, entry in st._storage.items():
        old = items.get(k)
        obj = entry[0]
        if old is None or old[0] is not obj or entry[1:] != old[1:]:
            out.append(k)
        elif isinstance(obj, torch.Tensor) and obj._version != versions.get(k):
            out.append(k)
        elif not isinstance(obj, (torch.Tensor, type(None), bool, int, float, str, tuple)):
            out.append(k)  # a mutable object: it may have changed in place
    return out


def _removed_keys(st: Storage, state) -> list:
    """Entries the client's storage held before the round and no longer does
    (Storage.remove)."""
    items, _ = state
    return [k for k in items if k not in st._storage]


def _distributed_rank() -> int:
    d = torch.distributed
    return d.get_rank() if d.is_available() and d.is_initialized() else 0


class CentralFLAlgorithm(object):
    def __init__(
        self,
        data_manager,
        metric_logger,
        num_clients,
        sample_scheme,
        sample_rate,
        model_def,
        epochs,
        criterion_def,
        optimizer_def=partial(torch.optim.SGD, lr=1.0),
        local_optimizer_def=partial(torch.optim.SGD, lr=0.1),
        lr_scheduler_def=None,
        local_lr_scheduler_def=None,
        r2r_local_lr_scheduler_def=None,
        batch_size=32,
        test_batch_size=64,
        device="cpu",
        *args,
        aggregator_factory=None,
        shard_over=None,
        shard_clients=None,
        client_reduction="chain",
        check_client_context=True,
        progress=False,
        **kwargs,
    ):
        sample_count = int(sample_rate * num_clients)
        if not 1 <= sample_count <= num_clients:
            raise Exception(
                "invalid client sample size for {}% of {} clients".format(sample_rate, num_clients)
            )
        model_def_ = getattr(model_def, "func", model_def)
        if not (inspect.isclass(model_def_) and issubclass(model_def_, nn.Module)) and not callable(
            model_def
        ):
            raise Exception("incompatiple model!")
        if isinstance(criterion_def, str) and hasattr(_scores, criterion_def):
            criterion_def = getattr(_scores, criterion_def)

        r2r_local_lr_scheduler = None
        if r2r_local_lr_scheduler_def is not None:
            if hasattr(local_optimizer_def, "keywords"):
                clr = local_optimizer_def.keywords["lr"]
            elif "lr" in inspect.signature(local_optimizer_def).parameters:
                clr = inspect.signature(local_optimizer_def).parameters["lr"].default
            else:
                raise Exception("lr not found in local optimizer class")
            dummy_opt = torch.optim.SGD(params=[torch.tensor([1.0, 1.0], requires_grad=True)],
                                        lr=clr)
            r2r_local_lr_scheduler = r2r_local_lr_scheduler_def(dummy_opt)
            if not hasattr(r2r_local_lr_scheduler, "get_last_lr"):
                sch = r2r_local_lr_scheduler
                sch.get_last_lr = lambda: sch._last_lr
            dummy_opt.step()

        global_dataloaders = {
            key: DataLoader(dataset, batch_size=test_batch_size, pin_memory=False)
            for key, dataset in data_manager.get_global_dataset().items()
        }
        oracle_dataset = data_manager.get_oracle_dataset()

        # size each round's HBM ring once for the clients it will receive, and
        # reduce HBM-resident client vectors in place: a message is dropped
        # right after receive_from_client, so its tensor can be handed over.
        # shard_over (not in the reference): spread each round's aggregation
        # over several GPUs by columns (fedsim_amd.sharding) -- "group" (the
        # default torch.distributed group: every rank runs this same round
        # loop, one process per GPU), a ProcessGroup, or a list of local
        # devices (one process driving several GPUs).  Opt-in: ranks of a
        # group that run different simulations must not be sharded together.
        # shard_clients (not in the reference): split each round's CLIENTS
        # over the ranks of a process group ("group" = the default group, or a
        # ProcessGroup): rank r trains one contiguous block of the sampled
        # clients, every rank receives every message (other ranks' vectors as
        # stand-ins) and the blocks are combined by ``client_reduction``:
        # "chain" (bit-exact) or "allreduce" (RCCL, normwise).  See
        # fedsim_amd.sharding.ClientShardedSerialAggregator.
        if shard_clients is not None:
            if aggregator_factory is not None or shard_over is not None:
                raise ValueError("shard_clients excludes aggregator_factory and shard_over")
            from ...sharding import ClientShardedSerialAggregator

            world = (torch.distributed.get_world_size(
                None if shard_clients == "group" else shard_clients)
                if torch.distributed.is_available() and torch.distributed.is_initialized()
                else 1)
            kw = dict(expected_rows=-(-sample_count // world), borrow=True, borrow_host=True,
                      mode=client_reduction)
            if shard_clients != "group":
                kw["group"] = shard_clients
            aggregator_factory = partial(ClientShardedSerialAggregator, **kw)
        if aggregator_factory is None:
            kw = dict(expected_rows=sample_count, borrow=True, borrow_host=True)
            if shard_over is None:
                aggregator_factory = partial(SerialAggregator, **kw)
            else:
                from ...sharding import ShardedSerialAggregator

                if isinstance(shard_over, (list, tuple)):
                    kw["devices"] = list(shard_over)
                elif shard_over != "group":
                    kw["group"] = shard_over
                aggregator_factory = partial(ShardedSerialAggregator, **kw)
        elif shard_over is not None:
            raise ValueError("pass either aggregator_factory or shard_over")
        self._aggregator_factory = aggregator_factory
        # client-sharded rounds: check that no client's send_to_client
        # message depends on an earlier client of the same round
        self._check_client_context = check_client_context
        # client-storage entries another rank wrote, kept in host memory
        # until this rank trains that client: {client_id: {key: device kind}}
        self._client_on_host = {}
        self._progress = progress
        self._server_memory = Storage()
        w = self._server_memory.write
        for key, val in (("data_manager", data_manager), ("num_clients", num_clients),
                         ("sample_count", sample_count), ("sample_scheme", sample_scheme),
                         ("oracle_dataset", oracle_dataset), ("last_client_sampled", None)):
            w(key, val, read_protected=True, write_protected=True)
        for key, val in (("test_batch_size", test_batch_size), ("optimizer_def", optimizer_def),
                         ("lr_scheduler_def", lr_scheduler_def),
                         ("r2r_local_lr_scheduler", r2r_local_lr_scheduler),
                         ("criterion_def", criterion_def), ("model_def", model_def),
                         ("metric_logger", metric_logger), ("device", device),
                         ("global_dataloaders", global_dataloaders), ("rounds", 0)):
            w(key, val, write_protected=True)

        self._client_memory = {k: Storage() for k in range(num_clients)}
        self._local_cfg = Storage()
        for key, val in (("epochs", epochs), ("batch_size", batch_size),
                         ("test_batch_size", test_batch_size), ("criterion_def", criterion_def),
                         ("local_optimizer_def", local_optimizer_def),
                         ("local_lr_scheduler_def", local_lr_scheduler_def)):
            self._local_cfg.write(key, val, write_protected=True)
        self._local_cfg.write("device", device)
        self._train_split_name = "train"
        self._server_scores = {key: dict() for key in global_dataloaders}
        self._client_scores = {key: dict() for key in data_manager.get_local_splits_names()}

        self.user_methods = dict(
            init=self.__class__.init,
            at_round_start=self.__class__.at_round_start,
            at_round_end=self.__class__.at_round_end,
            deploy=self.__class__.deploy,
            optimize=self.__class__.optimize,
            report=self.__class__.report,
            receive_from_client=self.__class__.receive_from_client,
            send_to_client=self.__class__.send_to_client,
            send_to_server=self.__class__.send_to_server,
        )
        for key, value in self.user_methods.items():
            if "self" in inspect.signature(value).parameters:
                raise Exception(
                    f"Remove `self` from {key} arguments. All user methods should be static!"
                )
        self.user_methods["init"](self._server_memory, *args, **kwargs)

    # ---- round plumbing (centralized_fl_algorithm.py:299-443) -------------
    def _sample_clients(self):
        mem = self._server_memory
        scheme = mem.read("sample_scheme", silent=True)
        count = mem.read("sample_count", silent=True)
        n = mem.read("num_clients", silent=True)
        last = mem.read("last_client_sampled", silent=True)
        if scheme == "uniform":
            return random.sample(range(n), count)
        if scheme == "sequential":
            last = -1 if last is None else last
            clients = [(i + 1) % n for i in range(last, last + count)]
            mem.write("last_client_sampled", clients[-1], silent=True)
            return clients
        raise NotImplementedError

    def _send_to_client(self, client_id):
        return self.user_methods["send_to_client"](self._server_memory, client_id=client_id)

    def _send_to_server(self, client_id, ctx_hook=None):
        r2r = self._server_memory.read("r2r_local_lr_scheduler")
        data_manager = self._server_memory.read("data_manager", silent=True)
        rounds = self._server_memory.read("rounds")
        cfg = self._local_cfg
        local_optimizer_def = cfg.read("local_optimizer_def")
        if r2r is not None:
            local_optimizer_def = partial(local_optimizer_def, lr=r2r.get_last_lr()[0])
        ctx = self._send_to_client(client_id)
        if ctx_hook is not None:
            ctx_hook(ctx)
        client_ctx = self.user_methods["send_to_server"](
            client_id, rounds, self._client_memory[client_id],
            data_manager.get_local_dataset(client_id), self.get_train_split_name(),
            self.get_local_scores(), cfg.read("epochs"), cfg.read("criterion_def")(),
            cfg.read("batch_size"), cfg.read("test_batch_size"), local_optimizer_def,
            cfg.read("local_lr_scheduler_def"), cfg.read("device"),
            ctx=ctx,
        )
        if not isinstance(client_ctx, dict):
            raise Exception("client should only return a dict!")
        return {**client_ctx, "client_id": client_id}

    def _receive_from_client(self, client_msg, serial_aggregator, appendix_aggregator):
        client_id = client_msg.pop("client_id")
        return self.user_methods["receive_from_client"](
            self._server_memory, client_id, client_msg, self.get_train_split_name(),
            serial_aggregator, appendix_aggregator,
        )

    def _optimize(self, serial_aggregator, appendix_aggregator):
        return self.user_methods["optimize"](self._server_memory, serial_aggregator,
                                             appendix_aggregator)

    def _report(self, round_scores, optimize_reports=None, deployment_points=None):
        mem = self._server_memory
        metric_logger = mem.read("metric_logger")
        rounds = mem.read("rounds")
        report_metrics = self.user_methods["report"](
            mem, mem.read("global_dataloaders", silent=True), rounds, round_scores,
            metric_logger, mem.read("device"), optimize_reports, deployment_points,
        )
        if metric_logger is not None and _distributed_rank() == 0:
            # ranks of a sharded run report the same scalars: log them once
            apply_on_dict(report_metrics, metric_logger.log_scalar, step=rounds)
        return report_metrics

    def _train(self, rounds, num_score_report_point=None):
        diverged = False
        cur_round = self._server_memory.read("rounds")
        score_aggregator = AppendixAggregator(max_deque_lenght=num_score_report_point)
        loop = _trange(rounds + 1) if self._progress else range(rounds + 1)
        for round_num in loop:
            self._at_round_start()
            round_serial_aggregator = self._aggregator_factory()
            round_appendix_aggregator = AppendixAggregator()
            # clients that train on the GPU vectorize straight into this
            # round's HBM slab (utils/slab_rows.py)
            with round_aggregator(round_serial_aggregator), handover_round():
                if hasattr(round_serial_aggregator, "client_block"):
                    diverged = self._client_sharded_round(round_serial_aggregator,
                                                          round_appendix_aggregator)
                else:
                    for client_id in self._sample_clients():
                        client_msg = self._send_to_server(client_id)
                        success = self._receive_from_client(client_msg, round_serial_aggregator,
                                                            round_appendix_aggregator)
                        del client_msg  # the aggregator may hold the message's tensor
                        if not success:
                            diverged = True
                            break
            if diverged:
                # drop the round's slab without launching
                del round_serial_aggregator
                return score_aggregator.pop_all()
            opt_reports = self._optimize(round_serial_aggregator, round_appendix_aggregator)
            deploy_point = self.user_methods["deploy"](self._server_memory)
            score_dict = self._report(self.get_global_scores(), opt_reports, deploy_point)
            score_aggregator.append_all(score_dict, step=cur_round)
            self._at_round_end(score_aggregator)
            self._server_memory.write("rounds", cur_round + round_num + 1, silent=True)
        return score_aggregator.pop_all()

    def _client_sharded_round(self, agg, appendix_aggregator) -> bool:
        """One round's clients under a ClientShardedSerialAggregator: this rank
        trains its block of the sampled clients, then every rank receives all
        the round's messages in the reference's order (other ranks' vectors as
        RemoteRow stand-ins), so the server state evolves identically on every
        rank.  Clients' own storages (AdaBest / FedDyn drift state) are
        shared with every rank after the round.  Returns ``diverged``.

        Checked on every rank alike (so all raise together, none hangs):
        * every rank sampled the same clients (a client that consumes Python
          ``random`` on one rank would otherwise shift the next rounds);
        * (``check_client_context``) every client's send_to_client message
          is the one it would get in the reference's sequential loop: at
          position p the message is recomputed after the receives of clients
          0..p-1 and its plain-data entries must equal what the client
          trained with.  AdaBest's ``average_sample`` (the running mean that
          receive_from_client updates, adabest.py:76-80,167-169) differs, so
          such an algorithm is refused instead of run on stale contexts."""
        clients = self._sample_clients()  # same seed, same list on every rank
        lo, hi = agg.client_block(len(clients))
        local, failure, ctx_fp, before = {}, None, {}, {}
        try:
            for p in range(lo, hi):
                cid = clients[p]
                self._client_to_device(cid, agg)
                before[p] = _storage_state(self._client_memory[cid])
                local[p] = self._send_to_server(
                    cid, ctx_hook=lambda ctx, p=p: ctx_fp.__setitem__(p, _context_fingerprint(ctx)))
        except Exception as e:  # noqa: BLE001 - re-raised below, after the exchange
            failure, local = e, {}
        # every rank reaches the exchange, so a failing client cannot leave
        # the others blocked in it; then every rank raises
        remote, extras = agg.exchange(local, len(clients), failed=failure is not None,
                                      extras=dict(clients=list(clients), ctx=ctx_fp))
        if failure is not None:
            raise failure
        if remote is None:
            raise RuntimeError("a client of another rank of this client-sharded round failed")
        if any(e["clients"] != list(clients) for e in extras):
            raise RuntimeError(
                "the ranks of a client-sharded round sampled different clients (%s): every "
                "rank must draw the same Python random numbers between rounds (a client "
                "that consumes Python's random module desynchronises them)"
                % "; ".join("rank %d: %s" % (r, e["clients"][:8]) for r, e in enumerate(extras)))
        contexts = {}
        for e in extras:
            contexts.update(e["ctx"])
        diverged_at = None
        for p in range(len(clients)):
            # a message without plain-data entries (FedAvg's: the model) has
            # nothing to compare, and send_to_client is not called twice
            if p > 0 and self._check_client_context and contexts.get(p):
                now = _context_fingerprint(self._send_to_client(clients[p]))
                if now != contexts.get(p):
                    keys = sorted(k for k in set(now or {}) | set(contexts.get(p) or {})
                                  if (now or {}).get(k) != (contexts.get(p) or {}).get(k))
                    raise RuntimeError(
                        f"client-sharded round: client {clients[p]} (position {p}) trained with "
                        f"a send_to_client message whose {keys} differ from the one the "
                        "reference's sequential loop gives it after the earlier clients' "
                        "receive_from_client; this algorithm's clients depend on each other in "
                        "arrival order (e.g. AdaBest's running average_sample) and cannot be "
                        "trained in parallel -- use shard_over (parameter sharding) instead")
            client_msg = local.pop(p) if p in local else remote[p]
            remote[p] = None
            success = self._receive_from_client(client_msg, agg, appendix_aggregator)
            del client_msg
            if not success:
                diverged_at = p
                break
        local.clear()
        # the reference stops training at the diverged client: clients after
        # it keep the storage they had before this round
        shared = []
        for p in range(lo, hi):
            if diverged_at is not None and p > diverged_at:
                self._restore_client(clients[p], before[p])
            else:
                shared.append((clients[p], before[p]))
        self._share_client_memory(agg, shared)
        return diverged_at is not None

    def _restore_client(self, cid, state) -> None:
        items, versions = state
        st = self._client_memory[cid]
        for k, (obj, _, _) in items.items():
            if isinstance(obj, torch.Tensor) and obj._version != versions.get(k):
                import warnings

                warnings.warn(f"client {cid}'s storage entry {k!r} was changed in place by a "
                              "client after the diverged one; it cannot be restored",
                              RuntimeWarning, stacklevel=3)
        st._storage = dict(items)

    def _client_to_device(self, cid, agg) -> None:
        """Entries other ranks wrote for this client wait in host memory
        until this rank trains it."""
        pending = self._client_on_host.pop(cid, None)
        if not pending:
            return
        dev = agg._reduce_device()
        st = self._client_memory[cid]
        for k, (kind, rg) in pending.items():
            obj, rp, wp = st._storage[k]
            st._storage[k] = (_from_host(("__fedsim_tensor__", obj, kind, rg), dev), rp, wp)

    def _share_client_memory(self, agg, trained) -> None:
        """Every rank gets the client-storage entries this round's other
        ranks wrote (only the entries that changed; tensors travel through
        host memory and stay there until this rank trains that client)."""
        import torch.distributed as dist

        if agg._solo:
            return
        mine = {}
        for cid, state in trained:
            st = self._client_memory[cid]
            keys, gone = _changed_keys(st, state), _removed_keys(st, state)
            if keys or gone:
                mine[cid] = ([(k, _to_host(st._storage[k][0]), st._storage[k][1],
                               st._storage[k][2]) for k in keys], gone)
        every = [None] * agg.world_size
        dist.all_gather_object(every, mine, group=agg._group)
        for r, mem in enumerate(every):
            if r == agg.rank:
                continue
            for cid, (items, gone) in mem.items():
                st = self._client_memory[cid]
                pending = self._client_on_host.setdefault(cid, {})
                for k in gone:  # Storage.remove on the rank that trained it
                    st._storage.pop(k, None)
                    pending.pop(k, None)
                for k, obj, rp, wp in items:
                    pending.pop(k, None)
                    if isinstance(obj, tuple) and len(obj) == 4 and obj[0] == "__fedsim_tensor__":
                        _, t, kind, rg = obj
                        pending[k] = (kind, rg)
                        obj = t.requires_grad_(rg) if rg else t
                    st._storage[k] = (obj, rp, wp)

    def _at_round_start(self) -> None:
        self.user_methods["at_round_start"](self._server_memory)

    def _at_round_end(self, score_aggregator) -> None:
        r2r = self._server_memory.read("r2r_local_lr_scheduler")
        if r2r is not None:
            r2r.step()
        self.user_methods["at_round_end"](self._server_memory, score_aggregator)

    def _get_round_scores(self, score_def_deck):
        rounds = self._server_memory.read("rounds")
        out = dict()
        for name, definition in score_def_deck.items():
            obj = definition()
            if rounds % obj.log_freq == 0:
                out[name] = obj
        return out

    # ---- public API (centralized_fl_algorithm.py:466-631) -----------------
    def train(self, rounds: int, num_score_report_point: Optional[int] = None,
              train_split_name="train") -> Optional[Dict[str, Optional[float]]]:
        from ...utils.aggregators import release_borrowed

        default_split_name = self._train_split_name
        self._train_split_name = train_split_name
        try:
            ans = self._train(rounds=rounds, num_score_report_point=num_score_report_point)
        finally:
            release_borrowed()  # the last round's borrowed client tensors
        self._train_split_name = default_split_name
        return ans

    def get_model_def(self):
        return self._server_memory.read("model_def")

    def get_server_storage(self):
        return self._server_memory

    def get_round_number(self):
        return self._server_memory.read("rounds")

    def get_train_split_name(self):
        return self._train_split_name

    def get_global_loader_split(self, split_name):
        return self._server_memory.read("global_dataloaders")[split_name]

    def get_device(self) -> str:
        return self._server_memory.read("device")

    def hook_local_score(self, score_def, score_name, split_name) -> None:
        self._client_scores[split_name][score_name] = score_def

    def hook_global_score(self, score_def, score_name, split_name) -> None:
        self._server_scores[split_name][score_name] = score_def

    def get_local_split_scores(self, split_name) -> Dict[str, Any]:
        return self._get_round_scores(self._client_scores[split_name])

    def get_global_split_scores(self, split_name):
        split_scores = self._get_round_scores(self._server_scores[split_name])
        return split_scores if len(split_scores) > 0 else None

    def get_local_scores(self) -> Dict[str, Any]:
        out = dict()
        for split_name in self._client_scores:
            s = self.get_local_split_scores(split_name)
            if s is not None:
                out[split_name] = s
        return out

    def get_global_scores(self) -> Dict[str, Any]:
        out = dict()
        for split_name in self._server_scores:
            s = self.get_global_split_scores(split_name)
            if s is not None:
                out[split_name] = s
        return out

    # ---- user methods (static; centralized_fl_algorithm.py:636-828) -------
    def init(server_storage, *args, **kwargs) -> None:
        pass

    def at_round_start(server_storage) -> None:
        pass

    def at_round_end(server_storage, score_aggregator) -> None:
        pass

    def send_to_client(server_storage, client_id):
        raise NotImplementedError("Algorithm is missing the required 'send_to_client' function")

    def send_to_server(id, rounds, storage, datasets, train_split_name, scores, epochs,
                       criterion, train_batch_size, inference_batch_size, optimizer_def,
                       lr_scheduler_def=None, device="cuda", ctx=None, *args, **kwargs):
        raise NotImplementedError("Algorithm is missing the required 'send_to_server' function")

    def receive_from_client(server_storage, client_id, client_msg, train_split_name,
                            serial_aggregator, appendix_aggregator) -> bool:
        raise NotImplementedError

    def optimize(server_storage, serial_aggregator, appendix_aggregator):
        raise NotImplementedError

    def deploy(server_storage):
        raise NotImplementedError

    def report(server_storage, dataloaders, round_scores, metric_logger, device,
               optimize_reports, deployment_points=None):
        raise NotImplementedError
