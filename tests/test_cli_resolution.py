"""``fedsim-cli fed-learn --algorithm ...`` resolution onto this package
(fedsim_amd/cli.py), restating fedsim_cli/utils.py:116-147 (decode_margs),
:33-69 (parse_class_from_file / get_definition), :186-192 (module list),
:221-230 (base-class argument guard), :235-236 (partial binding) and the
instantiation of fedsim_cli/fed_learn.py:372-389.

These tests check the grammar and the instantiation; the resolver's
outputs are pinned to the reference's own resolver in tests/test_cli_golden.py
(fixtures from tools/gen_golden_cli.py)."""
import os
from collections import OrderedDict
from functools import partial

import pytest
import torch

from conftest import REPO


def test_decode_margs_grammar():
    from fedsim_amd.cli import SearchSpace, decode_margs

    assert decode_margs(None) == (None, None, None)
    assert decode_margs(("FedAvg",)) == ("FedAvg", {}, OrderedDict())
    # click hands a single-string option over as characters: joined back
    assert decode_margs(tuple("FedAvg")) == ("FedAvg", {}, OrderedDict())
    name, args, hargs = decode_margs(("AdaBest", "mu:0.01", "beta:0.6"))
    assert (name, args, hargs) == ("AdaBest", {"mu": 0.01, "beta": 0.6}, OrderedDict())
    assert isinstance(args["mu"], float)
    name, args, hargs = decode_margs(("SGD", "lr:0.1", "momentum:Real:0-1", "nesterov:true"))
    assert args == {"lr": 0.1, "nesterov": True}
    assert hargs == OrderedDict(momentum=SearchSpace("Real", (0, 1)))
    with pytest.raises(Exception, match="invalid argument"):
        decode_margs(("FedAvg", "mu"))
    with pytest.raises(Exception, match="enetered correctly"):
        decode_margs(("FedAvg", "a:b:c:d"))


def test_algorithm_names_resolve_to_the_mi355x_path():
    from fedsim_amd.cli import ingest_algorithm
    from fedsim_amd.distributed.centralized import training

    for name in ("FedAvg", "AdaBest", "FedNova", "FedDyn", "FedProx", "FedDF"):
        ctx = ingest_algorithm((name,))
        assert ctx.definition.func is getattr(training, name)
    with pytest.raises(Exception, match="is not defined"):
        ingest_algorithm(("NoSuchAlgorithm",))


def test_base_class_arguments_are_protected():
    from fedsim_amd.cli import ingest_algorithm

    with pytest.raises(Exception, match="Not allowed to change parameters"):
        ingest_algorithm(("FedAvg", "num_clients:5"))


def _instantiate(definition):
    """fed_learn.py:372-389 with a synthetic data manager, on the CPU."""
    from fedsim_amd.scores import CrossEntropyScore
    from oracle import synthetic_fl as S

    return definition(
        data_manager=S.FakeDataManager(), metric_logger=None, num_clients=S.NUM_CLIENTS,
        sample_scheme="uniform", sample_rate=S.SAMPLE_RATE, model_def=S.TinyModel, epochs=1,
        criterion_def=partial(CrossEntropyScore, split="train"),
        optimizer_def=partial(torch.optim.SGD, lr=1.0),
        local_optimizer_def=partial(torch.optim.SGD, lr=0.1), lr_scheduler_def=None,
        local_lr_scheduler_def=None, r2r_local_lr_scheduler_def=None, batch_size=32,
        test_batch_size=64, device="cpu")


@pytest.mark.parametrize("tokens,expect", [
    (("AdaBest", "mu:0.01", "beta:0.6"), dict(mu=0.01, beta=0.6)),
    (("AdaBest",), dict(mu=0.1, beta=0.85)),  # the reference defaults (adabest.py:62)
    (("FedDyn", "alpha:0.05"), dict(alpha=0.05)),
])
def test_arguments_reach_init(tokens, expect):
    """BASELINE config 3's string binds through partial into the static
    init(server_storage, *args, **kwargs)."""
    from fedsim_amd.cli import ingest_algorithm

    ctx = ingest_algorithm(tokens)
    assert ctx.definition.keywords == {k: v for k, v in expect.items()
                                       if f"{k}:" in " ".join(tokens)}
    alg = _instantiate(ctx.definition)
    st = alg.get_server_storage()
    for k, v in expect.items():
        assert st.read(k) == v


def test_fedavg_string_instantiates():
    from fedsim_amd.cli import ingest_algorithm
    from fedsim_amd.distributed.centralized.training import FedAvg

    alg = _instantiate(ingest_algorithm(("FedAvg",)).definition)
    assert isinstance(alg, FedAvg)
    assert alg.get_server_storage().read("cloud_params").numel() == 454


def test_reference_cli_file_form_reaches_this_package():
    """The UNCHANGED reference CLI accepts ``--algorithm path/file:Class``
    (fedsim_cli/utils.py:33-46, 58-59): fedsim_amd/plugins.py is such a
    file, so no patch to the reference is needed to select this path."""
    from fedsim_amd.cli import get_definition, ingest_algorithm
    from fedsim_amd.distributed.centralized.training import AdaBest, FedAvg

    base = os.path.join(REPO, "fedsim_amd", "plugins")
    assert get_definition(base + ":FedAvg", []) is FedAvg
    ctx = ingest_algorithm((base + ":AdaBest", "mu:0.01", "beta:0.6"))
    assert ctx.definition.func is AdaBest and ctx.definition.keywords == dict(mu=0.01, beta=0.6)
