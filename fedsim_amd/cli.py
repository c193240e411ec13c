"""``--algorithm`` resolution of ``fedsim-cli fed-learn`` onto this package.

The reference CLI turns ``--algorithm FedAvg`` or ``--algorithm AdaBest
mu:0.01 beta:0.6`` into ``partial(AlgorithmClass, mu=0.01, beta=0.6)``
(fedsim_cli/utils.py:116-147 ``decode_margs``, :49-69 ``get_definition``,
:186-192 the module list, :221-230 the base-class argument guard, :235-236 the
``partial``) and instantiates it with the run's base-class arguments
(fedsim_cli/fed_learn.py:372-389), which hands the algorithm arguments to the
class's static ``init(server_storage, *args, **kwargs)``.

This module restates that resolution with this package's training module
FIRST in the lookup list, so the same strings select the MI355X path.  Two
ways to reach it from the unchanged reference CLI are documented in
INTEGRATION.md §3: the reference resolver's own ``path/file:Class`` form
pointing at ``fedsim_amd/plugins.py`` (no patch at all), or one line
adding ``fedsim_amd.distributed.centralized.training`` to the module list.

Parity: pinned to the reference's own resolver.  tools/gen_golden_cli.py
runs fedsim_cli/utils.py's ``ingest_fed_context`` in the build container
(skopt, absent here and used only for fed-tune's search spaces, replaced by
a stub that records their arguments) on 16 token lists; this restatement
gives the same algorithm entries and raises the same exceptions
(tests/test_cli_golden.py, tests/golden/cli_resolution.json).
Hyper-parameter search spaces (``lr:Real:0-1``, used only by fed-tune) are
parsed into ``SearchSpace`` tuples instead of ``eval``'d skopt objects, with
the same kind and arguments.
"""
from __future__ import annotations

import importlib.util
import inspect
import os
from collections import OrderedDict
from functools import partial
from typing import NamedTuple, Optional, Sequence, Tuple

import yaml

from .utils.misc import get_from_module

ALGORITHM_MODULES = [
    "fedsim_amd.distributed.centralized.training",
    "fedsim.distributed.centralized.training",
    "fedsim.distributed.decentralized.training",
]
SPACES = ("Real", "Integer", "Categorical")


class SearchSpace(NamedTuple):
    """``key:Real:lo-hi`` -- what the reference eval's into skopt.space.Real(lo, hi)."""

    kind: str
    args: Tuple


class ObjectContext(NamedTuple):
    name: str
    definition: object
    arguments: dict
    harguments: "OrderedDict"


def _space(kind: str, spec: str) -> SearchSpace:
    if kind not in SPACES:
        raise Exception(f"{kind} is not a search space ({', '.join(SPACES)})")
    vals = []
    for tok in spec.split("-"):
        v = yaml.safe_load(tok)
        vals.append(v)
    return SearchSpace(kind, tuple(vals))


def decode_margs(obj_and_args: Optional[Sequence[str]]):
    """``("AdaBest", "mu:0.01", "beta:0.6")`` -> ``("AdaBest", {"mu": 0.01,
    "beta": 0.6}, OrderedDict())``.  A name that arrives split into single
    characters (click's greedy option on one string) is joined back, as the
    reference does."""
    if obj_and_args is None:
        return None, None, None
    tokens = list(obj_and_args)
    if any(len(t) > 1 for t in tokens):
        name, arg_list = tokens[0], tokens[1:]
    else:
        name, arg_list = "".join(tokens), []
    args, hargs = dict(), OrderedDict()
    for arg in arg_list:
        if ":" not in arg:
            raise Exception(f"{arg} is invalid argument!")
        parts = arg.split(":")
        if not 2 <= len(parts) <= 3:
            raise Exception(f"{arg} does not seem to be enetered correctly!")
        if len(parts) == 3:
            hargs[parts[0]] = _space(parts[1], parts[2])
        else:
            args[parts[0]] = yaml.safe_load(parts[1])
    return name, args, hargs


def parse_class_from_file(s: str):
    """``path/to/file:Class`` -> the class, or None if the file is absent."""
    f, c = s.split(":")
    path = f + ".py"
    if not os.path.exists(path):
        return None
    spec = importlib.util.spec_from_file_location(os.path.dirname(path).replace(os.sep, "."),
                                                  path)
    module = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(module)
    return getattr(module, c)


def get_definition(name, modules):
    if name is None:
        return None
    if not isinstance(modules, list):
        modules = [modules]
    definition = None
    if ":" in name:
        definition = parse_class_from_file(name)
    else:
        for module in modules:
            try:
                definition = get_from_module(module, name)
            except ImportError:  # e.g. the reference package is not installed
                definition = None
            if definition is not None:
                break
    if definition is None:
        raise Exception(f"{name} is not defined in {modules}!")
    return definition


def ingest_algorithm(tokens: Sequence[str], modules=None) -> ObjectContext:
    """The ``algorithm`` entry of the reference's ingest_fed_context: decoded,
    resolved (this package first), guarded against overriding the base
    class's own arguments, and partially bound."""
    name, args, hargs = decode_margs(tokens)
    definition = get_definition(name, list(modules or ALGORITHM_MODULES))
    base = inspect.getmro(definition)[-2]  # the class right below object
    base_args = set(inspect.signature(base).parameters.keys())
    for key in args:
        if key in base_args:
            raise Exception(
                f"Not allowed to change parameters of {base} which is the parent of "
                f"algorithm class {definition}.Check other cli options")
    return ObjectContext(name, partial(definition, **args), args, hargs)
