"""Golden fixtures for ``--algorithm`` resolution, from the REFERENCE's own
CLI code (fedsim_cli/utils.py:116-147 ``decode_margs``, :33-69
``parse_class_from_file`` / ``get_definition``, :150-236
``ingest_fed_context``'s algorithm entry: the module list, the base-class
argument guard and the ``partial``).  Build container only.

The reference module imports skopt at top level for fed-tune's search
spaces, and skopt is not installed here.  This generator registers a
minimal ``skopt`` module whose ``space.Real / Integer / Categorical`` only
record their constructor arguments; the resolver's code paths run
unchanged, and a ``key:Real:lo-hi`` hyper-argument is recorded as what the
reference's ``eval`` built: the space's kind and arguments.

Every case runs ``ingest_fed_context`` with only the algorithm set (every
other component None, which the reference resolves to None) and records
the algorithm entry -- name, the class's name and defining module tail, the
partial's keywords, the arguments and hyper-arguments -- or the raised
exception's type and message.  Output: tests/golden/cli_resolution.json.

usage: python -B tools/gen_golden_cli.py
"""
from __future__ import annotations

import json
import os
import sys
import types

sys.dont_write_bytecode = True

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

# -- the algorithm strings a fed-learn user types (README / tests/test_cli.py)
CASES = [
    ["FedAvg"],
    list("FedAvg"),  # click's greedy option hands one string over as characters
    ["AdaBest", "mu:0.01", "beta:0.6"],
    ["AdaBest", "mu:0.1"],
    ["FedNova"],
    ["FedDyn", "mu:0.02"],
    ["FedProx", "mu:0.1"],
    ["FedDF", "global_train_split:valid", "global_epochs:2", "global_batch_size:32"],
    ["FedAvg", "num_clients:5"],          # base-class argument: refused
    ["AdaBest", "device:cpu"],            # base-class argument: refused
    ["AdaBest", "mu:Real:0-1", "beta:0.6"],
    ["AdaBest", "beta:Categorical:0.5-0.9", "mu:Integer:1-3"],
    ["FedAvg", "mu"],                     # malformed
    ["FedAvg", "a:b:c:d"],                # malformed
    ["FedAvg", "flag:true", "n:3", "x:1e-3", "s:hello"],
    ["NoSuchAlgorithm"],
]
FILE_CASES = ["fedsim_amd/plugins:FedAvg", "fedsim_amd/plugins:AdaBest",
              "fedsim_amd/plugins:FedDF"]


class _Space(object):
    def __init__(self, *args, **kw):
        self.args, self.kw = args, kw


def _install_stubs():
    skopt = types.ModuleType("skopt")
    space = types.ModuleType("skopt.space")
    for kind in ("Real", "Integer", "Categorical", "Space"):
        setattr(space, kind, type(kind, (_Space,), {}))
    skopt.space = space
    sys.modules["skopt"], sys.modules["skopt.space"] = skopt, space
    for name in ("fedsim", "fedsim.distributed", "fedsim.distributed.centralized",
                 "fedsim_cli"):
        mod = types.ModuleType(name)
        mod.__path__ = [os.path.join(REF, *name.split("."))]
        sys.modules[name] = mod


def _enc(v):
    if isinstance(v, _Space):
        return {"space": type(v).__name__, "args": list(v.args)}
    return v


def record(ctx):
    d = ctx.definition
    cls = d.func if hasattr(d, "func") else d
    return {"name": ctx.name, "class": cls.__name__,
            "module_tail": cls.__module__.split(".")[-1],
            "keywords": dict(getattr(d, "keywords", {})),
            "arguments": dict(ctx.arguments),
            "harguments": [[k, _enc(v)] for k, v in ctx.harguments.items()]}


def main():
    _install_stubs()
    import importlib

    cu = importlib.import_module("fedsim_cli.utils")
    none9 = [None] * 9
    out = {"cases": [], "file_cases": []}
    for tokens in CASES:
        args = list(none9)
        args[1] = tuple(tokens)
        try:
            res = {"ok": record(cu.ingest_fed_context(*args)["algorithm"])}
        except Exception as e:  # noqa: BLE001 -- the fixture records what was raised
            res = {"raise": type(e).__name__, "message": str(e)}
        out["cases"].append({"tokens": tokens, **res})
    for spec in FILE_CASES:
        path = os.path.join(REPO, spec)
        d = cu.get_definition(path, modules=["fedsim.distributed.centralized.training"])
        out["file_cases"].append({"spec": spec, "class": d.__name__,
                                  "module": d.__module__.rsplit(".", 1)[-1]})
    dst = os.path.join(REPO, "tests", "golden", "cli_resolution.json")
    with open(dst, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(dst, len(out["cases"]), "cases")


if __name__ == "__main__":
    main()
