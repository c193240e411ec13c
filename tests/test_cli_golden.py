"""``--algorithm`` resolution (fedsim_amd/cli.py) against the REFERENCE's own
resolver: tests/golden/cli_resolution.json is what fedsim_cli/utils.py's
``ingest_fed_context`` (decode_margs :116-147, get_definition :49-69, the
module list :186-192, the base-class guard :221-230, the partial :235-236)
returned or raised for each token list, run in the build container by
tools/gen_golden_cli.py (skopt, absent here, replaced by a stub that records
the search spaces' arguments; fed-learn never builds them).

Each case must give the same algorithm entry: name, class (this package's
class of the same name, defined in the module of the same name), partial
keywords, arguments and hyper-arguments -- or the same exception type and
message (module paths normalised: ``fedsim_amd.`` for ``fedsim.``).  The
reference resolver's ``path/file:Class`` form on fedsim_amd/plugins.py gives
the same classes as this package's own lookup.
"""
import json
import os

import pytest

from conftest import GOLDEN_DIR, REPO

with open(os.path.join(GOLDEN_DIR, "cli_resolution.json")) as _f:
    _GOLD = json.load(_f)


def _norm(msg: str) -> str:
    msg = msg.replace("fedsim_amd.", "fedsim.")
    return msg.split(" in [")[0]  # the module list differs by design (this package first)


def _record(ctx):
    from fedsim_amd.cli import SearchSpace

    d = ctx.definition
    cls = d.func
    enc = (lambda v: {"space": v.kind, "args": list(v.args)} if isinstance(v, SearchSpace)
           else v)
    return {"name": ctx.name, "class": cls.__name__,
            "module_tail": cls.__module__.split(".")[-1], "keywords": dict(d.keywords),
            "arguments": dict(ctx.arguments),
            "harguments": [[k, enc(v)] for k, v in ctx.harguments.items()]}


@pytest.mark.parametrize("case", _GOLD["cases"], ids=[" ".join(c["tokens"]) for c in _GOLD["cases"]])
def test_algorithm_entry_matches_reference_resolver(case):
    from fedsim_amd.cli import ingest_algorithm
    from fedsim_amd.distributed.centralized import training

    try:
        got = {"ok": _record(ingest_algorithm(tuple(case["tokens"])))}
    except Exception as e:  # noqa: BLE001 -- compared with what the reference raised
        got = {"raise": type(e).__name__, "message": _norm(str(e))}
    want = {k: v for k, v in case.items() if k != "tokens"}
    if "message" in want:
        want["message"] = _norm(want["message"])
    assert got == want
    if "ok" in got:  # the MI355X path's class, not the reference's
        assert got["ok"]["class"] in training.__all__ or hasattr(training, got["ok"]["class"])
        assert ingest_algorithm(tuple(case["tokens"])).definition.func.__module__.startswith(
            "fedsim_amd.")


@pytest.mark.parametrize("case", _GOLD["file_cases"], ids=[c["spec"] for c in _GOLD["file_cases"]])
def test_file_form_gives_this_package_classes(case):
    from fedsim_amd.cli import get_definition
    from fedsim_amd.distributed.centralized import training

    d = get_definition(os.path.join(REPO, case["spec"]), modules=[])
    assert d.__name__ == case["class"] and d.__module__.rsplit(".", 1)[-1] == case["module"]
    assert d is getattr(training, case["class"])
