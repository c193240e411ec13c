"""The algorithm classes under absolute imports, for the reference CLI's
``--algorithm path/file:Class`` form (fedsim_cli/utils.py:33-46 loads the
file as a stand-alone module, so it cannot use relative imports):

    fedsim-cli fed-learn --algorithm /path/to/repo/fedsim_amd/plugins:FedAvg
    fedsim-cli fed-learn --algorithm /path/to/repo/fedsim_amd/plugins:AdaBest mu:0.01 beta:0.6

selects the MI355X aggregation path with the CLI unchanged (the repository
root must be importable, e.g. on PYTHONPATH)."""
from fedsim_amd.distributed.centralized.training import (  # noqa: F401
    AdaBest,
    FedAvg,
    FedDF,
    FedDyn,
    FedNova,
    FedProx,
)
