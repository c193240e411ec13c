"""Small helpers the reference's utils package exports next to the
aggregators (fedsim/utils/random_utils.py:10-26, import_utils.py:8-22)."""
from __future__ import annotations

import importlib
import random

import numpy as np
import torch


def set_seed(seed, use_cuda) -> None:
    """Seed numpy, ``random`` and torch (and every HIP device, with
    deterministic cuDNN/MIOpen selection, when ``use_cuda``)."""
    np.random.seed(seed)
    random.seed(seed)
    torch.manual_seed(seed)
    if use_cuda:
        torch.backends.cudnn.deterministic = True
        torch.cuda.manual_seed_all(seed)


def get_from_module(module_name, entry_name):
    """``getattr(import_module(module_name), entry_name)``, or None when the
    module has no such member (ImportError still propagates)."""
    return getattr(importlib.import_module(module_name), entry_name, None)
