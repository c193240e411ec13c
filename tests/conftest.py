import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        manifest = json.load(f)
    with np.load(os.path.join(GOLDEN_DIR, "vectors.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    return manifest, arrays


def golden_cases():
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        return json.load(f)["cases"]


def bits(a):
    return np.ascontiguousarray(a, dtype=np.float32).view(np.uint32)
