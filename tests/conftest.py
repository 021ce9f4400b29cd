import glob
import os
import sys

import pytest
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)

GOLDEN_DIR = os.path.join(REPO, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI library)")


# fixtures without a model (checked by their own tests)
NON_MODEL = {"discrete_hist"}


def golden_names():
    return sorted(n for n in (os.path.splitext(os.path.basename(p))[0]
                              for p in glob.glob(os.path.join(GOLDEN_DIR, "*.pt"))) if n not in NON_MODEL)


_CACHE = {}


def load_golden(name):
    if name not in _CACHE:
        _CACHE[name] = torch.load(os.path.join(GOLDEN_DIR, f"{name}.pt"), weights_only=True)
    return _CACHE[name]


@pytest.fixture(scope="session")
def golden():
    return load_golden
