import gzip
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "golden.jsonl.gz")
GOLDEN_TIES = os.path.join(ROOT, "tests", "golden", "spm_ties.npz")
GOLDEN_NFKC = os.path.join(ROOT, "tests", "golden", "golden_nfkc.jsonl.gz")
BPE_PATH = os.path.join(ROOT, "models", "akshar.json")
SPM_PATH = os.path.join(ROOT, "models", "akshar.model")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X) and the built HIP engine")
    # The CPU suite (-m "not gpu") is mostly the host emulation of the tile kernels (64 threads per
    # emulated wave): it runs on 4 pytest-xdist workers unless -n was given, so the whole suite takes
    # minutes, not a quarter of an hour. GPU runs stay in one process.
    if (os.environ.get("PYTEST_XDIST_WORKER") is None and config.pluginmanager.hasplugin("xdist")
            and config.getoption("markexpr", "") == "not gpu" and not config.getoption("numprocesses", None)
            and not config.getoption("collectonly") and os.environ.get("AK_TEST_SERIAL") != "1"):
        config.option.numprocesses = 4
        config.option.dist = "load"
        config.option.tx = ["popen"] * 4


@pytest.fixture(scope="session")
def golden():
    with gzip.open(GOLDEN, "rt", encoding="utf-8") as f:
        return [json.loads(line) for line in f]


@pytest.fixture(scope="session")
def golden_nfkc():
    with gzip.open(GOLDEN_NFKC, "rt", encoding="utf-8") as f:
        return [json.loads(line) for line in f]


@pytest.fixture(scope="session")
def bpe_model():
    from akshar_amd.models import BPEModel
    return BPEModel(BPE_PATH)


@pytest.fixture(scope="session")
def spm_model():
    from akshar_amd.models import SPMModel
    return SPMModel(SPM_PATH)
