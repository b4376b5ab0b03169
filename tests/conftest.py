import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reconcile-rs_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "vectors.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle_lib():
    lib = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    import oracle
    return oracle


@pytest.fixture(scope="session")
def rsos_hip_lib():
    lib = os.path.join(ROOT, "reconcile-rs_amd", "rsos_hip", "_lib", "librsos_hip.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "reconcile-rs_amd")], check=True)
    import rsos_hip
    rsos_hip.lib()
    return rsos_hip


@pytest.fixture(scope="session")
def gpu(rsos_hip_lib):
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test on a host without a GPU")
    return torch.device("cuda:0")
