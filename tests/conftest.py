import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and the built libdwpa22000.so")
    config.addinivalue_line("markers", "slow: long-running")
    config.addinivalue_line("markers", "host_routing: a GPU test of the library's small-call host routing")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def dec(v):
    """JSON fixture value -> python (bytes for {'hex': ...})."""
    if isinstance(v, dict) and "hex" in v:
        return bytes.fromhex(v["hex"])
    if isinstance(v, list):
        return [dec(x) for x in v]
    return v


def job_args(j):
    line = j["line"].encode("latin-1")
    keys = [None if k is None else bytes.fromhex(k) for k in j["keys"]]
    pmk = bytes.fromhex(j["pmk"]) if j["pmk"] else False
    return line, keys, pmk, j["nc"]


@pytest.fixture(autouse=True)
def _device_path_for_gpu_tests(request, monkeypatch):
    """GPU tests measure the device path: the library's small-call routing to its host backend (ABI 4,
    dwpa_config.host_max_pmks) is off for them, so a one-key parity check runs the HIP kernels, not the CPU.  Tests
    marked host_routing exercise the routing and set it themselves.  DWPA_TEST_HOST_BACKEND=1 turns it around: every
    check call with a derive goes to the host backend (to run a GPU test's jobs through it on the GPU box's CPU)."""
    if request.node.get_closest_marker("gpu") and not request.node.get_closest_marker("host_routing"):
        host = os.environ.get("DWPA_TEST_HOST_BACKEND") == "1"
        monkeypatch.setenv("DWPA_HOST_MAX_PMKS", "1000000000" if host else "-1")
        monkeypatch.delenv("DWPA_CPU_FALLBACK", raising=False)
    yield


@pytest.fixture(scope="session")
def mixed():
    return load_golden("mixed.json")["jobs"]


@pytest.fixture(scope="session")
def kat():
    return load_golden("kat.json")


@pytest.fixture(scope="session")
def nc_windows():
    return load_golden("nc_windows.json")["jobs"]
