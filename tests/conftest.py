import base64
import json
import os
import sys
import zlib

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "java-rsync_amd"))
sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) device")
    config.addinivalue_line("markers", "slow: long-running parity sweep")


_GOLD = None


def golden():
    """tests/golden/cases.json with input blobs decoded (bytes)."""
    global _GOLD
    if _GOLD is None:
        with open(os.path.join(ROOT, "tests", "golden", "cases.json")) as f:
            d = json.load(f)
        blobs = {k: zlib.decompress(base64.b64decode(v)) for k, v in d["blobs"].items()}
        for c in d["cases"]:
            c["basis_bytes"] = None if c["basis"] is None else blobs[c["basis"]]
            c["src_bytes"] = blobs[c["src"]]
            c["seed_bytes"] = bytes.fromhex(c["seed"])
        _GOLD = d["cases"]
    return _GOLD


@pytest.fixture(scope="session")
def golden_cases():
    return golden()


def pytest_collection_finish(session):
    """Initialise torch's GPU runtime before any test touches librsynchip.

    torch ships its own HIP/HSA runtime (torch/lib) and librsynchip links the system one (/opt/rocm/lib).
    Measured on the MI355X box: when the system runtime initialises first (a librsynchip test before the
    first torch test), torch's initialisation then fails with "No HIP GPUs are available"; in the other
    order both work (bench.py and smoke() already initialise torch first)."""
    if not any(item.get_closest_marker("gpu") for item in session.items):
        return
    try:
        import torch
        if torch.cuda.is_available():
            torch.cuda.init()
    except Exception:  # no usable GPU: the gpu tests report it themselves
        pass


@pytest.fixture
def rsh_opt():
    """Sets librsynchip options (include/rsync_hip_debug.h) for one test: rsh_opt("k1_gather", 0).  Every option
    is back at its default afterwards."""
    import rsync_hip as R

    def setter(name, value):
        R.set_option(name, int(value))

    yield setter
    R.reset_options()
