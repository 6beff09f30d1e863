import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(params=["host", "device"])
def state_mode(request, monkeypatch):
    """Per-game pyspiel States host-resident (the default: the library's host
    build of the lane rules) or on device lanes (COUP_STATE_DEVICE=1): the
    facade tests run both."""
    from open_spiel_coup_amd import pyspiel
    monkeypatch.setattr(pyspiel, "DEVICE_STATES", request.param == "device")
    return request.param
