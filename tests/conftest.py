"""Test configuration.

Markers: ``gpu`` -- needs a real MI355X (run with ``-m gpu``); everything else runs on
CPU.  The oracle (oracle/) is importable here as the checker only.
"""

import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD GPU (MI355X) and the built HIP library")


@pytest.fixture(scope="session")
def golden():
    import json
    with open(os.path.join(ROOT, "tests", "golden", "rs_golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def ctx():
    import torch

    from alpenglow_amd import rs
    # torch's HIP runtime first: when the library's context initialises the device before
    # torch does, torch then reports "No HIP GPUs are available" in that process
    torch.zeros(1, device="cuda:0")
    c = rs.Context(0)
    yield c
    c.close()
