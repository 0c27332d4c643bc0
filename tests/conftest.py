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
    from alpenglow_amd import rs
    c = rs.Context(0)
    yield c
    c.close()
