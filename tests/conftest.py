"""pytest configuration: markers and import paths.

  -m "not gpu"  oracle vs golden vectors / the reference build, ABI and export
                checks, host logic, gloo multi-process tests (runs anywhere)
  -m gpu        parity of libmq's HIP path against the oracle (needs a gfx950 GPU)
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs libmq's HIP path")
    config.addinivalue_line("markers", "big: full-size (1e9-row) case")


@pytest.fixture(scope="session")
def refcpu():
    import refcpu as m
    m.build()
    return m


@pytest.fixture(scope="session")
def goldens():
    import json
    return json.load(open(os.path.join(ROOT, "tests", "golden", "goldens.json")))
