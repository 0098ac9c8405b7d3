import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")

import __graft_entry__  # noqa: E402

__graft_entry__.load_package()


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def golden_files(prefix):
    return sorted(glob.glob(os.path.join(GOLDEN, prefix + "*.json")))


def load_golden(path):
    with open(path) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import orcpy
    orcpy.build()
    return orcpy


@pytest.fixture(scope="session")
def gpu_ctx():
    __graft_entry__.build_hip()
    from glpk_js_amd import gk
    return gk.Context(0)
