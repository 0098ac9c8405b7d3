"""C-ABI surface checks that need no GPU: the library loads, exports every
entry point declared in include/glpk_mi355x.h, and refuses to run without
an MI355X instead of falling back to the CPU."""
import ctypes
import os
import re

import pytest

import __graft_entry__
from glpk_js_amd import gk

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "glpk_mi355x.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b(gk_[a-z0-9_]+)\s*\(", src))
    names -= {"gk_col_fn"}
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    __graft_entry__.build_hip()
    return ctypes.CDLL(gk.LIB_PATH)


def test_header_declares_core_entry_points():
    names = declared_functions()
    for n in ("gk_spx_primal", "gk_spx_dual", "gk_bfd_factorize", "gk_bfd_ftran", "gk_bfd_btran",
              "gk_bfd_update", "gk_ios_driver", "gk_last_error"):
        assert n in names


@pytest.mark.parametrize("name", declared_functions())
def test_library_exports_symbol(lib, name):
    assert hasattr(lib, name), f"{name} declared in include/glpk_mi355x.h but not exported"


def test_abi_version():
    L = gk.load_library()
    assert L.gk_abi_version() == 11


def test_no_cpu_fallback_without_device():
    L = gk.load_library()
    if L.gk_device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(gk.GkError):
        gk.Context(0)
