"""The JavaScript side of the boundary: N-API addon + shim (js/)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NODE = shutil.which("node")

pytestmark = pytest.mark.skipif(NODE is None, reason="node not installed")


def _addon():
    import __graft_entry__
    if not __graft_entry__.build_js():
        pytest.skip("node headers not installed (addon cannot be built)")


def test_addon_and_shim_cpu():
    """Addon exports, shim rebinding, and a loud failure without a device."""
    _addon()
    env = dict(os.environ)
    r = subprocess.run([NODE, os.path.join(ROOT, "js", "test_shim_cpu.js")], capture_output=True, text=True,
                       env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok"), r.stdout


@pytest.mark.gpu
def test_js_gpu_parity():
    """Every explicit LP fixture through the JS marshalling and the addon on the device."""
    _addon()
    r = subprocess.run([NODE, os.path.join(ROOT, "js", "test_gpu.js")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok js gpu parity" in r.stdout
