"""Device helpers of gk_device.h (wave-level candidate choice and
reductions) against naive host references: tools/check_wave.hip, built with
hipcc for gfx950 and run on the GPU (full and partial wave activity)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_wave_helpers_match_reference(tmp_path):
    exe = tmp_path / "check_wave"
    src = os.path.join(ROOT, "tools", "check_wave.hip")
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-o", str(exe), src], check=True,
                   timeout=300)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "OK (0 mismatches)" in r.stdout
