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


def test_js_native_presolver_cpu():
    """The native preprocessor through the JS marshalling (gk_core npp*,
    bound by the shim to the reference's npp_* names): reduced problems and
    recovered solutions of the presolve_* / mippre_* reference runs."""
    _addon()
    r = subprocess.run([NODE, os.path.join(ROOT, "js", "test_npp_cpu.js")], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.startswith("ok js npp"), r.stdout


@pytest.mark.gpu
def test_js_gpu_parity():
    """Every explicit LP fixture through the JS marshalling and the addon on the device."""
    _addon()
    r = subprocess.run([NODE, os.path.join(ROOT, "js", "test_gpu.js")], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok js gpu parity" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("ramp", ["0", "-1"], ids=["split", "rank0-starts-with-all"])
def test_js_sharded_bnb_two_processes(ramp):
    """glp_intopt sharded over two node processes (one GPU here: the TCP
    transport of the library's collective; RCCL between distinct GPUs) through
    the N-API boundary, on gap and C5s 12x30: both ranks return the
    reference's objective and the same incumbent, also when rank 1 starts
    with no open node (GK_RAMP_NODES < 0: the open-node exchange feeds it)."""
    import json
    import socket
    _addon()
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    names = ["gap", "c5s_12x30"]
    procs = []
    for rank in (0, 1):
        env = dict(os.environ, GK_WORLD_SIZE="2", GK_RANK=str(rank), GK_COMM_ADDR=f"127.0.0.1:{port}",
                   GK_RAMP_NODES=ramp)
        procs.append(subprocess.Popen([NODE, os.path.join(ROOT, "js", "test_sharded.js")] + names, env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True))
    outs = [p.communicate(timeout=300) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, o + e
    res = [[json.loads(line) for line in o.strip().splitlines()] for o, _ in outs]
    for k, name in enumerate(names):
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))["mip"]
        a, b = res[0][k], res[1][k]
        for r in (a, b):
            assert r["name"] == name and r["ret"] == ref["ret"] and r["mip_stat"] == ref["mip_stat"], r
            assert abs(r["mip_obj"] - ref["mip_obj"]) <= 1e-9 * max(1.0, abs(ref["mip_obj"])), r["mip_obj"]
        assert a["x"] == b["x"], f"{name}: the ranks disagree on the incumbent"
