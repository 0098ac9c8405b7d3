"""The library's collective for the sharded branch and bound (gk_comm,
glpk.js_amd/csrc/gk_comm.hip): the TCP all-gather through rank 0 among
several processes on this host, without a device (CPU), and the sharded
search through gk_ios_driver_comm with two ranks on one GPU (the TCP
transport: RCCL refuses two ranks on one device) — every rank ends with the
reference's objective and the same incumbent, including a rank that starts
with no open node."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import load_golden
from glpk_js_amd import gk, problems


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _allgather_worker(rank, size, port, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk as g
        c = g.Comm(None, rank, size, f"127.0.0.1:{port}", g.GK_COMM_TCP)
        out = []
        for k, n in enumerate((8, 1000, 70000)):
            blk = bytes(((rank * 7 + k + i) % 251) for i in range(n))
            out.append(c.allgather(blk))
        q.put((rank, c.backend, out))
        c.close()
    except Exception as e:          # reported to the parent
        q.put((rank, -1, repr(e)))


@pytest.mark.parametrize("size", [2, 3])
def test_comm_tcp_allgather_cpu(size):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_allgather_worker, args=(r, size, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(size)]
    for p in ps:
        p.join(timeout=60)
    for rank, backend, out in res:
        assert backend == gk.GK_COMM_TCP, out
        for k, n in enumerate((8, 1000, 70000)):
            want = [bytes(((r * 7 + k + i) % 251) for i in range(n)) for r in range(size)]
            assert out[k] == want


def _mip_worker(rank, size, port, name, ramp, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk as g, problems as pr
        d = load_golden(os.path.join(root, "tests", "golden", f"mip_{name}.json"))
        ctx = g.Context(0)
        comm = g.Comm(ctx, rank, size, f"127.0.0.1:{port}")
        P = g.GkProblem(ctx, pr.from_fixture(d))
        assert g.glp_simplex(P, g.SMCP(msg_lev=g.GLP_MSG_OFF)) == 0
        ret = g.glp_intopt(P, g.IOCP(msg_lev=g.GLP_MSG_OFF), comm=comm, ramp_nodes=ramp)
        q.put((rank, comm.backend, ret, P.mip_stat, P.mip_obj, P.col_mipx[1:].tolist(), P.mip_stats))
        comm.close()
    except Exception as e:
        q.put((rank, -1, repr(e), None, None, None, None))


@pytest.mark.gpu
@pytest.mark.parametrize("name,ramp", [("gap", 0), ("gap", -1), ("c5s_12x30", 0), ("c5s_12x20", -1)])
def test_gpu_sharded_bnb_library_comm(name, ramp):
    d = load_golden(os.path.join(os.path.dirname(__file__), "golden", f"mip_{name}.json"))
    ref = d["mip"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_mip_worker, args=(r, 2, port, name, ramp, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    xs = []
    for rank, backend, ret, stat, obj, x, stats in res:
        assert backend == gk.GK_COMM_TCP, ret
        assert ret == ref["ret"] and stat == ref["mip_stat"], (rank, ret, stat)
        assert abs(obj - ref["mip_obj"]) <= 1e-9 * max(1.0, abs(ref["mip_obj"])), (rank, obj)
        xs.append(x)
        print(name, "ramp", ramp, "rank", rank, stats)
    assert xs[0] == xs[1], "ranks disagree on the incumbent"
