"""Multi-process branch and bound (glpk.js_amd/shard.py, gk_ios_driver_sharded).

CPU: the exchange / winner-selection collectives with world_size 2 over gloo.
GPU: two ranks share the box's GPU (gloo for the incumbent exchange) and
solve MIP fixtures sharded; both must return the reference's objective and
the same incumbent."""
import json
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _comm_worker(rank, world, port, q):
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.load_package()
    from glpk_js_amd.shard import TorchComm
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    c = TorchComm()
    out = {}
    # exchange: min of the bests, any-active indicator
    out["ex1"] = c.exchange([5.0, 3.0][rank], [1, 0][rank])
    out["ex2"] = c.exchange([1e300, 7.0][rank], 0)
    out["total"] = c.total(rank + 1)
    # allgather_bytes: fixed-size byte blocks in rank order (the C driver's
    # open-node exchange), through raw addresses
    send = np.frombuffer(bytes([rank + 1] * 5), dtype=np.uint8).copy()
    recv = np.zeros(10, dtype=np.uint8)
    c.allgather_bytes(send.ctypes.data, 5, recv.ctypes.data)
    out["ag"] = recv.tolist()
    # finalize: rank 1 has the better objective; its x is broadcast
    x = np.full(4, float(rank))
    obj, have, xw, win = c.finalize([10.0, 2.0][rank], True, x)
    out["fin"] = (obj, have, xw.tolist(), win)
    # ties go to the lowest rank; no solution anywhere
    out["tie"] = c.finalize(3.0, True, np.full(2, float(rank)))[2].tolist()
    out["none"] = c.finalize(0.0, False, np.zeros(1))[1]
    dist.destroy_process_group()
    q.put((rank, out))


def _run_ranks(target, world, args, timeout):
    """Start `world` spawned ranks, collect one result each; a rank that dies
    or a run that exceeds `timeout` seconds fails the test (the remaining
    ranks are terminated, by their own PIDs)."""
    import queue
    import time
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port) + tuple(args) + (q,)) for r in range(world)]
    for p in ps:
        p.start()
    res, t_end = {}, time.time() + timeout
    try:
        while len(res) < world:
            try:
                r, out = q.get(timeout=1.0)
                res[r] = out
            except queue.Empty:
                dead = [p.exitcode for p in ps if p.exitcode not in (None, 0)]
                assert not dead, f"a rank died with exit code {dead}"
                assert time.time() < t_end, "ranks did not finish in time"
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.terminate()
    for p in ps:
        assert p.exitcode == 0
    return res


def test_torchcomm_gloo_world2():
    res = _run_ranks(_comm_worker, 2, (), 120)
    for r in range(2):
        o = res[r]
        assert o["ex1"] == (3.0, 1)
        assert o["ex2"] == (7.0, 0)
        assert o["total"] == 3.0
        assert o["ag"] == [1] * 5 + [2] * 5
        assert o["fin"] == (2.0, True, [1.0] * 4, 1)
        assert o["tie"] == [0.0, 0.0]
        assert o["none"] is False


def _bnb_worker(rank, world, port, names, q, ramp=0):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.load_package()
    from glpk_js_amd import gk, problems
    from glpk_js_amd.shard import TorchComm
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = TorchComm()
    ctx = gk.Context(0)
    out = {}
    for name in names:
        d = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))
        P = gk.GkProblem(ctx, problems.from_fixture(d))
        assert gk.glp_simplex(P, gk.SMCP(**d["root"]["opts"])) == 0
        ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_OFF), comm=comm, ramp_nodes=ramp)
        out[name] = (ret, P.mip_stat, P.mip_obj, P.col_mipx[1:].tolist(), P.mip_stats)
    dist.destroy_process_group()
    q.put((rank, out))


@pytest.mark.gpu
def test_sharded_bnb_two_ranks_one_gpu():
    names = ["c5s_12x20", "mixint8", "mixint11", "gap", "c5s_12x40", "c5s_12x42"]
    res = _run_ranks(_bnb_worker, 2, (names,), 240)
    for name in names:
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))["mip"]
        a, b = res[0][name], res[1][name]
        assert a[0] == b[0] == ref["ret"]
        assert a[1] == b[1] == ref["mip_stat"]
        assert abs(a[2] - ref["mip_obj"]) <= 1e-9 * max(1.0, abs(ref["mip_obj"]))
        assert a[2] == b[2] and a[3] == b[3], "ranks disagree on the incumbent"
        print(name, "lp_solves", a[4])


def _bnb_worker_root_split(rank, world, port, names, q):
    _bnb_worker(rank, world, port, names, q, ramp=-1)


@pytest.mark.gpu
def test_sharded_bnb_open_node_exchange():
    """Rank 1 starts with nothing (the root alone is split, to rank 0); the
    open-node exchange must hand it work: both ranks solve node LPs, rank 1
    receives nodes, and the result is the reference's (C5s 12x30: 15039)."""
    names = ["c5s_12x30", "gap"]
    res = _run_ranks(_bnb_worker_root_split, 2, (names,), 240)
    for name in names:
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))["mip"]
        a, b = res[0][name], res[1][name]
        assert a[0] == b[0] == ref["ret"]
        assert abs(a[2] - ref["mip_obj"]) <= 1e-9 * max(1.0, abs(ref["mip_obj"]))
        assert a[2] == b[2] and a[3] == b[3], "ranks disagree on the incumbent"
        assert a[4]["local_lp_solves"] > 0 and b[4]["local_lp_solves"] > 0, (a[4], b[4])
        assert b[4]["local_nodes_moved"] > 0, b[4]
        print(name, "rank0", a[4], "rank1", b[4])
