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


def _incumbent_worker(rank, size, port, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk as g
        c = g.Comm(None, rank, size, f"127.0.0.1:{port}", g.GK_COMM_TCP)
        seen = [c.incumbent(1.7976931348623157e308)]          # nothing published yet: DBL_MAX
        c.allgather(b"x")                                      # every rank has read the empty word
        vals = {0: [5.0, -3.25, 7.0], 1: [4.0, 2.0, -1e300], 2: [-0.0, 6.0, 1.0]}[rank]
        for v in vals:
            seen.append(c.incumbent(v))
        c.allgather(b"y")                                      # every rank has published all of its values
        seen.append(c.incumbent(1e308))
        q.put((rank, c.shared_incumbent, seen))
        c.close()
    except Exception as e:
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("size", [2, 3])
def test_comm_shared_incumbent_cpu(size):
    """The incumbent word the ranks of one host share between the exchange
    epochs (gk_comm_incumbent): an atomic minimum over an order-preserving
    image of the double — negative values, -0.0 and -1e300 included — so
    every rank reads the best objective any rank has published, and never a
    value worse than its own."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_incumbent_worker, args=(r, size, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(size)]
    for p in ps:
        p.join(timeout=60)
    vals = {0: [5.0, -3.25, 7.0], 1: [4.0, 2.0, -1e300], 2: [-0.0, 6.0, 1.0]}
    best = min(v for r in range(size) for v in vals[r])
    for rank, shared, seen in res:
        assert shared is True, seen
        assert seen[0] == 1.7976931348623157e308
        run = seen[0]
        for v, got in zip(vals[rank], seen[1:4]):
            run = min(run, v)
            assert got <= run                  # at least as good as everything this rank published
        assert seen[-1] == best                # after the barrier: the best of all ranks


def _mip_worker(rank, size, port, name, ramp, q, iocp=None):
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
        ret = g.glp_intopt(P, g.IOCP(msg_lev=g.GLP_MSG_OFF, **(iocp or {})), comm=comm, ramp_nodes=ramp)
        q.put((rank, comm.backend, ret, P.mip_stat, P.mip_obj, P.col_mipx[1:].tolist(), P.mip_stats))
        comm.close()
    except Exception as e:
        q.put((rank, -1, repr(e), None, None, None, None))


@pytest.mark.gpu
@pytest.mark.parametrize("name,ramp", [("gap", 0), ("gap", -1), ("c5s_12x30", 0), ("c5s_12x20", -1), ("c5s_12x40", 0), ("c5s_12x42", 0)])
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


@pytest.mark.gpu
@pytest.mark.parametrize("name,env", [("sparsebig2", {}), ("gap", {"GK_BNB_ENGINE_BYTES": "0"})],
                         ids=["sparsebig2", "gap-engine-forced"])
def test_gpu_sharded_bnb_engine_mode(monkeypatch, name, env):
    """The sharded search with every node LP on the engine (engine mode,
    DESIGN §7: each rank's batch solved concurrently on its own worker
    contexts): both ranks reach the reference's objective and agree on the
    incumbent."""
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    d = load_golden(os.path.join(os.path.dirname(__file__), "golden", f"mip_{name}.json"))
    ref = d["mip"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_mip_worker, args=(r, 2, port, name, 0, q)) for r in range(2)]
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
        assert stats["node_fallbacks"] == stats["lp_solves"], stats      # every node LP on the engine
        xs.append(x)
        print(name, "rank", rank, stats)
    assert xs[0] == xs[1], "ranks disagree on the incumbent"


def _two_mips_worker(rank, size, port, names, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk as g, problems as pr
        ctx = g.Context(0)
        comm = g.Comm(ctx, rank, size, f"127.0.0.1:{port}")
        out = []
        for name in names:
            d = load_golden(os.path.join(root, "tests", "golden", f"mip_{name}.json"))
            P = g.GkProblem(ctx, pr.from_fixture(d))
            assert g.glp_simplex(P, g.SMCP(msg_lev=g.GLP_MSG_OFF)) == 0
            ret = g.glp_intopt(P, g.IOCP(msg_lev=g.GLP_MSG_OFF), comm=comm)
            out.append((name, ret, P.mip_stat, P.mip_obj, P.col_mipx[1:].tolist()))
            del P
        q.put((rank, comm.shared_incumbent, out))
        comm.close()
    except Exception as e:
        q.put((rank, None, repr(e)))


@pytest.mark.gpu
def test_gpu_sharded_two_searches_one_comm():
    """Two different MIPs one after the other on ONE 2-rank communicator
    (the ranks share the incumbent word between epochs): the second search
    must not inherit the first one's incumbent — a maximisation with a large
    objective (C5s, 15039 -> -15039 in minimisation form) before a
    minimisation (gap, 261) would otherwise prune the whole second tree.
    Both searches reach the reference's optimum on both ranks."""
    names = ["c5s_12x20", "gap", "c5s_12x20"]
    refs = {n: load_golden(os.path.join(os.path.dirname(__file__), "golden", f"mip_{n}.json"))["mip"] for n in names}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_two_mips_worker, args=(r, 2, port, names, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for rank, shared, out in res:
        assert shared is True, (rank, out)
        for name, ret, stat, obj, x in out:
            ref = refs[name]
            assert ret == ref["ret"] and stat == ref["mip_stat"], (rank, name, ret, stat)
            assert abs(obj - ref["mip_obj"]) <= 1e-9 * max(1.0, abs(ref["mip_obj"])), (rank, name, obj)
    assert [o[4] for o in res[0][2]] == [o[4] for o in res[1][2]], "ranks disagree on an incumbent"


@pytest.mark.gpu
@pytest.mark.parametrize("name,gap", [("gap", 0.05), ("gap", 0.002), ("c5s_12x20", 0.01)])
def test_gpu_sharded_bnb_mip_gap(name, gap):
    """mip_gap > 0 in a sharded search: the stop is decided inside the sync
    epoch from the gathered incumbents and open bounds, so both ranks leave
    the search at the same epoch and meet in the final all-gather (no rank
    stops on its local gap and leaves the other waiting).  Both return the
    same code (0 or GLP_EMIPGAP) and incumbent, within the gap of the
    reference's optimum."""
    d = load_golden(os.path.join(os.path.dirname(__file__), "golden", f"mip_{name}.json"))
    opt = d["mip"]["mip_obj"]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_mip_worker, args=(r, 2, port, name, 0, q, {"mip_gap": gap})) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(2)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    assert res[0][2] == res[1][2], res
    for rank, backend, ret, stat, obj, x, stats in res:
        assert ret in (0, gk.GLP_EMIPGAP), (rank, ret)
        assert stat == (problems.GLP_OPT if ret == 0 else problems.GLP_FEAS), (rank, stat)
        assert abs(obj - opt) / (abs(obj) + 2.220446049250313e-16) <= gap + 1e-12, (rank, obj, opt)
        if ret == 0:
            assert abs(obj - opt) <= 1e-9 * max(1.0, abs(opt))
    assert res[0][5] == res[1][5], "ranks disagree on the incumbent"


@pytest.mark.gpu
def test_gpu_rccl_one_rank_after_torch_nccl():
    """The RCCL transport of gk_comm on hardware: torch.distributed first
    initialises its own NCCL (= RCCL) group in this process, then a one-rank
    gk_comm with GK_COMM_RCCL (ncclCommInitRank, nranks = 1, over the
    library's own dlopen'd librccl) all-gathers blocks and carries a
    glp_intopt through gk_ios_driver_comm (its final all-gather on RCCL)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_one_rank_worker, args=(free_port(), q))
    p.start()
    res = q.get(timeout=240)
    p.join(timeout=60)
    assert res[0] == "ok", res
    backend, blocks, ret, stat, obj, ref = res[1:]
    assert backend == gk.GK_COMM_RCCL
    assert blocks == [b"rccl-one-rank" * 100]
    assert ret == 0 and stat == problems.GLP_OPT
    assert abs(obj - ref) <= 1e-9 * max(1.0, abs(ref))


def _rccl_one_rank_worker(port, q):
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        t = torch.ones(4, device="cuda")
        dist.all_reduce(t)
        torch.cuda.synchronize()
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk as g, problems as pr
        ctx = g.Context(0)
        comm = g.Comm(ctx, 0, 1, f"127.0.0.1:{port + 1}", g.GK_COMM_RCCL)
        blocks = comm.allgather(b"rccl-one-rank" * 100)
        d = load_golden(os.path.join(root, "tests", "golden", "mip_gap.json"))
        P = g.GkProblem(ctx, pr.from_fixture(d))
        assert g.glp_simplex(P, g.SMCP(msg_lev=g.GLP_MSG_OFF)) == 0
        ret = g.glp_intopt(P, g.IOCP(msg_lev=g.GLP_MSG_OFF), comm=comm)
        q.put(("ok", comm.backend, blocks, ret, P.mip_stat, P.mip_obj, d["mip"]["mip_obj"]))
        comm.close()
        dist.destroy_process_group()
    except Exception as e:
        q.put(("error", repr(e)))
