"""Column-sharded pricing of one LP (gk_bfd_set_comm; SURVEY
§8(e)): every rank holds the problem and the factor, forms its slice of the
non-basic positions of each pivot row with the column pass, and the slices
are all-gathered before the ratio test (glpspx02.js:655-935 — eval_trow,
sort_trow, chuzc — then run on the whole row on every rank).

update_gamma's A w (glpspx02.js:1103-1134) is sharded the same way: each
rank sums the members of the reference space in its slice, and the
partials travel in the same exchange and are summed in rank order.  The
pivot row's values do not depend on the slicing, A w's rounding does (the
sum's association): every rank takes the same pivots (return code, pivot
count and objective bits equal across ranks — the run is deterministic),
and the objective is the reference's 978.22910129338311 (1024 x 4096
generator, tolerance 1e-9 relative).  With one rank (the RCCL test) the
sum is the single-GPU one and the run is the single-GPU column-pass run
(GK_FORCE_COLPASS=1) bit for bit.  Two and three ranks share the one GPU
through the library's TCP transport (RCCL refuses two ranks on one
device); three ranks do not divide n = 4096, so the last slice is the
short one."""
import json
import multiprocessing as mp
import os
import subprocess
import sys

import pytest

from test_comm import free_port

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_OBJ = 978.22910129338311

SINGLE = r"""
import json, sys
sys.path.insert(0, %r)
import __graft_entry__
__graft_entry__.load_package()
from glpk_js_amd import gk, problems
ctx = gk.Context(0)
P = gk.GkProblem(ctx, problems.gen_dense(1024, 4096, seed=42))
ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR))
print(json.dumps({"ret": ret, "it_cnt": P.it_cnt, "obj": float(P.obj_val).hex()}))
"""


SIM = r"""
import json, sys
sys.path.insert(0, %r)
import __graft_entry__
__graft_entry__.load_package()
from glpk_js_amd import gk, problems
ctx = gk.Context(0)
comm = gk.Comm(ctx, 0, 1, "127.0.0.1:%d")
P = gk.GkProblem(ctx, problems.gen_dense(1024, 4096, seed=42))
P.set_comm(comm)
ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR))
print(json.dumps({"ret": ret, "it_cnt": P.it_cnt, "obj": float(P.obj_val).hex(),
                  "ex": int(P.stats().shard_exchanges)}))
"""


def _sim(size):
    """One process forming all `size` ranks' slices in turn (GK_SHARD_SIM)."""
    env = dict(os.environ, GK_SHARD_ONE_RANK="1", GK_SHARD_SIM=str(size))
    r = subprocess.run([sys.executable, "-c", SIM % (ROOT, free_port())], capture_output=True, text=True, env=env,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def _worker(rank, size, port, q):
    try:
        sys.path.insert(0, ROOT)
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk, problems
        ctx = gk.Context(0)
        comm = gk.Comm(ctx, rank, size, f"127.0.0.1:{port}")
        P = gk.GkProblem(ctx, problems.gen_dense(1024, 4096, seed=42))
        P.set_comm(comm)
        ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR))
        q.put((rank, comm.backend, ret, P.it_cnt, float(P.obj_val).hex()))
        del P
        comm.close()
    except Exception as e:                       # noqa: BLE001 (reported to the parent)
        q.put((rank, -1, repr(e), None, None))


def _single():
    env = dict(os.environ, GK_FORCE_COLPASS="1")
    r = subprocess.run([sys.executable, "-c", SINGLE % ROOT], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])


def _rccl_worker(port, q):
    """One rank, GK_COMM_RCCL, the exchange forced on (GK_SHARD_ONE_RANK):
    every pivot row goes through ncclAllGather on the engine's stream."""
    try:
        os.environ["GK_SHARD_ONE_RANK"] = "1"
        sys.path.insert(0, ROOT)
        import torch
        import torch.distributed as dist
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=0, world_size=1)
        import __graft_entry__
        __graft_entry__.load_package()
        from glpk_js_amd import gk, problems
        ctx = gk.Context(0)
        comm = gk.Comm(ctx, 0, 1, f"127.0.0.1:{port + 1}", gk.GK_COMM_RCCL)
        P = gk.GkProblem(ctx, problems.gen_dense(1024, 4096, seed=42))
        P.set_comm(comm)
        ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR))
        ex = int(P.stats().shard_exchanges)
        q.put((0, comm.backend, ret, P.it_cnt, float(P.obj_val).hex(), ex))
        del P
        comm.close()
        dist.destroy_process_group()
    except Exception as e:                       # noqa: BLE001 (reported to the parent)
        q.put((0, -1, repr(e), None, None, None))


@pytest.mark.gpu
def test_gpu_lp_column_sharded_rccl_one_rank():
    """The RCCL branch of the sharded exchange (gk_comm_allgather_dev: the
    all-gather on the engine's stream, no host round trip) on hardware: one
    RCCL rank with the exchange forced on takes the single-GPU column-pass
    pivots, bit for bit, and every dual pivot's row went through it."""
    single = _single()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(free_port(), q))
    p.start()
    rank, backend, ret, it_cnt, obj, ex = q.get(timeout=240)
    p.join(timeout=60)
    assert backend != -1, ret
    from glpk_js_amd import gk
    assert backend == gk.GK_COMM_RCCL
    assert (ret, it_cnt, obj) == (single["ret"], single["it_cnt"], single["obj"]), (ret, it_cnt, obj, single)
    assert ex > 0, ex
    print("rccl one rank: pivots", it_cnt, "exchanges", ex)


@pytest.mark.gpu
@pytest.mark.parametrize("size", [2, 3])
def test_gpu_lp_column_sharded_same_pivots(size):
    single = _single()
    assert single["ret"] == 0
    assert abs(float.fromhex(single["obj"]) - REF_OBJ) <= 1e-9 * REF_OBJ
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_worker, args=(r, size, port, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(size)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for rank, backend, ret, it_cnt, obj in res:
        assert backend != -1, ret
        assert (ret, it_cnt, obj) == res[0][2:], ("ranks disagree", res)
    ret, it_cnt, obj = res[0][2:]
    assert ret == 0
    assert abs(float.fromhex(obj) - REF_OBJ) <= 1e-9 * REF_OBJ, (float.fromhex(obj), REF_OBJ)
    print("size", size, "pivots", it_cnt, "obj", float.fromhex(obj), "single-GPU pivots", single["it_cnt"],
          "bits equal to single", (ret, it_cnt, obj) == (single["ret"], single["it_cnt"], single["obj"]))
    # the simulated ranks (tools/shard_sim_prof.py's mode) are the real ones
    sim = _sim(size)
    assert (sim["ret"], sim["it_cnt"], sim["obj"]) == (ret, it_cnt, obj), (sim, res[0])
    assert sim["ex"] > 0
