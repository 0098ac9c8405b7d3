#!/usr/bin/env python3
"""Benchmark of the MI355X simplex core on BASELINE.json's HBM-roofline
configuration: the C3 dense random LP, m=4096, n=16384, fp64, dual simplex.

One *step* = one glp_simplex(SMCP{meth: GLP_DUAL, it_lim: P}) call that
continues from the basis the previous step left (P = 100 pivots by default),
i.e. the reference's own it_lim-bounded timing run ("first 300
pivots"), on inputs already resident in HBM.  `value` is simplex pivots/s of
the whole job: every rank solves its own replica (seed 42 + rank), so per-GPU
work is fixed as N grows ("scaling": "weak", replicas only for a single LP).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
(torchrun-launched for N > 1; RANK/LOCAL_RANK/WORLD_SIZE from the env).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import __graft_entry__  # noqa: E402

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# the two kernels that carry the headline pivot's time; the roofline is
# priced on whichever of them has the larger event time in the timed region
# (k_dual_row in rounds 5 and 6)
UPDATE_KERNEL = "k_dual_update"
ROW_KERNEL = "k_dual_row"
ROUND = "r06"
# the C port (oracle/) against the reference itself, both on one core of the
# build container on C3 from the slack basis: the port 285.8 pivots/s over a
# 20 s window (6,874 pivots, init_csa included), the reference node 9.4
# pivots/s over its first 300 pivots; later pivots cost more, so
# the ratio on the same window is larger still
PORT_OVER_NODE = 30.4


def load_profile(args):
    """rocprofv3 numbers of this exact command from profiles/ (written by
    tools/profile_round.sh with the command it profiled); {} when the
    committed profile is of a different command."""
    out = {}
    meta_p = os.path.join(ROOT, "profiles", f"{ROUND}_profile_meta.json")
    try:
        meta = json.load(open(meta_p))
    except Exception:
        return out
    want = {"steps": args.steps, "warmup": args.warmup, "pivots_per_step": args.pivots_per_step,
            "m": args.m, "n": args.n}
    if any(meta.get("args", {}).get(k) != v for k, v in want.items()):
        return out
    out["source"] = f"profiles/{ROUND}_kernel_stats_timed.json, profiles/{ROUND}_pmc_traffic.json " \
                    f"(command: {meta.get('cmd')}; head {meta.get('head')})"
    for kern in (UPDATE_KERNEL, ROW_KERNEL):
        try:
            stats = json.load(open(os.path.join(ROOT, "profiles", f"{ROUND}_kernel_stats_timed.json")))
            key = next(k for k in stats if k.startswith(kern))
            out.setdefault(kern, {})["rocprof_ms"] = round(stats[key]["avg_ns"] / 1e6, 5)
        except Exception:
            pass
        try:
            tr = json.load(open(os.path.join(ROOT, "profiles", f"{ROUND}_pmc_traffic.json")))["kernels"]
            key = next(k for k in tr if k.startswith(kern))
            out.setdefault(kern, {})["traffic"] = tr[key]["bytes_per_launch"]
        except Exception:
            pass
    return out


LEG = {"name": "setup"}


def leg(name):
    LEG["name"] = name


def log(rank, *a):
    if rank == 0:
        print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pivots-per-step", type=int, default=100)
    ap.add_argument("--m", type=int, default=4096)
    ap.add_argument("--n", type=int, default=16384)
    ap.add_argument("--cpu-seconds", type=float, default=20.0, help="bounded CPU-baseline sample (oracle)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))

    # torch first: the library then binds to the HIP runtime torch carries
    # (one runtime per process)
    import torch
    import torch.distributed as dist
    ndev = torch.cuda.device_count() if torch.cuda.is_available() else 0
    device = local_rank % max(1, ndev)          # more ranks than GPUs only in rehearsals
    if world > 1:
        backend = os.environ.get("GK_DIST_BACKEND") or ("nccl" if ndev else "gloo")
        dist.init_process_group(backend=backend)
    if ndev:
        torch.cuda.set_device(device)

    __graft_entry__.build_hip()
    __graft_entry__.load_package()
    from glpk_js_amd import gk, problems
    # the solver's printed lines (glp_simplex's xprintf) go to stderr: stdout
    # carries the one JSON line
    # (a warning is tagged with the bench leg and the iteration count at the
    # start of the call that printed it, so that it can be traced)
    gk.glp_set_print_func(lambda s: print(s + (f"  [{LEG['name']}]" if s.startswith(("Warning", "Error")) else ""),
                                          file=sys.stderr))

    def barrier():
        if world > 1:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    t_gen = time.time()
    prob = problems.gen_dense(args.m, args.n, seed=42 + rank)
    ctx = gk.Context(device)
    P = gk.GkProblem(ctx, prob)
    # the steps change the basis only: the bounds / costs version is declared
    # once (gk_lp.b_version, what the JS shim maintains on every mutator), so
    # each call skips init_csa's rebuild and its comparison with the resident
    # working set
    P.touch_bounds()
    assert P.factorize() == 0
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=args.pivots_per_step, msg_lev=gk.GLP_MSG_ERR)
    log(rank, f"[bench] generated C3 {args.m}x{args.n} in {time.time() - t_gen:.1f}s")

    restarts = [0]

    def step(tag="headline"):
        it0 = P.it_cnt
        leg(f"{tag} step from it_cnt={it0}")
        ret = gk.glp_simplex(P, parm)
        if ret not in (0, 8):
            raise RuntimeError(f"glp_simplex returned {ret}")
        if ret == 0:                    # optimum reached: restart from the slack basis
            P.row_stat[1:] = problems.GLP_BS
            P.col_stat[1:] = problems.GLP_NL
            P.valid = 0
            assert P.factorize() == 0
            restarts[0] += 1
        return P.it_cnt - it0

    for _ in range(args.warmup):
        step()
    # the basis the timed region starts from: the roofline and cross-check
    # passes below replay the same window of pivots from it
    saved = (P.row_stat.copy(), P.col_stat.copy(), P.it_cnt)

    def rewind():
        P.row_stat[:] = saved[0]
        P.col_stat[:] = saved[1]
        P.it_cnt = saved[2]
        P.valid = 0
        assert P.factorize() == 0

    ctx.mark(1)                         # timed region starts (kernel-trace window)
    barrier()
    t0 = time.perf_counter()
    piv = 0
    split = {"init": 0.0, "eval": 0.0, "batches": 0.0, "reinvert": 0.0, "total": 0.0}
    reinv = 0
    resident, skipped = 0, 0
    for _ in range(args.steps):
        piv += step()
        s_ = P.stats()
        split["init"] += s_.seconds_init
        split["eval"] += s_.seconds_eval
        split["batches"] += s_.seconds_batches
        split["reinvert"] += s_.seconds_reinvert
        split["total"] += s_.seconds_total
        reinv += s_.reinversions
        resident += s_.resident
        skipped += s_.evals_skipped
    barrier()
    dt = time.perf_counter() - t0
    ctx.mark(2)                         # timed region ends
    st = P.stats()

    # roofline pass: the same steps again (continuing), with the pivot
    # kernels' device-clock stamps and byte accounting on (gk_bfd_profile(4):
    # stores and a reduction on every pivot's critical path, so never inside
    # the timed region), graphs kept as in the timed region
    dev = {"ms": 0.0, "ms_b": 0.0, "launches": 0, "bytes": 0.0, "ms_r": 0.0, "launches_r": 0, "bytes_pivots": 0.0,
           "upd_ms": 0.0, "upd_launches": 0, "upd_bytes": 0.0, "pivots": 0}
    if rank == 0:
        rewind()
        P.profile(4)
        for _ in range(args.steps):
            dev["pivots"] += step("roofline pass")
            s_ = P.stats()
            dev["ms"] += s_.trow_dev_ms
            dev["ms_b"] += s_.trow_dev_ms_b
            dev["launches"] += s_.trow_dev_launches
            dev["bytes"] += s_.trow_bytes
            dev["ms_r"] += s_.trow_dev_ms_r
            dev["launches_r"] += s_.trow_dev_launches_r
            dev["bytes_pivots"] += s_.bytes_pivots
            dev["upd_ms"] += s_.upd_dev_ms
            dev["upd_launches"] += s_.upd_dev_launches
            dev["upd_bytes"] += s_.upd_bytes
        P.profile(0)

    # event pass: the same steps again, launched eagerly (event nodes inside
    # captured graphs are not timed by every HIP runtime), the pivot-row and
    # the fused update kernels each through hipExtLaunchKernelGGL with a
    # start and a stop event on the engine stream — the command processor's
    # timestamps of the dispatch itself, which is what a profiler reports
    trow = {"ms": 0.0, "launches": 0, "bytes": 0.0, "upd_ms": 0.0, "upd_launches": 0}
    if rank == 0:
        rewind()
        P.profile(True)
        for _ in range(args.steps):
            step("events pass")
            s_ = P.stats()
            trow["ms"] += s_.trow_ms
            trow["launches"] += s_.trow_launches
            trow["bytes"] += s_.trow_bytes
            trow["upd_ms"] += s_.upd_dev_ms
            trow["upd_launches"] += s_.upd_dev_launches
        P.profile(False)

    tot_piv, max_dt = piv, dt
    if world > 1:
        t = torch.tensor([float(piv)], dtype=torch.float64, device="cuda" if torch.cuda.is_available() else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        tot_piv = int(t.item())
        t = torch.tensor([dt], dtype=torch.float64, device=t.device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        max_dt = float(t.item())
    value = tot_piv / max_dt

    # roofline of the dominant kernel: of the two kernels that carry the
    # pivot's time, k_dual_row (chuzr, rho, the pivot row over the rows of AT
    # in the support of rho) and k_dual_update (pass-2 choice, FTRAN of the
    # entering column and the PSE vector over the dense columns of inv(B),
    # their product-form update, update_bbar / cbar / gamma, the next chuzr
    # candidates), the one with the larger total event time.  Per launch:
    # algorithmic bytes accumulated on the device in the stamp pass (DESIGN.md
    # §4: 8 ns n for k_dual_row; 16 m ns + 64 m + 29 n for k_dual_update, over
    # every update launch) over the duration between the kernel's start and
    # stop events (event pass).  The device-clock stamp timings and the
    # committed rocprof averages of the same command are reported beside it.
    roof = None
    kern = {}
    if rank == 0:
        for which, name in ((0, "pivot_row_pass"), (1, "dual_pse_A_w_dense"), (2, "ftran_Binv_x_dense"),
                            (3, "binv_rank1_dense")):
            ms_k, b_k = P.time_kernel(which, reps=10)
            kern[name] = {"ms": round(ms_k, 5), "bytes": b_k, "GBps": round(b_k / (ms_k * 1e-3) / 1e9, 1)}
        prof = load_profile(args)
        nl = max(1, dev["launches"])
        nr_ = max(1, dev["launches_r"])
        nu_ev = max(1, trow["upd_launches"])
        ne = max(1, trow["launches"])
        cands = {
            ROW_KERNEL: {"desc": "chuzr, rho = row p of inv(B), pivot row trow = -rho' N over the rows of A in the "
                                 "support of rho, ratio-test candidates",
                         "bytes": dev["bytes"] / nl, "ms": trow["ms"] / ne, "launches": trow["launches"],
                         "stamp_ms": dev["ms_r"] / nr_,
                         "stamp_timing": "last block exit of the kernel before it to its own last block exit"},
            UPDATE_KERNEL: {"desc": "pass-2 choice, FTRAN of the entering column and the PSE vector over the dense "
                                  "columns of inv(B), their product-form update, update_bbar/cbar/gamma, next chuzr "
                                  "candidates: one kernel",
                          "bytes": dev["upd_bytes"] / nu_ev, "ms": trow["upd_ms"] / nu_ev,
                          "launches": trow["upd_launches"],
                          "stamp_ms": dev["upd_ms"] / max(1, dev["upd_launches"]),
                          "stamp_timing": "block 0 entry to the last block exit"},
        }

        def entry(k):
            c = cands[k]
            pk = prof.get(k, {})
            ach = c["bytes"] / (c["ms"] * 1e-3) / 1e9 if c["ms"] > 0 else 0.0
            return {"kernel": k + " (" + c["desc"] + ")", "achieved": round(ach, 1),
                    "frac": round(ach / HBM_PEAK_GBS, 4), "ms_per_launch": round(c["ms"], 5),
                    "launches": c["launches"], "bytes_per_launch": round(c["bytes"]),
                    "traffic": pk.get("traffic"),
                    "traffic_over_algorithmic": round(pk["traffic"] / c["bytes"], 3)
                    if pk.get("traffic") and c["bytes"] > 0 else None,
                    "timing": "hipExtLaunchKernelGGL start/stop events of every launch of the event pass (the timed "
                              "region's steps replayed eagerly on the engine stream)",
                    "stamp_ms_per_launch": round(c["stamp_ms"], 5), "stamp_timing": c["stamp_timing"],
                    "rocprof_ms_per_launch": pk.get("rocprof_ms"),
                    "rocprof_frac": round(c["bytes"] / (pk["rocprof_ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
                    if pk.get("rocprof_ms") else None}

        dom = max(cands, key=lambda k: cands[k]["ms"] * cands[k]["launches"])
        other = ROW_KERNEL if dom == UPDATE_KERNEL else UPDATE_KERNEL
        e_dom = entry(dom)
        # the whole pivot (all kernels): the stamp pass's algorithmic bytes
        # per pivot times the timed region's pivots over its time
        step_bpp = dev["bytes_pivots"] / max(1, dev["pivots"])
        step_gbps = step_bpp * piv / max_dt / 1e9 if max_dt > 0 else 0.0
        roof = {"bound": "hbm", "achieved": e_dom["achieved"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": e_dom["frac"], "traffic": e_dom["traffic"]}
        roof.update({k: v for k, v in e_dom.items() if k not in roof})
        roof.update({"dominance": {k: round(cands[k]["ms"] * cands[k]["launches"], 3) for k in cands},
                     "profile_source": prof.get("source"), "second_kernel": entry(other),
                     "step_achieved": round(step_gbps, 1), "step_frac": round(step_gbps / HBM_PEAK_GBS, 4),
                     "step_bytes_per_pivot": round(step_bpp)})

    cpu = None
    extra = {}
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import orcpy   # CPU baseline leg only: the bit-faithful C port of the reference
        base = problems.gen_dense(args.m, args.n, seed=42, keep_dense=False)
        o = orcpy.OracleProb(base)
        del base
        t1 = time.perf_counter()
        o.simplex(meth=3, tm_lim=int(args.cpu_seconds * 1000))
        cdt = time.perf_counter() - t1
        cres = o.result()
        del o
        cpu = {"value": round(cres["it_cnt"] / cdt, 3), "unit": "pivots/s", "cores": 1, "kind": "port",
               "sample": f"oracle (C restatement of glpspx02.js) dual simplex on the same C3 4096x16384 "
                         f"instance from the slack basis, tm_lim={args.cpu_seconds:.0f}s: "
                         f"{cres['it_cnt']} pivots in {cdt:.1f}s incl. init_csa; reference node "
                         f"dist/glpk.js measured 9.4 pivots/s on this config (BASELINE.md)",
               # the port is not a proxy for the reference's speed: both timed
               # in the build container on the same instance
               "port_over_reference_node": PORT_OVER_NODE,
               "reference_node_pivots_per_s": 9.4}

    line = None
    if rank == 0:
        line = {
            "metric": "simplex pivots/s (dual, C3 dense 4096x16384 fp64)",
            "value": round(value, 2),
            "unit": "pivots/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1000.0 * max_dt / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SURVEY.md §8(d) splitmix64 C3 generator, seed 42+rank)",
            "config": {"workload": "C3 dense random LP m=4096 n=16384 (BASELINE.json configs[2]); "
                                   f"step = glp_simplex dual with it_lim={args.pivots_per_step} continuing "
                                   "from the previous basis",
                       "m": args.m, "n": args.n, "pivots_per_step": args.pivots_per_step,
                       "parallelism": f"replicas x{world}"},
            "roofline": roof,
            "cpu_baseline": cpu,
            "engine": {"ms_split_per_step": {k: round(1000.0 * v / args.steps, 3) for k, v in split.items()},
                       "bytes_per_pivot_roofline_pass": round(dev["bytes_pivots"] / max(1, dev["pivots"])),
                       "graphs_built_last_step": int(st.graphs_built),
                       "pivots": int(st.pivots), "reinversions_timed_region": reinv,
                       "batches": int(st.batches), "host_syncs": int(st.host_syncs),
                       "restarts": restarts[0], "resident_calls": resident, "evals_skipped": skipped,
                       "kernels": kern},
            "extra": {},
        }

    if not args.no_extra:
        if world == 1:
            del P
            extra = run_extra(gk, problems, ctx, prob)
        else:
            # B&B sharded over all ranks (subtree per GPU) through the
            # library's own collective (gk_comm: RCCL over xGMI between the
            # ranks' devices), every epoch's exchange inside the C driver.
            # The headline is measured by now: a failure of this context leg
            # is reported in the line, and a watchdog prints the line and
            # ends every rank should the collective hang
            import threading

            held = {"extra": {}}

            def _expire():
                if rank == 0:
                    line["extra"] = dict(held["extra"], error=f"multi-rank extras exceeded {EXTRA_MULTI_S:.0f} s")
                    print(json.dumps(line), flush=True)
                sys.stderr.flush()
                os._exit(3)            # a hang is a failure: non-zero exit after the line

            dog = threading.Timer(EXTRA_MULTI_S, _expire)
            dog.daemon = True
            dog.start()
            try:
                port = int(os.environ.get("MASTER_PORT", "29500")) + 7
                comm = gk.Comm(ctx, rank, world, f"{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{port}")
                # the deepest C5s instance (the reference: 813,077 node LPs, 27,575 s)
                extra = run_bnb(gk, problems, ctx, names=("c5s_12x42",), comm=comm)
                extra["bnb_comm_backend"] = {1: "tcp", 2: "rccl"}.get(comm.backend, comm.backend)
            except Exception as e:            # noqa: BLE001 (reported, the headline stands)
                extra = {"error": f"multi-rank B&B leg: {type(e).__name__}: {e}"}
            if "error" not in extra:
                # column-sharded pricing of one LP over the same communicator
                try:
                    del P
                    held["extra"] = extra                  # (what the watchdog prints should this leg hang)
                    extra["c3_mid_solve_sharded"] = run_mid_sharded(
                        gk, ctx, problems.gen_dense(args.m, args.n, seed=42), comm)   # one instance on every rank
                except Exception as e:        # noqa: BLE001
                    extra["c3_mid_solve_sharded"] = {"error": f"{type(e).__name__}: {e}"}
            dog.cancel()

    if rank == 0:
        line["extra"] = extra
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


EXTRA_MULTI_S = 240.0      # the multi-rank B&B leg's watchdog


def run_extra(gk, problems, ctx, c3):
    """Secondary configurations of BASELINE.json on the same GPU (C2s surrogate
    of configs[1]; C3 timed exactly as BASELINE.md times the reference: first
    300 dual pivots from the slack basis including setup); for context, not
    the headline."""
    out = {}
    P = gk.GkProblem(ctx, c3)
    leg("c3_first300_dual")
    t0 = time.perf_counter()
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, it_lim=300, msg_lev=gk.GLP_MSG_ERR))
    dt = time.perf_counter() - t0
    out["c3_first300_dual_incl_setup"] = {"ret": ret, "pivots": P.it_cnt, "seconds": round(dt, 4),
                                          "pivots_per_s": round(P.it_cnt / dt, 1),
                                          "reference_node_pivots_per_s": 9.4}
    del P
    # the primal (glp_simplex's default method) on the same instance, timed
    # like the headline: it_lim=100 steps continuing from the previous basis
    P = gk.GkProblem(ctx, c3)
    parm = gk.SMCP(meth=gk.GLP_PRIMAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    leg("c3_primal_steps")
    gk.glp_simplex(P, parm)
    t0 = time.perf_counter()
    it0 = P.it_cnt
    for _ in range(5):
        ret = gk.glp_simplex(P, parm)
    dt = time.perf_counter() - t0
    out["c3_primal_steps"] = {"ret": ret, "pivots": P.it_cnt - it0, "seconds": round(dt, 4),
                              "pivots_per_s": round((P.it_cnt - it0) / dt, 1),
                              "window": "pivots 100-600 from the slack basis, 5 steps of it_lim=100",
                              "reference_node_pivots_per_s": 4.0}
    del P
    for meth, name, ref_rate in ((gk.GLP_DUAL, "dual", 1813), (gk.GLP_PRIMAL, "primal", 1833)):
        p = problems.gen_c2s()
        P = gk.GkProblem(ctx, p)
        leg("c2s_" + name)
        t0 = time.perf_counter()
        ret = gk.glp_simplex(P, gk.SMCP(meth=meth, msg_lev=gk.GLP_MSG_ERR))
        dt = time.perf_counter() - t0
        out["c2s_" + name + "_full_solve"] = {"ret": ret, "obj": P.obj_val, "ref_obj": 357.82820943518834,
                                              "pivots": P.it_cnt, "seconds": round(dt, 4),
                                              "pivots_per_s": round(P.it_cnt / dt, 1),
                                              "reference_node_pivots_per_s": ref_rate}
        del P
    out["sparse_blocks_20k"] = run_sparse(gk, problems, ctx)
    out["c3_mid_solve"] = run_mid(gk, problems, ctx, c3)
    out["c3_full_dual"] = run_full(gk, ctx, c3)
    out.update(run_bnb(gk, problems, ctx))
    out["scale_c3"] = run_scale(gk, ctx, c3)
    return out


def run_sparse(gk, problems, ctx):
    """The sparse factor path (gk_sparse.hip) on the m = 20,020
    block-angular fixture (tests/golden/sparse_oracle_blocks_200x100x200+20:
    the oracle's objective and 89,265 pivots in 275 s on one core): the
    whole dual solve, and its roofline — the pivots' algorithmic bytes
    (accumulated per pivot: 12 B per L / U entry per sweep, 12 nnz(A) for
    the pivot row and again for A w, the Schur chain's Y / inv(M) reads,
    the O(m + n) vectors) over the solve's pivot-batch wall time."""
    gold = os.path.join(ROOT, "tests", "golden", "sparse_oracle_blocks_200x100x200+20.json")
    d = json.load(open(gold))
    prob = problems.gen_blocks(*d["args"])
    P = gk.GkProblem(ctx, prob)
    leg("sparse_blocks_20k")
    t0 = time.perf_counter()
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR))
    dt = time.perf_counter() - t0
    st = P.stats()
    bpp = st.bytes_pivots / max(1, st.pivots)
    gbps = st.bytes_pivots / max(1e-9, st.seconds_batches) / 1e9
    out = {"ret": ret, "obj": P.obj_val, "ref_obj": d["obj"],
           "obj_rel_err": abs(P.obj_val - d["obj"]) / max(1.0, abs(d["obj"])),
           "pivots": P.it_cnt, "oracle_pivots": d["it_cnt"], "seconds": round(dt, 2),
           "pivots_per_s": round(P.it_cnt / dt, 1), "oracle_seconds_1core": d["oracle_seconds"],
           "factor_sparse": int(st.factor_sparse), "refactorizations": int(st.reinversions),
           "seconds_batches": round(st.seconds_batches, 2), "seconds_lu": round(st.seconds_lu, 2),
           "bytes_per_pivot": round(bpp), "achieved_GBps_batches": round(gbps, 1),
           "frac_of_hbm_peak": round(gbps / HBM_PEAK_GBS, 4),
           "bound": "latency (dependent sweep levels), DESIGN §2f"}
    del P
    return out


def run_scale(gk, ctx, p, flags=0x31):
    """glp_scale_prob(GM | EQ | 2N) on C3 (gk_scale.hip):
    the device time of the scaling work with A resident (every sweep, each
    streaming the 12-byte entries of A once by rows or by columns, plus the
    row copy when one is built) against the sweeps' algorithmic bytes, and
    the whole call including the upload of A."""
    import ctypes as C
    import numpy as np
    ptr = np.ascontiguousarray(np.asarray(p.A_ptr, np.int32))
    ind = np.ascontiguousarray(np.asarray(p.A_ind, np.int32))
    val = np.ascontiguousarray(np.asarray(p.A_val, np.float64))
    rii, sjj, rep = np.ones(p.m), np.ones(p.n), np.zeros(13)
    ms, by = C.c_double(0.0), C.c_double(0.0)
    f = lambda a: a.ctypes.data_as(C.c_void_p)  # noqa: E731
    L = gk.load_library()
    L.gk_scale_prob_timed(ctx.h, p.m, p.n, f(ptr), f(ind), f(val), flags, f(rii), f(sjj), f(rep),   # warm-up
                          C.byref(ms), C.byref(by))
    t0 = time.perf_counter()
    ret = L.gk_scale_prob_timed(ctx.h, p.m, p.n, f(ptr), f(ind), f(val), flags, f(rii), f(sjj), f(rep),
                                C.byref(ms), C.byref(by))
    dt = time.perf_counter() - t0
    gbps = by.value / (ms.value * 1e-3) / 1e9 if ms.value > 0 else 0.0
    return {"ret": ret, "flags": flags, "nnz": int(ptr[-1]), "sweeps_ms": round(ms.value, 3),
            "sweep_bytes": by.value, "sweeps_GBps": round(gbps, 1), "frac_of_hbm_peak": round(gbps / 8000.0, 4),
            "seconds_incl_upload": round(dt, 4),
            "report": {"A": list(rep[0:3]), "GM": list(rep[3:6]), "EQ": list(rep[6:9]), "2N": list(rep[9:12])}}


def run_full(gk, ctx, c3):
    """The whole C3 dual solve from the slack basis in one glp_simplex call
    (the representative rate: the headline window is the cheap start of it),
    with its re-inversion time and a KKT certificate of the optimum
    (tests/kkt.py: primal / dual feasibility, complementary slackness, zero
    duality gap — the reference, at ~9 pivots/s, cannot finish this solve)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from kkt import dense_kkt
    P = gk.GkProblem(ctx, c3)
    leg("c3_full_dual")
    t0 = time.perf_counter()
    ret = gk.glp_simplex(P, gk.SMCP(meth=gk.GLP_DUAL, msg_lev=gk.GLP_MSG_ERR))
    dt = time.perf_counter() - t0
    st = P.stats()
    out = {"ret": ret, "obj": P.obj_val, "pivots": P.it_cnt, "seconds": round(dt, 2),
           "pivots_per_s": round(P.it_cnt / dt, 1), "reinversions": int(st.reinversions),
           "reinversion_seconds": round(st.seconds_reinvert, 2), "newton_refined": int(st.refinements),
           "panel_hits": int(st.panel_hits), "panel_refills": int(st.panel_refills)}
    try:
        res = dense_kkt(P, c3)
        out["kkt"] = {"certified": True, "gap": res["gap"], "max_residual": max(v for k, v in res.items())}
    except AssertionError as e:        # reported, not raised: the headline stands
        out["kkt"] = {"certified": False, "violation": str(e)[:300]}
    del P
    return out


def run_mid(gk, problems, ctx, c3, start=100000, steps=10):
    """C3 dual in its HBM-bound regime: the same instance advanced to pivot
    `start` (most of the basis structural: the pivot row is a column pass over
    all of A and the rank-1 update touches ~m dense columns of inv(B)), then
    `steps` it_lim=100 steps; algorithmic bytes per pivot as in the headline
    (the engine's device-side count)."""
    import torch
    P = gk.GkProblem(ctx, c3)
    adv = gk.SMCP(meth=gk.GLP_DUAL, it_lim=2000, msg_lev=gk.GLP_MSG_ERR)
    t0 = time.perf_counter()
    while P.it_cnt < start:
        leg(f"c3_mid advance from it_cnt={P.it_cnt}")
        if gk.glp_simplex(P, adv) != 8:
            return {"error": "solve ended before the window"}
    t_adv = time.perf_counter() - t0
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    gk.glp_simplex(P, parm)
    P.profile(4)                        # byte accounting on (the window's algorithmic bytes)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    piv, byts = 0, 0.0
    for _ in range(steps):
        it0 = P.it_cnt
        leg(f"c3_mid window from it_cnt={it0}")
        gk.glp_simplex(P, parm)
        piv += P.it_cnt - it0
        byts += P.stats().bytes_pivots
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    gbps = byts / dt / 1e9
    return {"window": f"pivots {start + 100}-{start + 100 + piv} of the full solve (381,750 pivots, "
                      f"profiles/r01_c3_full_dual.jsonl)", "pivots": piv, "seconds": round(dt, 4),
            "pivots_per_s": round(piv / dt, 1), "bytes_per_pivot": round(byts / max(piv, 1)),
            "algorithmic_GBps": round(gbps, 1), "frac_of_hbm_peak": round(gbps / HBM_PEAK_GBS, 4),
            "advance_seconds": round(t_adv, 1)}


def run_mid_sharded(gk, ctx, c3, comm, start=100000, steps=10):
    """C3 dual in the HBM-bound regime with column-sharded pricing
    (gk_bfd_set_comm): every rank advances the same instance to
    pivot `start` on its own (the same pivots on every rank), then the
    window of `steps` it_lim=100 calls runs with each pivot row's column pass
    split over the ranks and the slices all-gathered over comm; the time is
    the max over ranks.  The single-GPU window with the pricing panel is
    `c3_mid_solve` of the one-GPU run."""
    import struct
    P = gk.GkProblem(ctx, c3)
    adv = gk.SMCP(meth=gk.GLP_DUAL, it_lim=2000, msg_lev=gk.GLP_MSG_ERR)
    while P.it_cnt < start:
        leg(f"c3_mid_sharded advance from it_cnt={P.it_cnt}")
        if gk.glp_simplex(P, adv) != 8:
            return {"error": "solve ended before the window"}
    P.set_comm(comm)
    parm = gk.SMCP(meth=gk.GLP_DUAL, it_lim=100, msg_lev=gk.GLP_MSG_ERR)
    gk.glp_simplex(P, parm)
    comm.allgather(b"x")
    t0 = time.perf_counter()
    piv = 0
    for _ in range(steps):
        it0 = P.it_cnt
        leg(f"c3_mid_sharded window from it_cnt={it0}")
        gk.glp_simplex(P, parm)
        piv += P.it_cnt - it0
    dt = time.perf_counter() - t0
    dt = max(struct.unpack("d", blk)[0] for blk in comm.allgather(struct.pack("d", dt)))
    its = {struct.unpack("q", blk)[0] for blk in comm.allgather(struct.pack("q", int(P.it_cnt)))}
    P.set_comm(None)
    return {"window": f"pivots {start + 100}-{start + 100 + piv}", "ranks": comm.size, "pivots": piv,
            "seconds": round(dt, 4), "pivots_per_s": round(piv / dt, 1), "ranks_agree": len(its) == 1,
            "backend": {1: "tcp", 2: "rccl"}.get(comm.backend, comm.backend)}


def run_bnb(gk, problems, ctx, names=("gap", "c5s_12x30", "c5s_12x40", "c5s_12x42", "sparsebig4"), comm=None):
    """B&B configs (BASELINE.json configs[3], C5s surrogate of configs[4]):
    root glp_simplex + glp_intopt on the device; LP-relaxations/s = node LP
    solves (all ranks) / wall time of glp_intopt."""
    import json as _json
    out = {}
    gold = os.path.join(ROOT, "tests", "golden")
    refs = {"gap": (196, 0.0477), "c5s_12x30": (70506, 49.7)}
    for name in names:
        d = _json.load(open(os.path.join(gold, "mip_" + name + ".json")))
        ref_lps, ref_s = refs.get(name, (d["mip"]["lp_solves"], d["mip"]["seconds"]))
        prob = problems.from_fixture(d)
        leg("bnb_" + name)
        # one untimed search first (warm-up, as the LP legs have): the node
        # kernel's code object loads on its first launch and the search
        # buffers are allocated once per context (gk_ctx_mip_cache)
        W = gk.GkProblem(ctx, prob.copy())
        assert gk.glp_simplex(W, gk.SMCP(msg_lev=gk.GLP_MSG_ERR)) == 0
        gk.glp_intopt(W, gk.IOCP(msg_lev=gk.GLP_MSG_ERR), comm=comm)
        del W
        P = gk.GkProblem(ctx, prob)
        assert gk.glp_simplex(P, gk.SMCP(msg_lev=gk.GLP_MSG_ERR)) == 0
        t0 = time.perf_counter()
        ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_ERR), comm=comm)
        dt = dt_local = time.perf_counter() - t0
        if comm is not None:
            import struct
            dt = max(struct.unpack("d", blk)[0] for blk in comm.allgather(struct.pack("d", dt)))   # max over ranks
        lps = P.mip_stats.get("lp_solves", 0)
        per_rank = None
        if comm is not None:
            import struct
            blks = comm.allgather(struct.pack("qd", int(lps), dt_local))
            per_rank = [{"node_lps": struct.unpack("qd", b)[0], "seconds": round(struct.unpack("qd", b)[1], 4)}
                        for b in blks]
            lps = sum(r["node_lps"] for r in per_rank)                # all ranks
        # LP-relax/s counts every node LP the batched search solves, including
        # the speculative ones a sequential walk would have pruned: read it
        # with the time to the optimum and the node-LP counts beside it
        out["bnb_" + name] = {"ret": ret, "mip_obj": P.mip_obj, "ref_mip_obj": d["mip"]["mip_obj"],
                              "time_to_optimal_s": round(dt, 4), "reference_time_to_optimal_s": ref_s,
                              "time_speedup": round(ref_s / dt, 1) if dt > 0 else None,
                              "node_lps": lps, "reference_node_lps": ref_lps,
                              "node_lps_over_reference": round(lps / ref_lps, 2),
                              "lp_relax_per_s": round(lps / dt, 1),
                              "reference_lp_relax_per_s": round(ref_lps / ref_s, 1),
                              "nodes": P.mip_stats.get("nodes_created"),
                              "pp_fathomed": P.mip_stats.get("pp_fathomed"),
                              "node_fallbacks": P.mip_stats.get("node_fallbacks"),
                              "ranks": comm.size if comm is not None else 1}
        if per_rank is not None:
            out["bnb_" + name]["per_rank"] = per_rank
    return out


if __name__ == "__main__":
    main()
