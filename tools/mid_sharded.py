"""Rehearse bench.py's multi-rank column-sharded window on one GPU: N ranks
(default 2) share cuda:0 through the library's TCP transport and run
bench.run_mid_sharded on the C3 instance; prints each rank's result.

    python tools/mid_sharded.py [ranks] [start] [steps]
"""
import json
import multiprocessing as mp
import os
import socket
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _worker(rank, size, port, start, steps, q):
    sys.path.insert(0, ROOT)
    import bench
    import __graft_entry__
    __graft_entry__.load_package()
    from glpk_js_amd import gk, problems
    ctx = gk.Context(0)
    comm = gk.Comm(ctx, rank, size, f"127.0.0.1:{port}")
    try:
        r = bench.run_mid_sharded(gk, ctx, problems.gen_dense(4096, 16384, seed=42), comm,
                                  start=start, steps=steps)
    except Exception as e:  # noqa: BLE001
        r = {"error": repr(e)}
    q.put((rank, r))
    comm.close()


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    start = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, size, port, start, steps, q)) for r in range(size)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=600) for _ in range(size)], key=lambda t: t[0])
    for p in ps:
        p.join(timeout=60)
    for rank, r in res:
        print(json.dumps({"rank": rank, **r}), flush=True)
    sys.exit(0 if all("error" not in r for _, r in res) else 1)


if __name__ == "__main__":
    main()
