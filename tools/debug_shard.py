# two ranks on one GPU, gloo; prints progress (debug helper)
import json, os, sys, socket
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

def worker(rank, world, port, name):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    import __graft_entry__
    __graft_entry__.load_package()
    from glpk_js_amd import gk, problems
    from glpk_js_amd.shard import TorchComm
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    comm = TorchComm()
    n_ex = [0]
    orig = comm.exchange
    def ex(b, a):
        n_ex[0] += 1
        r = orig(b, a)
        if n_ex[0] <= 5 or n_ex[0] % 50 == 0:
            print(f"rank {rank} exchange #{n_ex[0]} in=({b:.4g},{a}) out={r}", flush=True)
        return r
    comm.exchange = ex
    ctx = gk.Context(0)
    d = json.load(open(os.path.join(ROOT, "tests", "golden", f"mip_{name}.json")))
    P = gk.GkProblem(ctx, problems.from_fixture(d))
    print(f"rank {rank} root", gk.glp_simplex(P, gk.SMCP(**d["root"]["opts"])), flush=True)
    try:
        ret = gk.glp_intopt(P, gk.IOCP(msg_lev=gk.GLP_MSG_OFF), comm=comm)
        print(f"rank {rank} ret {ret} obj {P.mip_obj} stats {P.mip_stats} exchanges {n_ex[0]}", flush=True)
    except Exception as e:
        print(f"rank {rank} FAILED {e!r}", flush=True)
        os._exit(3)
    dist.destroy_process_group()

if __name__ == "__main__":
    import torch.multiprocessing as mp
    s = socket.socket(); s.bind(("127.0.0.1", 0)); port = s.getsockname()[1]; s.close()
    name = sys.argv[1] if len(sys.argv) > 1 else "mixint8"
    mp.start_processes(worker, args=(2, port, name), nprocs=2, start_method="spawn")
