"""Multi-GPU branch and bound: one process per GPU.

Every rank runs gk_ios_driver_sharded on the same problem: identical
ramp-up batches, then a round-robin split of the frontier.  Every few
batches the native driver calls `TorchComm.allgather_bytes`, an all-gather
of a fixed-size byte block per rank: first {incumbent, best open bound, open
nodes, active} of every rank, then — when some rank is idle and another
holds open nodes — the node descriptors (bounds, warm-start basis, parent
information) the donors hand to the idle ranks (gk_mip.hip, shard_epoch).
`TorchComm.exchange` (all-reduce MIN of [best, -active]) is the older,
incumbent-only protocol; `TorchComm.finalize` picks the winning incumbent
(lowest objective, lowest rank on ties) and broadcasts it.  The backend is whatever process group is
initialised: "nccl" (RCCL over xGMI) on MI355X nodes, "gloo" for CPU tests.
"""
from __future__ import annotations

import numpy as np


class TorchComm:
    def __init__(self, group=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank = dist.get_rank(group)
        self.size = dist.get_world_size(group)
        backend = dist.get_backend(group)
        self.device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")

    def exchange(self, best: float, active: int) -> tuple[float, int]:
        """All-reduce MIN of (best, -active): global best and the number of
        ranks with open nodes (0 or the max indicator 1)."""
        t = self.torch.tensor([best, -float(active)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN, group=self.group)
        v = t.cpu().tolist()
        return v[0], int(-v[1])

    def allgather_bytes(self, send_ptr: int, nbytes: int, recv_ptr: int) -> None:
        """All-gather of nbytes from every rank (the C driver's buffers, raw
        addresses) into recv (size * nbytes, rank order)."""
        import ctypes
        torch, dist = self.torch, self.dist
        buf = np.empty(nbytes, dtype=np.uint8)
        ctypes.memmove(buf.ctypes.data, send_ptr, nbytes)
        t = torch.from_numpy(buf).to(self.device)
        outs = [torch.empty_like(t) for _ in range(self.size)]
        dist.all_gather(outs, t, group=self.group)
        for r, o in enumerate(outs):
            a = np.ascontiguousarray(o.cpu().numpy())
            ctypes.memmove(recv_ptr + r * nbytes, a.ctypes.data, nbytes)

    def total(self, v: float) -> float:
        t = self.torch.tensor([float(v)], dtype=self.torch.float64, device=self.device)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM, group=self.group)
        return float(t.item())

    def finalize(self, obj_min: float, have: bool, x: np.ndarray) -> tuple[float, bool, np.ndarray, int]:
        """Winner = lowest objective (minimisation form) with a solution, lowest
        rank on ties; its x is broadcast to every rank."""
        torch, dist = self.torch, self.dist
        key = torch.tensor([obj_min if have else float("inf"), float(self.rank)], dtype=torch.float64,
                           device=self.device)
        keys = [torch.zeros_like(key) for _ in range(self.size)]
        dist.all_gather(keys, key, group=self.group)
        ks = [k.cpu().tolist() for k in keys]
        best = min(range(self.size), key=lambda r: (ks[r][0], r))
        win_obj = ks[best][0]
        if win_obj == float("inf"):
            return float("inf"), False, x, best
        buf = torch.as_tensor(np.ascontiguousarray(x, dtype=np.float64), device=self.device).clone()
        dist.broadcast(buf, src=dist.get_global_rank(self.group, best) if self.group is not None else best,
                       group=self.group)
        return win_obj, True, buf.cpu().numpy(), best
