"""Inter-block exchange for the multisplitting drivers.

Replaces the reference's MPI point-to-point layer (src/utils/comm.c:126-141,
comm_sync_send_and_receive) and the residual-norm Allreduce over the block
roots (synchronous-multisplitting.c:189-196, utils.c:584-592):

* boundary exchange: each block sends only the plane(s) its neighbours'
  coupling rows read (the reference swaps whole block vectors, comm.c:135;
  A_ij is zero outside that plane, so the result is identical), over RCCL
  (torch.distributed backend "nccl") with grouped send/recv, or gloo on CPU;
* the sum of per-block squared norms is an all-gather followed by a sum in
  block order, so the result does not depend on the collective's reduction
  order (for 2 blocks this is the reference's a + b).

Two implementations share one interface:
  LocalComm  -- every block in this process (one GPU, or tests): device copies;
  TorchComm  -- one block per rank (one rank per GPU), torch.distributed.
"""
from __future__ import annotations

import math


class LocalComm:
    """All blocks live in this process; the exchange is a device-to-device copy
    of each neighbour's boundary plane into the block's halo."""

    def __init__(self):
        self.world = 1

    def alloc(self, ctx, n):
        from .petsc import Vec
        return Vec(ctx, n), None

    def exchange(self, blocks):
        by_id = {blk.layout.b: blk for blk in blocks}
        for blk in blocks:
            for nbr, halo_off, cnt, nbr_off in blk.layout.recv:
                src = by_id[nbr]
                src.x.copy_range_to(nbr_off, blk.halo, halo_off, cnt)

    def ordered_sum(self, blocks, values):
        """values[i] belongs to blocks[i]; sum in global block order."""
        tot = 0.0
        for _, v in sorted(zip([b.layout.b for b in blocks], values)):
            tot += v
        return tot

    def barrier(self):
        pass


class TorchComm:
    """One block per rank over a torch.distributed process group.  With the
    "nccl" backend (= RCCL on ROCm) the halo planes move GPU to GPU over xGMI
    inside one ncclGroupStart/End (batch_isend_irecv); with "gloo" (CPU tests)
    the same pattern runs on host tensors."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.device = device if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu"))

    def alloc(self, ctx, n):
        """A device buffer visible both to torch (for the collective) and to the
        HIP library (wrapped as a Vec over the same memory)."""
        from .petsc import Vec
        t = self.torch.zeros(max(int(n), 2), dtype=self.torch.float64, device=self.device)
        return Vec(ctx, n, device_ptr=t.data_ptr()), t

    def exchange_tensors(self, send: dict, recv: dict):
        """send/recv: {neighbour rank: tensor}.  Grouped point-to-point."""
        dist = self.dist
        ops = []
        for nbr, t in recv.items():
            ops.append(dist.P2POp(dist.irecv, t, nbr, self.group))
        for nbr, t in send.items():
            ops.append(dist.P2POp(dist.isend, t, nbr, self.group))
        if not ops:
            return
        if self.backend == "nccl":
            for req in dist.batch_isend_irecv(ops):
                req.wait()
        else:
            reqs = [op.op(op.tensor, op.peer, op.group) for op in ops]
            for r in reqs:
                r.wait()

    def exchange(self, blocks):
        (blk,) = blocks
        ctx = blk.ctx
        # pack my boundary planes (device copies on the block's stream)
        for nbr, off, cnt in blk.layout.send:
            blk.x.copy_range_to(off, blk.send_bufs[nbr][0], 0, cnt)
        ctx.synchronize()
        send = {nbr: blk.send_bufs[nbr][1][:cnt] for nbr, _, cnt in blk.layout.send}
        recv = {nbr: blk.halo_t[halo_off:halo_off + cnt] for nbr, halo_off, cnt, _ in blk.layout.recv}
        self.exchange_tensors(send, recv)
        if self.backend == "nccl":
            self.torch.cuda.synchronize(self.device)

    def allgather_scalar(self, v: float):
        torch = self.torch
        t = torch.tensor([float(v)], dtype=torch.float64, device=self.device)
        out = torch.zeros(self.world, dtype=torch.float64, device=self.device)
        self.dist.all_gather_into_tensor(out, t, group=self.group)
        return out.cpu().tolist()

    def ordered_sum(self, blocks, values):
        (v,) = values
        tot = 0.0
        for x in self.allgather_scalar(v):
            tot += x
        return tot

    def barrier(self):
        self.dist.barrier(group=self.group)


def sqrt(x):
    return math.sqrt(x)
