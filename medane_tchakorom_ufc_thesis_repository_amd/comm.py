"""Inter-block exchange for the multisplitting drivers.

Replaces the reference's MPI point-to-point layer (src/utils/comm.c:126-141,
comm_sync_send_and_receive) and the residual-norm Allreduce over the block
roots (synchronous-multisplitting.c:189-196, utils.c:584-592):

* boundary exchange: each block sends only the plane(s) its neighbours'
  coupling rows read (the reference swaps whole block vectors, comm.c:135;
  A_ij is zero outside that plane, so the result is identical), over RCCL
  (torch.distributed backend "nccl", grouped send/recv GPU to GPU over xGMI),
  or gloo (host tensors; CPU tests and single-GPU rehearsals);
* the sum of per-block squared norms is an all-gather followed by a sum in
  block order, so the result does not depend on the collective's reduction
  order (for 2 blocks this is the reference's a + b).

A block object provides: layout (utils.BlockLayout), pack_send(nbr) -> tensor
with the plane(s) for neighbour nbr, recv_buffer(nbr) -> tensor to receive
into, unpack_recv(), and, for LocalComm, copy_halo_from(block).

  LocalComm  -- every block in this process (one GPU or tests): direct copies;
  LibComm    -- one block per rank (one rank per GPU) over the library's own
                communicator (msp_comm): halo planes, residual sums and LSQR
                partials on ONE RCCL communicator, on the context's stream;
  TorchComm  -- one block per rank over torch.distributed collectives (CPU
                tests with test-double blocks, gloo).
"""
from __future__ import annotations


class LocalComm:
    """All blocks live in this process; the exchange is a device-to-device copy
    of each neighbour's boundary plane into the block's halo."""

    world = 1
    rank = 0
    backend = "local"

    def alloc(self, ctx, n):
        from .petsc import Vec
        return Vec(ctx, n), None

    def exchange(self, blocks):
        by_id = {blk.layout.b: blk for blk in blocks}
        for blk in blocks:
            blk.copy_halo_from(by_id)

    def ordered_sum(self, blocks, values):
        """values[i] belongs to blocks[i]; sum in global block order."""
        tot = 0.0
        for _, v in sorted(zip([b.layout.b for b in blocks], values)):
            tot += v
        return tot

    def barrier(self):
        pass

    def agree(self, token: int) -> bool:
        """Every block is in this process: one loop, one decision."""
        return True

    def lsqr_comm(self, ctx):
        """Every block is in this process: LSQR adds the block partials itself."""
        return None


class TorchComm:
    """One block per rank over a torch.distributed process group (block id =
    rank).  With "nccl" (= RCCL on ROCm) the halo planes move GPU to GPU inside
    one ncclGroupStart/End (batch_isend_irecv); with "gloo" the same pattern
    runs on host tensors (device planes are staged through the host)."""

    def __init__(self, group=None, device=None):
        import torch
        import torch.distributed as dist
        self.torch = torch
        self.dist = dist
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        if device is None:
            device = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
        self.device = device

    @property
    def device_buffers(self) -> bool:
        """Halo buffers live in HBM (nccl) or on the host (gloo)."""
        return self.backend == "nccl"

    def alloc(self, ctx, n):
        """A buffer visible to torch (for the collective) and, for nccl, to the
        HIP library (a Vec over the same device memory)."""
        from .petsc import Vec
        if self.device_buffers:
            t = self.torch.zeros(max(int(n), 2), dtype=self.torch.float64, device=self.device)
            # the zero fill runs on torch's stream; the library writes the buffer on its own
            self.torch.cuda.current_stream(self.device).synchronize()
            return Vec(ctx, n, device_ptr=t.data_ptr()), t
        return Vec(ctx, n), self.torch.zeros(max(int(n), 2), dtype=self.torch.float64)

    def exchange_tensors(self, send: dict, recv: dict):
        """send/recv: {neighbour rank: tensor}.  Grouped point-to-point."""
        dist = self.dist
        ops = [dist.P2POp(dist.irecv, t, nbr, self.group) for nbr, t in recv.items()]
        ops += [dist.P2POp(dist.isend, t, nbr, self.group) for nbr, t in send.items()]
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
        send = {nbr: blk.pack_send(nbr) for nbr, _, _ in blk.layout.send}
        recv = {nbr: blk.recv_buffer(nbr) for nbr, _, _, _ in blk.layout.recv}
        self.exchange_tensors(send, recv)
        if self.backend == "nccl":
            self.torch.cuda.current_stream(self.device).synchronize()
        blk.unpack_recv()

    def allgather_scalar(self, v: float):
        torch = self.torch
        dev = self.device if self.backend == "nccl" else torch.device("cpu")
        t = torch.tensor([float(v)], dtype=torch.float64, device=dev)
        if self.backend == "nccl":
            out = torch.zeros(self.world, dtype=torch.float64, device=dev)
            self.dist.all_gather_into_tensor(out, t, group=self.group)
            return out.cpu().tolist()
        outs = [torch.zeros(1, dtype=torch.float64) for _ in range(self.world)]
        self.dist.all_gather(outs, t, group=self.group)
        return [float(o[0]) for o in outs]

    def ordered_sum(self, blocks, values):
        (v,) = values
        tot = 0.0
        for x in self.allgather_scalar(v):       # rank order = block order
            tot += x
        return tot

    def barrier(self):
        self.dist.barrier(group=self.group)

    def agree(self, token: int) -> bool:
        """Every rank holds the same outer-loop token (msp_comm_agree's contract); raises on every rank if not."""
        got = self.allgather_scalar(float(token))
        bad = [r for r, v in enumerate(got) if v != got[0]]
        if bad:
            raise RuntimeError(f"ranks disagree on the outer loop state: rank 0 holds {int(got[0])}, "
                               f"rank {bad[0]} {int(got[bad[0]])}")
        return True

    def lsqr_comm(self, ctx):
        """The all-gather of LSQR's block partials (petsc.Comm): with "nccl" an
        RCCL communicator of its own (id broadcast over this group), enqueued
        on the context's stream; with "gloo" (or MSPLIT_LSQR_TRANSPORT=host) a
        host callback over this group's all_gather."""
        import os
        from .petsc import Comm
        if self.world == 1:
            return None
        transport = os.environ.get("MSPLIT_LSQR_TRANSPORT", "rccl" if self.backend == "nccl" else "host")
        if transport == "rccl":
            obj = [None]
            if self.rank == 0:
                try:
                    obj = [Comm.unique_id()]
                except Exception as e:                   # no usable librccl: every rank takes the other path
                    obj = [f"error: {e}"]
            self.dist.broadcast_object_list(obj, src=0, group=self.group)
            ok = isinstance(obj[0], bytes)
            comm = None
            if ok:
                try:
                    comm = Comm.rccl(ctx, self.world, self.rank, obj[0])
                except Exception as e:
                    ok, obj = False, [f"error: {e}"]
            # every rank must agree on the transport before the first all-gather
            flags = self.allgather_scalar(1.0 if ok else 0.0)
            if all(f == 1.0 for f in flags):
                return comm
            if comm is not None:
                comm.destroy()
            import sys
            print(f"msplit: own RCCL communicator unavailable ({obj[0] if not ok else 'on another rank'}); "
                  "LSQR partials go through the process group instead", file=sys.stderr)
        torch, dist, world, group = self.torch, self.dist, self.world, self.group
        dev = self.device if self.backend == "nccl" else torch.device("cpu")

        def allgather(a):
            t = torch.from_numpy(a).to(dev)
            out = torch.empty(world * t.numel(), dtype=t.dtype, device=dev)
            dist.all_gather_into_tensor(out, t, group=group)
            return out.cpu().numpy()
        return Comm.host(ctx, self.world, self.rank, allgather)


class LibComm:
    """One block per rank (block id = rank) over the library's msp_comm, the
    product's N > 1 path.  The boundary exchange is msp_comm_exchange_neighbors
    (comm.c:126-141 for chain neighbours: the planes to rank-1 / rank+1 and back,
    RCCL send/recv in one group enqueued on the context's stream -- no host
    synchronisation), the outer-residual sum is msp_comm_sum_ordered (rank order,
    synchronous-multisplitting.c:192) and the LSQR block partials go over the
    same communicator, so each rank holds one RCCL communicator.
    torch.distributed only broadcasts its id (and runs barriers).

    transport "rccl" (default with the nccl process group) or "host" (the
    library's host-callback transport over the process group's all_gather: gloo
    rehearsals, e.g. two ranks sharing one GPU, which RCCL refuses)."""

    device_buffers = True
    lsqr_comm_owned = False     # GpuMinimizer must not destroy it: the exchange uses it too

    def __init__(self, ctx, group=None, transport: str | None = None):
        import torch
        import torch.distributed as dist
        from .petsc import Comm
        self.torch, self.dist, self.group = torch, dist, group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.backend = dist.get_backend(group)
        self.transport = transport or ("rccl" if self.backend == "nccl" else "host")
        self.ctx = ctx
        self.comm = None
        if self.transport == "rccl":
            dev = (torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl"
                   else torch.device("cpu"))

            def agree(flag: bool) -> bool:  # every rank takes the same path (MPI_Allreduce MIN, host/main.c)
                t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=dev)
                dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
                return bool(int(t.item()))

            # readiness before the collective ncclCommInitRank: a rank that cannot load RCCL (or rank 0 that
            # cannot get an id) must not leave the others blocked inside init, so all ranks agree first.  Only
            # rank 0 creates the id (ncclGetUniqueId starts a bootstrap root thread and socket, as in
            # host/main.c); the others test that the library loads.
            err, uid = None, None
            try:
                if self.rank == 0:
                    uid = Comm.unique_id()
                elif not Comm.rccl_available():
                    err = RuntimeError("librccl.so.1 could not be loaded")
            except Exception as e:
                err = e
            ready = agree(err is None)
            if ready:
                obj = [uid if self.rank == 0 else None]
                dist.broadcast_object_list(obj, src=0, group=group)
                try:
                    self.comm = Comm.rccl(ctx, self.world, self.rank, obj[0])
                except Exception as e:          # e.g. ranks sharing a GPU, which RCCL refuses on every rank
                    err = e
            # a failure inside init itself is assumed symmetric (RCCL fails on every rank, as for ranks
            # sharing a GPU); the agreement below then moves every rank to the host transport
            ok = ready and agree(err is None)
            if not ok:
                if self.comm is not None:
                    self.comm.destroy()
                    self.comm = None
                if self.rank == 0:
                    import sys
                    print(f"msplit: RCCL communicator unavailable ({err or 'on another rank'}); "
                          "using the host transport over the process group", file=sys.stderr)
                self.transport = "host"
        if self.transport == "host":
            dev = torch.device("cuda", torch.cuda.current_device()) if self.backend == "nccl" else torch.device("cpu")
            world = self.world

            def allgather(a):
                t = torch.from_numpy(a).to(dev)
                out = torch.empty(world * t.numel(), dtype=t.dtype, device=dev)
                dist.all_gather_into_tensor(out, t, group=group)
                return out.cpu().numpy()
            self.comm = Comm.host(ctx, self.world, self.rank, allgather)

    def alloc(self, ctx, n):
        from .petsc import Vec
        return Vec(ctx, n), None

    def exchange(self, blocks):
        (blk,) = blocks
        L = blk.layout
        lo_src = hi_src = lo_dst = hi_dst = 0
        count = 0
        for nbr, off, cnt in L.send:
            count = cnt
            if nbr == self.rank - 1:
                lo_src = off
            else:
                hi_src = off
        for nbr, hoff, cnt, _ in L.recv:
            if cnt != count:
                raise ValueError("msp_comm_exchange_neighbors moves equal planes both ways")
            if nbr == self.rank - 1:
                lo_dst = hoff
            else:
                hi_dst = hoff
        if count:
            self.comm.exchange_neighbors(blk.x, lo_src, hi_src, blk.halo, lo_dst, hi_dst, count)

    def ordered_sum(self, blocks, values):
        (v,) = values
        return float(self.comm.sum_ordered([v])[0])

    def barrier(self):
        self.dist.barrier(group=self.group)

    def agree(self, token: int) -> bool:
        """msp_comm_agree over the library communicator (raises petsc's MsplitError on every rank on a mismatch)."""
        return self.comm.agree(token)

    def lsqr_comm(self, ctx):
        return self.comm

    def close(self):
        if getattr(self, "comm", None) is not None:
            self.ctx.synchronize()
            self.comm.destroy()
            self.comm = None
