"""Asynchronous multisplitting (AM) over the GPU inner solve.

Mirrors src/asynchronous-multisplitting/asynchronous-multisplitting_prime.c:
setup (:131-330: spanning tree, detection state, ||b||), the loop (:333-392)
and the final exchange and report (:394-427), generalised from 2 blocks to a
chain of nb blocks.  Blocks never wait for each other: each one takes the
newest iterate its neighbours have published (if newer than the last one it
took), solves, publishes its own boundary plane stamped (PhaseTag, iteration),
and runs one step of the decentralised convergence detection
(conv_detection_prime.c, in C: csrc/conv_detect.c).  Messages travel through
newest-value slots in shared memory (csrc/amsg.c) -- the reference's MPI
Isend / Iprobe-drain layer (comm.c:455-554) -- between one process per GPU
(TorchComm) or between the blocks of one process (LocalComm, which runs the
blocks round-robin: a deterministic schedule the tests replay on the oracle).

Stop test per block (:359): local ||rhs_i - A_ii x_i|| <= max(atol, rtol/sqrt(nb) ||b||)
(the reference's rtol/sqrt(2) for its 2 blocks), then the detection protocol
decides the global stop.

variant "amam_local" is src/asynchronous-multisplitting-asynchronous-minimization-local/
asynchronous-multisplitting-asynchronous-minimization-local_prime.c:371-431: per
outer iteration s asynchronous inner steps (each stamped with the inner-step
count), S_i(:,k) = x_i, then the block-local minimization x_i = S_i LSQR(A_ii S_i,
rhs_i) and one detection step.  variant "amam_semi_local" is
asynchronous-multisplitting-asynchronous-minimization-semi-local_prime.c:350-420: each
inner step is followed by a second receive and S_i(:,k) = [neighbour planes | x_i];
then R_i = A_block S_i, alpha_i = LSQR(R_i, b_i) and x_minimized = S_i alpha_i, which
the reference computes but never scatters back, and the detection step.
variant "amam_global" is asynchronous-multisplitting-asynchronous-minimization-
global_prime.c:370-470: the same inner steps, then R_i = A_block S_i is sent to
every block and the newest rows of every other block are taken (newest-value
broadcast, csrc/abcast.c), alpha = LSQR over the replicated R and the global b,
x_minimized = S_i alpha replaces x_i and the block's view of its neighbours, and
the local test is ||b_i - A_block x_minimized|| (:437-438).
"""
from __future__ import annotations

import math
import os
import time
import uuid
from dataclasses import dataclass, field

from .petsc import AsyncBroadcast, AsyncMessages, ConvDetection


@dataclass
class AMResult:
    iterations: list = field(default_factory=list)     # outer iterations of each local block
    inner_its: list = field(default_factory=list)      # total inner GMRES iterations of each local block
    phase_tags: list = field(default_factory=list)
    norm0: float = 0.0
    final_norm: float = float("nan")
    error: float = float("nan")
    elapsed: float = 0.0
    trace: list = field(default_factory=list)          # (block, iteration, local norm, state, phase tag)
    timers: dict = field(default_factory=dict)         # host seconds per phase, summed over local blocks
    converged: bool = True                             # False: stopped at max_iterations (stop_at_limit)
    transport: str = "host"                            # "device" (HBM slots, xGMI) or "host" (shared memory)
    states: list = field(default_factory=list)         # detection state of each local block at the end (FINISHED)
    discarded: list = field(default_factory=list)      # messages / R blocks discarded unread at shutdown, per block
    in_flight: list = field(default_factory=list)      # own sends still in flight at shutdown (completed), per block


class AsyncBlock:
    """The asynchronous state of one block root: its message slots, its
    convergence-detection instance and its counters."""

    def __init__(self, blk, name: str, owner: bool, strict: bool, bcast_cap: int = 0):
        L = blk.layout
        self.blk = blk
        self.am = AsyncMessages(name, L.nb, L.b, max(L.plane, 1), owner)
        self.bcast = AsyncBroadcast(name + "_R", L.nb, L.b, bcast_cap, owner) if bcast_cap else None
        self.bcast_cap = bcast_cap
        nbrs = [nbr for nbr, *_ in L.recv]            # spanning tree = chain; dependencies = the same blocks
        self.cvd = ConvDetection(self.am, L.b, nbrs, nbrs, strict)
        self.it = 0
        self.steps = 0                                  # number_of_inner_times_outer_iterations (AMAM)
        self.inner = 0
        self.state = ConvDetection.NORMAL
        self.tag = 0
        self.local_norm = math.inf
        self.timers = {"solve": 0.0, "exchange": 0.0, "minimize": 0.0, "detect": 0.0}

    def _timed(self, key, fn, *args):
        t0 = time.perf_counter()
        r = fn(*args)
        self.timers[key] += time.perf_counter() - t0
        return r

    def _receive(self):
        """comm_async_probe_and_receive_prime: newest iterate of each dependency."""
        blk, L = self.blk, self.blk.layout
        for d, (nbr, hoff, cnt, _) in enumerate(L.recv):
            got, (tag, it) = blk.async_recv(self.am, nbr, hoff, cnt)
            if got and self.cvd.data_received(d, tag, it):
                blk.async_accept(hoff, cnt)

    def _publish(self, stamp: int):
        """comm_async_test_and_send_prime: the planes the neighbours read, (PhaseTag, stamp)."""
        for nbr, off, cnt in self.blk.layout.send:
            self.blk.async_send(self.am, nbr, off, cnt, self.tag, stamp)

    def _detect(self, norm0, rtol, atol, trace, block_norm: bool = False):
        blk, L = self.blk, self.blk.layout
        # MatResidual(A_ii, rhs, x) + VecNorm; AMAM-global: MatResidual(A_block, b_i, x_minimized)
        self.local_norm = math.sqrt(blk.block_residual_sq() if block_norm else blk.local_residual_sq())
        under = self.local_norm <= max(atol, rtol / math.sqrt(L.nb) * norm0)
        self.cvd.step(under)                                          # detection + receives
        self.it += 1
        self.state, self.tag = self.cvd.state()
        if trace is not None:
            trace.append((L.b, self.it, self.local_norm, self.state, self.tag))

    def iterate(self, norm0: float, rtol: float, atol: float, trace=None, variant: str = "am", s: int = 0):
        blk = self.blk
        T = self._timed
        if variant == "am":                                           # asynchronous-multisplitting_prime.c:333-377
            T("exchange", self._receive)
            blk.update_rhs()
            self.inner += T("solve", blk.solve)
            T("exchange", self._publish, self.it)
        elif variant in ("amam_semi_local", "amam_global"):          # AMAM-semi-local_prime.c:350-420,
            for k in range(s):                                        # AMAM-global_prime.c:378-413
                T("exchange", self._receive)
                blk.update_rhs()
                self.inner += T("solve", blk.solve)
                T("exchange", self._publish, self.steps)
                T("exchange", self._receive)
                blk.store_column(k)
                self.steps += 1
            if variant == "amam_global":
                T("minimize", blk.global_async_minimize, self.bcast)
            else:
                T("minimize", blk.semi_local_minimize, False)
        else:                                                         # AMAM-local_prime.c:371-404
            for k in range(s):
                T("exchange", self._receive)
                blk.update_rhs()
                self.inner += T("solve", blk.solve)
                T("exchange", self._publish, self.steps)
                blk.store_local_column(k)
                self.steps += 1
            T("minimize", blk.local_minimize)
        T("detect", self._detect, norm0, rtol, atol, trace, variant == "amam_global")

    def enable_device(self):
        """Device slots / buffers in this block's HBM (xGMI peer copies between GPUs).  The R
        broadcast takes two buffers, or one when two would not leave a quarter of the GPU's HBM free
        (the library's rule, msp_abcast_enable_device with nbuf 0; configs[3] scale: DESIGN.md section
        6.5); MSPLIT_ABCAST_NBUF forces 1 or 2."""
        self.am.enable_device(self.blk.ctx)
        if self.bcast is not None:
            nbuf = int(os.environ.get("MSPLIT_ABCAST_NBUF", "0"))
            self.bcast_nbuf = self.bcast.enable_device(self.blk.ctx, nbuf if nbuf in (1, 2) else 0)

    def discard_pending(self):
        """comm_discard_pending_messages and the MPI_Cancel of the pending sends
        (AMAM-global_prime.c:522-572): (discarded unread, own sends in flight)."""
        d, f = self.am.discard_pending()
        if self.bcast is not None:
            d2, f2 = self.bcast.discard_pending()
            d, f = d + d2, f + f2
        return d, f

    def close_peers(self):
        self.am.close_peers()
        if self.bcast is not None:
            self.bcast.close_peers()

    def close(self):
        self.cvd.destroy()
        self.am.destroy()
        if self.bcast is not None:
            self.bcast.destroy()


def _channel_name(comm) -> str:
    name = f"/msplit_am_{os.getpid()}_{uuid.uuid4().hex[:12]}"
    if getattr(comm, "world", 1) > 1:
        obj = [name if comm.rank == 0 else None]
        comm.dist.broadcast_object_list(obj, src=0, group=comm.group)
        name = obj[0]
    return name


def am_solve(blocks, comm, rtol: float, atol: float = 1e-100, max_iterations: int = 100000,
             strict: bool = False, record: bool = False, monitor=None, variant: str = "am", s: int = 0,
             stop_at_limit: bool = False, transport: str | None = None) -> AMResult:
    """The asynchronous multisplitting loop (asynchronous-multisplitting_prime.c:333-392);
    variant "amam_local" adds the block-local minimization every s inner steps
    (the blocks must have setup_local_minimization(s)), "amam_semi_local" the
    semi-local one (setup_minimization(s)), "amam_global" the global one
    (setup_global_async_minimization(s)).  At max_iterations the run raises, or
    (stop_at_limit, for timing runs) every block stops and the result says
    converged = False.  transport: "device" (payloads in the senders' HBM, peer copies
    over xGMI; the default for GpuBlocks) or "host" (staged through shared memory)."""
    if variant not in ("am", "amam_local", "amam_semi_local", "amam_global"):
        raise ValueError(f"unknown asynchronous variant {variant}")
    res = AMResult()
    # global_norm_0 = computeFinalResidualNorm at x = 0 (:322)
    res.norm0 = math.sqrt(comm.ordered_sum(blocks, [blk.norm0_sq() for blk in blocks]))
    name = _channel_name(comm)
    ordered = sorted(blocks, key=lambda b: b.layout.b)
    cap = 0
    if variant == "amam_global":                     # the largest block (of R, or Gram part) any block broadcasts
        cap = ordered[0].bcast_cap()
        if getattr(ordered[0], "minimization", "lsqr") == "lsqr":
            cap = max(R.shape[0] * R.shape[1] for R in ordered[0].R_rep)
    asyncs = {}
    owner_here = ordered[0].layout.b == 0
    if owner_here:                                   # block 0 creates the regions, the others open them
        asyncs[0] = AsyncBlock(ordered[0], name, True, strict, cap)
    comm.barrier()
    for blk in ordered:
        if blk.layout.b not in asyncs:
            asyncs[blk.layout.b] = AsyncBlock(blk, name, False, strict, cap)
    comm.barrier()
    if transport is None:
        transport = "device" if all(getattr(b, "async_transport", "host") == "device" for b in ordered) else "host"
    if transport not in ("device", "host"):
        raise ValueError(f"unknown transport {transport}")
    if transport == "device":                        # every block exports its slots before anyone sends
        for ab in asyncs.values():
            ab.enable_device()
        comm.barrier()
    for blk in blocks:                               # x_j = 0; updateLocalRHS before the loop (:329)
        blk.reset_halo()
        blk.update_rhs()
    comm.barrier()
    trace = [] if record else None
    t0 = time.perf_counter()
    active = [asyncs[b.layout.b] for b in ordered]
    while active:
        for ab in active:                            # round-robin over the blocks of this process
            ab.iterate(res.norm0, rtol, atol, trace, variant, s)
            if monitor:
                monitor(ab.blk.layout.b, ab.it, ab.local_norm, ab.state, ab.tag)
        active = [ab for ab in active if ab.state != ConvDetection.FINISHED]
        if any(ab.it >= max_iterations for ab in active):
            if not stop_at_limit:
                raise RuntimeError(f"asynchronous multisplitting did not terminate in {max_iterations} iterations")
            res.converged = False
            break
    comm.barrier()
    res.elapsed = time.perf_counter() - t0
    comm.exchange(blocks)                            # comm_sync_send_and_receive_final (:396)
    res.final_norm = math.sqrt(comm.ordered_sum(blocks, [blk.block_residual_sq() for blk in blocks]))
    res.error = math.sqrt(comm.ordered_sum(blocks, [blk.error_sq() for blk in blocks]))
    for blk in blocks:
        ab = asyncs[blk.layout.b]
        res.iterations.append(ab.it)
        res.inner_its.append(ab.inner)
        res.phase_tags.append(ab.tag)
        res.states.append(ab.state)
        for k, v in ab.timers.items():
            res.timers[k] = res.timers.get(k, 0.0) + v
    res.trace = trace or []
    res.transport = transport
    comm.barrier()
    for blk in blocks:                               # drain and cancel (every rank is past its loop)
        d, f = asyncs[blk.layout.b].discard_pending()
        res.discarded.append(d)
        res.in_flight.append(f)
    comm.barrier()
    for ab in asyncs.values():                       # unmap the peers' slots before anyone frees its own
        ab.close_peers()
    comm.barrier()
    for ab in asyncs.values():
        if ab.blk.layout.b != 0:
            ab.close()
    comm.barrier()
    if 0 in asyncs:
        asyncs[0].close()                            # the owner unlinks the region last
    return res
