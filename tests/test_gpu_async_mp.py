"""The asynchronous transports across processes on the GPU: device slots and
buffers in the sender's HBM, opened by the receivers through HIP IPC (the
xGMI mailboxes; on the one-GPU box both processes share cuda:0, so the peer
copies are same-device copies through the IPC mapping).  Two processes per
test, spawned fresh (no fork of a GPU-initialised parent)."""
import multiprocessing as mp
import os
import sys

import numpy as np
import pytest

from test_distributed_gloo import _free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _transport_worker(rank, name, n_msgs, n, q, nbuf=2):
    sys.path.insert(0, ROOT)
    import time
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import AsyncBroadcast, AsyncMessages, Context, DenseMat, Vec
    ctx = Context(0)
    if rank == 1:
        t0 = time.time()
        while True:                                   # the owner (rank 0) creates the regions first
            try:
                am = AsyncMessages(name, 2, 1, n, owner=False)
                bc = AsyncBroadcast(name + "_R", 2, 1, n * 3, owner=False)
                break
            except Exception:
                if time.time() - t0 > 60:
                    raise
                time.sleep(0.05)
    else:
        am = AsyncMessages(name, 2, 0, n, owner=True)
        bc = AsyncBroadcast(name + "_R", 2, 0, n * 3, owner=True)
    am.enable_device(ctx)
    bc.enable_device(ctx, nbuf)
    while am.attached() < 2:
        time.sleep(0.01)
    ok = True
    if rank == 1:                                     # the writer: planes and dense blocks stamped k
        v = Vec(ctx, n)
        D = DenseMat(ctx, n, 3)
        for k in range(1, n_msgs + 1):
            v.set(float(k))
            posted = am.stats()[0]
            am.send_vec(0, [k, k], v, 0, n)
            while k == n_msgs and am.stats()[0] == posted:  # skipped (comm_async_test_and_send_prime's MPI_Test:
                time.sleep(0.001)                            # the last copy not yet published, or the reader still
                am.send_vec(0, [k, k], v, 0, n)              # holds the free buffer): the last plane must land
            if k % 10 == 0 or k == n_msgs:
                for j in range(3):
                    D.set_column(j, 0, v)
                while not bc.publish_dense(D):
                    pass
        am.send(0, AsyncMessages.VERDICT, [n_msgs, 1])
        got_done = False
        while not got_done:                           # wait for the reader before unmapping anything
            got_done = am.recv(0, AsyncMessages.VERDICT, 1)[0]
            time.sleep(0.01)
        am.close_peers()
        bc.close_peers()
        sent, skipped = am.stats()
        am.destroy()
        bc.destroy()
        q.put((rank, ok and sent >= 1 and sent + skipped >= n_msgs, sent, skipped))
        return
    y = Vec(ctx, n)
    R = DenseMat(ctx, n, 3)
    last, taken, last_r, done = 0, 0, 0, False
    while not done or last < n_msgs or last_r < n_msgs:
        got, ints, _ = am.recv_vec(1, 2, y, 0, n)
        if got:
            a = y.get_array()
            ok = ok and ints[0] == ints[1] > last and bool(np.all(a == float(ints[0])))
            last, taken = ints[0], taken + 1
        if bc.fetch_dense(1, R):
            a = R.get_values()
            ok = ok and bool(np.all(a == a[0, 0])) and a[0, 0] > last_r
            last_r = a[0, 0]
        done = done or am.recv(1, AsyncMessages.VERDICT, 2)[0]
    am.close_peers()                                  # unmap the writer's slots, then let it free them
    bc.close_peers()
    am.send(1, AsyncMessages.VERDICT, [1])
    time.sleep(0.5)
    am.destroy()
    bc.destroy()
    q.put((rank, ok, taken, last))


def _inflight_worker(rank, name, n, q):
    sys.path.insert(0, ROOT)
    import time
    import torch  # noqa: F401
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import AsyncBroadcast, AsyncMessages, Context, DenseMat, Vec
    ctx = Context(0)
    if rank == 1:
        t0 = time.time()
        while True:
            try:
                am = AsyncMessages(name, 2, 1, n, owner=False)
                bc = AsyncBroadcast(name + "_R", 2, 1, n * 2, owner=False)
                break
            except Exception:
                if time.time() - t0 > 60:
                    raise
                time.sleep(0.05)
    else:
        am = AsyncMessages(name, 2, 0, n, owner=True)
        bc = AsyncBroadcast(name + "_R", 2, 0, n * 2, owner=True)
    am.enable_device(ctx)
    bc.enable_device(ctx, 2)
    while am.attached() < 2:
        time.sleep(0.01)
    if rank == 1:                       # the sender: its last send still queued on the stream at shutdown
        v = Vec(ctx, n)
        v.set(7.0)
        busy = Vec(ctx, 1 << 27)        # 1 GiB: milliseconds of stream work ahead of the send's copy and publish
        busy.set(1.0)
        for _ in range(12):
            busy.scale(-1.0)            # (VecScale returns at once for 1.0)
        am.send_vec(0, [7, 7], v, 0, n)
        discarded, in_flight = am.discard_pending()    # the MPI_Cancel point: the send cannot be withdrawn (a DMA),
        sent, skipped = am.stats()                      # so the drain completes it (and syncs the stream)
        D = DenseMat(ctx, n, 2)                         # an R block, queued the same way behind stream work
        v.set(9.0)
        D.set_column(0, 0, v)
        D.set_column(1, 0, v)
        for _ in range(12):
            busy.scale(-1.0)
        published = bc.publish_dense(D)
        bdisc, bflight = bc.discard_pending()
        am.send(0, AsyncMessages.VERDICT, [1])
        while not am.recv(0, AsyncMessages.VERDICT, 1)[0]:
            time.sleep(0.01)
        am.close_peers()
        bc.close_peers()
        am.destroy()
        bc.destroy()
        q.put((rank, in_flight, sent, skipped, published, bflight))
        return
    while not am.recv(1, AsyncMessages.VERDICT, 1)[0]:  # the sender has drained
        time.sleep(0.01)
    y = Vec(ctx, n)
    got, ints, m = am.recv_vec(1, 2, y, 0, n)
    ok = got and ints == [7, 7] and m == n and bool(np.all(y.get_array() == 7.0))
    R = DenseMat(ctx, n, 2)
    ok = ok and bc.fetch_dense(1, R) and bool(np.all(R.get_values() == 9.0))
    am.close_peers()
    bc.close_peers()
    am.send(1, AsyncMessages.VERDICT, [1])
    time.sleep(0.5)
    am.destroy()
    bc.destroy()
    q.put((rank, ok))


def test_send_in_flight_at_shutdown_is_completed():
    """The end of an asynchronous run (AMAM-global_prime.c:522-572: MPI_Cancel of the sends still pending, then
    comm_discard_pending_messages): a plane send whose copy and publish are still queued behind milliseconds of
    stream work when the sender drains is counted in flight, completed by the drain (a DMA cannot be withdrawn), and
    its plane reaches the receiver whole; the same for an R block published through the broadcast."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/msplit_inflight_{os.getpid()}"
    n = 1 << 22
    procs = [ctx.Process(target=_inflight_worker, args=(r, name, n, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][1]                                    # the receiver got the whole plane
    assert out[1][1] == 1 and out[1][2] == 1 and out[1][3] == 0, out[1]   # one send, posted, in flight at the drain
    assert out[1][4] and out[1][5] == 1, out[1]                           # the R block likewise


@pytest.mark.parametrize("nbuf", [2, 1])
def test_device_slots_cross_process_whole_and_newest(nbuf):
    """Every plane and block a receiver takes from the sender's HBM is whole and
    newer than the last, and the last one arrives (R broadcast with two device
    buffers, or one).  Plane sends and receives never wait on the host: the
    stream publishes each plane behind its copy and releases the buffer a
    receiver copied, and a send that finds its free buffer still being read is
    skipped (counted in stats), as the reference's MPI_Test-gated Isend."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    name = f"/msplit_ipc_{os.getpid()}_{nbuf}"
    n, n_msgs = 1 << 16, 400
    procs = [ctx.Process(target=_transport_worker, args=(r, name, n_msgs, n, q, nbuf)) for r in range(2)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=300) for _ in range(2)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0][1] and out[1][1]
    assert out[0][3] == n_msgs and out[0][2] >= 1


def _am_worker(rank, world, port, problem, q):
    sys.path.insert(0, ROOT)
    import time
    from datetime import timedelta
    import torch  # noqa: F401
    import torch.distributed as dist
    from medane_tchakorom_ufc_thesis_repository_amd.asynchronous import am_solve
    from medane_tchakorom_ufc_thesis_repository_amd.comm import TorchComm
    from medane_tchakorom_ufc_thesis_repository_amd.multisplitting import make_blocks
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Options
    # a rank stuck in a collective raises after 240 s instead of holding the others (and the test) forever
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=timedelta(seconds=240))
    try:
        variant, dim, nx, ny, nz, s, max_it, rtol = problem[:8]
        minimization = problem[8] if len(problem) > 8 else "lsqr"
        peclet = problem[9] if len(problem) > 9 else None
        b = rank
        opts = Options(f"-inner{b + 1}_ksp_max_it {max_it} -inner{b + 1}_ksp_rtol 1e-20 -inner{b + 1}_pc_type none "
                       f"-outer{b + 1}_ksp_type lsqr -outer{b + 1}_ksp_convergence_test default "
                       f"-outer{b + 1}_ksp_lsqr_exact_mat_norm -outer{b + 1}_ksp_atol 1e-100 "
                       f"-outer{b + 1}_ksp_max_it 70 -outer{b + 1}_ksp_rtol 1e-15")
        ctx = Context(0)
        comm = TorchComm()
        (blk,) = make_blocks(ctx, dim, nx, ny, nz, world, [rank], opts, comm, peclet=peclet)
        if variant == "amam_global":
            blk.setup_global_async_minimization(s, minimization=minimization)
        last = [None]
        tdir = os.environ.get("MSPLIT_TEST_TRACE_DIR")   # diagnostics: every iteration's detection state per rank
        tf = open(os.path.join(tdir, f"rank{rank}.txt"), "w", buffering=1) if tdir else None
        import medane_tchakorom_ufc_thesis_repository_amd.asynchronous as A
        mine = {}
        orig = A.AsyncBlock.__init__

        def init(self, *a, **kw):
            orig(self, *a, **kw)
            mine["ab"] = self
            if tf is not None:  # every data message the detection is offered: (dependency, tag, stamp, taken)
                dr = self.cvd.data_received

                def logged(d, tag, it, _dr=dr):
                    ok = _dr(d, tag, it)
                    tf.write(f"R {d} {tag} {it} {int(ok)}\n")
                    return ok
                self.cvd.data_received = logged
        A.AsyncBlock.__init__ = init

        def progress(b, it, ln, st, tag):   # state changes and every 500th iteration on stderr (visible with -s)
            if tf is not None and "ab" in mine:
                ab = mine["ab"]
                links = [ab.am.link_info(nb) for nb, *_ in ab.blk.layout.recv]
                tf.write(f"{it} {ln:.3e} {ab.cvd.info()} {ab.am.stats()} {time.time():.4f} {links}\n")
            if (st, tag) != last[0] or it % 500 == 0:
                print(f"rank {rank} iteration {it} local residual {ln:.3e} state {st} tag {tag}", file=sys.stderr,
                      flush=True)
                last[0] = (st, tag)
        res = am_solve([blk], comm, rtol=rtol, max_iterations=int(os.environ.get("MSPLIT_TEST_MAX_ITS", "20000")),
                       variant=variant, s=s, monitor=progress)
        q.put((rank, res.iterations[0], res.phase_tags[0], res.norm0, res.final_norm, res.transport, res.states[0],
               res.discarded[0], res.in_flight[0]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,problem,nbuf", [(2, ("am", 3, 8, 8, 16, 0, 5, 1e-6), "2"),
                                                (2, ("amam_global", 3, 8, 8, 16, 4, 5, 1e-6), "2"),
                                                (3, ("amam_global", 3, 8, 8, 18, 4, 5, 1e-6), "1"),
                                                (2, ("amam_global", 3, 8, 8, 16, 4, 5, 1e-6, "rtr"), "2"),
                                                (3, ("amam_global", 3, 8, 8, 18, 4, 5, 1e-6, "rtr"), "1")])
def test_am_processes_device_transport(world, problem, nbuf, monkeypatch):
    """One process per block, truly asynchronous, planes (and for AMAM-global the
    R rows, with two or one HBM buffers) through HBM slots opened by IPC: the
    detection ends every block in the same phase with one global final residual
    below the threshold."""
    monkeypatch.setenv("MSPLIT_ABCAST_NBUF", nbuf)       # inherited by the spawned workers
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_am_worker, args=(r, world, port, problem, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = sorted([q.get(timeout=600) for _ in range(world)])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(o[5] == "device" for o in out)
    assert all(o[3] == out[0][3] and o[4] == out[0][4] for o in out)
    assert out[0][4] <= 1e-4 * out[0][3]
    assert all(o[2] == out[0][2] for o in out)
    assert all(o[6] == 3 for o in out)                    # every block FINISHED (constants.h State)


PE = (0.5, 0.25, -0.3)


@pytest.mark.parametrize("problem,nbuf", [
    (("am", 3, 8, 8, 32, 0, 5, 1e-6), "2"),
    (("am", 3, 8, 8, 32, 0, 5, 1e-6, "lsqr", PE), "2"),
    (("amam_global", 3, 8, 8, 32, 4, 5, 1e-6), "2"),
    (("amam_global", 3, 8, 8, 32, 4, 5, 1e-6), "1"),
    (("amam_global", 3, 8, 8, 32, 4, 5, 1e-6, "lsqr", PE), "1"),
    (("amam_global", 3, 8, 8, 32, 4, 5, 1e-6, "rtr"), "2"),
    (("amam_global", 3, 8, 8, 32, 4, 5, 1e-6, "rtr", PE), "1"),
], ids=["am", "am-convdiff", "amam-lsqr-nbuf2", "amam-lsqr-nbuf1", "amam-lsqr-convdiff-nbuf1", "amam-rtr-nbuf2",
        "amam-rtr-convdiff-nbuf1"])
def test_am_eight_processes_device_transport(problem, nbuf, monkeypatch):
    """configs[3]/[4]'s world size: 8 processes, one block each, truly asynchronous on the one GPU -- the planes
    and (AMAM-global) the R rows or Gram parts through HBM slots opened by IPC, the detection over a chain of
    diameter 7 (conv_detection_prime.c:11-210; AMAM-global_prime.c:371-481).  Every process ends FINISHED in one
    phase tag, all report the same global final residual below the threshold, each drains the messages still
    pending and completes its sends still in flight (comm_discard_pending_messages and the MPI_Cancel calls,
    AMAM-global_prime.c:522-572), and every process exits 0."""
    world = 8
    monkeypatch.setenv("MSPLIT_ABCAST_NBUF", nbuf)
    # one hardware queue per rank.  This GPU's KFD node maps 24 compute queues (topology `num_cp_queues`, recorded in
    # profiles/r06/async8/kfd_props.txt); HIP gives each process up to four.  Eight ranks plus a pytest parent that
    # has run GPU tests (its own four queues) oversubscribe those slots, and the scheduler then runs the processes
    # one at a time: one rank ran 600 iterations alone in 5 s while the seven others sat at their second (and, with
    # no iteration cap, forever: the hang of the first suite run).  With one queue per rank the eight interleave
    # and the run terminates in ~30 iterations per rank (profiles/r06/async8/).  Not a property of the asynchronous
    # protocol: configs[3]/[4] run one process per GPU.
    monkeypatch.setenv("GPU_MAX_HW_QUEUES", os.environ.get("MSPLIT_TEST_WORKER_HW_QUEUES", "1"))
    tdir = os.environ.get("MSPLIT_TEST_TRACE_DIR")
    if tdir:                                               # diagnostics: what the GPU holds before the ranks start
        import subprocess
        with open(os.path.join(tdir, "parent_vram.txt"), "w") as f:
            f.write(subprocess.run(["rocm-smi", "--showmeminfo", "vram", "--showpids"], capture_output=True,
                                   text=True, timeout=60).stdout)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_am_worker, args=(r, world, port, problem, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        out = sorted([q.get(timeout=300) for _ in range(world)])
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.exitcode is None:
                p.kill()
    assert [p.exitcode for p in procs] == [0] * world
    assert [o[0] for o in out] == list(range(world))
    assert all(o[5] == "device" for o in out)
    assert all(o[6] == 3 for o in out), [o[6] for o in out]          # FINISHED
    assert len({o[2] for o in out}) == 1, [o[2] for o in out]        # one phase tag
    assert all(o[3] == out[0][3] and o[4] == out[0][4] for o in out)
    assert out[0][4] <= 1e-4 * out[0][3]
    assert all(o[7] >= 0 and o[8] >= 0 for o in out)
    print("iterations", [o[1] for o in out], "discarded", [o[7] for o in out], "in_flight", [o[8] for o in out])


def _comm_worker(rank, world, port, q):
    sys.path.insert(0, ROOT)
    import torch
    import torch.distributed as dist
    from medane_tchakorom_ufc_thesis_repository_amd.comm import TorchComm
    from medane_tchakorom_ufc_thesis_repository_amd.petsc import Context, Vec
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        ctx = Context(0)
        os.environ["MSPLIT_LSQR_TRANSPORT"] = "host"
        comm = TorchComm().lsqr_comm(ctx)               # the host-callback msp_comm over gloo
        n, p = 40, 6
        src = Vec.from_array(ctx, 1000.0 * rank + np.arange(n, dtype=np.float64))
        dst = Vec.from_array(ctx, np.full(2 * p, -1.0))
        comm.exchange_neighbors(src, 0, n - p, dst, 0, p, p)   # first plane down, last plane up
        got = dst.get_array()
        s = comm.sum_ordered(np.array([rank + 0.1, 2.0 ** -rank]))
        q.put((rank, got, s))
        comm.destroy()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


def test_comm_exchange_neighbors_host_transport_three_ranks():
    """msp_comm_exchange_neighbors / msp_comm_sum_ordered across three processes
    (host transport over gloo): each rank receives exactly its neighbours'
    boundary planes and every rank holds the same rank-ordered sum."""
    world, n, p = 3, 40, 6
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_comm_worker, args=(r, world, port, q)) for r in range(world)]
    for pr in procs:
        pr.start()
    out = sorted([q.get(timeout=300) for _ in range(world)], key=lambda t: t[0])
    for pr in procs:
        pr.join(timeout=60)
        assert pr.exitcode == 0
    for rank, got, s in out:
        lo = 1000.0 * (rank - 1) + np.arange(n - p, n) if rank > 0 else np.full(p, -1.0)
        hi = 1000.0 * (rank + 1) + np.arange(p) if rank < world - 1 else np.full(p, -1.0)
        assert np.array_equal(got, np.concatenate([lo, hi]))
        exp0 = 0.0
        for r in range(world):
            exp0 += r + 0.1
        assert s[0] == exp0 and s[1] == 1.0 + 0.5 + 0.25
