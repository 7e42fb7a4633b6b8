"""Deterministic replay of asynchronous multisplitting (AM) for the tests.

TEST INFRASTRUCTURE ONLY (imported by tests/ alone).  Restates, independently
of the product's C code (csrc/amsg.c, csrc/conv_detect.c) and driver
(asynchronous.py):

  * the AM loop, src/asynchronous-multisplitting/asynchronous-multisplitting_prime.c:333-392
    (newest iterate per dependency, RHS update, inner GMRES, publish, local
    residual, threshold rtol/sqrt(nb)*||b||, detection step), and the final
    synchronous exchange and residual (:394-427);
  * the convergence detection of src/utils/conv_detection_prime.c (Algorithm 5.15),
    including its test of the pointer `UnderThreashold` (never false) during
    verification, over a chain spanning tree;
  * the drain-to-newest message semantics of comm.c:455-554 and the detection's
    Iprobe/Recv loops, as newest-value slots,

on the round-robin schedule the product uses when all blocks live in one
process: blocks iterate in block order, a message is visible as soon as it is
sent.  The arithmetic is the oracle's (oracle/oracle.c via pyoracle, DBR order),
so the product must replay it bit for bit.
"""
from __future__ import annotations

import math

import numpy as np

NORMAL, WAIT4VERIFICATION, VERIFICATION, FINISHED = 0, 1, 2, 3
DATA, PARTIAL_CV, VERIFICATION_MSG, RESPONSE, VERDICT = 0, 1, 2, 3, 4


class Slots:
    """Newest message per (src, dst, kind); each receiver remembers what it took."""

    def __init__(self):
        self.slot = {}
        self.seen = {}

    def send(self, src, dst, kind, payload):
        seq = self.slot.get((src, dst, kind), (0, None))[0] + 1
        self.slot[(src, dst, kind)] = (seq, payload)

    def recv(self, src, dst, kind):
        seq, payload = self.slot.get((src, dst, kind), (0, None))
        if seq == 0 or self.seen.get((src, dst, kind)) == seq:
            return None
        self.seen[(src, dst, kind)] = seq
        return payload


class Detector:
    """conv_detection_prime.c for one block root (chain tree)."""

    def __init__(self, rank, neighbors, net: Slots, strict=False):
        self.rank = rank
        self.nbrs = list(neighbors)
        self.net = net
        self.strict = strict
        self.phase = 0
        self.last_iter = [-1] * len(self.nbrs)
        self.newer = [False] * len(self.nbrs)
        self.responses = [0] * len(self.nbrs)
        self.response_sent = False
        self._initialize_state()

    # -- the reference's helpers
    def _reinit_pseudo_period(self):
        self.pp_begin = self.pp_end = False
        self.newer = [False] * len(self.nbrs)

    def _initialize_state(self):
        self.not_recvd = len(self.nbrs)
        self.got_pcv = [False] * len(self.nbrs)
        self.elected = False
        self.local_cv = False
        self.pcv_sent = False
        self._reinit_pseudo_period()
        self.state = NORMAL

    def _initialize_verification(self):
        self._reinit_pseudo_period()
        self.phase += 1
        self.responses = [0] * len(self.nbrs)
        self.response_sent = False

    def _send(self, dst, kind, payload):
        self.net.send(self.rank, dst, kind, payload)

    def data_received(self, d, tag, it):
        if self.last_iter[d] < it and (self.state != VERIFICATION or tag == self.phase):
            self.last_iter[d] = it
            self.newer[d] = True
            return True
        return False

    def step(self, under):
        self._detect(under)
        self._recv_partial_cv()
        self._recv_verification()
        self._recv_response()
        self._recv_verdict()

    def _detect(self, under):
        veto = (not under) if self.strict else False     # the reference compares a pointer with PETSC_FALSE
        if self.state == NORMAL:
            if not under:
                self._reinit_pseudo_period()
            elif not self.pp_begin:
                self.pp_begin = True
            elif self.pp_end:
                self.local_cv = True
                if self.not_recvd == 0:
                    self.elected = True
                    self._initialize_verification()
                    for n in self.nbrs:
                        self._send(n, VERIFICATION_MSG, (self.phase,))
                    self.state = VERIFICATION
                elif self.not_recvd == 1:
                    for i, n in enumerate(self.nbrs):
                        if not self.got_pcv[i]:
                            self._send(n, PARTIAL_CV, (self.phase,))
                            break
                    self.pcv_sent = True
                    self.state = WAIT4VERIFICATION
            elif all(self.newer):
                self.pp_end = True
        elif self.state == WAIT4VERIFICATION:
            if veto:
                self.local_cv = False
        elif self.state == VERIFICATION:
            negative = -1 in self.responses
            if self.elected:
                if veto or not self.local_cv or negative:
                    self.phase += 1
                    for n in self.nbrs:
                        self._send(n, VERDICT, (self.phase, -1))
                    self._initialize_state()
                elif self.pp_end:
                    if 0 not in self.responses:
                        if not negative:
                            for n in self.nbrs:
                                self._send(n, VERDICT, (self.phase, 1))
                            self.state = FINISHED
                        else:
                            self.phase += 1
                            for n in self.nbrs:
                                self._send(n, VERDICT, (self.phase, -1))
                            self._initialize_state()
                elif all(self.newer):
                    self.pp_end = True
            elif not self.response_sent:
                if veto or not self.local_cv or negative:
                    for i, n in enumerate(self.nbrs):
                        if not self.got_pcv[i]:
                            self._send(n, RESPONSE, (self.phase, -1))
                            break
                    self.response_sent = True
                elif self.pp_end:
                    if self.responses.count(0) == 1:
                        asking = self.nbrs[self.responses.index(0)]
                        ok = self.responses.count(1) == len(self.nbrs) - 1
                        self._send(asking, RESPONSE, (self.phase, 1 if ok else -1))
                        self.response_sent = True
                elif all(self.newer):
                    self.pp_end = True

    def _recv_partial_cv(self):
        for i, n in enumerate(self.nbrs):
            m = self.net.recv(n, self.rank, PARTIAL_CV)
            if m is None or m[0] != self.phase:
                continue
            self.got_pcv[i] = True
            self.not_recvd -= 1
            if self.not_recvd == 0 and self.pcv_sent and max(self.rank, n) == self.rank:
                self.elected = True
                self._initialize_verification()
                for k in self.nbrs:
                    self._send(k, VERIFICATION_MSG, (self.phase,))
                self.state = VERIFICATION

    def _recv_verification(self):
        for n in self.nbrs:
            m = self.net.recv(n, self.rank, VERIFICATION_MSG)
            if m is None or m[0] != self.phase + 1:
                continue
            self._initialize_verification()
            self.state = VERIFICATION
            for k in self.nbrs:
                if k != n:
                    self._send(k, VERIFICATION_MSG, (self.phase,))

    def _recv_response(self):
        for i, n in enumerate(self.nbrs):
            m = self.net.recv(n, self.rank, RESPONSE)
            if m is not None and m[0] == self.phase:
                self.responses[i] = m[1]

    def _recv_verdict(self):
        for n in self.nbrs:
            m = self.net.recv(n, self.rank, VERDICT)
            if m is None:
                continue
            if m[1] == 1:
                self.state = FINISHED
            else:
                self._initialize_state()
                self.phase = m[0]
            for k in self.nbrs:
                if k != n:
                    self._send(k, VERDICT, (self.phase, m[1]))


def _block_rows(po, dim, nx, ny, nz, nb, b, peclet=None):
    """Block b's rows of the reference operator (Poisson) or the convection-diffusion one."""
    N = nx * ny * (nz if dim == 3 else 1)
    rows = N // nb
    if peclet is not None and any(peclet):
        return po.convdiff_rows(dim, nx, ny, nz, b * rows, (b + 1) * rows, peclet)
    if dim == 3:
        ppb = nz // nb
        return po.poisson3d_rows(nx, ny, nz, b * ppb, (b + 1) * ppb)
    return po.poisson2d_rows(nx, ny, b * rows, (b + 1) * rows)


def am_roundrobin(po, dim, nx, ny, nz, nb, rtol, inner: dict, atol=1e-100, max_iterations=100000, strict=False,
                  variant="am", s=0, outer: dict | None = None, peclet=None):
    """Replay AM (or, variant "amam_local", AMAM-local: s inner steps then the
    block-local LSQR minimization, AMAM-local_prime.c:371-431) on nb blocks, round-robin.  Returns a dict with per-block
    iterations / inner iterations / phase tags, the trace of (block, iteration,
    local norm, state, phase tag), the final iterate, final residual and error."""
    mode = po.REDUCE_DBR
    nz = nz if dim == 3 else 1
    N = nx * ny * nz
    if dim == 3:
        plane, rows = nx * ny, N // nb
    else:
        plane, rows = ny, N // nb
    blocks = []
    for b in range(nb):
        r0, r1 = b * rows, (b + 1) * rows
        Ab = _block_rows(po, dim, nx, ny, nz, nb, b, peclet)
        Aii, Aoff = po.split(Ab, r0, r1)
        bb = Ab.mult(np.ones(N))
        nbrs = [k for k in (b - 1, b + 1) if 0 <= k < nb]
        blocks.append(dict(b=b, r0=r0, r1=r1, Ab=Ab, Aii=Aii, Aoff=Aoff, rhs_b=bb, x=np.zeros(rows),
                           view=np.zeros(N), nbrs=nbrs, it=0, inner=0))
    net = Slots()
    dets = [Detector(blk["b"], blk["nbrs"], net, strict) for blk in blocks]
    norm0 = math.sqrt(sum_ordered([po.norm2(blk["rhs_b"], mode) ** 2 for blk in blocks]))
    thr = max(atol, rtol / math.sqrt(nb) * norm0)
    opts = dict(inner, guess_nonzero=1, uirnorm=1, reduce_mode=mode)
    trace = []

    def plane_for(blk, nbr):         # the plane of blk that nbr's coupling rows read
        return blk["x"][:plane].copy() if nbr < blk["b"] else blk["x"][rows - plane:].copy()

    def store(blk, nbr, data):       # nbr's plane into blk's view of x
        lo = nbr * rows + (rows - plane if nbr < blk["b"] else 0)
        blk["view"][lo:lo + plane] = data

    outer = dict(outer or {}, reduce_mode=mode)

    def receive(blk, det):
        for d, nbr in enumerate(blk["nbrs"]):
            m = net.recv(nbr, blk["b"], DATA)
            if m is not None and det.data_received(d, m[0], m[1]):
                store(blk, nbr, m[2])

    def inner_step(blk, det, stamp):
        rhs = blk["Aoff"].residual(blk["rhs_b"], blk["view"])
        blk["x"], r = po.gmres(blk["Aii"], rhs, x0=blk["x"], **opts)
        blk["inner"] += r["its"]
        for nbr in blk["nbrs"]:
            net.send(blk["b"], nbr, DATA, (det.phase, stamp, plane_for(blk, nbr)))
        return rhs

    active = list(range(nb))
    while active:
        for bi in active:
            blk, det = blocks[bi], dets[bi]
            if variant == "am":
                receive(blk, det)
                rhs = inner_step(blk, det, blk["it"])
            else:
                S = np.zeros((rows, s), order="F")
                for k in range(s):
                    receive(blk, det)
                    inner_step(blk, det, blk.setdefault("steps", 0))
                    S[:, k] = blk["x"]
                    blk["steps"] += 1
                R = np.stack([blk["Aii"].mult(np.ascontiguousarray(S[:, k])) for k in range(s)], axis=1)
                rhs = blk["Aoff"].residual(blk["rhs_b"], blk["view"])
                alpha, _ = po.lsqr([R], [rhs], **outer)
                blk["x"] = po.dense_mult(S, alpha)
            ln = po.norm2(blk["Aii"].residual(rhs, blk["x"]), mode)
            det.step(ln <= thr)
            blk["it"] += 1
            trace.append((blk["b"], blk["it"], ln, det.state, det.phase))
            if blk["it"] >= max_iterations:
                raise RuntimeError("no termination")
        active = [bi for bi in active if dets[bi].state != FINISHED]
    x = np.concatenate([blk["x"] for blk in blocks])
    fin, err = [], []
    for blk in blocks:                                # final synchronous exchange, full-row residual
        rr = blk["Ab"].residual(blk["rhs_b"], x)
        fin.append(po.norm2(rr, mode) ** 2)
        err.append(po.norm2(blk["x"] - 1.0, mode) ** 2)
    return {"iterations": [blk["it"] for blk in blocks], "inner_its": [blk["inner"] for blk in blocks],
            "phase_tags": [d.phase for d in dets], "trace": trace, "x": x, "norm0": norm0,
            "final_norm": math.sqrt(sum_ordered(fin)), "error": math.sqrt(sum_ordered(err))}


def sum_ordered(values):
    t = 0.0
    for v in values:
        t += v
    return t


def smsm_local(po, dim, nx, ny, nz, nb, s, rtol, inner: dict, outer: dict, atol=1e-100, max_outer=1000,
               peclet=None):
    """SMSM with block-local minimization (synchronous-multisplitting-synchronous-
    minimization-local.c): s times {rhs_i, inner GMRES, exchange, S_i(:,k) = x_i},
    R_i = A_ii S_i, rhs_i, x_i = S_i LSQR(R_i, rhs_i); stop when every block's
    ||rhs_i - A_ii x_i|| <= max(atol, rtol/sqrt(nb) ||b||).  Oracle arithmetic (DBR)."""
    mode = po.REDUCE_DBR
    nz = nz if dim == 3 else 1
    N = nx * ny * nz
    rows = N // nb
    blocks = []
    for b in range(nb):
        r0, r1 = b * rows, (b + 1) * rows
        Ab = _block_rows(po, dim, nx, ny, nz, nb, b, peclet)
        Aii, Aoff = po.split(Ab, r0, r1)
        blocks.append(dict(r0=r0, Ab=Ab, Aii=Aii, Aoff=Aoff, rhs_b=Ab.mult(np.ones(N))))
    x = np.zeros(N)        # every block's own rows
    view = np.zeros(N)     # what the blocks last exchanged (x_j of updateLocalRHS)
    norm0 = math.sqrt(sum_ordered([po.norm2(blk["rhs_b"], mode) ** 2 for blk in blocks]))
    thr = max(atol, rtol / math.sqrt(nb) * norm0)
    opts = dict(inner, guess_nonzero=1, uirnorm=1, reduce_mode=mode)
    outer = dict(outer, reduce_mode=mode)
    hist, lits_all, inner_all = [], [], []
    outer_its = 0
    while True:
        S = [np.zeros((rows, s), order="F") for _ in range(nb)]
        its_outer = []
        for k in range(s):
            rhs = [blk["Aoff"].residual(blk["rhs_b"], view) for blk in blocks]
            its = []
            xn = x.copy()
            for b, blk in enumerate(blocks):
                xb, r = po.gmres(blk["Aii"], rhs[b], x0=x[blk["r0"]:blk["r0"] + rows], **opts)
                xn[blk["r0"]:blk["r0"] + rows] = xb
                its.append(r["its"])
            x = xn
            view = x.copy()                              # the exchange: every block sees every x_j
            its_outer.append(its)
            for b, blk in enumerate(blocks):
                S[b][:, k] = x[blk["r0"]:blk["r0"] + rows]
        norms, lits = [], []
        xn = x.copy()
        for b, blk in enumerate(blocks):
            R = np.stack([blk["Aii"].mult(np.ascontiguousarray(S[b][:, k])) for k in range(s)], axis=1)
            rhs = blk["Aoff"].residual(blk["rhs_b"], view)
            alpha, r = po.lsqr([R], [rhs], **outer)
            xb = po.dense_mult(S[b], alpha)
            xn[blk["r0"]:blk["r0"] + rows] = xb
            lits.append(r["its"])
            norms.append(po.norm2(blk["Aii"].residual(rhs, xb), mode))
        x = xn                                           # own rows minimized; view unchanged until the next exchange
        hist.append(norms)
        lits_all.append(lits)
        inner_all.append(its_outer)
        outer_its += 1
        if all(n <= thr for n in norms) or outer_its >= max_outer:
            break
    fin = [po.norm2(blk["Ab"].residual(blk["rhs_b"], x), mode) ** 2 for blk in blocks]
    err = [po.norm2(x[blk["r0"]:blk["r0"] + rows] - 1.0, mode) ** 2 for blk in blocks]
    return {"outer_its": outer_its, "norm0": norm0, "hist": hist, "lsqr_its": lits_all, "inner_its": inner_all,
            "x": x, "final_norm": math.sqrt(sum_ordered(fin)), "error": math.sqrt(sum_ordered(err))}


def _blocks_ext(po, dim, nx, ny, nz, nb, peclet=None):
    """Block rows with the ext column space [plane below | own | plane above]."""
    nz = nz if dim == 3 else 1
    N = nx * ny * nz
    rows = N // nb
    plane = nx * ny if dim == 3 else ny
    out = []
    for b in range(nb):
        r0, r1 = b * rows, (b + 1) * rows
        Ab = _block_rows(po, dim, nx, ny, nz, nb, b, peclet)
        Aii, Aoff = po.split(Ab, r0, r1)
        lo = plane if b > 0 else 0
        hi = plane if b < nb - 1 else 0
        rp, c, v = Ab.arrays()
        Aext = po.Mat.from_arrays(rows, lo + rows + hi, rp, c - (r0 - lo), v)
        out.append(dict(b=b, r0=r0, r1=r1, lo=lo, hi=hi, Ab=Ab, Aii=Aii, Aoff=Aoff, Aext=Aext,
                        rhs_b=Ab.mult(np.ones(N)), x=np.zeros(rows), view=np.zeros(N),
                        nbrs=[k for k in (b - 1, b + 1) if 0 <= k < nb], it=0, inner=0, steps=0))
    return out, N, rows, plane


def _ext_col(blk, rows):
    r0, lo, hi = blk["r0"], blk["lo"], blk["hi"]
    return np.concatenate([blk["view"][r0 - lo:r0], blk["x"], blk["view"][r0 + rows:r0 + rows + hi]])


def _apply_ext(blk, xe, rows):
    r0, lo, hi = blk["r0"], blk["lo"], blk["hi"]
    blk["x"] = xe[lo:lo + rows].copy()
    blk["view"][r0 - lo:r0] = xe[:lo]
    blk["view"][r0 + rows:r0 + rows + hi] = xe[lo + rows:]


def smsm_semi_local(po, dim, nx, ny, nz, nb, s, rtol, inner: dict, outer: dict, atol=1e-100, max_outer=1000,
                    peclet=None):
    """SMSM with semi-local minimization (synchronous-multisplitting-synchronous-
    minimization-semi-local.c): s times {rhs_i, inner GMRES, exchange, S_i(:,k) = x
    over the block's rows and neighbour planes}, R_i = A_block S_i (own rows),
    alpha_i = LSQR(R_i, b_i), local test on the last inner iterate, then x_i and the
    block's view of its neighbours <- S_i alpha_i; stop when every block passes."""
    mode = po.REDUCE_DBR
    blocks, N, rows, plane = _blocks_ext(po, dim, nx, ny, nz, nb, peclet)
    norm0 = math.sqrt(sum_ordered([po.norm2(blk["rhs_b"], mode) ** 2 for blk in blocks]))
    thr = max(atol, rtol / math.sqrt(nb) * norm0)
    opts = dict(inner, guess_nonzero=1, uirnorm=1, reduce_mode=mode)
    outer = dict(outer, reduce_mode=mode)
    hist, lits_all = [], []
    outer_its = 0
    while True:
        S = [np.zeros((blk["lo"] + rows + blk["hi"], s), order="F") for blk in blocks]
        rhs = [None] * nb
        for k in range(s):
            for blk in blocks:
                rhs[blk["b"]] = blk["Aoff"].residual(blk["rhs_b"], blk["view"])
            for blk in blocks:
                blk["x"], r = po.gmres(blk["Aii"], rhs[blk["b"]], x0=blk["x"], **opts)
            for blk in blocks:                              # exchange
                for nbr in blk["nbrs"]:
                    o = blocks[nbr]
                    blk["view"][o["r0"]:o["r0"] + rows] = o["x"]
            for blk in blocks:
                S[blk["b"]][:, k] = _ext_col(blk, rows)
        norms, lits, alphas = [], [], []
        for blk in blocks:
            R = np.stack([blk["Aext"].mult(np.ascontiguousarray(S[blk["b"]][:, k])) for k in range(s)], axis=1)
            alpha, r = po.lsqr([R], [blk["rhs_b"]], **outer)
            alphas.append(alpha)
            lits.append(r["its"])
            norms.append(po.norm2(blk["Aii"].residual(rhs[blk["b"]], blk["x"]), mode))
        for blk, alpha in zip(blocks, alphas):
            _apply_ext(blk, po.dense_mult(S[blk["b"]], alpha), rows)
        hist.append(norms)
        lits_all.append(lits)
        outer_its += 1
        if all(n <= thr for n in norms) or outer_its >= max_outer:
            break
    for blk in blocks:                                      # final exchange
        for nbr in blk["nbrs"]:
            o = blocks[nbr]
            blk["view"][o["r0"]:o["r0"] + rows] = o["x"]
    x = np.concatenate([blk["x"] for blk in blocks])
    fin = [po.norm2(blk["Ab"].residual(blk["rhs_b"], x), mode) ** 2 for blk in blocks]
    err = [po.norm2(blk["x"] - 1.0, mode) ** 2 for blk in blocks]
    return {"outer_its": outer_its, "norm0": norm0, "hist": hist, "lsqr_its": lits_all, "x": x,
            "final_norm": math.sqrt(sum_ordered(fin)), "error": math.sqrt(sum_ordered(err))}


def amam_semi_local_roundrobin(po, dim, nx, ny, nz, nb, s, rtol, inner: dict, outer: dict, atol=1e-100,
                               max_iterations=100000, strict=False, peclet=None):
    """AMAM with semi-local minimization (asynchronous-multisplitting-asynchronous-
    minimization-semi-local_prime.c:350-420), round-robin: s asynchronous inner
    steps, each followed by a second receive and S_i(:,k) = [neighbour planes | x_i];
    R_i = A_block S_i, alpha_i = LSQR(R_i, b_i), x_minimized = S_i alpha_i -- which
    the reference computes but never scatters back (the iterate is unchanged) --;
    the local test on the last inner iterate; one detection step."""
    mode = po.REDUCE_DBR
    blocks, N, rows, plane = _blocks_ext(po, dim, nx, ny, nz, nb, peclet)
    net = Slots()
    dets = [Detector(blk["b"], blk["nbrs"], net, strict) for blk in blocks]
    norm0 = math.sqrt(sum_ordered([po.norm2(blk["rhs_b"], mode) ** 2 for blk in blocks]))
    thr = max(atol, rtol / math.sqrt(nb) * norm0)
    opts = dict(inner, guess_nonzero=1, uirnorm=1, reduce_mode=mode)
    outer = dict(outer, reduce_mode=mode)
    trace = []

    def receive(blk, det):
        for d, nbr in enumerate(blk["nbrs"]):
            m = net.recv(nbr, blk["b"], DATA)
            if m is not None and det.data_received(d, m[0], m[1]):
                lo = nbr * rows + (rows - plane if nbr < blk["b"] else 0)
                blk["view"][lo:lo + plane] = m[2]

    active = list(range(nb))
    while active:
        for bi in active:
            blk, det = blocks[bi], dets[bi]
            S = np.zeros((blk["lo"] + rows + blk["hi"], s), order="F")
            for k in range(s):
                receive(blk, det)
                rhs = blk["Aoff"].residual(blk["rhs_b"], blk["view"])
                blk["x"], r = po.gmres(blk["Aii"], rhs, x0=blk["x"], **opts)
                blk["inner"] += r["its"]
                for nbr in blk["nbrs"]:
                    pl = blk["x"][:plane].copy() if nbr < blk["b"] else blk["x"][rows - plane:].copy()
                    net.send(blk["b"], nbr, DATA, (det.phase, blk["steps"], pl))
                receive(blk, det)
                S[:, k] = _ext_col(blk, rows)
                blk["steps"] += 1
            R = np.stack([blk["Aext"].mult(np.ascontiguousarray(S[:, k])) for k in range(s)], axis=1)
            alpha, _ = po.lsqr([R], [blk["rhs_b"]], **outer)
            po.dense_mult(S, alpha)                         # x_minimized, not used by the reference
            ln = po.norm2(blk["Aii"].residual(rhs, blk["x"]), mode)
            det.step(ln <= thr)
            blk["it"] += 1
            trace.append((blk["b"], blk["it"], ln, det.state, det.phase))
            if blk["it"] >= max_iterations:
                raise RuntimeError("no termination")
        active = [bi for bi in active if dets[bi].state != FINISHED]
    x = np.concatenate([blk["x"] for blk in blocks])
    fin = [po.norm2(blk["Ab"].residual(blk["rhs_b"], x), mode) ** 2 for blk in blocks]
    err = [po.norm2(blk["x"] - 1.0, mode) ** 2 for blk in blocks]
    return {"iterations": [blk["it"] for blk in blocks], "inner_its": [blk["inner"] for blk in blocks],
            "phase_tags": [d.phase for d in dets], "trace": trace, "x": x, "norm0": norm0,
            "final_norm": math.sqrt(sum_ordered(fin)), "error": math.sqrt(sum_ordered(err))}


def amam_global_roundrobin(po, dim, nx, ny, nz, nb, s, rtol, inner: dict, outer: dict, atol=1e-100,
                           max_iterations=100000, strict=False, peclet=None, minimization="lsqr"):
    """AMAM with global minimization (asynchronous-multisplitting-asynchronous-
    minimization-global_prime.c:370-470), round-robin: s asynchronous inner steps,
    each followed by a second receive and S_i(:,k) = [neighbour planes | x_i];
    R_i = A_block S_i is broadcast, every other block's newest R rows are taken
    (zeros before the first), alpha = LSQR(R, b) over all nb row blocks in block
    order, x_minimized = S_i alpha replaces x_i and the view of the neighbour
    planes, the local test is ||b_i - A_block x_minimized||, one detection step.

    minimization "rtr": outer_solver (utils.c:972-996) -- block i broadcasts
    [R_i^T R_i | R_i^T b_i] (the oracle's orc_dense_gram) instead of its rows; the
    newest parts are summed elementwise in block order from 0.0 and the outer LSQR
    (same options) solves R^T R alpha = R^T b."""
    mode = po.REDUCE_DBR
    blocks, N, rows, plane = _blocks_ext(po, dim, nx, ny, nz, nb, peclet)
    net = Slots()
    dets = [Detector(blk["b"], blk["nbrs"], net, strict) for blk in blocks]
    norm0 = math.sqrt(sum_ordered([po.norm2(blk["rhs_b"], mode) ** 2 for blk in blocks]))
    thr = max(atol, rtol / math.sqrt(nb) * norm0)
    opts = dict(inner, guess_nonzero=1, uirnorm=1, reduce_mode=mode)
    outer = dict(outer, reduce_mode=mode)
    published = [None] * nb                                 # newest R rows each block sent
    for blk in blocks:
        if minimization == "rtr":
            blk["Rrep"] = [np.zeros((s, s + 1), order="F") for _ in range(nb)]
        else:
            blk["Rrep"] = [np.zeros((rows, s), order="F") for _ in range(nb)]
        blk["taken"] = [0] * nb
    versions = [0] * nb
    b_all = [blk["rhs_b"] for blk in blocks]
    trace, lsqr_its = [], []

    def receive(blk, det):
        for d, nbr in enumerate(blk["nbrs"]):
            m = net.recv(nbr, blk["b"], DATA)
            if m is not None and det.data_received(d, m[0], m[1]):
                lo = nbr * rows + (rows - plane if nbr < blk["b"] else 0)
                blk["view"][lo:lo + plane] = m[2]

    active = list(range(nb))
    while active:
        for bi in active:
            blk, det = blocks[bi], dets[bi]
            S = np.zeros((blk["lo"] + rows + blk["hi"], s), order="F")
            for k in range(s):
                receive(blk, det)
                rhs = blk["Aoff"].residual(blk["rhs_b"], blk["view"])
                blk["x"], r = po.gmres(blk["Aii"], rhs, x0=blk["x"], **opts)
                blk["inner"] += r["its"]
                for nbr in blk["nbrs"]:
                    pl = blk["x"][:plane].copy() if nbr < blk["b"] else blk["x"][rows - plane:].copy()
                    net.send(blk["b"], nbr, DATA, (det.phase, blk["steps"], pl))
                receive(blk, det)
                S[:, k] = _ext_col(blk, rows)
                blk["steps"] += 1
            R = np.asfortranarray(np.stack([blk["Aext"].mult(np.ascontiguousarray(S[:, k])) for k in range(s)],
                                           axis=1))
            if minimization == "rtr":
                R = po.dense_gram(R, blk["rhs_b"], mode)    # [R_i^T R_i | R_i^T b_i]
            blk["Rrep"][bi] = R
            published[bi] = R.copy()                        # comm_async_test_and_send_min
            versions[bi] += 1
            for j in range(nb):                             # comm_async_probe_and_receive_min
                if j != bi and versions[j] > blk["taken"][j]:
                    blk["Rrep"][j] = published[j].copy()
                    blk["taken"][j] = versions[j]
            if minimization == "rtr":
                G = np.zeros((s, s + 1), order="F")
                for part in blk["Rrep"]:                    # block order, from 0.0
                    G = G + part
                alpha, lr = po.lsqr([np.asfortranarray(G[:, :s])], [np.ascontiguousarray(G[:, s])], **outer)
            else:
                alpha, lr = po.lsqr(blk["Rrep"], b_all, **outer)
            lsqr_its.append(lr["its"])
            _apply_ext(blk, po.dense_mult(S, alpha), rows)
            ln = po.norm2(blk["Aext"].residual(blk["rhs_b"], _ext_col(blk, rows)), mode)
            det.step(ln <= thr)
            blk["it"] += 1
            trace.append((blk["b"], blk["it"], ln, det.state, det.phase))
            if blk["it"] >= max_iterations:
                raise RuntimeError("no termination")
        active = [bi for bi in active if dets[bi].state != FINISHED]
    x = np.concatenate([blk["x"] for blk in blocks])
    fin = [po.norm2(blk["Ab"].residual(blk["rhs_b"], x), mode) ** 2 for blk in blocks]
    err = [po.norm2(blk["x"] - 1.0, mode) ** 2 for blk in blocks]
    return {"iterations": [blk["it"] for blk in blocks], "inner_its": [blk["inner"] for blk in blocks],
            "phase_tags": [d.phase for d in dets], "trace": trace, "x": x, "norm0": norm0, "lsqr_its": lsqr_its,
            "final_norm": math.sqrt(sum_ordered(fin)), "error": math.sqrt(sum_ordered(err))}
