"""The reference's executables as entry points over the GPU path.

    python -m medane_tchakorom_ufc_thesis_repository_amd.drivers <program> [options]

<program> is one of the reference's drivers (src/<program>/<program>[_prime].c):
gmres_solution, synchronous-multisplitting,
synchronous-multisplitting-synchronous-minimization-{global,local,semi-local},
asynchronous-multisplitting,
asynchronous-multisplitting-asynchronous-minimization-{global,local,semi-local}.

Options are the reference's: -m (mesh lines) -n (mesh columns) -s -npb -rtol
-atol (read with PetscOptionsGet*, e.g. synchronous-multisplitting.c:44-48),
and the inner/outer solvers' -inner{b}_ksp_* / -outer{b}_ksp_* keys.  The
drivers are 2D like the reference's; -dim 3 -p <planes> selects the 3D 7-point
operator (m x n x p, z-slabs) and -peclet px,py,pz the convection-diffusion
one.  -npb must be 1 (one GPU per block).

Blocks: one per rank under torch.distributed.run (nccl = RCCL when GPUs are
visible, else gloo), or -nb <blocks> in one process (round-robin on one GPU).
Output follows the reference's printFinalResidualNorm / printElapsedTime /
computeError lines (utils.c:665-730), plus -json for one JSON line.
"""
from __future__ import annotations

import json
import os
import sys

PROGRAMS = {
    "gmres_solution": ("gmres", None),
    "synchronous-multisplitting": ("sm", None),
    "synchronous-multisplitting-synchronous-minimization-global": ("smsm", "global"),
    "synchronous-multisplitting-synchronous-minimization-local": ("smsm", "local"),
    "synchronous-multisplitting-synchronous-minimization-semi-local": ("smsm", "semi_local"),
    "asynchronous-multisplitting": ("am", "am"),
    "asynchronous-multisplitting-asynchronous-minimization-global": ("am", "amam_global"),
    "asynchronous-multisplitting-asynchronous-minimization-local": ("am", "amam_local"),
    "asynchronous-multisplitting-asynchronous-minimization-semi-local": ("am", "amam_semi_local"),
}


def parse(argv):
    """(program, Options, problem dict); raises ValueError on a bad command line."""
    from .petsc import Options
    if not argv or argv[0] not in PROGRAMS:
        raise ValueError(f"first argument must be one of: {', '.join(PROGRAMS)}")
    prog = argv[0]
    opts = Options(argv[1:])
    p = {
        "m": opts.get_int("m", 256), "n": opts.get_int("n", 256), "s": opts.get_int("s", 4),
        "npb": opts.get_int("npb", 1), "rtol": opts.get_real("rtol", 1e-6), "atol": opts.get_real("atol", 1e-100),
        "dim": opts.get_int("dim", 2), "p": opts.get_int("p", 0), "nb": opts.get_int("nb", 0),
        "max_outer": opts.get_int("max_outer", 100000), "json": opts.get_bool("json", False),
        "peclet": None,
    }
    pe = opts.get_string("peclet", None)
    if pe is not None:
        vals = [float(v) for v in pe.split(",")]
        if len(vals) != 3:
            raise ValueError("-peclet takes px,py,pz")
        p["peclet"] = tuple(vals)
    if p["npb"] != 1:
        raise ValueError("-npb must be 1: one GPU (one process) per block")
    if p["dim"] not in (2, 3):
        raise ValueError("-dim is 2 or 3")
    if p["dim"] == 3 and p["p"] <= 0:
        p["p"] = p["n"]
    if PROGRAMS[prog][0] != "gmres" and p["s"] < 1 and PROGRAMS[prog][1] not in (None, "am"):
        raise ValueError("-s must be >= 1 for the minimization variants")
    return prog, opts, p


def _report(prog, p, out, rank):
    if rank != 0:
        return
    if p["json"]:
        print(json.dumps(dict(program=prog, **out)), flush=True)
        return
    if prog == "gmres_solution":                       # gmres_solution.c:81-91
        print("======================== ")
        print(f"Number of iterations of GMRES : {out['outer_its']} ")
        print(f"Right hand side norm : {out['b_norm']:e} ")
        print(f"GMRES residual norm : {out['final_norm']:e} ")
        print(f"||r(i)||/||b|| : {out['final_norm'] / out['b_norm']:e} ")
        print("======================== ")
        print(f"Erreur : {out['error']:e} ")
        return
    print(f"Elapsed time (iterations):   {out['elapsed']:f}  seconds ")
    if "outer_its" in out:
        print(f"Total number of iterations (outer_iterations) = {out['outer_its']} ")
    if "iterations" in out:
        for b, it in enumerate(out["iterations"]):
            print(f"[ Block rank {b} ] Total number of iterations (outer_iterations) = {it} ")
    print(f"Final residual norm 2 = {out['final_norm']:e} ")
    print(f"Erreur  : {out['error']:e}  ")


def run(argv) -> dict:
    prog, opts, p = parse(argv)
    kind, variant = PROGRAMS[prog]
    import torch
    from .comm import LocalComm, TorchComm
    from .petsc import Context
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        if not dist.is_initialized():
            if torch.cuda.device_count() > 0:
                torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")) % torch.cuda.device_count())
                dist.init_process_group("nccl", device_id=torch.device("cuda", torch.cuda.current_device()))
            else:
                dist.init_process_group("gloo")
    dev = torch.cuda.current_device() if torch.cuda.device_count() > 0 else 0
    ctx = Context(dev)
    # -msplit_reduction seq: PETSc's reduction order on the device (the parity mode, msp_ctx_set_reduction)
    red = opts.get_string("msplit_reduction", "dbr").lower()
    if red not in Context.REDUCTIONS:
        raise ValueError(f"-msplit_reduction {red}: expected one of {sorted(Context.REDUCTIONS)}")
    ctx.set_reduction(red)
    dim, nx, ny, nz = p["dim"], p["m"], p["n"], p["p"] or 1
    if kind == "gmres":
        out = _gmres(ctx, opts, p)
        _report(prog, p, out, rank)
        return out
    if world > 1:
        comm = TorchComm()
        nb, ids = world, [rank]
    else:
        comm = LocalComm()
        nb = p["nb"] or 2
        ids = list(range(nb))
    from .multisplitting import make_blocks, smsm_local_solve, smsm_semi_local_solve, smsm_solve, sm_solve, \
        GpuMinimizer
    blocks = make_blocks(ctx, dim, nx, ny, nz, nb, ids, opts, comm, p["peclet"])
    s, rtol, atol = p["s"], p["rtol"], p["atol"]
    if kind == "sm":
        r = sm_solve(blocks, comm, rtol, atol, p["max_outer"])
        fin = r.hist[-1] if r.hist else float("nan")
        out = {"outer_its": r.outer_its, "final_norm": fin, "error": r.error, "elapsed": r.elapsed,
               "hist": list(r.hist)}
    elif kind == "smsm":
        if variant == "global":
            for blk in blocks:
                blk.setup_minimization(s)
            mini = GpuMinimizer(ctx, blocks, comm, opts)
            r = smsm_solve(blocks, comm, s, mini, rtol, atol, p["max_outer"])
            mini.close()
        elif variant == "local":
            for blk in blocks:
                blk.setup_local_minimization(s, opts)
            r = smsm_local_solve(blocks, comm, s, rtol, atol, p["max_outer"])
        else:
            for blk in blocks:
                blk.setup_minimization(s)
            r = smsm_semi_local_solve(blocks, comm, s, rtol, atol, p["max_outer"])
        out = {"outer_its": r.outer_its, "final_norm": r.final_norm, "error": r.error, "elapsed": r.elapsed,
               "hist": list(r.hist), "lsqr_its": list(getattr(r, "lsqr_its", []))}
    else:
        from .asynchronous import am_solve
        for blk in blocks:
            if variant == "amam_global":
                blk.setup_global_async_minimization(s)
            elif variant == "amam_local":
                blk.setup_local_minimization(s, opts)
            elif variant == "amam_semi_local":
                blk.setup_minimization(s)
        r = am_solve(blocks, comm, rtol, atol, p["max_outer"], variant=variant, s=s)
        out = {"iterations": r.iterations, "final_norm": r.final_norm, "error": r.error, "elapsed": r.elapsed}
    _report(prog, p, out, rank)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()
    return out


def _gmres(ctx, opts, p):
    """gmres_solution.c: one KSPSolve on the whole operator (b = A 1, x0 = 0), options prefix-free."""
    import time
    from .petsc import KSP, Mat, Vec
    dim, nx, ny, nz = p["dim"], p["m"], p["n"], p["p"] or 1
    if dim == 2:       # poisson2DMatrix numbering: m lines of n columns -> box (n fast, m slow)
        A = Mat.box_convdiff(ctx, 2, ny, nx, 1, False, False, p["peclet"] or (0.0, 0.0, 0.0))
    else:
        A = Mat.box_convdiff(ctx, 3, nx, ny, nz, False, False, p["peclet"] or (0.0, 0.0, 0.0))
    n = A.shape[0]
    u = Vec(ctx, n)
    u.set(1.0)
    b = Vec(ctx, n)
    A.mult(u, b)
    x = Vec(ctx, n)
    ksp = KSP(ctx)
    ksp.set_operators(A)
    ksp.set_from_options(opts)
    ctx.synchronize()
    t0 = time.perf_counter()
    ksp.solve(b, x)
    ctx.synchronize()
    dt = time.perf_counter() - t0
    e = Vec(ctx, n)
    e.waxpy(-1.0, u, x)
    return {"outer_its": ksp.get_iteration_number(), "reason": ksp.get_converged_reason(), "b_norm": b.norm(),
            "final_norm": ksp.get_residual_norm(), "error": e.norm(), "elapsed": dt}


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    try:
        run(argv)
    except ValueError as e:
        print(f"error: {e}", file=sys.stderr)
        print(__doc__, file=sys.stderr)
        return 2
    return 0


if __name__ == "__main__":
    sys.exit(main())
