"""Benchmark: image_warping 4096x4096 fp32 Gauss-Newton + PCG through the Opt C ABI.

One step = one Opt_ProblemStep (one GN iteration: J^T F + Jacobi preconditioner from the
arrays bound at that Step fused with the first PCG apply, then lIterations - 1 passes of
{residual update, p-update, J^T J p apply, delta update, the four PCG sums}, X += delta,
cost). Inputs are resident in HBM before the timed region starts.

  value       PCG unknowns processed per second over the whole job:
              n_unknowns * lIterations * steps / wall time of the timed steps
  roofline    the dominant kernel (the in-loop J^T J p pass, iw_apply_res): its duration
              from HIP events on its launches (plan stream) over K more steps after the
              timed ones; init_kernel: the same for iw_jtf_apply
  cpu_baseline the oracle (C restatement of the reference's GN/PCG, pthreads over rows
              as backend_cpu_mt) timing one whole GN step on this host's cores, in the
              same unit, plus apply-only rates on all cores and on one; rank 0 at N=1

Multi-GPU (--gpus N): the 4096² image is split into N row slabs, one per rank
(OptAMD_PlanSetDecomposition over an RCCL communicator; the reference's outer-dimension
split, backend_cpu_mt.t:716-737): per PCG iteration one all-reduce of four fp64 scalars
(r.z, p.Ap, r.W Ap, Ap.W Ap: the fused pass takes beta's numerator from their identity)
and one halo-row exchange. Total work is fixed, so the scaling is strong. Launch either
under torch.distributed.run (WORLD_SIZE must then equal --gpus, else the script exits
with status 2), or plainly: `python bench.py --gpus N` then starts the N rank processes
itself (before anything touches the GPU) and exits with the worst child status.
`--dry-run` prints each rank's environment and slab as JSON and touches no GPU.

--workload shape_from_shading: BASELINE config 3 (4096² fp32 LM + PCG, the config
north_star tiles across the node) through the same slabs (halo 2, ComputedArray planes
exchanged after each precompute, r.z and q all-reduced together).
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "PCG JᵀJ·p throughput (unknowns/s) + GN iters/s, image_warping 4096² fp32"
METRIC_SFS = "PCG JᵀJ·p throughput (unknowns/s) + LM iters/s, shape_from_shading 4096² fp32"
SFS_APPLY_BYTES_PER_PX = 34
PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# Compulsory HBM bytes per pixel of the in-loop apply kernel iw_apply:
# always Angle 4 + UrShape 8 + flag 1 + r 12 + angle-channel pre 4 read, p 12 + Ap 12 written;
# from PCG iteration 1 on also p_old 12 read and delta 12 written; from iteration 2 on
# also delta 12 read.
def apply_bytes_per_px(i: int, liter: int = 10) -> int:
    b = 4 + 8 + 1 + 12 + 4 + 12 + 12
    if i >= 1:
        b += 12 + 12
    if i >= 2:
        b += 12
    if i == liter - 1:
        b -= 12   # the last iteration's Ap is not stored (nothing reads it)
    return b


# HBM traffic of the in-loop apply from the committed rocprofv3 PMC summary of the same
# kernels (tools/measure_r04.sh: separate --pmc FETCH_SIZE / WRITE_SIZE passes over this
# bench). FETCH_SIZE reads exactly 1/2 of the bytes on gfx950 for 1/4/8/16-B-per-lane
# streaming reads and WRITE_SIZE is exact (profiles/r01_fetchcal.json, 1 GiB arrays), so
# traffic = 2 FETCH_SIZE + WRITE_SIZE, averaged over the lIterations in-loop launches.
PMC_FILE = os.path.join(ROOT, "profiles", "r06_pmc.json")
APPLY_VARIANT = {0: "iw_apply<float, 1, 0,", 1: "iw_apply<float, 2, 1,", 2: "iw_apply<float, 2, 2,"}


# PCG iteration i >= 1 as ONE pass (iw_apply_res: the apply with the previous iteration's
# residual update folded in): Angle 4 + UrShape 8 + flag 1 + angle pre 4 + r_{i-1} 12 +
# Ap_{i-1} 12 + p_{i-1} 12 read, p_i 12 written; r_i 12 + Ap_i 12 written except in the last
# iteration (nothing reads them). The delta update, deferred (OPT_AMD_IW_DEFER, default on):
# none in odd iterations; i = 2 reads p_0 12 and writes delta 12; even i >= 4 read delta 12 +
# p_{i-2} 12 and write delta 12. Per iteration (OPT_AMD_IW_DEFER=0): delta 12 written, and
# read from i = 2 on.
IW_DEFER = os.environ.get("OPT_AMD_IW_DEFER", "1") != "0"


def res_bytes_per_px(i: int, liter: int = 10, defer: bool = IW_DEFER) -> int:
    b = 4 + 8 + 1 + 4 + 12 + 12 + 12 + 12
    if i == 1 and liter >= 3:
        b -= 12   # P0: pass 1 forms p_0 = pre r_0 from the r_0 it reads (p_0 is never stored)
    if i < liter - 1:
        b += 24
    if defer:
        b += 0 if i % 2 == 1 else (24 if i == 2 else 36)
    else:
        b += 12 if i == 1 else 24
    return b


RES_KERNEL = "iw_apply_res"


def res_variant(i: int, defer: bool = IW_DEFER, liter: int = 10) -> str:
    """The iw_apply_res instantiation PCG iteration i >= 1 runs (<T, DM, NT, E, P0>)."""
    if defer:
        dm, e = (0, 0) if i % 2 == 1 else ((1, 1) if i == 2 else (2, 1))
    else:
        dm, e = (1 if i == 1 else 2), 0
    p0 = "true" if liter >= 3 and (i == 1 or (defer and i == 2)) else "false"
    return f"iw_apply_res<float, {dm}, 2, {e}, {p0}>"


# PCG iteration i >= 1 as iw_pcg (the default on one GPU, round 5): iw_apply_res with
# Ap_{i-1} recomputed from p_{i-1} instead of read back, and Ap_i never stored: Angle 4 +
# UrShape 8 + flag 1 + angle pre 4 + r_{i-1} 12 + p_{i-1} 12 read, p_i 12 written, r_i 12
# written except in the last iteration; P0 and the deferred delta as iw_apply_res. With every
# p_i kept (OPT_AMD_IW_ALLP, the default for lIterations 2..16) no pass carries a delta term:
# iw_update_all reads the L p vectors once at the end. Since round 6 the passes without P0
# recompute the angle pre from the stencil geometry (PRC) instead of reading it: 4 B/px less.
PCG_KERNEL = "iw_pcg"
IW_ALLP = os.environ.get("OPT_AMD_IW_ALLP", "1") != "0"
IW_PRC = os.environ.get("OPT_AMD_IW_PCG_PRC", "1") != "0"


def allp_on(liter: int) -> bool:
    return IW_ALLP and 2 <= liter <= 16


def pcg_bytes_per_px(i: int, liter: int = 10, defer: bool = IW_DEFER) -> int:
    b = 4 + 8 + 1 + 4 + 12 + 12 + 12
    if i == 1 and liter >= 3:
        b -= 12   # P0: p_0 = pre r_0 from the r_0 the pass reads
    if i < liter - 1:
        b += 12
    if allp_on(liter):
        if IW_PRC and not (i == 1 and liter >= 3):
            b -= 4   # PRC: no angle pre read
        return b
    if defer:
        b += 0 if i % 2 == 1 else (24 if i == 2 else 36)
    else:
        b += 12 if i == 1 else 24
    return b


def pcg_variant(i: int, defer: bool = IW_DEFER, liter: int = 10) -> str:
    """The iw_pcg instantiation PCG iteration i >= 1 runs (<T, DM, E, P0, SNT, U2, PF2, REC, PRC>)."""
    if allp_on(liter):
        dm, e, defer = 0, 0, False
    elif defer:
        dm, e = (0, 0) if i % 2 == 1 else ((1, 1) if i == 2 else (2, 1))
    else:
        dm, e = (1 if i == 1 else 2), 0
    p0 = "true" if liter >= 3 and (i == 1 or (defer and i == 2)) else "false"
    u2 = int(os.environ.get("OPT_AMD_IW_PCG_U2", "1"))   # the plan's default: two rows per trip
    prc = allp_on(liter) and IW_PRC and p0 == "false" and u2 != 2
    return (f"iw_pcg<float, {dm}, {e}, {p0}, false, {'true' if u2 >= 1 else 'false'}, "
            f"{'true' if u2 == 2 else 'false'}, false, {'true' if prc else 'false'}>")


# PCGInit1 fused with the first apply (iw_jtf_apply, one strip pass): Offset 8 + Angle 4 +
# UrShape 8 + Constraints 8 + Mask 4 read; r 12 + angle pre 4 + flag 1 + Ap 12 written, and
# p 12 only when lIterations <= 2 (from 3 on, passes 1 and 2 form p_0 = pre r_0 themselves).
INIT_KERNEL = "iw_jtf_apply"


def init_bytes_per_px(liter: int = 10, ap: bool = True) -> int:
    """ap: Ap_0 stored (iw_apply_res reads it back); iw_pcg recomputes it, so with the
    iw_pcg loop iw_jtf_apply stores no Ap."""
    return 8 + 4 + 8 + 8 + 4 + 12 + 4 + 1 + (12 if ap else 0) + (12 if liter <= 2 else 0)


# The step's two other kernels (HIP-event timed like the passes): iw_update reads the flag 1,
# Offset 8, Angle 4, delta 12, p_{L-1} 12 (+ p_{L-2} 12 when the deferred pair is pending,
# lIterations even) and writes Offset + Angle 12; iw_cost reads Offset 8, Angle 4, UrShape 8,
# Constraints 8, Mask 4 — or, with the Step's flags (OPT_AMD_IW_COST_FLAGS, default on), Offset 8,
# Angle 4, UrShape 8, the flag 1 (Constraints only at the workload's few fit pixels, not counted).
STEP_KERNELS = ("iw_jtf_apply", "iw_pcg", "iw_update", "iw_cost")   # iw_update: iw_update_all with allp


def update_bytes_per_px(liter: int = 10) -> int:
    if allp_on(liter):   # iw_update_all: flag, Offset, Angle, r_0 + angle pre (p_0 formed), p_1..p_{L-1}
        return 1 + 8 + 4 + (16 if liter >= 3 else 12) + 12 * (liter - 1) + 12
    return 1 + 8 + 4 + (12 if liter >= 2 else 0) + 12 + (12 if liter % 2 == 0 else 0) + 12


COST_BYTES_PER_PX = 21 if os.environ.get("OPT_AMD_IW_COST_FLAGS", "1") != "0" else 32


def pmc_traffic(liter: int, first: int = 0, res=False):
    try:
        with open(PMC_FILE) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    total = 0.0
    for i in range(first, liter):
        key = (pcg_variant(i, liter=liter) if res == "pcg" else res_variant(i, liter=liter) if res
               else APPLY_VARIANT[min(i, 2)])
        hit = [v for k, v in ks.items() if key in k]
        if not hit or "FETCH_SIZE" not in hit[0] or "WRITE_SIZE" not in hit[0]:
            return None
        total += (2.0 * hit[0]["FETCH_SIZE"] + hit[0]["WRITE_SIZE"]) * 1024.0
    return total / (liter - first)


def pmc_limiter(liter: int, first: int = 0):
    """What the in-loop iw_pcg passes wait on, from the same PMC summary's SQ pass: the
    launch-weighted fractions of wave cycles parked on memory / barriers (SQ_WAIT_ANY),
    stalled at issue (SQ_WAIT_INST_ANY) and issuing VALU (SQ_ACTIVE_INST_VALU)."""
    try:
        with open(PMC_FILE) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    acc = {"SQ_WAIT_ANY": 0.0, "SQ_WAIT_INST_ANY": 0.0, "SQ_ACTIVE_INST_VALU": 0.0}
    for i in range(first, liter):
        hit = [v for k, v in ks.items() if pcg_variant(i, liter=liter) in k]
        if not hit or not hit[0].get("SQ_WAVE_CYCLES") or any(c not in hit[0] for c in acc):
            return None
        for c in acc:
            acc[c] += hit[0][c] / hit[0]["SQ_WAVE_CYCLES"] / (liter - first)
    return {"wait_memory": round(acc["SQ_WAIT_ANY"], 3), "wait_issue": round(acc["SQ_WAIT_INST_ANY"], 3),
            "valu_active": round(acc["SQ_ACTIVE_INST_VALU"], 3),
            "source": os.path.relpath(PMC_FILE, ROOT) + " (fractions of SQ_WAVE_CYCLES)"}


PMC_FILE_SFS = os.path.join(ROOT, "profiles", "r06_pmc_sfs.json")


def pmc_traffic_sfs():
    """The same for the shape_from_shading leg: the in-loop J^T J p strip (sfs_strip<float,
    false, false>) from the committed PMC summary of that workload (tools/measure_r04.sh)."""
    try:
        with open(PMC_FILE_SFS) as f:
            ks = json.load(f)["kernels"]
    except (OSError, ValueError, KeyError):
        return None
    hit = [v for k, v in ks.items() if "sfs_strip<float, false, false>" in k]
    if not hit or "FETCH_SIZE" not in hit[0] or "WRITE_SIZE" not in hit[0]:
        return None
    return (2.0 * hit[0]["FETCH_SIZE"] + hit[0]["WRITE_SIZE"]) * 1024.0


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=4096)
    ap.add_argument("--liter", type=int, default=10)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--workload", default="image_warping", choices=["image_warping", "shape_from_shading"])
    ap.add_argument("--dry-run", action="store_true",
                    help="print each rank's launch environment and slab rows as JSON; no GPU work")
    return ap.parse_args()


# stencil radius (halo rows) of each workload's energy; checked against the plan's
# OptAMD_PlanHalo in the real run
HALO = {"image_warping": 2, "shape_from_shading": 2}


def rank_env():
    """(world, rank, local_rank) from the launcher's environment (torch.distributed.run or
    spawn_ranks)."""
    return (int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0")),
            int(os.environ.get("LOCAL_RANK", "0")))


def free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def visible_gpus():
    """GPUs this process could open, counted without any GPU runtime: the visibility
    variables if one is set, else the KFD topology's GPU nodes (simd_count > 0); None when
    neither can be read (each rank then checks its own device, main())."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([d for d in v.split(",") if d.strip() != ""])
    try:
        import glob
        n = 0
        for f in glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties"):
            for line in open(f):
                if line.startswith("simd_count") and int(line.split()[1]) > 0:
                    n += 1
        return n
    except (OSError, ValueError):
        return None


def spawn_ranks(args) -> int:
    """--gpus N > 1 without a launcher: start N copies of this script, one per GPU, with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set (what
    torch.distributed.run sets). This process never touches the GPU (it only waits), so the
    children own their devices; if any child fails the others are stopped and the worst
    status is returned. Rank 0 prints the JSON line."""
    import subprocess

    n = args.gpus
    if not args.dry_run:
        have = visible_gpus()   # counted without torch / HIP: this process never opens the GPU
        if have is not None and have < n:
            print(f"bench.py: --gpus {n} but only {have} GPU(s) visible", file=sys.stderr, flush=True)
            return 2
    port = os.environ.get("MASTER_PORT") or str(free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    status = 0
    pending = list(procs)
    while pending:
        for p in list(pending):
            rc = p.poll()
            if rc is None:
                continue
            pending.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 1
                for q in pending:   # a failed rank leaves the others blocked in a collective
                    q.kill()
        time.sleep(0.05)
    return status


def dry_run(args, world, rank, local):
    """One JSON line per rank: what the real run would use (no torch, no GPU)."""
    from opt_amd import distributed as dd

    sl = dd.slab(args.size, rank, world, HALO[args.workload]) if world > 1 else None
    print(json.dumps({"rank": rank, "local_rank": local, "world": world, "device": f"cuda:{local}",
                      "master": f"{os.environ.get('MASTER_ADDR', '')}:{os.environ.get('MASTER_PORT', '')}",
                      "workload": args.workload, "size": args.size,
                      "slab": ([sl.y_lo, sl.y_hi] if sl else [0, args.size]),
                      "mem_rows": ([sl.mem_lo, sl.mem_hi] if sl else [0, args.size])}), flush=True)


def host_cores():
    """CPUs this process may actually run on: the affinity mask, capped by the cgroup
    CPU quota (the GPU box grants a share of a larger machine; os.cpu_count() shows the
    whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        quota, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(w, n_unknowns, liter):
    """The oracle (oracle/image_warping.c, the reference's GN/PCG restated in C with
    pthreads over rows, as backend_cpu_mt splits its kernels, backend_cpu_mt.t:350-414)
    on the host: one whole GN step (JᵀF + preconditioner, `liter` PCG iterations, update,
    cost) on every available core, in the headline's unit (unknowns x lIterations per
    second), plus the JᵀJ·p apply alone on all cores and on one core (a 512-row sample)."""
    from oracle import oracle

    cores = host_cores()
    t0 = time.perf_counter()
    oracle.iw_solve(w, 1, liter, nthreads=cores)
    t_step = time.perf_counter() - t0
    rng = np.random.default_rng(0)
    p = rng.normal(size=n_unknowns).astype(np.float32)
    reps, t0 = 0, time.perf_counter()
    while reps < 3 or time.perf_counter() - t0 < 3.0:
        oracle.iw_apply_jtj(w, p, nthreads=cores)
        reps += 1
    t_apply = (time.perf_counter() - t0) / reps
    rows = 512
    ws = {**w, "H": rows, "Offset": w["Offset"][: 2 * w["W"] * rows], "Angle": w["Angle"][: w["W"] * rows],
          "UrShape": w["UrShape"][: 2 * w["W"] * rows], "Constraints": w["Constraints"][: 2 * w["W"] * rows],
          "Mask": w["Mask"][: w["W"] * rows]}
    n1 = 3 * w["W"] * rows
    reps1, t0 = 0, time.perf_counter()
    while reps1 < 2 or time.perf_counter() - t0 < 2.0:
        oracle.iw_apply_jtj(ws, p[:n1], nthreads=1)
        reps1 += 1
    t_apply1 = (time.perf_counter() - t0) / reps1
    return {
        "value": n_unknowns * liter / t_step,
        "unit": "unknowns/s",
        "cores": cores,
        "kind": "port",
        "sample": f"one GN step ({liter} PCG iterations, incl. the init cost) of the full {w['W']}x{w['H']} "
                  f"problem, oracle/image_warping.c on {cores} threads: {t_step:.2f} s",
        "gn_iters_per_s": 1.0 / t_step,
        "apply_unknowns_per_s": n_unknowns / t_apply,
        "apply_unknowns_per_s_1core": n1 / t_apply1,
        "cpu_model": cpu_model(),
    }


def cpu_baseline_sfs(w, W, H, liter):
    """Config 3's comparator: the oracle (oracle/sfs_impl.h, the reference's
    shape_from_shading energy and LM/PCG loop restated in C) timing ONE LM step
    (precompute, J^T F, `liter` PCG iterations, model cost, cost) of the full W x H
    workload, every stencil pass split over row slabs on all the host cores this process
    may use, per-thread sums added in thread order (backend_cpu_mt.t:350-414, 716-737), in
    the headline's unit (unknowns x lIterations per second)."""
    from oracle import oracle

    cores = host_cores()
    t0 = time.perf_counter()
    oracle.sfs_solve(w, 1, liter, lm=True, nthreads=cores)
    dt = time.perf_counter() - t0
    return {
        "value": W * H * liter / dt,
        "unit": "unknowns/s",
        "cores": cores,
        "kind": "port",
        "sample": f"one LM step ({liter} PCG iterations, incl. precompute and both costs) of the full {W}x{H} "
                  f"workload, oracle/sfs_impl.h over row slabs on {cores} threads: {dt:.2f} s",
        "lm_iters_per_s": 1.0 / dt,
        "cpu_model": cpu_model(),
    }
def main():
    args = parse()
    if args.gpus < 1:
        print("bench.py: --gpus must be >= 1", file=sys.stderr, flush=True)
        return 2
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args)
    world, rank, local = rank_env()
    if world != args.gpus:
        print(f"bench.py: launched with WORLD_SIZE={world} but --gpus {args.gpus}; refusing to report "
              f"a {world}-rank run as {args.gpus}", file=sys.stderr, flush=True)
        return 2
    if args.dry_run:
        dry_run(args, world, rank, local)
        return 0
    import torch

    if local >= torch.cuda.device_count():
        print(f"bench.py: rank {rank} needs device {local}, {torch.cuda.device_count()} visible", file=sys.stderr,
              flush=True)
        return 2
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist_mod

        dist = dist_mod
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    from opt_amd import OptSolver, api, workloads
    from opt_amd import distributed as dd

    W = H = args.size
    sfs = args.workload == "shape_from_shading"
    if sfs:
        w = workloads.shape_from_shading(W, H, seed=3)
        s = OptSolver([W, H], os.path.join(ROOT, "energies", "shape_from_shading.t"), "LMGPU")
    else:
        w = workloads.image_warping(W, H, seed=1234)
        s = OptSolver([W, H], os.path.join(ROOT, "energies", "image_warping.t"), "gaussNewtonGPU")
    n_unknowns = s.unknown_count()   # global
    comm = None
    lw = w
    sl = None
    if world > 1:
        lib = api.load_library()
        idbuf = torch.zeros(128, dtype=torch.uint8)
        if rank == 0:
            raw = (ctypes.c_uint8 * 128)()
            assert lib.OptAMD_RcclUniqueId(raw) == 0
            idbuf = torch.tensor(list(raw), dtype=torch.uint8)
        idbuf = idbuf.cuda()
        dist.broadcast(idbuf, 0)
        idraw = (ctypes.c_uint8 * 128)(*idbuf.cpu().tolist())
        comm = lib.OptAMD_CommCreateRccl(idraw, rank, world)
        assert comm, "RCCL communicator"
        assert lib.OptAMD_CommSize(comm) == world and lib.OptAMD_CommRank(comm) == rank
        assert s.halo() == HALO[args.workload], (s.halo(), args.workload)
        sl = dd.slab(H, rank, world, s.halo())
        s.set_decomposition(comm, sl.y_lo, sl.y_hi)
        lw = dd.local_image(w, sl, dd.SFS_CHANNELS if sfs else dd.IW_CHANNELS)
    if sfs:
        prm = [float(v) for v in w["params"]] + [torch.from_numpy(np.ascontiguousarray(lw[k])).cuda()
                                                 for k in ("X", "D_i", "Im", "edgeMaskR", "edgeMaskC")]
    else:
        prm = [torch.from_numpy(lw[k]).cuda() for k in ("Offset", "Angle", "UrShape", "Constraints", "Mask")] + \
              [w["w_fitSqrt"], w["w_regSqrt"]]
    # warmup, the K timed steps (no instrumentation), then K more steps with the apply
    # kernel timed by HIP events on its launches (the roofline's kernel duration), so
    # the headline's timed region carries no instrumentation at all
    total_steps = args.warmup + 2 * args.steps
    s.set_solver_params({"nIterations": total_steps + 1, "lIterations": args.liter})
    s.init(prm)
    for _ in range(args.warmup):
        s.step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        s.step()
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    if dist:
        t = torch.tensor([dt], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    s.set_kernel_timing(2)  # HIP events on the apply kernel's launches only
    for _ in range(args.steps):
        s.step()
    torch.cuda.synchronize()
    kname = s.apply_kernel_name()
    n_apply, apply_ms = s.kernel_stat(kname)
    n_init, init_ms = (0, 0.0) if sfs else s.kernel_stat(INIT_KERNEL)
    res = False
    if not sfs:
        n_res, res_ms = s.kernel_stat(RES_KERNEL)
        n_pcg, pcg_ms = s.kernel_stat(PCG_KERNEL)
        if n_pcg:   # the loop ran as iw_pcg passes (one GPU): the dominant kernel
            kname, n_apply, apply_ms, res = PCG_KERNEL, n_pcg, pcg_ms, "pcg"
        elif n_res:   # as iw_apply_res passes (row slabs, OPT_AMD_IW_APFREE=0)
            kname, n_apply, apply_ms, res = RES_KERNEL, n_res, res_ms, True
    kstats = {k: s.kernel_stat(k) for k in STEP_KERNELS}
    s.set_kernel_timing(0)
    # the in-loop applies of one step: PCG iterations first..liter-1 (first = 1 when the
    # first iteration's apply ran inside iw_jtf_apply)
    first = 0 if sfs else args.liter - int(round(n_apply / max(1, args.steps)))
    avg_apply_s = (apply_ms / 1e3) / max(1, n_apply)
    npx = W * (sl.rows if sl else H)
    ch = 1 if sfs else 3          # unknowns per pixel
    if sfs:   # sfs_strip: SURVEY.md §8d's per-pixel apply bytes
        bpp = SFS_APPLY_BYTES_PER_PX
    else:
        per = pcg_bytes_per_px if res == "pcg" else res_bytes_per_px if res else apply_bytes_per_px
        bpp = sum(per(i, args.liter) for i in range(first, args.liter)) / (args.liter - first)
    achieved = bpp * npx / avg_apply_s / 1e9
    # the pure apply (reads p) timed separately for the kernel-only unknowns/s
    n_local = ch * W * (sl.mem_rows if sl else H)
    p = torch.randn(n_local, device="cuda")
    Ap = torch.empty_like(p)
    pure_us = s.time_apply(prm, p, Ap, 20)
    kind = "LM" if sfs else "GN"
    n_ranks = api.load_library().OptAMD_CommSize(comm) if comm else 1   # what the solver ran on
    rows = [H // world] * (world - 1) + [H - (world - 1) * (H // world)]
    result = {
        "metric": METRIC_SFS if sfs else METRIC,
        "value": n_unknowns * args.liter * args.steps / dt,
        "unit": "unknowns/s",
        "n_gpus": n_ranks,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": 1000.0 * dt / args.steps,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f32",
        "data": f"synthetic (seeded {args.workload} inputs, SURVEY.md §8d)",
        "config": {
            "workload": f"{args.workload} {W}x{H} fp32 {kind}+PCG, lIterations={args.liter}",
            "unknowns": n_unknowns,
            "parallelism": (f"row-slabs x{n_ranks} of {rows[0]}" + (f"/{rows[-1]}" if rows[-1] != rows[0] else "")
                            + f" rows (halo {HALO[args.workload]}; RCCL: {2 if sfs else 1} allreduce + 1 halo "
                              "exchange per PCG iteration)" if n_ranks > 1 else "single"),
        },
        f"{kind.lower()}_iters_per_s": args.steps / dt,
        "apply_unknowns_per_s": ch * npx * world / avg_apply_s,
        "pure_apply_us": pure_us,
        "pure_apply_unknowns_per_s": ch * npx * world / (pure_us * 1e-6),
        "roofline": {
            "kernel": kname,
            "bound": "hbm",
            "achieved": achieved,
            "peak": PEAK_HBM_GBS,
            "unit": "GB/s",
            "frac": achieved / PEAK_HBM_GBS,
            "traffic": (None if world != 1 or args.size != 4096 else
                        pmc_traffic_sfs() if sfs else pmc_traffic(args.liter, first, res)),
            "traffic_unit": "bytes per launch (2 FETCH_SIZE + WRITE_SIZE, "
                            f"{os.path.relpath(PMC_FILE_SFS if sfs else PMC_FILE, ROOT)})",
            "avg_us": avg_apply_s * 1e6,
            "launches": n_apply,
            "bytes_per_px": bpp,
            # the pass is bound by VALU issue, not HBM, when wait_issue dominates
            "limiter": (pmc_limiter(args.liter, first) if res == "pcg" and world == 1 and args.size == 4096
                        else None),
        },
    }
    if n_init:
        init_s = (init_ms / 1e3) / n_init
        ibpp = init_bytes_per_px(args.liter, ap=res != "pcg")
        ach = ibpp * npx / init_s / 1e9
        result["init_kernel"] = {"kernel": INIT_KERNEL, "avg_us": init_s * 1e6, "launches": n_init,
                                 "bytes_per_px": ibpp, "achieved": ach, "frac": ach / PEAK_HBM_GBS}
    if not sfs:   # every kernel of the step: launches per step, average duration, HBM rate
        per_px = {"iw_jtf_apply": init_bytes_per_px(args.liter, ap=res != "pcg"), "iw_pcg": bpp,
                  "iw_update": update_bytes_per_px(args.liter), "iw_cost": COST_BYTES_PER_PX}
        ks = {}
        for k in STEP_KERNELS:
            n, ms = kstats[k]
            if n:
                us = 1e3 * ms / n
                ks[k] = {"per_step": n / args.steps, "avg_us": us, "bytes_per_px": per_px[k],
                         "frac": per_px[k] * npx / (us * 1e-6) / 1e9 / PEAK_HBM_GBS}
        result["step_kernels"] = ks
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        result["cpu_baseline"] = (cpu_baseline_sfs(w, W, H, args.liter) if sfs
                                  else cpu_baseline(w, n_unknowns, args.liter))
    if rank == 0:
        print(json.dumps(result), flush=True)
    s.close()
    if comm:
        api.load_library().OptAMD_CommDestroy(comm)
    if dist:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
