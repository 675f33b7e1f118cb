#!/usr/bin/env python3
"""bench.py -- CG matvecs/s + raster Mpix/s of the MI355X LM hot path (BASELINE.json metric).

Workload (BASELINE.json configs[2], the 1-GPU LM config; configs[3] at N = 8): P = 1M synthetic
Gaussians, SH degree 3, one 1920x1080 view per GPU (views sharded, weak scaling), random-init
model / seeded cameras / GT = render of a perturbed copy (SURVEY §8(d) recipe; no datasets here).

One step = one CG iteration of the LM solve: the fused (J^T J + D) p over the whole view batch
(per view: tangent preprocess -> fused JVP->VJP tile pass -> gather-sum backward; then one RCCL
all-reduce of the param-space vector when N > 1) plus the CG vector updates, device resident.
The primal forward / sort is done once per LM step (outside the timed region, reported as
raster Mpix/s from a separate timed loop of full forwards).  Before the W warm-up and K timed steps,
untimed CG calls run for ~200 ms so the GPU clocks are at the steady state of a running solve
(reported as "clock_settle"; the first call after the host-side setup runs ~15% slower).

    python bench.py [--gpus N] [--steps K] [--warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...
Prints ONE JSON line on rank 0.
"""
import argparse
import ctypes
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "gaussian-splatting-lm_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "CG matvecs/sec + raster Mpix/s, 1M Gaussians @1080p, 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md chip table)
RASTER_STREAMS = int(os.environ.get("GSLM_RASTER_STREAMS", "8"))  # renders in flight for `raster_streams` in the line


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--sh", type=int, default=3)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--views-per-gpu", type=int, default=1)
    ap.add_argument("--s0", type=float, default=0.005)
    ap.add_argument("--cpu-tiles", type=int, default=64)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--forward-steps", type=int, default=None)
    ap.add_argument("--val-views", type=int, default=50, help="line-search validation views (train_jvp.py:214-216)")
    ap.add_argument("--no-side", action="store_true", help="headline + roofline only (profiling runs)")
    ap.add_argument("--no-rank-slices", action="store_true",
                    help="skip the per-rank memory / time slices of configs[3] and configs[4] (N = 1 only)")
    return ap.parse_args()


def spawn_ranks(args):
    """`python bench.py --gpus N` without a launcher: start N ranks as child processes (one per GPU, RCCL) with the
    torchrun environment, before this process touches the GPU, and exit with the worst child's code.  Rank 0's
    stdout (the JSON line) passes through."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    procs = []
    for r in range(args.gpus):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(args.gpus), LOCAL_WORLD_SIZE=str(args.gpus),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else subprocess.DEVNULL))
    # poll every rank: the first one that fails ends the others (survivors would block in a collective until
    # RCCL's own timeout), and the whole job has a deadline
    deadline = time.monotonic() + float(os.environ.get("GSLM_BENCH_TIMEOUT_S", "1500"))
    codes = [None] * len(procs)
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
        failed = [c for c in codes if c not in (None, 0)]
        if failed or time.monotonic() > deadline:
            if not failed:
                print("bench.py: ranks still running after the deadline, terminating", file=sys.stderr)
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            return (failed or [124])[0]
        time.sleep(0.2)
    return max(codes, key=abs)


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn_ranks(args))
    # stdout carries exactly the one JSON line: everything else written to fd 1 -- RCCL prints its version banner
    # there at communicator setup -- goes to stderr
    sys.stdout.flush()
    json_out = os.fdopen(os.dup(1), "w")
    os.dup2(2, 1)
    world_size = int(os.environ.get("WORLD_SIZE", "1"))
    if world_size != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_size}: launch one rank per GPU "
                         f"(torchrun --nproc-per-node {args.gpus} bench.py --gpus {args.gpus}, or bench.py --gpus N alone)")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # GSLM_BENCH_DIST=gloo rehearses the multi-rank path with several ranks on one GPU (host-staged
    # collectives); the driver's runs use RCCL ("nccl"), one rank per GPU.
    backend = os.environ.get("GSLM_BENCH_DIST", "nccl")
    dev_index = local_rank if backend == "nccl" else local_rank % max(torch.cuda.device_count(), 1)
    # GSLM_FORCE_COLLECTIVES=1 at one rank (the one-rank RCCL rehearsal, gslm.parallel.collectives_on): a one-rank
    # process group, every collective of the exchange picked by GSLM_BENCH_EXCHANGE (default "auto") issued to it
    forced = os.environ.get("GSLM_FORCE_COLLECTIVES") == "1"
    if world_size > 1 or forced:
        if forced and world_size == 1:
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", "29531")
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("WORLD_SIZE", "1")
        torch.cuda.set_device(dev_index)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", dev_index)

    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem, cgls_fused
    from gslm.model import synthetic_gaussians
    from gslm.parallel import ShardedLMProblem, shard_views

    n_views = world_size * args.views_per_gpu
    W, H = args.width, args.height
    cams_all = orbit_cameras(n_views, W, H, seed=1)
    mine = shard_views(n_views, rank, world_size)
    cams = [cams_all[i] for i in mine]
    bg = torch.zeros(3)

    # GT (seed 2): render of the model with f_dc / opacity / scaling perturbed by N(0, 0.01^2)
    pert = synthetic_gaussians(args.P, args.sh, seed=0, s0=args.s0, device="cpu", n_cams=n_views)
    g2 = torch.Generator().manual_seed(2)
    with torch.no_grad():
        pert._features_dc += 0.01 * torch.randn(pert._features_dc.shape, generator=g2)
        pert._opacity += 0.01 * torch.randn(pert._opacity.shape, generator=g2)
        pert._scaling += 0.01 * torch.randn(pert._scaling.shape, generator=g2)
    pert.to(device)
    gt_prob = LMProblem(pert, [c.to(device) for c in cams], bg, device=device)
    gt_prob.evaluate()
    for c, vr in zip(cams, gt_prob.views):
        c.original_image = vr.color.clamp(0, 1).clone()
    del gt_prob
    # the line search's validation views (train_jvp.py:214-216: 50 cameras), GT from the same perturbed model; each
    # rank renders the GT of the views its LossEvaluator will hold (lm_step shards them with shard_views)
    val_all = orbit_cameras(args.val_views, W, H, seed=5) if not args.no_side else []
    mine_val = shard_views(len(val_all), rank, world_size)
    for c0 in range(0, len(mine_val), 8):
        chunk = [val_all[i].to(device) for i in mine_val[c0:c0 + 8]]
        vp = LMProblem(pert, chunk, bg, device=device)
        vp.evaluate()
        for c, vr in zip(chunk, vp.views):
            c.original_image = vr.color.clamp(0, 1).clone()
        del vp
    del pert
    torch.cuda.empty_cache()

    torch.cuda.reset_peak_memory_stats(device)
    model = synthetic_gaussians(args.P, args.sh, seed=0, s0=args.s0, device="cpu", n_cams=n_views).to(device)
    resident0 = torch.cuda.memory_allocated(device)  # the model + the GT images of the training / validation views
    # one view per problem (N = 1): the SH-rest group of the CG vectors is carried as its 3 coordinates in
    # the view's SH-rest span (GSLM_MV_SH_REST_PROJECTED); several views: the full layout
    prob = ShardedLMProblem(model, cams, bg, all_cams=cams_all, device=device, sh_projection="auto",
                            exchange=os.environ.get("GSLM_BENCH_EXCHANGE", "auto"))
    prob.evaluate()
    g = prob.rhs(prob.zeros())
    torch.cuda.synchronize()
    n_rendered = prob.num_rendered()

    def barrier():
        if world_size > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world_size > 1:
            t = torch.tensor([x], dtype=torch.float64, device=device)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            return float(t.item())
        return x

    # ---------------- GPU clock settle.  The GPU idles through the host-side scene setup, and its clocks need
    # ~150 ms of this load to reach their steady state: after 2 s idle the first timed CG call runs 0.83-0.87 ms per
    # iteration, after 150 ms of untimed CG calls 0.74 (tools/exp/cg_warm.py, profiles/r02/cg_clock_warmup.json; full
    # forwards warm it less).  An LM solve keeps the GPU busy, so the headline is the steady-state rate: untimed CG
    # calls run for >= 200 ms first (reported as "clock_settle"), then the W warm-up steps and the K timed ones.
    # (every rank runs the same number of calls: the sharded exchanges hold collectives)
    # (every rank runs the same number of calls: the sharded exchanges hold collectives; the second call's time
    # sizes the loop, the first one also allocates the CG vectors)
    t_settle0 = time.perf_counter()
    cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False)
    torch.cuda.synchronize()
    t_call = time.perf_counter()
    cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False)
    torch.cuda.synchronize()
    t_call = time.perf_counter() - t_call
    n_calls = max(int(max_over_ranks(math.ceil(0.2 / max(t_call, 1e-3)))) - 2, 0)
    for _ in range(n_calls):
        cgls_fused(prob, g, max_iter=10, restart_iter=10, check_every=False)
        torch.cuda.synchronize()
    settle = {"cg_iterations": 10 * (2 + n_calls), "ms": 1e3 * (time.perf_counter() - t_settle0)}

    # ---------------- timed: K CG iterations (fused matvec + vector ops), no host sync inside
    cgls_fused(prob, g, max_iter=max(args.warmup, 1), restart_iter=max(args.warmup, 1), check_every=False)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    x, _ = cgls_fused(prob, g, max_iter=args.steps, restart_iter=args.steps, check_every=False)
    torch.cuda.synchronize()
    barrier()
    t_cg = max_over_ranks(time.perf_counter() - t0)
    ms_per_step = 1e3 * t_cg / args.steps

    # the same K iterations with the reference's stopping tests each iteration (conjugate_gradient.py:88-117: delta,
    # the residual monitor b^2 - <x, g> - <x, s>, the gamma tolerance), evaluated on the device (gslm_cg_monitor; the
    # monitor's two dots fused into the update pass): what an iteration of train_jvp.py's CGLS costs in full.  The
    # timed loop above skips only those scalar tests (its iterates are identical while no test fires).  Warm-up
    # first: the monitor's kernels load on their first launch.
    cgls_fused(prob, g, max_iter=max(args.warmup, 1), restart_iter=max(args.warmup, 1), check_every=True)
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _, info_chk = cgls_fused(prob, g, max_iter=args.steps, restart_iter=args.steps, check_every=True)
    torch.cuda.synchronize()
    barrier()
    t_chk = max_over_ranks(time.perf_counter() - t0)
    # device memory of the CG solve: the torch allocator's peak since the model was created (model,
    # the problem's library workspaces -- geometry, binning, image state, scratch per view -- the weights and the CG
    # vectors); nothing else is resident on this rank
    loc0 = getattr(prob, "local", prob)
    peak_mem = {"cg_loop": {"max_allocated_gb": peak_gb(device), "resident_before_gb": resident0 / 1e9,
                            "workspace_gb": cuda_tensor_bytes(loc0.views) / 1e9,
                            "note": "torch.cuda.max_memory_allocated from the model's creation through the timed CG "
                                    "loops (model, every view's library workspaces, weights, CG vectors); "
                                    "resident_before_gb = the model and the GT images of the training and validation "
                                    "views; workspace_gb = the views' gslm workspaces alone"}}
    del loc0
    cg_checked = {"ms_per_step": 1e3 * t_chk / args.steps, "view_matvec_per_s": n_views * args.steps / t_chk,
                  "iters_before_stop": info_chk["iters"], "stop": info_chk.get("stop"),
                  "note": "the timed K iterations with the reference's stopping tests on the device each iteration "
                          "(stop 0: none fired; a fired test leaves the later launches returning at once)"}

    # the same CG loop on the reference's full param-space layout (59 floats per Gaussian at SH 3), for
    # comparison when the projected SH-rest layout ran above
    cg_full = None
    if prob.layout.rest_projected:
        pf = LMProblem(model, cams, bg, device=device, sh_projection=False)
        pf.evaluate()
        gf = pf.rhs(pf.zeros())
        cgls_fused(pf, gf, max_iter=max(args.warmup, 1), restart_iter=max(args.warmup, 1), check_every=False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        cgls_fused(pf, gf, max_iter=args.steps, restart_iter=args.steps, check_every=False)
        torch.cuda.synchronize()
        tf = time.perf_counter() - t0
        cg_full = {"ms_per_step": 1e3 * tf / args.steps, "view_matvec_per_s": n_views * args.steps / tf,
                   "note": "CG iteration with the SH-rest group in the reference's layout (3(K-1) floats per Gaussian)"}
        del pf, gf
        torch.cuda.empty_cache()

    # per-rank stage times of the sharded product (GaussianShardedOperator: tangent records for every view, the two
    # all-to-alls, the tile pass + screen sums of this rank's views, the shard's gather), HIP events around each
    # stage of a few extra products outside the timed region
    shard_stages = None
    if getattr(prob, "exchange", None) == "gaussian" and hasattr(prob, "stage_times"):
        shard_stages = prob.stage_times(g, reps=max(args.steps, 5))

    # ---------------- raster Mpix/s: full forwards (preprocess, depth sort, binning, tile sort, ranges, blend) through
    # the device-count form (gslm_rasterize_dev: the pair count stays on the device, no host round trip between the
    # preprocess and the binning); each render's count is checked against its list capacity after the timed loop.
    # `raster_sync_mpix_s`: the same forwards with the count read back per view (gslm_forward's protocol, as upstream)
    fsteps = args.forward_steps or args.steps
    from gslm.params import raw_gaussians
    graw = raw_gaussians(model)
    for vr in prob.views:
        vr.forward(graw, prob.stream)
    counts = torch.zeros(max(fsteps, 1) * len(prob.views), dtype=torch.int32, device=device)
    caps = [vr.capacity() for vr in prob.views]
    barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(fsteps):
        for j, vr in enumerate(prob.views):
            vr.forward_dev(graw, prob.stream, n_out=counts.data_ptr() + 4 * (it * len(prob.views) + j))
    torch.cuda.synchronize()
    barrier()
    t_fwd = max_over_ranks(time.perf_counter() - t0)
    cnt = counts.view(max(fsteps, 1), len(prob.views)).tolist()
    if any(c[j] > caps[j] for c in cnt[:fsteps] for j in range(len(caps))):
        raise RuntimeError(f"raster timing: a pair count exceeded its list capacity ({cnt[0]} vs {caps})")
    mpix = n_views * W * H * fsteps / t_fwd / 1e6
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(fsteps):
        for vr in prob.views:
            vr.forward(graw, prob.stream)
    torch.cuda.synchronize()
    barrier()
    t_fwd_sync = max_over_ranks(time.perf_counter() - t0)  # (leaves every view in forward()'s exact layout)
    mpix_sync = n_views * W * H * fsteps / t_fwd_sync / 1e6
    # ---------------- roofline of the dominant kernel: the fused JVP->VJP tile pass (k_render_matvec)
    loc = getattr(prob, "local", prob)  # the rank's own LMProblem (full P) under a sharded operator
    vr = loc.views[0]
    xv = prob.gather_full(x) if getattr(prob, "exchange", None) == "gaussian" else x
    vs = loc.layout.grads_struct(xv)
    ys = loc.layout.grads_struct(loc.zeros(), accumulate=True)
    lib, check = _lib.lib, _lib.check

    def stage(mask):
        opts = _lib.GslmMatvecOpts()
        opts.stages = mask | (8 if mask == 4 else 0)  # the gather in its CG form: overwrite + D v
        opts.flags = 1 | loc.mv_flags  # GSLM_MV_TAIL_CLEAN: the geometry's derived state built (opts0), as in the CG loop
        opts.damp7 = loc._damps if mask == 4 else None
        check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(graw), ctypes.byref(vs),
                                      loc.weights[0].data_ptr(), 1, vr.geom.data_ptr(), vr.binning.data_ptr(),
                                      vr.N, vr.image.data_ptr(), vr.scratch.data_ptr(), vr.scratch.numel(),
                                      ctypes.byref(ys), ctypes.byref(opts), loc.stream))

    opts0 = _lib.GslmMatvecOpts()
    # RENDER once without GSLM_MV_TAIL_CLEAN (the forwards above rewrote the binning): the row map and, with the
    # projected LM rows, the linearisation record rebuilt -- the state every CG iteration after the first sees
    opts0.stages = 2
    opts0.flags = loc.mv_flags
    check(lib.gslm_matvec_view_ex(ctypes.byref(vr.view), ctypes.byref(graw), ctypes.byref(vs), loc.weights[0].data_ptr(),
                                  1, vr.geom.data_ptr(), vr.binning.data_ptr(), vr.N, vr.image.data_ptr(),
                                  vr.scratch.data_ptr(), vr.scratch.numel(), ctypes.byref(ys), ctypes.byref(opts0),
                                  loc.stream))
    stage(1)
    stage(2)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    reps = max(args.steps, 5)
    ev0.record()
    for _ in range(reps):
        stage(2)
    ev1.record()
    torch.cuda.synchronize()
    render_ms = ev0.elapsed_time(ev1) / reps
    # per-stage times (tangent, gather) for the breakdown
    def time_stage(mask, n=reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            stage(mask)
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n
    tangent_ms = time_stage(1)
    gather_ms = time_stage(4)
    N0, HW = vr.N, W * H
    # algorithmic bytes of one k_render_matvec launch (SURVEY §8(d) per-unit figures):
    #   per (tile, Gaussian) entry: JVP pass primal gather 44 + tangent gather 40,
    #   VJP pass primal gather 44 + one gradient row 40 (plain store, replaces the atomic RMW)
    #   per pixel: n_contrib 4 + final_T 4 + weight 12
    alg_strict = 168 * N0 + 20 * HW
    # SURVEY 8(d)'s own per-unit figures for the two passes the fused kernel runs (B_jvp's 84 N_dup + 16 HW and B_vjp's
    # 124 N_dup + 24 HW, whose 2 x 40 B per entry is the atomic read-modify-write the row store replaces): `achieved`
    # is priced on them as the task prescribes; the stricter 168 N + 20 HW above is kept beside it
    alg_bytes = 208 * N0 + 40 * HW
    achieved = alg_bytes / (render_ms * 1e-3) / 1e9
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_render_matvec.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("P") == args.P and pm.get("width") == W and pm.get("height") == H:
                traffic = pm.get("hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None

    # list entries any pixel of their tile can blend (sum over tiles of max n_contrib): the tile passes read only
    # these (positions past a tile's last blended entry are skipped), N_dup counts every binned pair
    ts = tile_stats(vr, args.P)
    alg_visited = 168 * ts["visited_entries"] + 20 * HW
    # forward raster against SURVEY 8(d)'s B_fwd per view (params 4F P, preprocess state 48 P, 88 per list entry:
    # key/value write 12 + one sort read/write 24 + range scan 8 + render gather 44, 24 per pixel)
    F = 11 + 3 * (args.sh + 1) ** 2
    b_fwd = 4 * F * args.P + 48 * args.P + 88 * N0 + 24 * HW
    fwd_s = t_fwd / fsteps / max(len(prob.views), 1)
    raster_roofline = {"bound": "hbm", "achieved": b_fwd / fwd_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                       "frac": b_fwd / fwd_s / 1e9 / HBM_PEAK_GBS, "alg_bytes_per_view": b_fwd,
                       "model": "SURVEY 8(d) B_fwd = 4F P + 48 P + 88 N_dup + 24 HW, over the full forward "
                                "(preprocess, depth sort, binning, tile sort, ranges, blend; the pair count on the "
                                "device, gslm_rasterize_dev)"}

    # the side measurements below run on one view and need the memory of the batch's problem back
    # (at configs[4], 5M Gaussians x 32 4K views, that is ~100 GB)
    n_views_local = len(loc.views)
    sh_proj = prob.layout.rest_projected
    exchange = prob.exchange if (world_size > 1 or forced) else "none"
    view0 = prob.views[0].view if prob.views else None
    del prob, loc, vr, vs, ys, x, xv, g
    torch.cuda.empty_cache()

    raster_streams = None

    fb = c0_gpu = lm = lm_tv = lm_ref = ssim = fo = dropin = None
    if not args.no_side:
        # ---------------- BASELINE configs[2] / [3] as train_jvp.py runs it, on every rank: one full LM step (loss,
        # J^T b, CGLS with 10 iterations and the reference's stopping tests, the 7-point line search on the
        # reference's 50 validation views), sharded over the ranks; and with the training batch as the validation set
        torch.cuda.reset_peak_memory_stats(device)
        resident = torch.cuda.memory_allocated(device)
        lm = time_lm_step(model, cams_all, val_all, bg)
        from gslm.lm import _VAL_CACHE
        ev = _VAL_CACHE.get("last")
        peak_mem["lm_step"] = {"max_allocated_gb": peak_gb(device), "resident_before_gb": resident / 1e9,
                               "evaluator_workspace_gb": (cuda_tensor_bytes(ev[1]) / 1e9) if ev else None,
                               "note": "configs[2] LM step (evaluate, J^T b, CGLS 10 with the stopping tests, the line "
                                       "search on the validation views): allocator peak over its timed reps; "
                                       "evaluator_workspace_gb = the validation evaluator kept across LM steps "
                                       "(its per-view depth orders, union lists and slot workspaces)"}
        del ev
        lm_tv = time_lm_step(model, cams_all, cams_all, bg, reps=3, with_timing=False)
        # the reference's own CGLS schedule, max_iter = 2, restart_iter = 1 (train_jvp.py:254-256; SURVEY 8(d) config 3
        # "the reference-schedule (2 x 1) variant is also reported")
        lm_ref = time_lm_step(model, cams_all, val_all, bg, iters=2, restart=1, reps=3)
        # ---------------- BASELINE configs[1]: 100k Gaussians SH 3, one 1080p view, forward + backward
        # through the drop-in autograd surface (GaussianRasterizer, the reference's render() path)
        fb = time_drop_in_fwd_bwd(device, W, H, args.s0, reps=max(args.steps, 5)) if rank == 0 else None
        c0_gpu = time_config0_gpu(device) if rank == 0 else None
        # the drop-in operator at the headline size: what an unchanged train_jvp.py pays per matvec / matvec_T /
        # evaluate_loss (tests/test_jvp_timing.py:71-106 through the reference's call shapes)
        torch.cuda.reset_peak_memory_stats(device)
        resident = torch.cuda.memory_allocated(device)
        dropin = time_dropin_solver_ops(model, cams[0], bg, reps=11) if rank == 0 else None
        peak_mem["dropin_solver_ops"] = {"max_allocated_gb": peak_gb(device), "resident_before_gb": resident / 1e9,
                                         "note": "the drop-in J u / J^T v / forward calls through render() at the "
                                                 "headline size (autograd graphs, dual tensors, rasterizer buffers)"}
        # the SSIM residual (disable_ssim=False): CG iteration on the same view(s)
        ssim = time_ssim_cg(model, cams[:1], bg, steps=args.steps) if world_size == 1 else None
        # first-order path: the fused Adam step at the bench model's size and one train.py
        # iteration (render, L1 + SSIM loss, backward, densification statistics, Adam) at configs[1]'s size
        fo = time_first_order(device, W, H, args.s0, P_adam=args.P, sh=args.sh) if rank == 0 else None

    # ---------------- what one rank of the 8-GPU configs holds, emulated on this GPU (N = 1 only)
    rank_slices = None
    if world_size == 1 and not forced and not args.no_side and not args.no_rank_slices:
        rank_slices = rank_slice_memory(model, cams_all, val_all, bg, device)

    # ---------------- the raster forwards with RASTER_STREAMS renders in flight on as many HIP streams (independent
    # renders overlap, a render's launch-bound sort passes beside another's blend) -- a throughput over many renders,
    # reported beside the one-stream rate, which stays `raster_mpix_s`.  Run LAST among the GPU measurements: after a
    # burst of 8-stream work the process's later kernels run slower (the stage timing measured k_render_matvec 7% over
    # rocprof's solo average; the LM step 96.3 ms against 91-92 in tools/exp/lm_phases.py on the same box, every
    # phase 6-10% slower, profiles/r06/ab_bench_order/), which an LM run that never issues such a burst does not see
    if not args.no_side and view0 is not None:
        from gslm.lm import ViewRaster
        S = RASTER_STREAMS
        rasters = [ViewRaster(view0, device) for _ in range(S)]
        graw2 = raw_gaussians(model)
        streams = [torch.cuda.Stream(device) for _ in range(S)]
        for r, st in zip(rasters, streams):
            r.forward(graw2, st.cuda_stream)
        capz = [r.capacity() for r in rasters]
        cnt_s = torch.zeros(max(fsteps, 1) * S, dtype=torch.int32, device=device)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for it in range(fsteps):
            for j, (r, st) in enumerate(zip(rasters, streams)):
                r.forward_dev(graw2, st.cuda_stream, n_out=cnt_s.data_ptr() + 4 * (it * S + j))
        torch.cuda.synchronize()
        t_s = time.perf_counter() - t0
        cs = cnt_s.view(max(fsteps, 1), S).tolist()
        if any(c[j] > capz[j] for c in cs[:fsteps] for j in range(S)):
            raise RuntimeError("raster_streams: a pair count exceeded its list capacity")
        raster_streams = {"streams": S, "renders": S * fsteps, "mpix_s": S * fsteps * W * H / t_s / 1e6,
                          "ms_per_render": 1e3 * t_s / (S * fsteps),
                          "note": f"{S} independent forwards of view 0 in flight on {S} HIP streams (gslm_rasterize_dev, "
                                  "counts checked after the loop): render throughput, not one forward's latency "
                                  "(raster_mpix_s / forward_ms_per_view)"}
        del rasters, streams
        torch.cuda.empty_cache()


    # ---------------- CPU baseline (rank 0, N = 1 only): the oracle on host cores, bounded sample
    cpu = None
    if rank == 0 and world_size == 1 and not args.no_cpu_baseline and not args.no_side:
        from oracle.cpu_baseline import cpu_matvec_rate
        cm = synthetic_gaussians(args.P, args.sh, seed=0, s0=args.s0, device="cpu")
        cc = orbit_cameras(1, W, H, seed=1)[0]
        threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count()
        r = cpu_matvec_rate(cm, cc, torch.zeros(3), n_tiles=args.cpu_tiles, repeats=3, threads=threads)
        from oracle.cpu_baseline import cpu_config0_times, cpu_config1_forward, host_info
        c0 = cpu_config0_times(repeats=5, threads=threads)
        c1 = cpu_config1_forward(repeats=5, threads=threads, W=W, H=H, s0=args.s0)
        cpu = {"value": 1.0 / r["matvec_s"], "unit": "view-matvec/s", "cores": r["threads"], "kind": "port",
               "sample": (f"oracle/torch_raster.py (PyTorch CPU, {r['threads']} threads, {r['cpu_model']}): "
                          f"all {args.P} Gaussians through preprocess+binning with forward-AD and autograd "
                          f"(t_gauss={r['t_gauss']:.2f}s, timed whole), blend JVP+VJP on {r['n_tiles']} of "
                          f"{r['ntiles']} tiles spread over the 1080p frame (t_tiles={r['t_tiles']:.3f}s, timed on "
                          f"their own) scaled by {r['ntiles']}/{r['n_tiles']}; each phase the median of 3"),
               "raster_mpix_s": W * H / r["forward_s"] / 1e6,
               "host": host_info(),
               "threads_note": "OMP_NUM_THREADS threads: the CPU share the GPU box gives one GPU's job (16 of the "
                               "host's threads; os.cpu_count() counts the whole 8-GPU host, whose other threads "
                               "belong to the other GPUs' jobs, so timing on all of them would not be this "
                               "job's baseline)",
               "configs1_forward": c1,
               "configs0": dict(c0, config="BASELINE configs[0]: 2000 Gaussians SH0, one 256x256 view, oracle "
                                           "forward / JVP / VJP, 1 warm-up + median of 5, no extrapolation")}

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": n_views * args.steps / t_cg,
            "unit": "view-matvec/s (one (J^T J + D) application per 1080p view, 1M Gaussians)",
            "n_gpus": world_size, "ranks": dist.get_world_size() if world_size > 1 else 1,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (seeded Gaussians / orbit cameras / GT = render of perturbed model)",
            "config": {"workload": f"LM CG iteration, {args.P} Gaussians SH{args.sh}, {args.views_per_gpu}x{W}x{H} "
                                   f"view(s) per GPU (BASELINE configs[2]; configs[3] at 8 GPUs)",
                       "P": args.P, "sh_degree": args.sh, "width": W, "height": H,
                       "views_total": n_views, "parallelism": f"views sharded x{world_size}",
                       "exchange": exchange, "sh_rest_projected": bool(sh_proj)},
            "cg_matvecs_per_s": args.steps / t_cg,
            "cg_checked": cg_checked,
            "clock_settle": dict(settle, note="untimed CG calls before the warm-up and timed steps: the GPU clocks "
                                              "at their steady state, as in a running LM solve"),
            "raster_mpix_s": mpix,
            "forward_ms_per_view": 1e3 * t_fwd / fsteps / max(n_views_local, 1),
            "raster_sync": {"mpix_s": mpix_sync, "forward_ms_per_view": 1e3 * t_fwd_sync / fsteps / max(n_views_local, 1),
                            "note": "the same forwards with the pair count read back by the host before the binning "
                                    "(gslm_forward's protocol, as the upstream forward)"},
            "raster_streams": raster_streams,
            "num_rendered": n_rendered,
            "stage_ms": {"tangent_preprocess": tangent_ms, "render_matvec": render_ms, "gather_backward": gather_ms},
            "roofline": {"bound": "hbm", "kernel": "k_render_matvec", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "alg_bytes_per_launch": alg_bytes, "avg_launch_ms": render_ms,
                         "frac_strict": alg_strict / (render_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "alg_bytes_strict": alg_strict,
                         "frac_visited": alg_visited / (render_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                         "alg_bytes_visited": alg_visited,
                         "note": "SURVEY 8(d): B_jvp + B_vjp tile terms, (84 + 124) B per list entry + (16 + 24) B "
                                 "per pixel; frac_strict: 168 B per entry (no atomic RMW: one plain row store) + 20 B "
                                 "per pixel; frac_visited: the strict model over the entries a pixel of their tile "
                                 "can blend (sum over tiles of max n_contrib)"},
            "raster_roofline": raster_roofline,
            "tile_stats": ts,
            "cpu_baseline": cpu,
            "raster_fwd_bwd": fb,
            "configs0_gpu": c0_gpu,
            "dropin_solver_ops": dropin,
            "sharded_stage_ms": shard_stages,
            "lm_step": lm,
            "lm_step_val_is_train": lm_tv,
            "lm_step_ref_schedule": lm_ref,
            "ssim_cg": ssim,
            "first_order": fo,
            "cg_full_layout": cg_full,
            "peak_mem": dict(peak_mem, rank_slices=rank_slices),
        }
        json_out.write(json.dumps(line) + "\n")
        json_out.flush()
    if dist.is_initialized():
        dist.barrier()
        from gslm.parallel import close_native_comms
        close_native_comms()  # (GSLM_COMM=native) every rank at the same point, before the process group goes
        dist.destroy_process_group()


def rank_slice_memory(model, cams_all, val_all, bg, device):
    """Device memory (and time) of one rank's share of the multi-GPU configs, run on this GPU:
      configs3_lm_step   BASELINE configs[3] at 8 ranks: the LM step of one rank -- its one 1080p training view and its
                         ceil(50 / 8) = 7 validation views, 1M Gaussians (the model replicated; at one rank the CG
                         vectors are full-P, an upper bound of the sharded rank's P / 8 slices);
      configs4_cg_slice  BASELINE configs[4] at 8 ranks: rank 0's CG iterations of the Gaussian-sharded product over
                         its 4 of 32 4K views, 5M Gaussians (GaussianShardedOperator(emulate=(0, 8)): the collectives
                         replaced by same-shape local copies)."""
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem, cgls_fused, clear_val_cache, lm_step
    from gslm.model import synthetic_gaussians
    from gslm.parallel import GaussianShardedOperator
    out = {}
    clear_val_cache()
    torch.cuda.empty_cache()
    if val_all:
        saved = [t.detach().clone() for t in model.params()]
        torch.cuda.reset_peak_memory_stats(device)
        res = torch.cuda.memory_allocated(device)
        n_val = -(-len(val_all) // 8)
        t0 = time.perf_counter()
        o = lm_step(model, [cams_all[0]], val_all[:n_val], bg, max_iter=10, restart_iter=10)
        torch.cuda.synchronize()
        t_lm = time.perf_counter() - t0  # (one step, cold: workspaces allocated inside)
        with torch.no_grad():
            for t, s0 in zip(model.params(), saved):
                if t is not model._xyz:
                    t.copy_(s0)
        out["configs3_lm_step"] = {"max_allocated_gb": peak_gb(device), "resident_before_gb": res / 1e9,
                                   "train_views": 1, "val_views": n_val, "P": int(model._xyz.shape[0]),
                                   "first_step_ms": 1e3 * t_lm, "best_alpha": o["best_alpha"]}
        del saved, o
        clear_val_cache()
        torch.cuda.empty_cache()
    P5, W4, H4, per, n = 5_000_000, 3840, 2160, 4, 8
    torch.cuda.reset_peak_memory_stats(device)
    res = torch.cuda.memory_allocated(device)
    cams = [c.to(device) for c in orbit_cameras(n * per, W4, H4, seed=1)]
    m5 = synthetic_gaussians(P5, 3, seed=0, s0=0.005, device="cpu", n_cams=n * per).to(device)
    mine = cams[:per]
    g5 = torch.Generator().manual_seed(7)
    for c in mine:
        c.original_image = torch.rand(3, H4, W4, generator=g5).to(device)
    local = LMProblem(m5, mine, bg, device=device, sh_projection=False)
    local.evaluate()
    op = GaussianShardedOperator(local, all_cams=cams, emulate=(0, n))
    gs = op.rhs(op.zeros())
    cgls_fused(op, gs, max_iter=2, restart_iter=2, check_every=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cgls_fused(op, gs, max_iter=3, restart_iter=3, check_every=False)
    torch.cuda.synchronize()
    t_it = (time.perf_counter() - t0) / 3
    out["configs4_cg_slice"] = {"max_allocated_gb": peak_gb(device), "resident_before_gb": res / 1e9, "P": P5,
                                "views_on_rank": per, "ranks": n, "width": W4, "height": H4,
                                "workspace_gb": cuda_tensor_bytes(local.views) / 1e9,
                                "num_rendered": [vr.N for vr in local.views],
                                "emulated_cg_ms_per_iteration": 1e3 * t_it,
                                "note": "rank 0 of 8, collectives as local copies (compute only)"}
    del op, local, gs, m5, cams, mine
    torch.cuda.empty_cache()
    return out


def cuda_tensor_bytes(*objs, depth=3):
    """Bytes of the distinct CUDA tensors reachable from objs through attributes, lists, tuples and dicts (depth-
    limited): the library workspaces a ViewRaster / LossEvaluator holds (geometry, binning, image state, scratch)."""
    seen, total = set(), 0

    def walk(o, d):
        nonlocal total
        if isinstance(o, torch.Tensor):
            if o.is_cuda:
                st = o.untyped_storage()
                if st.data_ptr() not in seen:
                    seen.add(st.data_ptr())
                    total += st.nbytes()
            return
        if d <= 0:
            return
        if isinstance(o, (list, tuple)):
            for x in o:
                walk(x, d - 1)
        elif isinstance(o, dict):
            for x in o.values():
                walk(x, d - 1)
        elif hasattr(o, "__dict__") and not isinstance(o, type):
            for x in vars(o).values():
                walk(x, d - 1)

    for o in objs:
        walk(o, depth)
    return total


def peak_gb(device):
    return torch.cuda.max_memory_allocated(device) / 1e9


def tile_stats(vr, P):
    """N_dup, visited entries (sum over tiles of the max n_contrib of their pixels) and the mean n_contrib per
    pixel of one preprocessed view (SURVEY 8(d) asks for N_dup and the mean blended count per pixel)."""
    from gslm import _lib
    H, W = vr.H, vr.W
    nc = torch.zeros(H * W, dtype=torch.int32, device=vr.device)
    _lib.check(_lib.lib.gslm_inspect(vr.geom.data_ptr(), P, vr.binning.data_ptr(), vr.N, H, W, vr.image.data_ptr(),
                                     None, None, None, None, nc.data_ptr(), None, _lib.stream_handle(vr.device)))
    gy, gx = (H + 15) // 16, (W + 15) // 16
    pad = torch.zeros(gy * 16, gx * 16, dtype=torch.int32, device=vr.device)
    pad[:H, :W] = nc.view(H, W)
    per_tile = pad.view(gy, 16, gx, 16).amax(dim=(1, 3))
    return {"num_rendered": int(vr.N), "visited_entries": int(per_tile.sum()),
            "visited_frac": float(per_tile.sum()) / max(int(vr.N), 1),
            "mean_n_contrib_per_pixel": float(nc.double().mean()), "tiles": gx * gy}


def time_config0_gpu(device, reps=20):
    """BASELINE configs[0] on the GPU through the drop-in rasterizer (forward, forward-mode JVP, VJP): 2000 Gaussians,
    SH 0, one 256x256 view, median of `reps` host-timed calls (each includes the num_rendered read-back)."""
    import torch.autograd.forward_ad as fwAD
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    m = synthetic_gaussians(2000, 0, seed=0, s0=0.005, device="cpu").to(device)
    cam = orbit_cameras(1, 256, 256, seed=1)[0].to(device)
    st = GaussianRasterizationSettings(
        image_height=256, image_width=256, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=torch.zeros(3, device=device), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=0, campos=cam.camera_center, prefiltered=False, debug=False,
        antialiasing=False)
    rast = GaussianRasterizer(st)
    a = {"means3D": m.get_xyz.detach(), "opacities": m.get_opacity.detach(), "scales": m.get_scaling.detach(),
         "rotations": m.get_rotation.detach(), "shs": m.get_features.detach().contiguous()}
    g3 = torch.Generator().manual_seed(3)
    tang = {k: torch.randn(v.shape, generator=g3).to(device) for k, v in a.items()}
    dcol = torch.randn(3, 256, 256, generator=torch.Generator().manual_seed(4)).to(device)
    m2 = torch.zeros_like(a["means3D"])

    def fwd():
        with torch.no_grad():
            rast(means2D=m2, **a)

    def jvp():
        with torch.no_grad(), fwAD.dual_level():
            fwAD.unpack_dual(rast(means2D=m2, **{k: fwAD.make_dual(v, tang[k]) for k, v in a.items()})[0]).tangent

    def vjp():
        leaves = {k: v.clone().requires_grad_(True) for k, v in a.items()}
        (rast(means2D=m2, **leaves)[0] * dcol).sum().backward()

    out = {"config": "BASELINE configs[0] on the GPU: 2000 Gaussians SH0, one 256x256 view, drop-in rasterizer, "
                     "median of host-timed calls"}
    for name, fn in (("forward", fwd), ("jvp", jvp), ("vjp", vjp)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_ms"] = 1e3 * sorted(ts)[len(ts) // 2]
    return out


def _events_ms(fn, reps):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def time_first_order(device, W, H, s0, P_adam=1_000_000, sh=3, P_train=100_000, reps=10):
    """gslm_adam_step (FusedAdam) vs torch.optim.Adam (foreach) over the six training_setup groups of a
    P_adam-Gaussian model, and one train.py iteration (gslm.train.Trainer.step, no densification) at
    P_train Gaussians, one WxH view."""
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    from gslm.optim import FusedAdam
    from gslm.train import OptimizationParams, Trainer
    K = (sh + 1) ** 2
    shapes = {"xyz": (P_adam, 3), "f_dc": (P_adam, 1, 3), "f_rest": (P_adam, K - 1, 3), "opacity": (P_adam, 1),
              "scaling": (P_adam, 3), "rotation": (P_adam, 4)}
    out = {}
    for name, cls in (("fused", FusedAdam), ("torch", torch.optim.Adam)):
        ps = [torch.nn.Parameter(torch.randn(s_, device=device)) for s_ in shapes.values()]
        for p in ps:
            p.grad = torch.randn_like(p)
        opt = cls([{"params": [p], "lr": 1e-3} for p in ps], lr=0.0, eps=1e-15)
        out[name] = _events_ms(opt.step, reps)
        del ps, opt
    floats = sum(math.prod(s_) for s_ in shapes.values())
    adam = {"config": f"Adam step over the 6 parameter groups of {P_adam} Gaussians SH{sh} ({floats} floats)",
            "fused_ms": out["fused"], "torch_foreach_ms": out["torch"],
            "fused_gbs": 28.0 * floats / (out["fused"] * 1e-3) / 1e9,
            "note": "28 B per float (read p, g, m, v; write p, m, v) over the fused launch's time"}
    torch.cuda.empty_cache()
    m = synthetic_gaussians(P_train, sh, seed=0, s0=s0, device="cpu").to(device)
    m.spatial_lr_scale = 1.0
    cam = orbit_cameras(1, W, H, seed=1)[0].to(device)
    cam.original_image = torch.rand(3, H, W, device=device)
    opt = OptimizationParams(densify_from_iter=10 ** 9)  # statistics every step, no densification
    m.training_setup(opt)
    tr = Trainer(m, [cam], opt=opt)
    it = [1]

    def step():
        tr.step(it[0], viewpoint_cam=cam)
        it[0] += 1
    t_ms = _events_ms(step, reps)
    return {"adam": adam, "train_step": {
        "config": f"one train.py iteration, {P_train} Gaussians SH{sh}, 1x{W}x{H} view: render + "
                  "(1-l) L1 + l (1-SSIM) + backward + densification statistics + Adam", "ms": t_ms}}


def time_ssim_cg(model, cams, bg, steps=10):
    """CG iterations of the LM normal equations with the SSIM residual ([r1; r2], lambda_dssim 0.2):
    per view J v -> image-space factor (separable 11-tap SSIM JVP / VJP) -> seeded VJP -> gather."""
    from gslm.lm import LMProblem, cgls_fused
    prob = LMProblem(model, cams, bg, ssim=True, sh_projection="auto")
    prob.evaluate()
    g = prob.rhs(prob.zeros())
    cgls_fused(prob, g, max_iter=2, restart_iter=2, check_every=False)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    cgls_fused(prob, g, max_iter=steps, restart_iter=steps, check_every=False)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / steps
    return {"config": f"CG iteration with the SSIM residual, {len(cams)} view(s) (batch_training_loss.py:18-30)",
            "ms_per_step": 1e3 * t, "view_matvec_per_s": len(cams) / t}


def time_lm_step(model, cams, val_cams, bg, iters=10, reps=5, with_timing=True, restart=None):
    """gslm.lm.lm_step (train_jvp.py:221-289) with max_iter = iters, restart_iter = restart (default iters) and the
    reference's stopping
    tests (on the device), the line search over `val_cams`; every rank calls it (the training and validation views
    are sharded over the ranks inside).  The model is restored after each step, so every rep solves the same
    problem.  `ms` is the median of `reps` individually synchronised steps (max over ranks per rep), with the spread
    beside it; the phase breakdown (evaluate + J^T b, CG, line search) comes from one more step with timing=True."""
    from gslm.lm import lm_step
    saved = [t.detach().clone() for t in model.params()]

    def restore():
        # xyz is masked (train_jvp.py:221-227): lm_step never writes it, and copying it anyway would bump its version
        # and drop the validation views' cached depth orders, which in train_jvp.py's loop live across LM steps
        with torch.no_grad():
            for t, s0 in zip(model.params(), saved):
                if t is not model._xyz:
                    t.copy_(s0)

    restart = iters if restart is None else restart
    out = lm_step(model, cams, val_cams, bg, max_iter=iters, restart_iter=restart)  # warm-up (workspaces, clocks)
    restore()
    torch.cuda.synchronize()
    if dist.is_initialized():
        dist.barrier()
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        out = lm_step(model, cams, val_cams, bg, max_iter=iters, restart_iter=restart)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
        restore()  # (outside the timed region: bench bookkeeping, not part of train_jvp.py's step)
        torch.cuda.synchronize()
    if dist.is_initialized():
        tt = torch.tensor(ts, dtype=torch.float64, device=saved[0].device)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        ts = tt.tolist()
    srt = sorted(ts)
    t = srt[len(srt) // 2] if len(srt) % 2 else 0.5 * (srt[len(srt) // 2 - 1] + srt[len(srt) // 2])
    sched = f"{iters} iterations" if restart == iters else f"max_iter {iters} x restart_iter {restart} (the reference's schedule)"
    res = {"config": f"full LM step, {len(cams)} training view(s) over {out['ranks']} rank(s), CGLS {sched} "
                     f"with the reference's stopping tests + 7-point line search on {len(val_cams)} validation "
                     "view(s) (train_jvp.py:237-279; BASELINE configs[2], configs[3] at 8 GPUs)",
           "ms": 1e3 * t, "reps": reps, "ms_min": 1e3 * srt[0], "ms_max": 1e3 * srt[-1],
           "ms_mean": 1e3 * sum(srt) / len(srt),
           "cg_iters": out["cg"]["iters"], "val_views": len(val_cams), "ranks": out["ranks"],
           "val_renders_per_rank": 7 * -(-len(val_cams) // out["ranks"]),
           "loss_start": out["start_loss"], "loss_final": out["final_val_loss"], "best_alpha": out["best_alpha"],
           "line_search": out["line_search"]}
    if with_timing:
        # the phases, and the validation loss at the starting parameters (loss_start is the TRAINING view's loss: the
        # line search's losses are over the validation views, so loss_val_start is the one loss_final compares with)
        o2 = lm_step(model, cams, val_cams, bg, max_iter=iters, restart_iter=restart, timing=True, val_at_start=True)
        restore()
        res["breakdown_ms"] = {k: v for k, v in o2["timing"].items() if k != "val_start_ms"}
        res["loss_val_start"] = o2["val_start_loss"]
        res["ms_per_val_render"] = o2["timing"]["line_search_ms"] / res["val_renders_per_rank"]
        # the same step with train_jvp.py's render order (update, render, ...: every render bins its view)
        o3 = lm_step(model, cams, val_cams, bg, max_iter=iters, restart_iter=restart, timing=True, line_search="exact")
        restore()
        res["line_search_exact_ms"] = o3["timing"]["line_search_ms"]
        res["exact_equal"] = (o3["trace"] == o2["trace"] and o3["final_val_loss"] == o2["final_val_loss"])
    return res


def time_dropin_solver_ops(model, cam, bg, reps=5):
    """The drop-in path an unchanged train_jvp.py runs, at the headline size: tests/test_jvp_timing.py:71-106's three
    timings through the reference's call shapes on this build's diff_gaussian_rasterization (gslm.train.render =
    gaussian_renderer.render, activations in PyTorch, GaussianRasterizer's autograd Function):
      matvec    J u: forward-mode AD (GaussianModel.make_dual, solver_functions.py:83-99) through the render and the
                disable_ssim residual m clamp(R) - gt (batch_training_loss.py:10-17)
      matvec_T  J^T v: the render again with grad, then the two .backward calls of the [r; r] pair
                (loss_image_state.py:93-97, solver_functions.py:101-132)
      forward   evaluate_loss: render + residual + loss_scalar (solver_functions.py:31-53)
    Median of `reps` host-timed calls, each synchronised (the reference's script does not synchronise)."""
    import types
    import torch.autograd.forward_ad as fwAD
    from gslm.train import PipelineParams, render
    pipe = PipelineParams()
    gt = cam.original_image
    m = cam.alpha_mask
    g3 = torch.Generator().manual_seed(3)
    u = types.SimpleNamespace(**{f"{k}_grad": torch.randn(t.shape, generator=g3).to(t.device) for k, t in
                                 zip(("xyz", "features_dc", "features_rest", "scaling", "rotation", "opacity", "exposure"),
                                     model.params())})
    v = torch.randn(gt.shape, generator=torch.Generator().manual_seed(4)).to(gt.device)

    def residual():
        img = render(cam, model, pipe, bg.to(gt.device))["render"]
        return img * m - gt if m is not None else img - gt

    def matvec():
        with torch.no_grad(), fwAD.dual_level(), model.make_dual(u):
            return fwAD.unpack_dual(residual()).tangent

    def matvec_T():
        model.zero_grad()
        r = residual()
        r.backward(v, retain_graph=True)  # the L1 slot
        r.backward(v)                     # the aliased "ssim" slot
        return model._opacity.grad

    def forward():
        with torch.no_grad():
            r = residual()
            return 2.0 * (r.double() ** 2).sum()

    out = {"config": f"{model._xyz.shape[0]} Gaussians SH{model.active_sh_degree}, 1x{cam.image_width}x"
                     f"{cam.image_height} view, drop-in rasterizer through render() (tests/test_jvp_timing.py:71-106)"}
    for name, fn in (("matvec", matvec), ("matvec_T", matvec_T), ("forward", forward)):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        out[name + "_ms"] = 1e3 * sorted(ts)[len(ts) // 2]
    model.zero_grad()
    return out


def time_drop_in_fwd_bwd(device, W, H, s0, P=100_000, sh=3, reps=10):
    """Forward + backward of one view through diff_gaussian_rasterization (activated leaves with
    requires_grad, dL/dcolor ~ N(0, 1) seed 4: SURVEY §8(d) config 2)."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
    from gslm.cameras import orbit_cameras
    from gslm.model import synthetic_gaussians
    m = synthetic_gaussians(P, sh, seed=0, s0=s0, device="cpu").to(device)
    cam = orbit_cameras(1, W, H, seed=1)[0].to(device)
    st = GaussianRasterizationSettings(
        image_height=H, image_width=W, tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5),
        bg=torch.zeros(3, device=device), scale_modifier=1.0, viewmatrix=cam.world_view_transform,
        projmatrix=cam.full_proj_transform, sh_degree=sh, campos=cam.camera_center, prefiltered=False,
        debug=False, antialiasing=False)
    leaves = [t.detach().clone().requires_grad_(True) for t in
              (m.get_xyz, m.get_opacity, m.get_scaling, m.get_rotation, m.get_features)]
    means2D = torch.zeros(P, 3, device=device, requires_grad=True)
    g4 = torch.Generator(device="cpu").manual_seed(4)
    dcolor = torch.randn(3, H, W, generator=g4).to(device)
    rast = GaussianRasterizer(raster_settings=st)

    def step():
        color, _, _ = rast(means3D=leaves[0], means2D=means2D, opacities=leaves[1], scales=leaves[2],
                           rotations=leaves[3], shs=leaves[4])
        color.backward(dcolor)

    step()
    torch.cuda.synchronize()
    # median of per-step times: each step already synchronises once (the num_rendered read-back the
    # upstream forward also does), and the host-side autograd work makes single steps noisy
    ts = []
    for _ in range(max(reps, 20)):
        t0 = time.perf_counter()
        step()
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    return {"config": f"{P} Gaussians SH{sh}, 1x{W}x{H} view, forward + backward via GaussianRasterizer "
                      "(BASELINE configs[1])", "ms": 1e3 * t, "mpix_s": W * H / t / 1e6}


if __name__ == "__main__":
    main()
