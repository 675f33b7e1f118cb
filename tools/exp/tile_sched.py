"""Experiment: where k_render_matvec's wave-visits go, and how much of the launch its tile schedule can leave idle.

At the bench config (1M Gaussians SH3, one 1080p view: the scene of tools/mv_ab.py) the forward runs on the GPU and
gslm_inspect copies out the point list, the tile ranges, n_contrib and the render records.  Then, in torch on the
GPU (float32, the tile passes' exponent and alpha test; not bit-exact with the kernels, statistics only), per list
entry and 8x8 quadrant (one wave of a tile block):

  reach[e, q]   some pixel of the quadrant passes the alpha test (what the quadrant mask approximates from above)
  visit[e, q]   reach and the entry lies before the quadrant's largest n_contrib (the wave's bound wm_q): the
                J v pass and the VJP pass each run one wave-iteration for it
  valid[e, q]   lanes of such a visit that blend (also below their own n_contrib)

and reports the valid-lane fraction, the quadrant-count distribution of visited entries, the VJP's barrier cost
(per 128-entry batch the busiest wave sets the pace: sum over batches of the max against the free-running max and
the mean) and a list schedule of the tiles in k_tile_order's longest-first order onto the chip's resident blocks
(256 CUs x 8 blocks), each block's time modelled from its visits, against perfect packing.
    python tools/exp/tile_sched.py [--P 1000000] [--out gpurun_out/tile_sched.json]"""
import argparse
import ctypes
import heapq
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--P", type=int, default=1_000_000)
    ap.add_argument("--W", type=int, default=1920)
    ap.add_argument("--H", type=int, default=1080)
    ap.add_argument("--slots", type=int, default=2048)
    ap.add_argument("--out", default="gpurun_out/tile_sched.json")
    a = ap.parse_args()
    from gslm import _lib
    from gslm.cameras import orbit_cameras
    from gslm.lm import LMProblem
    from gslm.model import synthetic_gaussians
    dev = torch.device("cuda", 0)
    W, H = a.W, a.H
    cams = orbit_cameras(1, W, H, seed=1)
    model = synthetic_gaussians(a.P, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to(dev)
    prob = LMProblem(model, cams, torch.zeros(3), device=dev)
    prob.evaluate()
    torch.cuda.synchronize()
    vr = prob.views[0]
    N, P = vr.N, a.P
    gx, gy = (W + 15) // 16, (H + 15) // 16
    ntiles = gx * gy
    pl = torch.empty(N, dtype=torch.int32, device=dev)
    rg = torch.empty(ntiles * 2, dtype=torch.int32, device=dev)
    nc = torch.empty(H * W, dtype=torch.int32, device=dev)
    rec = torch.empty(P * 12, dtype=torch.float32, device=dev)
    _lib.check(_lib.lib.gslm_inspect(vr.geom.data_ptr(), P, vr.binning.data_ptr(), N, H, W, vr.image.data_ptr(),
                                     pl.data_ptr(), rg.data_ptr(), None, None, nc.data_ptr(), rec.data_ptr(),
                                     _lib.stream_handle()))
    torch.cuda.synchronize()
    rg = rg.view(ntiles, 2).long()
    lens = rg[:, 1] - rg[:, 0]
    rec = rec.view(P, 12)
    nc = nc.view(H, W).long()
    # per tile and quadrant: the wave bound wm_q = min(max n_contrib over the quadrant's pixels, list length)
    ncp = torch.zeros(gy * 16, gx * 16, dtype=torch.long, device=dev)
    ncp[:H, :W] = nc
    q4 = ncp.view(gy, 2, 8, gx, 2, 8).amax(dim=(2, 5))          # [gy, qy, gx, qx]
    wm = q4.permute(0, 2, 1, 3).reshape(ntiles, 4)              # quadrant index q = 2 qy + qx
    wm = torch.minimum(wm, lens[:, None])
    # entries: tile and list position
    tile_of = torch.repeat_interleave(torch.arange(ntiles, device=dev), lens)
    pos = torch.arange(N, device=dev) - rg[tile_of, 0]
    gid = pl.long()
    lane = torch.arange(64, device=dev)
    lx, ly = (lane & 7).float(), (lane >> 3).float()
    reach = torch.zeros(N, 4, dtype=torch.bool, device=dev)
    vcnt = torch.zeros(N, 4, dtype=torch.int16, device=dev)
    CH = 1 << 18
    for s in range(0, N, CH):
        e = slice(s, min(N, s + CH))
        t = tile_of[e]
        r = rec[gid[e]]
        x, y, ca, cb, cc, op = (r[:, i:i + 1] for i in range(6))
        for q in range(4):
            px = (t % gx * 16 + 8 * (q & 1)).float()[:, None] + lx[None]
            py = (t // gx * 16 + 8 * (q >> 1)).float()[:, None] + ly[None]
            dx, dy = x - px, y - py
            power = -0.5 * (ca * dx * dx + cc * dy * dy) - cb * dx * dy
            alpha = torch.clamp(op * torch.exp(power), max=0.99)
            inside = (px < W) & (py < H)
            ok = (power <= 0) & (alpha >= 1.0 / 255.0) & inside
            reach[e, q] = ok.any(1)
            pxi, pyi = px.long().clamp(max=W - 1), py.long().clamp(max=H - 1)
            below = pos[e][:, None] < nc[pyi, pxi]
            vcnt[e, q] = (ok & below).sum(1).to(torch.int16)
    visit = reach & (pos[:, None] < wm[tile_of])
    V = int(visit.sum())
    anyv = visit & (vcnt > 0)
    out = {"P": P, "N": N, "tiles": ntiles, "wave_visits": V,
           "visits_with_a_blending_lane": int(anyv.sum()),
           "valid_lane_frac": float(vcnt[visit].float().sum() / (64.0 * max(V, 1))),
           "entries_visited": int(visit.any(1).sum()),
           "quadrants_per_visited_entry": {str(k): int(((visit.sum(1) == k)).sum()) for k in range(1, 5)},
           "reach_without_bound": int(reach.sum())}
    # per tile: J v pass (free-running waves) and VJP pass (128-entry batches from n_eff down, barrier per batch)
    vis_t = torch.zeros(ntiles, 4, dtype=torch.long, device=dev).index_add_(0, tile_of, visit.long())
    n_eff = wm.amax(1)
    bidx = torch.where(pos < n_eff[tile_of], (n_eff[tile_of] - 1 - pos) // 128, torch.full_like(pos, -1))
    nb_max = int(bidx.max()) + 1
    key = tile_of * nb_max + bidx.clamp(min=0)
    per_b = torch.zeros(ntiles * nb_max, 4, dtype=torch.long, device=dev)
    sel = bidx >= 0
    per_b.index_add_(0, key[sel], visit[sel].long())
    per_b = per_b.view(ntiles, nb_max, 4)
    vjp_sync = per_b.amax(2).sum(1)
    nbat = (n_eff + 127) // 128
    jvp_free = vis_t.amax(1)
    mean_q = vis_t.float().mean(1)
    out["vjp_barrier_cost"] = {"sum_batches_busiest_wave": int(vjp_sync.sum()), "busiest_wave_total": int(jvp_free.sum()),
                               "mean_wave_total": float(mean_q.sum()), "batches": int(nbat.sum())}
    # list schedule: block time = JVP (busiest wave) + VJP (sum of batch maxima) + per-batch overhead (units of visits)
    for ovh in (0, 8):
        cost = (jvp_free + vjp_sync + ovh * nbat).double().cpu().numpy()
        order = np.argsort(-lens.cpu().numpy(), kind="stable")
        slots = [0.0] * a.slots
        heapq.heapify(slots)
        for t in order:
            t0 = heapq.heappop(slots)
            heapq.heappush(slots, t0 + cost[t])
        makespan = max(slots)
        ideal = cost.sum() / a.slots
        out[f"schedule_ovh{ovh}"] = {"makespan": makespan, "ideal": ideal, "idle_frac": 1 - ideal / makespan,
                                     "max_block": float(cost.max()), "mean_block": float(cost.mean())}
    hist = np.percentile(lens.cpu().numpy(), [50, 90, 99, 100]).tolist()
    out["list_len_p50_p90_p99_max"] = hist
    out["n_eff_p50_p90_p99_max"] = np.percentile(n_eff.cpu().numpy(), [50, 90, 99, 100]).tolist()
    # per-tile arrays for offline schedule experiments (orders, cost models)
    vjp_vis_t = per_b.sum(1)
    np.savez(os.path.splitext(a.out)[0] + ".npz", lens=lens.cpu().numpy(), wm=wm.cpu().numpy(), vis=vis_t.cpu().numpy(),
             vjp_sync=vjp_sync.cpu().numpy(), nbat=nbat.cpu().numpy(), vjp_vis=vjp_vis_t.cpu().numpy(),
             valid=torch.zeros(ntiles, 4, dtype=torch.long, device=dev).index_add_(
                 0, tile_of, torch.where(visit, vcnt.long(), torch.zeros_like(vcnt, dtype=torch.long))).cpu().numpy())
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
