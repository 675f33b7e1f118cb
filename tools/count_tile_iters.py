"""Experiment helper: counts tile-pass wave iterations and valid lanes of one fused matvec at the bench
config.  Needs the counter build: make -C gaussian-splatting-lm_amd/csrc OUTDIR=../build_cnt EXTRA=-DGSLM_EXPERIMENT_COUNT"""
import ctypes, os, sys, torch
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "gaussian-splatting-lm_amd")]
os.environ["GSLM_LIB"] = os.path.join(os.getcwd(), "gaussian-splatting-lm_amd",
                                      sys.argv[1] if len(sys.argv) > 1 else "build_cnt", "libgslm.so")
from gslm import _lib
from gslm.cameras import orbit_cameras
from gslm.model import synthetic_gaussians
from gslm.lm import LMProblem
W, H = 1920, 1080
cams = orbit_cameras(1, W, H, seed=1)
pert = synthetic_gaussians(1_000_000, 3, seed=0, s0=0.005, device="cpu", n_cams=1).to("cuda")
gp = LMProblem(pert, [c.to("cuda") for c in cams], torch.zeros(3))
gp.evaluate()
cams[0].original_image = gp.views[0].color.clamp(0, 1).clone() * 0.9
prob = LMProblem(pert, cams, torch.zeros(3))
prob.evaluate()
g = prob.rhs(prob.zeros())
v = torch.randn(g.numel(), device="cuda")
lo, hi = prob.layout.offsets["xyz"]; v[lo:hi] = 0
lo, hi = prob.layout.offsets["exposure"]; v[lo:hi] = 0
lib = _lib.lib
buf = (ctypes.c_ulonglong * 8)()
lib.gslm_dbg_read(buf, 1)
y = prob.zeros()
prob.matvec(v, y); torch.cuda.synchronize()
lib.gslm_dbg_read(buf, 1)
c = list(buf)
print("N_dup", prob.views[0].N, "pixels", W * H)
print("JVP wave-iters", c[0], "valid lanes", c[1], "frac", c[1] / max(c[0], 1) / 64)
print("VJP wave-iters", c[2], "valid lanes", c[3], "frac", c[3] / max(c[2], 1) / 64, "none-valid iters", c[4])
# per-tile timeline of the same matvec (wall clock, 100 MHz)
import numpy as np
ntiles = ((W + 15) // 16) * ((H + 15) // 16)
tb = (ctypes.c_ulonglong * (3 * ntiles))()
prob.matvec(v, y); torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(); prob.matvec(v, y); e1.record(); torch.cuda.synchronize()
print("matvec ms (events)", e0.elapsed_time(e1))
lib.gslm_dbg_tiles(tb, ntiles)
t = np.array(list(tb), dtype=np.float64).reshape(ntiles, 3)
t0 = t[:, 0].min()
print("raw tick span", t[:, 2].max() - t0)
t = (t - t0) / 100.0  # us at the documented 100 MHz wall clock
jv = t[:, 1] - t[:, 0]; vj = t[:, 2] - t[:, 1]; tot = t[:, 2] - t[:, 0]
print("kernel span us", t[:, 2].max(), "sum tile us", tot.sum(), "mean", tot.mean(), "max", tot.max())
print("jvp sum", jv.sum(), "vjp sum", vj.sum())
order = np.argsort(-tot)
print("top 10 tiles (us):", np.round(tot[order[:10]], 1), "at start", np.round(t[order[:10], 0], 1))
ends = np.sort(t[:, 2])
print("time when 50/90/99/100% tiles done:", [round(ends[int(q * (ntiles - 1))], 1) for q in (0.5, 0.9, 0.99, 1.0)])
rg = torch.zeros(ntiles * 2, dtype=torch.int32, device="cuda")
vr = prob.views[0]
_lib.check(lib.gslm_inspect(vr.geom.data_ptr(), 1_000_000, vr.binning.data_ptr(), vr.N, H, W, None, None,
                            rg.data_ptr(), None, None, None, None, _lib.stream_handle()))
torch.cuda.synchronize()
r = rg.view(-1, 2).cpu().numpy().astype(np.int64)
n = r[:, 1] - r[:, 0]
print("list length: mean", n.mean(), "max", n.max(), "empty tiles", (n == 0).sum(), "corr(n, time)", np.corrcoef(n, tot)[0, 1])
np.save("gpurun_out/tile_times.npy", np.concatenate([t, n[:, None]], axis=1))
