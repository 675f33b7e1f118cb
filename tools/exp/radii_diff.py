"""Experiment: where do GPU and oracle radii differ at 1M / 1080p?"""
import os, sys, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gaussian-splatting-lm_amd"), os.path.join(ROOT, "tests")]
import test_gpu_fullsize as T
from test_gpu_raster import _gpu_forward_internals
from oracle import torch_raster as tr
from scenes import activated, oracle_settings
model, cam = T._scene(1_000_000)
a = activated(model)
st = oracle_settings(cam, 3)
with torch.no_grad():
    pre = tr.preprocess(a["means3D"], torch.zeros_like(a["means3D"]), a["opacities"], a["shs"], None,
                        a["scales"], a["rotations"], None, st)
G = _gpu_forward_internals(model, cam, 3)
d = (G["radii"] != pre["radii"]).nonzero().reshape(-1)
print("mismatches", d.numel(), d[:10].tolist())
print("gpu", G["radii"][d[:10]].tolist(), "oracle", pre["radii"][d[:10]].tolist())
print("tiles gpu", G["tiles"][d[:10]].tolist(), "oracle", pre["tiles_touched"][d[:10]].tolist())
# float64 restatement of the same Gaussians
a64 = {k: v[d[:10]].double() for k, v in a.items()}
class S: pass
st64 = tr.settings_from_camera(cam, torch.zeros(3, dtype=torch.float64), 3)
st64.viewmatrix = st64.viewmatrix.double(); st64.projmatrix = st64.projmatrix.double(); st64.campos = st64.campos.double()
with torch.no_grad():
    p64 = tr.preprocess(a64["means3D"], torch.zeros_like(a64["means3D"]), a64["opacities"], a64["shs"], None,
                        a64["scales"], a64["rotations"], None, st64)
print("f64 radii", p64["radii"].tolist())
c = p64["conic"]
print("f64 conic", c[:3].tolist())
import ctypes
from diff_gaussian_rasterization import _gaussians, forward_buffers
from gslm import _lib
from scenes import gpu_settings
ag = {k: v.to("cuda") for k, v in a.items()}
view = _lib.view_from_settings(gpu_settings(cam, 3))
P = ag["means3D"].shape[0]
g = _gaussians(P, ag["means3D"], ag["opacities"].reshape(-1).contiguous(), ag["scales"], ag["rotations"], None, ag["shs"], None, None)
color, radii, invd, geom, binning, image, N = forward_buffers(view, g, "cuda")
rec = torch.zeros(P * 12, dtype=torch.float32, device="cuda")
_lib.check(_lib.lib.gslm_inspect(geom.data_ptr(), P, binning.data_ptr(), N, 1080, 1920, image.data_ptr(), None, None, None, None, None, rec.data_ptr(), _lib.stream_handle()))
torch.cuda.synchronize()
r = rec.view(P, 12).cpu()
vis = pre["radii"] > 0
for name, gcol, oc in (("x", r[:, 0], pre["xy"][:, 0]), ("y", r[:, 1], pre["xy"][:, 1]), ("ca", r[:, 2], pre["conic"][:, 0]),
                       ("cb", r[:, 3], pre["conic"][:, 1]), ("cc", r[:, 4], pre["conic"][:, 2]), ("op", r[:, 5], pre["opacity"]),
                       ("r", r[:, 6], pre["rgb"][:, 0]), ("invz", r[:, 9], 1.0 / pre["depth"])):
    mm = (gcol[vis] != oc[vis]).sum().item()
    print(name, "bit mismatches among visible:", mm)
for i in d[:2].tolist():
    print(i, "gpu conic", r[i, 2:5].tolist(), "oracle", pre["conic"][i].tolist())
print("cpu capability", torch.backends.cpu.get_cpu_capability())
R = tr.quat_to_rotmat(a["rotations"]); s = a["scales"]; L = R * s[:, None, :]
S = L @ L.transpose(1, 2)
E = tr.compute_cov3d(a["scales"], 1.0, a["rotations"])
B = torch.stack([S[:,0,0],S[:,0,1],S[:,0,2],S[:,1,1],S[:,1,2],S[:,2,2]],1)
print("cov3d bmm vs elementwise mismatch frac", (E != B).any(1).float().mean().item())
import numpy as np
i = int(d[0])
c00, c01, c11 = [np.float32(v) for v in pre["cov2d"][i].tolist()]
det = np.float32(c00 * c11 - c01 * c01)
mid = np.float32(np.float32(0.5) * np.float32(c00 + c11))
q = np.float32(max(np.float32(mid * mid - det), np.float32(0.1)))
lam1 = np.float32(mid + np.sqrt(q))
r3 = np.float32(np.float32(3.0) * np.sqrt(lam1))
print("c", c00, c01, c11, "det", det, "mid", mid, "q", q, "lam1", repr(lam1), "3sqrt", repr(r3), "ceil", np.ceil(r3))
print("f64 3sqrt(lam1)", 3 * math.sqrt(float(lam1)) if False else 3 * np.sqrt(np.float64(lam1)))
vals = torch.rand(1 << 22) * 400 + 1
g = torch.sqrt(vals.cuda()).cpu(); cpu = torch.sqrt(vals)
print("torch cuda sqrt vs cpu mismatch", (g != cpu).sum().item())
