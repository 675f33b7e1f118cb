"""Experiment: is torch's CPU float32 sqrt correctly rounded on this host?"""
import numpy as np, torch
vals = torch.rand(1 << 22) * 400 + 1
t = torch.sqrt(vals).numpy(); n = np.sqrt(vals.numpy())
print("cpu", torch.backends.cpu.get_cpu_capability(), "torch.sqrt vs np.sqrt mismatches", int((t != n).sum()))
t1 = torch.sqrt(vals[:7]).numpy(); print("short tensor mismatches", int((t1 != n[:7]).sum()))
d = torch.rand(1 << 22) + 0.5
print("div mismatches", int(((vals / d).numpy() != (vals.numpy() / d.numpy())).sum()))
print("exp mismatches vs np", int((torch.exp(-d).numpy() != np.exp(-d.numpy())).sum()))
