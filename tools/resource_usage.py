"""Kernel resource usage of the library sources as the Makefile builds them (hipcc -O3 with its flags, gfx950,
-Rpass-analysis=kernel-resource-usage): VGPRs, the compiler's waves-per-SIMD bound and static LDS per kernel, demangled.
    python tools/resource_usage.py > profiles/<round>/resource_usage.txt"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "gaussian-splatting-lm_amd", "csrc")
FLAGS = ["-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off", "-munsafe-fp-atomics",
         "-I../../include", "-I.", "-Rpass-analysis=kernel-resource-usage", "--cuda-device-only", "-c", "-o", os.devnull]
TILE = {"jvp.hip", "backward.hip", "render_fwd.hip"}  # -fno-slp-vectorize, as the Makefile


def demangle(names):
    out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True,
                         text=True).stdout.splitlines()
    return out if len(out) == len(names) else names


def main():
    rows = []
    for f in sorted(x for x in os.listdir(CSRC) if x.endswith(".hip")):
        extra = ["-fno-slp-vectorize"] if f in TILE else []
        r = subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, f], cwd=CSRC, capture_output=True, text=True)
        cur = None
        for line in r.stderr.splitlines():
            m = re.search(r"remark: Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1), "file": f}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+(VGPRs|Occupancy \[waves/SIMD\]|LDS Size \[bytes/block\]): (\d+)", line)
            if m and cur is not None:
                cur[m.group(1).split()[0]] = int(m.group(2))
    names = demangle([r["name"] for r in rows])
    print("Kernel resource usage on gfx950 (tools/resource_usage.py: hipcc -O3 with the Makefile's flags,\n"
          "-Rpass-analysis=kernel-resource-usage; static LDS only -- dynamic LDS is added at launch; occupancy = the\n"
          "compiler's waves-per-SIMD bound from VGPRs and LDS).\n")
    for r, n in sorted(zip(rows, names), key=lambda t: (t[0]["file"], t[1])):
        if not r["name"].startswith("_Z"):
            continue
        n = n.split("(")[0][:70]
        print(f"{r['file']:16s} {n:72s} VGPRs: {r.get('VGPRs', '?'):<4} Occupancy [waves/SIMD]: {r.get('Occupancy', '?'):<2}"
              f" LDS [bytes/block]: {r.get('LDS', '?')}")


if __name__ == "__main__":
    sys.exit(main())
