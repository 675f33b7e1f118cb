# variant: the tangent kernel's geometry formed after the fused direction update (the round-5 order)
p = "tangent.hip"
s = open(p).read()
old = """    if (act) compute_geo<RAW>(v, g, i, clampw[i], e);
"""
assert old in s
s = s.replace(old, "")
old = """    __syncthreads();
    if (t.rest) {
      t.rest = s_rest;
      t.rest_base = (int64_t)blockIdx.x * blockDim.x;
    }
  }
  if (!act) return;"""
new = """    __syncthreads();
    if (t.rest) {
      t.rest = s_rest;
      t.rest_base = (int64_t)blockIdx.x * blockDim.x;
    }
    if (act) compute_geo<RAW>(v, g, i, clampw[i], e);
  }
  if (!act) return;"""
assert old in s
s = s.replace(old, new)
open(p, "w").write(s)
