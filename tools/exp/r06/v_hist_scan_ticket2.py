# variant: v_hist_scan_ticket.py without the device-scope fences -- the counts go out as agent-scope (write-through)
# atomic stores drained by a wait on the vector memory counter before the ticket, and the scanning blocks read them
# with agent-scope atomic loads, so no block writes back its L2.
import runpy, os
runpy.run_path(os.path.join(os.path.dirname(os.path.abspath(__file__)), "v_hist_scan_ticket.py"))
s = open("sort.hip").read()
a = """  hist[(int64_t)tid * nblocks + blockIdx.x] = cnt[tid];
  __syncthreads();
  if (tid == 0) {
    __threadfence();
    s_ticket = (int)atomicAdd(ctr, 1u);
  }"""
assert a in s
s = s.replace(a, """  __hip_atomic_store(hist + (int64_t)tid * nblocks + blockIdx.x, cnt[tid], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __builtin_amdgcn_s_waitcnt(0);
  __syncthreads();
  if (tid == 0) s_ticket = (int)__hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);""")
a = """      if (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)nblocks) break;"""
assert a in s
s = s.replace(a, """      if (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (uint32_t)nblocks) break;""")
a = """  __syncthreads();
  __threadfence();
  uint32_t* h = hist + (int64_t)d * nblocks;"""
assert a in s
s = s.replace(a, """  __syncthreads();
  uint32_t* h = hist + (int64_t)d * nblocks;""")
open("sort.hip", "w").write(s)
