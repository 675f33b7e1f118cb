# variant: vjp_tile without the barrier at the top of each batch (redundant: the post-hit-loop barrier and the
# post-publish barrier already order every LDS access of consecutive batches)
p = "gslm_tile.hpp"
s = open(p).read()
old = """    const int cnt = min(BATCH, base + 1);
    __syncthreads();
    uint32_t my_slot = 0;"""
assert old in s
s = s.replace(old, """    const int cnt = min(BATCH, base + 1);
    uint32_t my_slot = 0;""")
open(p, "w").write(s)
