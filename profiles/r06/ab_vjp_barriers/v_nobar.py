# TIMING ONLY (wrong products, records and hit words race): v_nosync + no barrier after the batch's publish either --
# the VJP batch loop with no block barrier at all: the most any barrier-free VJP design could save before its own
# costs (per-wave gathers, arrival counters)
import os
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "v_nosync.py")).read())
p = "gslm_tile.hpp"
s = open(p).read()
old = """    publish_quad_masks(my_mask, s_bits);
    __syncthreads();
    // the batch's hit words in order"""
assert old in s
s = s.replace(old, """    publish_quad_masks(my_mask, s_bits);
    __builtin_amdgcn_wave_barrier();
    // the batch's hit words in order""")
open(p, "w").write(s)
