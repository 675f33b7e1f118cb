# TIMING ONLY (wrong products): v_nostart + no barrier between the hit loop and the combine -- what the VJP's
# combine barrier costs at most
import os
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "v_nostart.py")).read())
p = "gslm_tile.hpp"
s = open(p).read()
old = """    }
    __syncthreads();
    // rows only for the entries some wave visited"""
assert old in s
s = s.replace(old, """    }
    // rows only for the entries some wave visited""")
open(p, "w").write(s)
