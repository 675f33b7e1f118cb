# timing variant (round 6): k_render_matvec's VJP pass in 256-entry batches (half the block barriers; 39 KB of LDS
# per block -> 4 blocks per CU), the one batch size round 4 did not run (profiles/r04/ab/vjp_batch64_rejected/)
s = open("jvp.hip").read()
a = "constexpr int MATVEC_BATCH = 128;"
assert a in s
s = s.replace(a, "constexpr int MATVEC_BATCH = 256;")
open("jvp.hip", "w").write(s)
