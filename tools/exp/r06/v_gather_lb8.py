# timing variant (round 6): k_gather_lm's projected-layout instantiation at __launch_bounds__(256, 8) (the tree: 5,
# which the compiler meets with 76 VGPRs, 6 waves per SIMD)
s = open("gather.hip").read()
a = "__launch_bounds__(256, PROJ ? 5 : 1) void k_gather_lm("
assert a in s
s = s.replace(a, "__launch_bounds__(256, PROJ ? 8 : 1) void k_gather_lm(")
open("gather.hip", "w").write(s)
