# variant: the tangent kernel (k_preprocess_jvp) held to 5 waves per SIMD (__launch_bounds__(256, 5): <= 96 VGPRs
# against the 121 the compiler picks at 4 waves)
s = open("tangent.hip").read()
a = "__global__ __launch_bounds__(256) void k_preprocess_jvp(ViewK v, GaussK g, GaussK t, const float* __restrict__ m2t,"
assert a in s
s = s.replace(a, "__global__ __launch_bounds__(256, 5) void k_preprocess_jvp(ViewK v, GaussK g, GaussK t, const float* __restrict__ m2t,")
open("tangent.hip", "w").write(s)
