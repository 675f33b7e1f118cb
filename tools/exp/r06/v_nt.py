# timing-only variant (round 6): nontemporal stores for the CG loop's streamed outputs -- the update's s, the
# gather's y, the LM gradient rows -- to test whether less dirty L2 at the kernel boundaries shortens the gaps
# between the iteration's kernels (each boundary writes back the XCDs' L2s).
s = open("cg.hip").read()
a = "    s4[i] = sv;\n"
assert a in s
s = s.replace(a, "    __builtin_nontemporal_store(sv.x, &s[4 * i]); __builtin_nontemporal_store(sv.y, &s[4 * i + 1]);\n"
                 "    __builtin_nontemporal_store(sv.z, &s[4 * i + 2]); __builtin_nontemporal_store(sv.w, &s[4 * i + 3]);\n")
open("cg.hip", "w").write(s)
s = open("gslm_gather.hpp").read()
for a, b in (("    y[base + k] = out;\n", "    __builtin_nontemporal_store(out, &y[base + k]);\n"),
             ("        o.y[2][base + e] = out;\n", "        __builtin_nontemporal_store(out, &o.y[2][base + e]);\n")):
    assert a in s
    s = s.replace(a, b)
open("gslm_gather.hpp", "w").write(s)
s = open("gslm_tile.hpp").read()
a = """    rows[2 * (size_t)slot + 0] = make_float4(t[2], t[3], t[4], t[5]);
    rows[2 * (size_t)slot + 1] = make_float4(t[6], t[7], t[8], 0.f);"""
assert a in s
s = s.replace(a, """    float* rf = reinterpret_cast<float*>(rows + 2 * (size_t)slot);
    __builtin_nontemporal_store(t[2], rf + 0); __builtin_nontemporal_store(t[3], rf + 1);
    __builtin_nontemporal_store(t[4], rf + 2); __builtin_nontemporal_store(t[5], rf + 3);
    __builtin_nontemporal_store(t[6], rf + 4); __builtin_nontemporal_store(t[7], rf + 5);
    __builtin_nontemporal_store(t[8], rf + 6); __builtin_nontemporal_store(0.f, rf + 7);""")
open("gslm_tile.hpp", "w").write(s)
