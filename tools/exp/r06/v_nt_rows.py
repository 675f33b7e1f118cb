# timing-only variant (round 6): nontemporal stores for the LM gradient rows only (v_nt.py's third part)
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
