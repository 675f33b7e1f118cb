# timing-only variant (round 6): nontemporal stores for the gather's y only (v_nt.py's second part)
s = open("gslm_gather.hpp").read()
for a, b in (("    y[base + k] = out;\n", "    __builtin_nontemporal_store(out, &y[base + k]);\n"),
             ("        o.y[2][base + e] = out;\n", "        __builtin_nontemporal_store(out, &o.y[2][base + e]);\n")):
    assert a in s
    s = s.replace(a, b)
open("gslm_gather.hpp", "w").write(s)
