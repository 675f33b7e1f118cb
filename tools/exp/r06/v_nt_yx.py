# timing-only variant (round 6): nontemporal stores for the gather's y and the deferred x update in the tangent kernel
# (x is read again only by the next iteration's tangent kernel); GSLM_NT_S=1 also the update's s
import os
exec(open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "v_nt_y.py")).read())
s = open("tangent.hip").read()
for a, b in (("        if (with_x) xp.p[k][xp.xoff + gi] = xv[n] + a * pv[n];\n",
              "        if (with_x) __builtin_nontemporal_store(xv[n] + a * pv[n], &xp.p[k][xp.xoff + gi]);\n"),
             ("          if (with_x) p[xp.xoff + e] = xu[u] + a * pu[u];\n",
              "          if (with_x) __builtin_nontemporal_store(xu[u] + a * pu[u], &p[xp.xoff + e]);\n")):
    assert a in s
    s = s.replace(a, b)
open("tangent.hip", "w").write(s)
if os.environ.get("GSLM_NT_S") == "1":
    s = open("cg.hip").read()
    a = "    s4[i] = sv;\n"
    assert a in s
    s = s.replace(a, "    __builtin_nontemporal_store(sv.x, &s[4 * i]); __builtin_nontemporal_store(sv.y, &s[4 * i + 1]);\n"
                     "    __builtin_nontemporal_store(sv.z, &s[4 * i + 2]); __builtin_nontemporal_store(sv.w, &s[4 * i + 3]);\n")
    open("cg.hip", "w").write(s)
