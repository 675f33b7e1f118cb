# variant: the J v visit waits for its tangent half only after the primal alpha (the empty asm pin moved below it)
p = "jvp.hip"
s = open(p).read()
old = """      const float4 a = s[j], b = s[64 + j], C = s[128 + j], D = s[192 + j];
      asm volatile("" : : "v"(b.z), "v"(b.w), "v"(C.x), "v"(C.y), "v"(C.z), "v"(C.w), "v"(D.x), "v"(D.y), "v"(D.z),
                   "v"(D.w));
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gpower(a.z, a.w, b.x, dx, dy);
      const float G = gexp(power);
      const float alpha = fminf(0.99f, b.y * G);"""
assert old in s
s = s.replace(old, """      const float4 a = s[j], b = s[64 + j], C = s[128 + j], D = s[192 + j];
      const float dx = a.x - pxf, dy = a.y - pyf;
      const float power = gpower(a.z, a.w, b.x, dx, dy);
      const float G = gexp(power);
      const float alpha = fminf(0.99f, b.y * G);
      asm volatile("" : : "v"(b.z), "v"(b.w), "v"(C.x), "v"(C.y), "v"(C.z), "v"(C.w), "v"(D.x), "v"(D.y), "v"(D.z),
                   "v"(D.w));""")
open(p, "w").write(s)
