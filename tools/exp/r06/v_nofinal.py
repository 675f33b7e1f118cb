# timing-only variant (round 6): the CG loop's two dot finalisations (gamma' after the update, <p, Ap> after the
# gather) not launched -- prices what fusing them into their producers' last block could save.  Wrong scalars.
s = open("cg.hip").read()
a = """  hipLaunchKernelGGL(k_dot_final, dim3(1), dim3(DOT_THREADS), 0, st, (const double*)scratch, DOT_BLOCKS, gam_new_dev);
  GSLM_LAUNCH_CHECK();
  return GSLM_OK;
}"""
assert a in s
s = s.replace(a, "  GSLM_LAUNCH_CHECK();\n  return GSLM_OK;\n}")
open("cg.hip", "w").write(s)
s = open("api.hip").read()
a = "  if (dot_out) return gslm_dot_finalize(part, (int32_t)((b.g.P + 255) / 256), dot_out, stream);\n  return GSLM_OK;\n}"
assert a in s
s = s.replace(a, "  return GSLM_OK;\n}")
open("api.hip", "w").write(s)
