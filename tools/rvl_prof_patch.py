"""Build-variant generator (profiling only, never the product): a copy of
csrc/tbf_render.hip in which every wave of k_rv_core_lds accumulates s_memtime cycles per
segment of rvl_pair on lane 0 and adds them, per wave index, to a device array read back
by tbf_debug_rvl_prof (tools/rvl_prof.py):
  0 pair start -> first barrier (ring load, or state load + first plan)
  1 the barrier before the group loop (first inputs)
  2 read phase (workers) / planning (planner)      per group
  3 first barrier wait                             per group
  4 write phase                                    per group
  5 second barrier wait                            per group
  6 after the loop -> end (ring and state stores)
  7 groups (count)

usage: python tools/rvl_prof_patch.py OUT.hip"""
import sys
from pathlib import Path

SRC = Path(__file__).resolve().parents[1] / "tunebfree_amd" / "csrc" / "tbf_render.hip"


def sub(s, old, new, count=1):
    assert s.count(old) == count, (old, s.count(old))
    return s.replace(old, new)


def main():
    s = SRC.read_text()
    head = ("__device__ unsigned long long g_rvlprof[16][8];\n"
            "#define RVP_T() ({ asm volatile (\"\" ::: \"memory\"); __builtin_amdgcn_s_memtime (); })\n")
    s = sub(s, "/* one (instance, channel) of a k_rv_core_lds launch */", head + "/* one (instance, channel) of a k_rv_core_lds launch */")
    a = s.index("__device__ __forceinline__ void rvl_pair (")
    b = s.index("\n}\n", a)
    body = s[a:b]
    body = sub(body, "\tconst int      tid  = threadIdx.x;\n",
               "\tconst int      tid  = threadIdx.x;\n\tunsigned long long pt[8] = {0, 0, 0, 0, 0, 0, 0, 0};\n"
               "\tunsigned long long t0 = RVP_T (), t1;\n")
    # the first two barriers (before the loops)
    body = sub(body, "\t__syncthreads ();\n\tint cntv", "\t__syncthreads ();\n\tt1 = RVP_T (); pt[0] += t1 - t0; t0 = t1;\n\tint cntv")
    body = sub(body, "\t__syncthreads ();\n\t/* the workers and the planner run separate loops",
               "\t__syncthreads ();\n\tt1 = RVP_T (); pt[1] += t1 - t0; t0 = t1;\n\t/* the workers and the planner run separate loops")
    # the worker loop
    body = sub(body, "#pragma unroll 1\n\t\tfor (uint32_t g = 0; g < nGrp; g++) {\n\t\t\tconst int  nb  =",
               "#pragma unroll 1\n\t\tfor (uint32_t g = 0; g < nGrp; g++) {\n\t\t\tpt[7]++;\n\t\t\tconst int  nb  =")
    body = sub(body, "\t\t\t__syncthreads ();\n\t\t\t/* ---- write phase ---- */",
               "\t\t\tt1 = RVP_T (); pt[2] += t1 - t0; t0 = t1;\n\t\t\t__syncthreads ();\n"
               "\t\t\tt1 = RVP_T (); pt[3] += t1 - t0; t0 = t1;\n\t\t\t/* ---- write phase ---- */")
    body = sub(body, "#endif\n\t\t\t__syncthreads ();\n\t\t}\n#undef RVL_C",
               "#endif\n\t\t\tt1 = RVP_T (); pt[4] += t1 - t0; t0 = t1;\n"
               "\t\t\t__syncthreads ();\n\t\t\tt1 = RVP_T (); pt[5] += t1 - t0; t0 = t1;\n\t\t}\n#undef RVL_C")
    # the planner loop: planning as the "read phase", its two barriers
    body = sub(body, "\t\t\t__syncthreads ();\n\t\t\t__syncthreads ();\n\t\t}\n",
               "\t\t\tpt[7]++;\n\t\t\tt1 = RVP_T (); pt[2] += t1 - t0; t0 = t1;\n\t\t\t__syncthreads ();\n"
               "\t\t\tt1 = RVP_T (); pt[3] += t1 - t0; t0 = t1;\n\t\t\t__syncthreads ();\n"
               "\t\t\tt1 = RVP_T (); pt[5] += t1 - t0; t0 = t1;\n\t\t}\n")
    body += ("\n\tt1 = RVP_T (); pt[6] += t1 - t0;\n"
             "\tif ((threadIdx.x & 63) == 0)\n\t\tfor (int k = 0; k < 8; k++)\n"
             "\t\t\tatomicAdd (&g_rvlprof[threadIdx.x >> 6][k], pt[k]);")
    s = s[:a] + body + s[b:]
    s += ("\nextern \"C\" int tbf_debug_rvl_prof (unsigned long long* out, int reset)\n{\n"
          "\tif (hipMemcpyFromSymbol (out, HIP_SYMBOL (g_rvlprof), sizeof (g_rvlprof)) != hipSuccess)\n\t\treturn -5;\n"
          "\tif (reset) {\n\t\tstatic unsigned long long z[16][8];\n"
          "\t\tif (hipMemcpyToSymbol (HIP_SYMBOL (g_rvlprof), z, sizeof (z)) != hipSuccess)\n\t\t\treturn -5;\n\t}\n"
          "\treturn 0;\n}\n")
    Path(sys.argv[1]).write_text(s)


if __name__ == "__main__":
    main()
