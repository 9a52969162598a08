"""Build-variant generator (profiling only, never the product): a copy of
csrc/tbf_render.hip whose k_whirl accumulates s_memtime cycles per phase of stage_whirl on
lane 0 and writes them, as floats, over the first 16 output samples of instances 0..7
(tools/whirl_prof.py reads them back).  usage: python tools/whirl_prof_patch.py OUT.hip"""
import sys
from pathlib import Path

src = (Path(__file__).resolve().parents[1] / "tunebfree_amd" / "csrc" / "tbf_render.hip").read_text()


def ins_after(s, anchor, text, nth=1):
    i = -1
    for _ in range(nth):
        i = s.index(anchor, i + 1)
    j = i + len(anchor)
    return s[:j] + text + s[j:]


s = src
s = s.replace("\tint          ap;\n};", "\tint          ap;\n\tunsigned long long wp[16], wplast;\n};", 1)
mark = lambda k: f"\n\t\tif (threadIdx.x == 0) {{ const unsigned long long _t = __builtin_amdgcn_s_memtime (); sm.wp[{k}] += _t - sm.wplast; sm.wplast = _t; }}"
# block start (whirl_speed) and per-sub-block phases
s = ins_after(s, "\t\tsm.brake = brake;\n\t}\n\twave_sync ();", mark(9))
s = ins_after(s, "\t\twave_sync ();\n\t\tif (!sm.aReady) {", mark(1).replace("\n\t\t", "\n\t\t\t"))
s = ins_after(s, "\t\t}\n\t\twave_sync ();\n\t\t/* the filter outputs: horn B -> xf", "", 1)
s = s.replace("\t\t}\n\t\twave_sync ();\n\t\t/* the filter outputs: horn B -> xf",
              "\t\t}\n\t\twave_sync ();" + mark(3) + "\n\t\t/* the filter outputs: horn B -> xf", 1)
s = ins_after(s, "\t\t\t\tst.drumAngle = de;\n\t\t\t}\n\t\t}\n\t\twave_sync ();", mark(4))
s = ins_after(s, "\t\tconst float xd2v = (float)((0.4 * xd1v) + (0.4 * xd1p));\n\t\twave_sync ();", mark(5))
s = s.replace("\t\t\tbool okr[WH_RG];", mark(6).replace("\n\t\t", "\n\t\t\t") + "\n\t\t\tbool okr[WH_RG];")
s = s.replace("\t\t/* ---- outputs (whirlProc2 outHL/outHR/outDL/outDR + whirlProc3 mix) ---- */",
              mark(7)[1:] + "\n\t\t/* ---- outputs (whirlProc2 outHL/outHR/outDL/outDR + whirlProc3 mix) ---- */")
s = ins_after(s, "\t\t\tst.outpos = (st.outpos + TBF_SUB) & 2047u;\n\t\twave_sync ();", mark(8))
s = s.replace("\tif (lane == 0) {\n\t\tint brake;", mark(10)[1:].replace("\t\tif", "\tif", 1) + "\n\tif (lane == 0) {\n\t\tint brake;")
# init and write-out in k_whirl
s = s.replace("\t\tsm.ap     = 0;\n\t}\n",
              "\t\tsm.ap     = 0;\n\t}\n\tif (threadIdx.x < 16) sm.wp[threadIdx.x] = 0;\n"
              "\tif (threadIdx.x == 0) sm.wplast = __builtin_amdgcn_s_memtime ();\n", 1)
s = s.replace("\twave_sync ();\n\tcopy_words (S, &sm.st);\n\tfor (uint32_t i = threadIdx.x; i < 4u * W; i += NL)\n\t\twr[i] = sm.wring[i / W][i % W];\n}",
              "\twave_sync ();\n\tcopy_words (S, &sm.st);\n\tfor (uint32_t i = threadIdx.x; i < 4u * W; i += NL)\n\t\twr[i] = sm.wring[i / W][i % W];\n"
              "\tif (inst < 8 && threadIdx.x < 16) P.outL[(size_t)inst * P.outStride + P.outOffset + threadIdx.x] = (float)sm.wp[threadIdx.x];\n}")
assert s.count("sm.wp[") >= 11, s.count("sm.wp[")
Path(sys.argv[1]).write_text(s)
