"""Build-variant generator (profiling only, never the product): a copy of
csrc/tbf_render.hip whose k_whirl instance waves accumulate s_memtime cycles per phase on
lane 0 (the filter wave: its filter work and its barrier waits) and write them, as floats,
over the first 16 output samples of instances 0..7 (tools/whirl_prof.py reads them back).
usage: python tools/whirl_prof_patch.py OUT.hip"""
import sys
from pathlib import Path

src = (Path(__file__).resolve().parents[1] / "tunebfree_amd" / "csrc" / "tbf_render.hip").read_text()


def sub(s, old, new):
    assert s.count(old) == 1, (old, s.count(old))
    return s.replace(old, new)


def mark(k, ind="\t"):
    return (f"\n{ind}if ((threadIdx.x & 63) == 0) {{ const unsigned long long _t = __builtin_amdgcn_s_memtime (); "
            f"I.wp[{k}] += _t - I.wplast; I.wplast = _t; }}")


s = src
s = sub(s, "\tint32_t      bf[NL];            /* the launch's per-block control",
        "\tunsigned long long wp[16], wplast;\n\tint32_t      bf[NL];            /* the launch's per-block control")
# whirl_sub phases
s = sub(s, "\tI.xf[4 + n] = I.hb[k & 1][n];\n", "\tI.xf[4 + n] = I.hb[k & 1][n];" + mark(1) + "\n")
s = sub(s, "\t\t\tst.drumAngle = okd ? d0 + (double)TBF_SUB * Dd : wrap1 (angBuf[2 * TBF_SUB - 1] + drumIncr);\n\t}\n\twave_sync ();",
        "\t\t\tst.drumAngle = okd ? d0 + (double)TBF_SUB * Dd : wrap1 (angBuf[2 * TBF_SUB - 1] + drumIncr);\n\t}\n\twave_sync ();" + mark(4))
s = sub(s, "\tconst float xd2v = (float)((0.4 * xd1v) + (0.4 * I.xd1[n]));\n\twave_sync ();",
        "\tconst float xd2v = (float)((0.4 * xd1v) + (0.4 * I.xd1[n]));\n\twave_sync ();" + mark(5))
s = sub(s, "\t\tbool okr[WH_RG];", mark(6, "\t\t")[1:] + "\n\t\tbool okr[WH_RG];")
s = sub(s, "\t/* the horn outputs (whirlProc2 outHL / outHR); the drum outputs follow the shelves */",
        mark(7)[1:] + "\n\t/* the horn outputs (whirlProc2 outHL / outHR); the drum outputs follow the shelves */")
s = sub(s, "\t\tst.outpos = (st.outpos + TBF_SUB) & 2047u;\n\twave_sync ();\n}",
        "\t\tst.outpos = (st.outpos + TBF_SUB) & 2047u;\n\twave_sync ();" + mark(8) + "\n}")
# k_whirl: staging, block start, block end, barrier
s = sub(s, "\t\t\txnx = inB[(size_t)min (k + 4, nSub - 1) * TBF_SUB + lane];\n",
        "\t\t\txnx = inB[(size_t)min (k + 4, nSub - 1) * TBF_SUB + lane];" + mark(0, "\t\t\t") + "\n")
s = sub(s, "\t\t\t\t\t\tI.brake = brake;\n\t\t\t\t\t}\n\t\t\t\t\twave_sync ();",
        "\t\t\t\t\t\tI.brake = brake;\n\t\t\t\t\t}\n\t\t\t\t\twave_sync ();" + mark(9, "\t\t\t\t\t"))
s = sub(s, "\t\t\t\t\t\t\tif (I.brake & 2) I.st.drumIncr = 0;\n\t\t\t\t\t\t}\n\t\t\t\t\t\twave_sync ();",
        "\t\t\t\t\t\t\tif (I.brake & 2) I.st.drumIncr = 0;\n\t\t\t\t\t\t}\n\t\t\t\t\t\twave_sync ();" + mark(11, "\t\t\t\t\t\t"))
s = sub(s, "\t\t\tp1 = p0;\n\t\t}\n\t\t__syncthreads ();\n\t}\n",
        "\t\t\tp1 = p0;\n\t\t}" + mark(13, "\t\t") + "\n\t\t__syncthreads ();" + mark(12, "\t\t") + "\n\t}\n")
s = sub(s, "\tif (live) {\n\t\tcopy_words (&I.st, S);",
        "\tif (lane < 16) I.wp[lane] = 0;\n\tif (lane == 0) I.wplast = __builtin_amdgcn_s_memtime ();\n\tif (live) {\n\t\tcopy_words (&I.st, S);")
s = sub(s, "\t\tfor (uint32_t i = lane; i < 4u * W; i += NL)\n\t\t\twr[i] = (&I.wring[0][0])[i];\n\t}\n}",
        "\t\tfor (uint32_t i = lane; i < 4u * W; i += NL)\n\t\t\twr[i] = (&I.wring[0][0])[i];\n"
        "\t\tif (inst < 8 && lane < 16) P.outL[(size_t)inst * P.outStride + P.outOffset + lane] = (float)I.wp[lane];\n\t}\n}")
# the filter wave: work (14) and barrier waits (15), into instance 0's slots
s = sub(s, "\tfloat z0 = I.st.fz[rr][0], z1 = I.st.fz[rr][1];\n#pragma unroll 1\n\tfor (int k = -2; k <= nSub + 1; k++) {",
        "\tfloat z0 = I.st.fz[rr][0], z1 = I.st.fz[rr][1];\n\tunsigned long long _f0 = __builtin_amdgcn_s_memtime (), _f1, fw = 0, fb = 0;\n"
        "#pragma unroll 1\n\tfor (int k = -2; k <= nSub + 1; k++) {")
s = sub(s, "\t\t\t\t\tif (isnan (z1))\n\t\t\t\t\t\tz1 = 0.f;\n\t\t\t\t}\n\t\t\t}\n\t\t}\n\t\t__syncthreads ();\n\t}\n",
        "\t\t\t\t\tif (isnan (z1))\n\t\t\t\t\t\tz1 = 0.f;\n\t\t\t\t}\n\t\t\t}\n\t\t}\n"
        "\t\t_f1 = __builtin_amdgcn_s_memtime (); fw += _f1 - _f0; _f0 = _f1;\n\t\t__syncthreads ();\n"
        "\t\t_f1 = __builtin_amdgcn_s_memtime (); fb += _f1 - _f0; _f0 = _f1;\n\t}\n"
        "\tif (lane == 0) { sm.in[0].wp[14] = fw; sm.in[0].wp[15] = fb; }\n")
Path(sys.argv[1]).write_text(s)
