"""Build-variant generator (profiling only, never the product): a copy of
csrc/tbf_render.hip in which one single-wave kernel accumulates s_memtime cycles per
segment between its syncs (a marker after every __syncthreads / wave_sync of the named
device functions) on lane 0 and writes them, as floats, over the first 32 output samples
of instances 0..7 (tools/phase_prof.py reads them back).

usage: python tools/phase_prof_patch.py tonegen OUT.hip  (profile with tools/phase_prof.py --chain 1)"""
import re
import sys
from pathlib import Path

SRC = Path(__file__).resolve().parents[1] / "tunebfree_amd" / "csrc" / "tbf_render.hip"
CFG = {
    "tonegen": dict(lds="struct TgLds {", funcs=["__device__ __forceinline__ void stage_tonegen ("],
                    kernel="k_tonegen (const tbf_launch P", init_after="\tTgLds&              sm = smv[part];\n",
                    end="\t\tfor (uint32_t i = lane; i < sizeof (tbf_tg_state) / 4; i += NL)\n\t\t\tdst[i] = src[i];\n\t}\n}"),
}

def main():
    which, out = sys.argv[1], sys.argv[2]
    c = CFG[which]
    s = SRC.read_text()
    i = s.index(c["lds"])
    j = s.index("\n};", i)
    s = s[:j] + "\n\tunsigned long long pp[32], pplast;" + s[j:]
    k = 0
    for f in c["funcs"]:
        a = s.index(f)
        b = s.index("\n}\n", a)
        body = s[a:b]

        def mark(m):
            nonlocal k
            k += 1
            assert k < 32
            return (m.group(0) + f" if (threadIdx.x == 0) {{ asm volatile (\"\" ::: \"memory\"); const unsigned long long _t = "
                    f"__builtin_amdgcn_s_memtime (); sm.pp[{k}] += _t - sm.pplast; sm.pplast = _t; }}")
        body = re.sub(r"(__syncthreads|wave_sync) \(\);", mark, body)
        s = s[:a] + body + s[b:]
    a = s.index(c["kernel"])
    b = s.index(c["init_after"], a) + len(c["init_after"])
    s = s[:b] + "\n\tif (threadIdx.x < 32) sm.pp[threadIdx.x] = 0;\n\tif (threadIdx.x == 0) sm.pplast = __builtin_amdgcn_s_memtime ();" + s[b:]
    e = s.index(c["end"], a)
    s = s[:e] + c["end"][:-1] + ("\tif (inst < 8 && threadIdx.x < 32) P.outL[(size_t)inst * P.outStride + P.outOffset + "
                                  "threadIdx.x] = (float)sm.pp[threadIdx.x];\n}") + s[e + len(c["end"]):]
    Path(out).write_text(s)
    print(f"{k} markers")


if __name__ == "__main__":
    main()
