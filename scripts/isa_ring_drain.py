#!/usr/bin/env python3
"""Static check of the hot wgemm instantiations (tests/test_kernel_resources.py's HOT_WGEMM):
per kernel, the s_waitcnt vmcnt(0) and the 64-bit register copies between the first weight-
stream load and the first MFMA of EVERY path (a vmcnt(0) there drains the primed weight ring
before compute starts).  usage: isa_ring_drain.py dir_with_lm_gemm_<unit>.s"""
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def hot():
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests",
                            "test_kernel_resources.py")).read()
    block = src[src.index("HOT_WGEMM = ["):src.index("]", src.index("HOT_WGEMM = ["))]
    return re.findall(r'"([^"]+)"', block)


def mangle(a):
    parts = [{"false": "Lb0E", "true": "Lb1E"}.get(x.strip(), f"Li{x.strip()}E") for x in a.split(",")]
    return "_ZN3tts12wgemm_kernelI" + "".join(parts) + "EEvNS_9WgemmArgsE"


def main():
    d = sys.argv[1]
    units = ["lm_gemm_store", "lm_gemm_resid", "lm_gemm_logits", "lm_gemm_swiglu"]
    srcs = {u: open(os.path.join(d, u + ".s")).read().splitlines() for u in units}
    for h in hot():
        name = mangle(h) + ":"
        for u, s in srcs.items():
            idx = [k for k, l in enumerate(s) if l.startswith(name)]
            if not idx:
                continue
            i = idx[0]
            j = next(k for k in range(i, len(s)) if s[k].strip().startswith(".Lfunc_end"))
            b = [l.strip() for l in s[i:j]]
            # every first-MFMA after a block of stream loads: scan stream-load -> next MFMA windows
            res = []
            k = 0
            while k < len(b):
                if b[k].startswith("buffer_load_dwordx4") and b[k].endswith(" nt"):
                    mf = next((q for q in range(k, len(b)) if b[q].startswith("v_mfma")), None)
                    if mf is None:
                        break
                    seg = b[k:mf]
                    res.append((sum(1 for l in seg if l == "s_waitcnt vmcnt(0)"),
                                sum(1 for l in seg if l.startswith("v_mov_b64"))))
                    k = mf
                k += 1
            print(f"{h:52s} {u:15s} windows {len(res):3d}  with vmcnt(0): {sum(1 for r in res if r[0])}  "
                  f"copies: {sum(r[1] for r in res)}")
            break


if __name__ == "__main__":
    main()
