"""Static check of the wgemm kernels' ISA: full vmcnt(0) drains around the weight stream.

usage: python scripts/isa_waits.py file.s [name-substring ...]
  (file.s from `hipcc -O3 --offload-arch=gfx950 --cuda-device-only -S lm_gemm_<epi>.hip`)

For each kernel with an LDS-DMA prologue (global_load_lds) it reports, on the GEMM path:
  scratch     scratch stores (register spills) in the whole function
  pre_stream  s_waitcnt vmcnt(0) between the A rows' DMA and the first weight-stream load:
              the stream is then issued only after the A rows landed (serial latency)
  pre_norm    vmcnt(0) between the explicit landing wait (vmcnt(n) + s_barrier) and the next
              LDS read: the primed weight ring is drained before the RMSNorm prologue
"""
import re
import sys


def functions(lines):
    i = 0
    while i < len(lines):
        m = re.match(r"^(_Z\S+):", lines[i])
        if m:
            j = i
            while j < len(lines) and not lines[j].strip().startswith(".Lfunc_end"):
                j += 1
            yield m.group(1), lines[i:j]
            i = j
        i += 1


def analyse(body):
    t = [l.strip() for l in body]
    res = {"scratch": sum(1 for l in t if l.startswith("scratch_store"))}
    dma = next((k for k, l in enumerate(t) if l.startswith("global_load_lds")), None)
    if dma is None:
        return res
    nt = next((k for k in range(dma, len(t)) if t[k].startswith(("global_load_dwordx4", "buffer_load_dwordx4")) and t[k].endswith(" nt")), None)
    if nt is None:
        return res
    res["pre_stream"] = sum(1 for k in range(dma, nt) if t[k].startswith("s_waitcnt vmcnt(0)"))
    land = None
    for k in range(nt, len(t) - 2):
        m = re.match(r"s_waitcnt vmcnt\((\d+)\)$", t[k])
        if m and int(m.group(1)) > 0 and t[k + 1] == "s_barrier":
            land = k
            break
    if land is not None:
        rd = next((k for k in range(land, len(t)) if t[k].startswith("ds_read")), len(t))
        res["pre_norm"] = sum(1 for k in range(land, rd) if t[k].startswith("s_waitcnt vmcnt(0)"))
    return res


def main():
    lines = open(sys.argv[1]).read().split("\n")
    subs = sys.argv[2:]
    for name, body in functions(lines):
        if all(s in name for s in subs):
            print(f"{name[20:80]}  {analyse(body)}")


if __name__ == "__main__":
    main()
