#!/usr/bin/env python3
"""Static ISA scan of the kernels for the two patterns that cost rounds 3-5 the most:

  1. `s_waitcnt vmcnt(0)` inside a loop after a global store in the same loop: gfx9 counts loads and
     stores in one in-order `vmcnt`, so such a wait drains every store issued before it (a table load
     the compiler sank into a store branch, a uniform table read as a vector load);
  2. per-loop instruction mix: VALU, SALU, 64-bit scalar multiply chains (`s_mul_hi_u32`), `s_nop`
     hazard padding, LDS and global instructions.

    python tools/isa_scan.py [KERNEL_SUBSTRING] [--src FILE] [--top N]

Compiles the source with hipcc (--cuda-device-only -S, gfx950) into /tmp and reads the assembly; the
loop structure comes from the compiler's `Loop Header` / `Header=` block comments."""
import argparse
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def compile_asm(src):
    out = os.path.join(tempfile.gettempdir(), "isa_scan_%d.s" % os.getpid())
    cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "--offload-arch=gfx950", "-munsafe-fp-atomics",
           "--cuda-device-only", "-S", "-I" + os.path.join(ROOT, "gr-dvbt2ll_amd", "csrc"), src, "-o", out]
    subprocess.run(cmd, check=True, capture_output=True)
    return open(out).read()


def loops_of(body):
    """(loop header, [instruction lines]) in program order, from the block comments"""
    cur, loops = None, collections.OrderedDict()
    for line in body.splitlines():
        if line.startswith((".LBB", "; %bb")):
            hdr = re.search(r"Header=(BB\d+_\d+)", line)
            top = re.search(r"=>This (Inner )?Loop Header", line)
            name = line.split(":")[0].strip().lstrip(".").replace("; %bb.", "bb")
            cur = name.replace("LBB", "BB") if top else (hdr.group(1) if hdr else None)
            continue
        t = line.strip()
        if cur and t and line.startswith("\t") and not t.startswith((";", ".")):
            loops.setdefault(cur, []).append(t)
    return loops


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel", nargs="?", default="kernel")
    ap.add_argument("--src", default=os.path.join(ROOT, "gr-dvbt2ll_amd", "csrc", "t2_kernels.hip"))
    ap.add_argument("--top", type=int, default=4, help="largest loops listed per kernel")
    a = ap.parse_args()
    s = compile_asm(a.src)
    for m in re.finditer(r"^(_Z\w+):", s, flags=re.M):
        name = m.group(1)
        if a.kernel not in name or "kernel" not in name:
            continue
        body = s[m.start():s.find(".Lfunc_end", m.start())]
        demangled = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print("== %s" % demangled[:100])
        loops = loops_of(body)
        drains = []
        for lp, ins in loops.items():
            stored = False
            for t in ins:
                if t.startswith(("global_store", "buffer_store", "global_atomic")):
                    stored = True
                if stored and t.startswith("s_waitcnt") and "vmcnt(0)" in t:
                    drains.append(lp)
        for lp, n in collections.Counter(drains).items():
            print("   store-draining vmcnt(0) in loop %s: %d" % (lp, n))
        big = sorted(loops.items(), key=lambda kv: -len(kv[1]))[:a.top]
        for lp, ins in big:
            ops = collections.Counter(t.split()[0] for t in ins)
            valu = sum(v for k, v in ops.items() if k.startswith("v_"))
            salu = sum(v for k, v in ops.items() if k.startswith("s_"))
            ds = sum(v for k, v in ops.items() if k.startswith("ds_"))
            gl = sum(v for k, v in ops.items() if k.startswith(("global_", "buffer_")))
            print("   loop %-9s %5d instr: VALU %4d SALU %4d (s_mul_hi %3d, s_nop %3d) LDS %3d global %3d" % (
                lp, len(ins), valu, salu, ops["s_mul_hi_u32"], ops["s_nop"], ds, gl))
    return 0


if __name__ == "__main__":
    sys.exit(main())
