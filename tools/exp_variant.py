"""Build an experiment variant of the kernel library from textual edits of t2_kernels.hip.

    python tools/exp_variant.py NAME EDITS.py

EDITS.py defines EDITS = [(old, new), ...]; each `old` must occur exactly once in the product
source.  The edited copy is compiled to exp_build/libNAME.so with the product's host objects, so
the product source never carries experiment switches (wrong-output variants included).
"""
import pathlib
import runpy
import subprocess
import sys

ROOT = pathlib.Path(__file__).resolve().parents[1]
C = ROOT / "gr-dvbt2ll_amd" / "csrc"
OUT = ROOT / "exp_build"


def main():
    name, edits_file = sys.argv[1], sys.argv[2]
    edits = runpy.run_path(edits_file)["EDITS"]
    src = (C / "t2_kernels.hip").read_text()
    for old, new in edits:
        n = src.count(old)
        if n != 1:
            sys.exit(f"edit target occurs {n} times: {old[:80]!r}")
        src = src.replace(old, new)
    OUT.mkdir(exist_ok=True)
    hip = OUT / f"t2_kernels_{name}.hip"
    hip.write_text(src)
    subprocess.run(["make", "-s", "-C", str(C)], check=True)
    obj = OUT / f"k_{name}.o"
    hipcc = "/opt/rocm/bin/hipcc"
    subprocess.run([hipcc, "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950", "-munsafe-fp-atomics",
                    f"-I{C}", "-c", str(hip), "-o", str(obj)], check=True)
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o", str(OUT / f"lib{name}.so"),
                    str(C / "_obj" / "t2_plan.o"), str(obj), str(C / "_obj" / "t2_capi.o")], check=True)
    print("built", OUT / f"lib{name}.so")


if __name__ == "__main__":
    main()
