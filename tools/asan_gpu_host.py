"""Host AddressSanitizer + UBSan run of the product's C ABI on the GPU box (verdict r3: t2_capi.cpp was not
under ASan).  `make -C gr-dvbt2ll_amd/csrc asan-host` (build container) instruments the host code of
libdvbt2ll_hip.so (handles, planner, launch wrappers; -Xarch_host, device code untouched) and of its two
native drivers:
  - dvbt2ll_tx, the CLI transmitter: the chain (dvbt2ll_chain_create / the streaming host ring: H2D of the
    TS, the kernels, D2H of the IQ), cf32 and sc16 with the output gain, batches of frames; and its --mplp
    mode (dvbt2ll_chain_create_mplp with its quad tables and per-PLP layouts, run_plps_host) for a 3-PLP
    frame and a frame with TIME_IL_TYPE 1 and sub-sliced Type-2 PLPs (multi-PLP host code);
  - gr_flowgraph, the GR-style scheduler over the header-only adapters: every block's make /
    output_multiple / forecast / general_work with ragged noutput_items and TS chunks / consume_each.
Each run's IQ must equal, byte for byte, the same command with the uninstrumented build (whose IQ the
GPU tests check against the oracle); any sanitizer report aborts the run.  This script never touches
the GPU itself (only its child processes do).  Usage: python tools/asan_gpu_host.py [outdir]"""
import os
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
from dvbt2ll.configs import CONFIGS, MPLP_CONFIGS, IF_CONFIGS, ts_for_frames  # noqa: E402  (numpy only)

PLAIN = {"tx": ROOT / "gr-dvbt2ll_amd" / "dvbt2ll" / "dvbt2ll_tx", "fg": ROOT / "tests" / "adapter" / "gr_flowgraph"}
ASAN = {"tx": ROOT / "build" / "asan_host" / "dvbt2ll_tx", "fg": ROOT / "build" / "asan_host" / "gr_flowgraph"}
# quarantine_size_mb: large enough that the quarantine never recycles during the HIP runtime's teardown at
# exit -- recycling a freed device-allocator chunk after the device runtime has unloaded trips the ROCm ASan
# runtime's own CHECK (sanitizer_allocator_device.h "!dev_runtime_unloaded_", seen once a run frees ~100 MB
# of device buffers, e.g. the streaming ring's); a larger quarantine only widens use-after-free detection
ENV = dict(os.environ,
           ASAN_OPTIONS="protect_shadow_gap=0:detect_leaks=0:verify_asan_link_order=0:halt_on_error=1:"
                        "quarantine_size_mb=4096",
           UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")


def fg_params(cfg):
    return [str(int(v)) for v in cfg.fm_args()] + [str(int(v)) for v in
                                                   (cfg.misogroup, cfg.equalization, cfg.bandwidth, cfg.tsrate)]


def run(kind, tool, args, out, log):
    r = subprocess.run([str(tool)] + args(out), capture_output=True, text=True, timeout=240,
                       env=ENV if kind == "asan" else None)
    log.write("$ %s %s\n%s%s\n" % (tool, " ".join(args(out)), r.stdout[-2000:], r.stderr[-6000:]))
    if r.returncode != 0:
        raise SystemExit("%s run failed (exit %d): %s" % (kind, r.returncode, r.stderr[-3000:]))
    return Path(out).read_bytes()


def main():
    outdir = Path(sys.argv[1] if len(sys.argv) > 1 else ROOT / "gpurun_out" / "asan_host")
    outdir.mkdir(parents=True, exist_ok=True)
    cases = []
    for name, nfr in (("cfg1", 4), ("cfg1q", 3), ("cfg4", 2), ("cfg3", 2)):
        cfg = CONFIGS[name]
        ts, base = ts_for_frames(cfg, 0, nfr + 1)
        assert base == 0
        tsf = outdir / ("%s.ts" % name)
        tsf.write_bytes(ts.tobytes())
        for fmt, gain, batch in (("cf32", "1", "1"), ("sc16", "0.2", "2")):
            cases.append(("tx", "%s_%s" % (name, fmt),
                          lambda o, n=name, t=tsf, f=fmt, g=gain, b=batch, k=nfr:
                          ["--preset", n, "--in", str(t), "--out", o, "--format", f, "--gain", g, "--batch", b,
                           "--frames", str(k)]))
        if name != "cfg3":
            cases.append(("fg", "%s_flowgraph" % name,
                          lambda o, t=tsf, c=cfg, k=nfr: [str(t), o, str(k), "7"] + fg_params(c)))
    for name in ("mplp3_4k", "mix_4k"):
        m = {**MPLP_CONFIGS, **IF_CONFIGS}[name]
        n = 4 * m.unit_frames
        ins = []
        for k, p in enumerate(m.plps):
            ts, base = ts_for_frames(p, 0, n, seed=k + 1)
            f = outdir / ("%s_p%d.ts" % (name, k))
            f.write_bytes(ts.tobytes())
            ins += ["--in", str(f)]
        cases.append(("tx", "%s_mplp" % name,
                      lambda o, nm=name, i=ins, k=n, u=m.unit_frames:
                      ["--mplp", nm, *i, "--out", o, "--batch", str(2 * u), "--frames", str(k)]))
    for tool in ASAN.values():   # the instrumented drivers really load the sanitizer runtime and library
        deps = subprocess.run(["ldd", str(tool)], capture_output=True, text=True, check=True).stdout
        assert "libclang_rt.asan" in deps and str(ROOT / "build" / "asan_host" / "libdvbt2ll_hip.so") in deps, deps
    with open(outdir / "asan_host.log", "w") as log:
        for tool, label, args in cases:
            if not PLAIN[tool].exists() or not ASAN[tool].exists():
                raise SystemExit("missing %s or %s: build first" % (PLAIN[tool], ASAN[tool]))
            want = run("plain", PLAIN[tool], args, str(outdir / ("%s.plain" % label)), log)
            got = run("asan", ASAN[tool], args, str(outdir / ("%s.asan" % label)), log)
            same = want == got
            print("%-18s %-10s %9d bytes  asan == plain: %s" % (label, tool, len(got), same), flush=True)
            if not same:
                raise SystemExit("IQ differs between the instrumented and the plain build: %s" % label)
            for f in (outdir / ("%s.plain" % label), outdir / ("%s.asan" % label)):
                f.unlink()
    print("asan_host ok: %d runs of the host-instrumented C ABI, no sanitizer report, IQ identical" % len(cases))


if __name__ == "__main__":
    main()
