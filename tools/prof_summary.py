#!/usr/bin/env python3
"""Condense one GPU session directory (tools/gpu_session.sh -> gpurun_out/<tag>) into
profiles/<round>_<tag>_summary.md (+ the bench JSON line) for the judge:

    python tools/prof_summary.py r2a r2

kernel-trace statistics come from the rocprofv3 rocpd database of the `trace` step (same bench
command, --slots 1), the per-kernel HIP-event launch times and PMC traffic from bench.json, the
IQ error statistics from the parity tests (IQ_STATS)."""
import glob
import json
import os
import shutil
import sqlite3
import sys
from collections import defaultdict


def kernel_stats(db):
    c = sqlite3.connect(db)
    rows = defaultdict(list)
    for name, start, end in c.execute("select name, start, end from kernels"):
        rows[name].append((end - start) / 1e3)
    tot = sum(sum(v) for v in rows.values())
    out = []
    for name, v in sorted(rows.items(), key=lambda kv: -sum(kv[1])):
        out.append((name, len(v), sum(v) / len(v), min(v), max(v), 100 * sum(v) / tot))
    return out


def kernel_stats_csv(path):
    import csv
    out = []
    for r in csv.DictReader(open(path)):
        out.append((r["Name"], int(r["Calls"]), float(r["AverageNs"]) / 1e3, float(r["MinNs"]) / 1e3,
                    float(r["MaxNs"]) / 1e3, float(r["Percentage"])))
    return out


def main(tag, rnd):
    src = os.path.join("gpurun_out", tag)
    lines = ["# GPU session %s (%s)" % (tag, rnd), ""]
    dbs = glob.glob(os.path.join(src, "trace", "*.db"))
    csvs = glob.glob(os.path.join(src, "trace", "*kernel_stats.csv"))
    stats = kernel_stats(dbs[0]) if dbs else (kernel_stats_csv(csvs[0]) if csvs else None)
    if csvs:
        shutil.copy(csvs[0], os.path.join("profiles", "%s_%s_kernel_stats.csv" % (rnd, tag)))
    if stats:
        lines += ["## kernel trace (`rocprofv3 --kernel-trace --stats`, bench.py --slots 1 --steps 10 --warmup 2)", "",
                  "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
        for name, n, avg, mn, mx, pct in stats:
            lines.append("| %s | %d | %.1f | %.1f | %.1f | %.1f |" % (name[:60], n, avg, mn, mx, pct))
        lines.append("")
    bj = os.path.join(src, "bench.json")
    if os.path.exists(bj) and os.path.getsize(bj):
        b = json.loads(open(bj).read().strip().splitlines()[-1])
        shutil.copy(bj, os.path.join("profiles", "%s_%s_bench.json" % (rnd, tag)))
        lines += ["## bench.py (default run): %.1f G IQ samples/s, %.3f ms/step, %.3g FEC blocks/s" % (
            b["value"] / 1e3, b["ms_per_step"], b["fec_blocks_per_sec"]), "",
            "| kernel | HIP-event avg ms | min bytes/launch | achieved GB/s | frac | PMC bytes/launch | PMC/min |",
            "|---|---|---|---|---|---|---|"]
        for k, e in b.get("rooflines", {}).items():
            lines.append("| %s | %.4f | %.4g | %.0f | %.3f | %s | %s |" % (
                k, e["avg_launch_ms"], e["min_bytes_per_launch"], e["achieved"], e["frac"],
                "%.4g" % e["traffic"] if e.get("traffic") else "-",
                "%.3f" % e["traffic_over_min"] if e.get("traffic_over_min") else "-"))
        fec = b.get("rooflines", {}).get("fec", {})
        if "valu_wave_instr_per_block" in fec:
            lines += ["", "FEC passes: %.3g FEC blocks/s, %.0f VALU + %.0f SALU wave-instructions per block, VALU issue "
                          "%.2f of peak" % (fec["fec_blocks_per_s"], fec["valu_wave_instr_per_block"],
                                            fec["salu_wave_instr_per_block"], fec["valu_issue_frac"])]
        lines.append("")
    st = os.path.join(src, "iq_stats.jsonl")
    if os.path.exists(st):
        by = defaultdict(list)
        for ln in open(st):
            r = json.loads(ln)
            by[r["N"]].append(r)
        lines += ["## IQ error vs a float64 IFFT of the oracle carriers (all GPU parity tests)", "",
                  "| FFT | symbols | max rel RMS | max of max/rms | pocketfft f32 rel RMS (max) | ratio (max) |",
                  "|---|---|---|---|---|---|"]
        for N, rs in sorted(by.items()):
            lines.append("| %d | %d | %.3g | %.3g | %.3g | %.2f |" % (
                N, len(rs), max(r["rel_rms"] for r in rs), max(r["max_rel"] for r in rs),
                max(r["f32_rel_rms"] for r in rs), max(r["rel_rms"] / r["f32_rel_rms"] for r in rs)))
        lines.append("")
    sq = os.path.join(src, "pmc_sq.txt")
    if os.path.exists(sq):
        shutil.copy(sq, os.path.join("profiles", "%s_%s_pmc_sq.txt" % (rnd, tag)))
        lines += ["SQ counters per launch (tools/gpu_pmc.sh): `profiles/%s_%s_pmc_sq.txt`" % (rnd, tag), ""]
    for f in ("pytest.log", "smoke.log"):
        p = os.path.join(src, f)
        if os.path.exists(p):
            tail = [ln for ln in open(p).read().splitlines() if ln.strip()][-1:]
            lines.append("%s: `%s`" % (f, tail[0] if tail else ""))
    out = os.path.join("profiles", "%s_%s_summary.md" % (rnd, tag))
    open(out, "w").write("\n".join(lines) + "\n")
    print(out)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
