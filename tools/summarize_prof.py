"""Condense a gpurun_out/prof/<tag> rocprofv3 session (kernel-trace --stats + PMC passes) into
profiles/<round>_<tag>_*.{csv,md} for the judge.   python tools/summarize_prof.py r1b r1"""
import csv
import glob
import os
import shutil
import sys
from collections import defaultdict

tag, rnd = sys.argv[1], sys.argv[2]
src = os.path.join("gpurun_out", "prof")
dst = "profiles"
os.makedirs(dst, exist_ok=True)
stats = glob.glob(os.path.join(src, "trace_%s" % tag, "*kernel_stats.csv"))
lines = ["# rocprofv3 summary %s (%s)" % (rnd, tag), ""]
if stats:
    out = os.path.join(dst, "%s_%s_kernel_stats.csv" % (rnd, tag))
    shutil.copy(stats[0], out)
    lines += ["## kernel trace (`rocprofv3 --kernel-trace --stats`, bench.py --steps 10 --warmup 2)", "",
              "| kernel | calls | avg us | min us | max us | % |", "|---|---|---|---|---|---|"]
    for r in csv.DictReader(open(stats[0])):
        lines.append("| %s | %s | %.1f | %.1f | %.1f | %.1f |" % (r["Name"][:40], r["Calls"], float(r["AverageNs"]) / 1e3,
                                                               float(r["MinNs"]) / 1e3, float(r["MaxNs"]) / 1e3,
                                                               float(r["Percentage"])))
    j = os.path.join(src, "trace_%s.json" % tag)
    if os.path.exists(j):
        shutil.copy(j, os.path.join(dst, "%s_%s_trace_bench.json" % (rnd, tag)))
lines += ["", "## PMC passes (`rocprofv3 --pmc <set>`, bench.py --pmc-child --steps 2 --warmup 1), mean per launch", "",
          "| kernel | counter | mean per launch |", "|---|---|---|"]
rows = defaultdict(list)
for fn in sorted(glob.glob(os.path.join(src, "pmc_%s_*" % tag, "**", "*counter_collection.csv"), recursive=True)):
    for r in csv.DictReader(open(fn)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "")
        k = k.split("<")[0] + ("<%s>" % r["Kernel_Name"].split("<")[1].split(">")[0] if "<" in r["Kernel_Name"] else "")
        rows[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(rows.items()):
    if "rocclr" in k:
        continue
    lines.append("| %s | %s | %.4g |" % (k[:48], c, sum(v) / len(v)))
lines += ["", "FETCH_SIZE / WRITE_SIZE are KiB; on gfx950 FETCH_SIZE counts half the read bytes",
          "(MI355X_MICROARCH.md): HBM read bytes = FETCH_SIZE x 1024 x 2."]
open(os.path.join(dst, "%s_%s_summary.md" % (rnd, tag)), "w").write("\n".join(lines) + "\n")
print("\n".join(lines))
