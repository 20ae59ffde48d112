#!/usr/bin/env python3
"""Attribute the cross-step overlap of the pipelined bench from a rocprofv3 kernel trace.

    python tools/overlap_trace.py TRACE_kernel_trace.csv [--skip N]

bench.py issues step s on HIP stream s % slots (3 slots by default), so the FEC + map + OFDM kernels of step
s + 1 may start while step s's kernels are still draining.  From the dispatch records (start / end per kernel,
its queue) this prints, over the timed steps:

  * the per-kernel mean durations, and the wall time of the whole sequence (first start -> last end);
  * busy = the union of the kernel intervals, idle = wall - busy (gaps with no kernel running), and
    overlap = sum(durations) - busy (time two or more kernels ran at once);
  * the overlap split by the pair of kernels that shared it (which kernel's tail ran beside which head);
  * per-kernel "stretch": its mean duration while it overlapped another kernel vs alone.

Kernel names are reduced to the chain's stage names (bbch, ldpc_map, ofdm32, ofdm, fill/other)."""
import argparse
import collections
import csv
import re
import sys

STAGES = (("bbch", "fec"), ("ldpc_map", "map"), ("ofdm32", "ofdm"), ("ofdm", "ofdm"))


def stage(name):
    for key, st in STAGES:
        if re.search(r"\b%s_kernel" % key, name) or ("::%s_kernel" % key) in name:
            return st
    return "other"


def load(path):
    rows = list(csv.DictReader(open(path)))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        s = int(r.get("Start_Timestamp") or r.get("BeginNs"))
        e = int(r.get("End_Timestamp") or r.get("EndNs"))
        q = r.get("Stream_Id") or r.get("Queue_Id") or "0"
        ks.append({"name": name, "stage": stage(name), "start": s, "end": e, "queue": q})
    ks.sort(key=lambda k: k["start"])
    return ks


def analyse(ks):
    ks = [k for k in ks if k["stage"] != "other"]
    if not ks:
        return None
    t0, t1 = ks[0]["start"], max(k["end"] for k in ks)
    # sweep: union and per-pair overlap (a pair's share of time when exactly those two ran)
    ev = []
    for i, k in enumerate(ks):
        ev.append((k["start"], 1, i))
        ev.append((k["end"], -1, i))
    ev.sort(key=lambda x: (x[0], x[1]))
    active = set()
    busy = 0
    pair = collections.Counter()
    multi = 0
    over_t = collections.Counter()   # per kernel: time it ran beside another
    last = t0
    for t, d, i in ev:
        dt = t - last
        if active and dt > 0:
            busy += dt
            if len(active) >= 2:
                multi += dt * (len(active) - 1)
                names = sorted(ks[j]["stage"] for j in active)
                if len(active) == 2:
                    pair["%s || %s" % tuple(names)] += dt
                else:
                    pair[" || ".join(names)] += dt
                for j in active:
                    over_t[j] += dt
        last = t
        if d > 0:
            active.add(i)
        else:
            active.discard(i)
    dur = collections.defaultdict(list)
    alone = collections.defaultdict(list)
    shared = collections.defaultdict(list)
    for i, k in enumerate(ks):
        dd = k["end"] - k["start"]
        dur[k["stage"]].append(dd)
        (shared if over_t[i] > 0.02 * dd else alone)[k["stage"]].append(dd)
    total = sum(k["end"] - k["start"] for k in ks)
    return {"wall": t1 - t0, "busy": busy, "idle": (t1 - t0) - busy, "sum": total, "overlap": total - busy,
            "pairs": pair, "dur": dur, "alone": alone, "shared": shared, "n": len(ks)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--skip", type=int, default=0, help="dispatches to drop from the start (warmup, other passes)")
    ap.add_argument("--take", type=int, default=0, help="dispatches to keep after --skip (0 = all)")
    a = ap.parse_args()
    ks = [k for k in load(a.trace) if k["stage"] != "other"][a.skip:]   # skip / take count chain dispatches
    if a.take:
        ks = ks[:a.take]
    r = analyse(ks)
    if r is None:
        print("no chain kernels in", a.trace)
        return 1
    ms = lambda ns: ns / 1e6  # noqa: E731
    print("%d chain dispatches: wall %.3f ms, kernel sum %.3f ms, busy (union) %.3f ms, idle %.3f ms, "
          "overlap (sum - union) %.3f ms" % (r["n"], ms(r["wall"]), ms(r["sum"]), ms(r["busy"]), ms(r["idle"]),
                                             ms(r["overlap"])))
    print("overlap by kernels sharing it:")
    for p, t in r["pairs"].most_common():
        print("  %-30s %.3f ms" % (p, ms(t)))
    print("per-kernel mean duration (all / alone / while overlapping another, >2 % of it):")
    for st in sorted(r["dur"]):
        f = lambda v: ("%.4f (%d)" % (ms(sum(v) / len(v)), len(v))) if v else "-"  # noqa: E731
        print("  %-6s %s  alone %s  overlapped %s" % (st, f(r["dur"][st]), f(r["alone"][st]), f(r["shared"][st])))
    return 0


if __name__ == "__main__":
    sys.exit(main())
