#!/usr/bin/env python3
"""One-frame latency calls, direct launches vs hipGraph mode, for a kernel + HIP API trace.

    rocprofv3 --kernel-trace --hip-trace -f csv -d DIR -o gt -- python3 tools/graph_trace.py run
    python3 tools/graph_trace.py analyse DIR

`run` issues 20 direct calls, then 20 graph calls with the same arguments, then 20 graph calls with a
different frame each (every node's arguments rewritten), each call synchronised (bench.py's latency_1_frame).
`analyse` splits the kernel dispatches into those three groups (3 kernels per call) and reports, per call, the
time from the call's first HIP API record to its first kernel's start (launch), the gaps between its kernels,
the kernels' durations and the end of the last kernel to the synchronisation's return."""
import csv
import glob
import os
import statistics
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
N = 20


def run():
    sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames
    cfg = CONFIGS["cfg3"]
    ch = dvbt2ll.Chain(cfg, max_frames=64)
    ts, base = ts_for_frames(cfg, 0, 64)
    ts_d = torch.from_numpy(ts).cuda()
    iq = torch.empty((ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()

    def call(frame):
        ch.run_device(ts_d.data_ptr(), base, len(ts), frame, 1, iq.data_ptr(), st.cuda_stream)
        st.synchronize()

    for _ in range(5):
        call(0)
    for _ in range(N):
        call(0)
    ch.set_graph(True)
    for _ in range(5):
        call(0)
    for _ in range(N):
        call(0)
    for k in range(N):
        call(1 + k)
    ch.set_graph(False)
    torch.cuda.synchronize()
    time.sleep(0.2)


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def analyse(d):
    ks = sorted(rows(d, "*kernel_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    ks = [r for r in ks if "_kernel" in r["Kernel_Name"] and "rocclr" not in r["Kernel_Name"]]
    api = sorted(rows(d, "*hip_api_trace.csv"), key=lambda r: int(r["Start_Timestamp"]))
    # groups: 5 warm + N direct, 5 warm + N graph, N graph with new arguments; 3 kernels per call
    calls = [ks[i:i + 3] for i in range(0, len(ks) - len(ks) % 3, 3)]
    if len(calls) < 2 * 5 + 3 * N:
        print("expected %d calls, found %d" % (2 * 5 + 3 * N, len(calls)))
        return 1
    groups = {"direct": calls[5:5 + N], "graph (same arguments)": calls[10 + N:10 + 2 * N],
              "graph (new arguments)": calls[10 + 2 * N:10 + 3 * N]}
    syncs = [r for r in api if r["Function"] in ("hipStreamSynchronize",)]
    for name, cs in groups.items():
        launch, gap1, gap2, dur, tail, total = [], [], [], [], [], []
        for c in cs:
            s0, e0 = int(c[0]["Start_Timestamp"]), int(c[0]["End_Timestamp"])
            s1, e1 = int(c[1]["Start_Timestamp"]), int(c[1]["End_Timestamp"])
            s2, e2 = int(c[2]["Start_Timestamp"]), int(c[2]["End_Timestamp"])
            # the call's API records: those after the previous synchronisation returned
            prev = [int(r["End_Timestamp"]) for r in syncs if int(r["End_Timestamp"]) <= s0]
            t_call = min((int(r["Start_Timestamp"]) for r in api
                          if int(r["Start_Timestamp"]) >= (prev[-1] if prev else 0) and int(r["Start_Timestamp"]) <= s0),
                         default=s0)
            nxt = [int(r["End_Timestamp"]) for r in syncs if int(r["End_Timestamp"]) >= e2]
            t_ret = nxt[0] if nxt else e2
            launch.append(s0 - t_call); gap1.append(s1 - e0); gap2.append(s2 - e1)
            dur.append((e0 - s0) + (e1 - s1) + (e2 - s2)); tail.append(t_ret - e2); total.append(t_ret - t_call)
        med = lambda v: statistics.median(v) / 1e3  # noqa: E731
        print("%-24s call->1st kernel %6.1f us | gaps %5.1f %5.1f us | kernels %6.1f us | last end->sync return "
              "%5.1f us | total %6.1f us" % (name, med(launch), med(gap1), med(gap2), med(dur), med(tail), med(total)))
    return 0


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "run":
        run()
    elif len(sys.argv) > 2 and sys.argv[1] == "analyse":
        sys.exit(analyse(sys.argv[2]))
    else:
        print(__doc__)
