"""Decode per-workgroup phase timestamps from an OFDM_VARIANT=8 build (experiment only).
Run on the GPU box after swapping exp_build/libvar8.so in as the product library."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg3"]
B = 64
ch = dvbt2ll.Chain(cfg, max_frames=B)
ts, base = ts_for_frames(cfg, 0, B)
ts_d = torch.from_numpy(ts).cuda()
per = ch.iq_per_frame
iq = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
for _ in range(3):
    ch.run_device(ts_d.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
w = iq.cpu().numpy().reshape(-1).view(np.uint32)
info = ch.info
N, G, Nsym = info["fft_size"], info["guard_interval"], info["num_symbols"]
rows = []
for f in range(B):
    for j in range(Nsym):
        o = (f * per + 2048 + j * (N + G)) * 2
        rows.append(w[o:o + 10].astype(np.int64))
a = np.array(rows)
t0 = a[:, 0]
t0 = (t0 - t0.min()) & 0xFFFFFFFF
d = a[:, 1:9]
names = (["fill0", "scatter0", "fft0", "hold E", "fill1", "scatter1", "fft1", "combine"] if N < 32768 else
         ["scatter0", "scatter1+read", "stageA", "exch1", "stageB", "exch2", "stageC", "store"])
prev = np.zeros(len(a), np.int64)
print("phase durations (us), median / p90 over %d workgroups" % len(a))
for i, n in enumerate(names):
    cur = d[:, i]
    dur = (cur - prev) * 0.01
    print("  %-9s %7.2f %7.2f" % (n, np.median(dur), np.percentile(dur, 90)))
    prev = cur
tot = d[:, 7] * 0.01
print("  total     %7.2f %7.2f" % (np.median(tot), np.percentile(tot, 90)))
span = (t0 + d[:, 7]).max() * 0.01
print("kernel span from first WG start: %.1f us; WG start spread: %.1f us" % (span, t0.max() * 0.01))
cus = np.unique(a[:, 9])
print("distinct hw ids:", len(cus))
