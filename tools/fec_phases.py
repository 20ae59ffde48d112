"""Decode per-block phase timestamps from a FEC_VARIANT=1 build (experiment only)."""
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
iq = torch.empty((B * ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
for _ in range(3):
    ch.run_device(ts_d.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
nb = B * ch.info["fec_blocks_per_frame"]
cw = ch.debug_codewords(nb)
w = cw[:, :44].copy().view(np.uint32).astype(np.int64)
names = ["geometry", "raw stage", "crc-8", "payload+hdr", "scramble", "bch", "ldpc D", "ldpc rows", "prefix", "output"]
prev = np.zeros(nb, np.int64)
print("FEC phase durations (us), median / p90 over %d blocks" % nb)
for i, n in enumerate(names):
    cur = w[:, i + 1]
    dur = (cur - prev) * 0.01
    print("  %-12s %7.2f %7.2f" % (n, np.median(dur), np.percentile(dur, 90)))
    prev = cur
t0 = (w[:, 0] - w[:, 0].min()) & 0xFFFFFFFF
print("  total        %7.2f" % np.median(w[:, len(names)] * 0.01))
print("span %.1f us, start spread %.1f us" % (((t0 + w[:, len(names)]).max()) * 0.01, t0.max() * 0.01))
