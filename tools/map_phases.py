"""Decode per-block phase timestamps from a MAP_VARIANT=1 build (experiment only)."""
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path[:0] = [str(ROOT / "gr-dvbt2ll_amd"), str(ROOT / "tests")]
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402
import plan_probe as PP  # noqa: E402

cfg = CONFIGS[sys.argv[1] if len(sys.argv) > 1 else "cfg3"]
B = 64
ch = dvbt2ll.Chain(cfg, max_frames=B)
ts, base = ts_for_frames(cfg, 0, B)
ts_d = torch.from_numpy(ts).cuda()
iq = torch.empty((B * ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
for _ in range(3):
    ch.run_device(ts_d.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
plan = PP.frame_plan(cfg.fm_args())
part = PP.chain_layout(cfg)["part"]
F = plan["F"]
pairs = ch.debug_cell_pairs(plan["S"]).astype(np.int64)
cs = plan["cs"]
rows = []
for r in range(F):
    # TI-store index c (row c // 5, column c % 5) = cell-interleaved position (c % 5) * cs/5 + c // 5
    t = [(c % 5) * (cs // 5) + c // 5 for c in range(12)]
    pos = [int(part[PP.ti_dest(plan, np.array([r]), np.array([tt]))[0]]) for tt in t]
    h = [pairs[p] for p in pos]
    rows.append(np.array([h[2 * i] | (h[2 * i + 1] << 16) for i in range(6)], np.int64))
a = np.array(rows)
names = ["cw load", "cell idx", "qam+ci", "ti store"]
prev = np.zeros(len(a), np.int64)
print("map phases (us), median / p90 over %d blocks of frame 0" % len(a))
for i, n in enumerate(names):
    cur = a[:, i + 1]
    print("  %-9s %7.2f %7.2f" % (n, np.median((cur - prev) * 0.01), np.percentile((cur - prev) * 0.01, 90)))
    prev = cur
print("  total     %7.2f" % np.median(a[:, 4] * 0.01))
