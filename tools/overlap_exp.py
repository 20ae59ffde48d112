"""Experiment: how do chain calls overlap on the GPU?  cfg3, 64 frames per call, IQ rate of
  serial      one stream
  alt S       S slots, calls alternating over S streams (dvbt2ll_chain_set_slots)
(A third mode, FEC + map on one stream and OFDM on another so step s+1's FEC + map run beside
step s's OFDM, measured 129.6 GSps against 133.6 for "alt 2" and was dropped.)"""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
import torch  # noqa: E402
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402

B = 64
cfg = CONFIGS["cfg3"]
ch = dvbt2ll.Chain(cfg, max_frames=B)
ch.set_slots(3)
per = ch.iq_per_frame
ts = []
for r in range(2):
    t, base = ts_for_frames(cfg, r * B, B)
    ts.append((torch.from_numpy(t).cuda(), base, len(t), r * B))
iq = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(3)]
streams = [torch.cuda.Stream() for _ in range(3)]


def run(mode, S, steps=24, warm=4):
    ch.set_slots(S)

    def step(s):
        t, base, n, first = ts[s % 2]
        if mode == "serial":
            ch.run_device(t.data_ptr(), base, n, first, B, iq[s % S].data_ptr(), streams[0].cuda_stream)
        else:
            ch.run_device(t.data_ptr(), base, n, first, B, iq[s % S].data_ptr(), streams[s % S].cuda_stream)

    for s in range(warm):
        step(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        step(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return steps * B * per / dt / 1e6


for rep in range(2):
    for mode, S in (("serial", 1), ("alt", 2), ("alt", 3)):
        print("%-6s slots %d: %.0f Msps" % (mode, S, run(mode, S)), flush=True)
