"""Experiment: do independent chain handles on separate HIP streams overlap on the GPU?
Prints the IQ rate of 1 handle on 1 stream against H handles on H streams (cfg3)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
import torch  # noqa: E402
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402


def run(nh, B, steps=24, warm=4):
    cfg = CONFIGS["cfg3"]
    chains = [dvbt2ll.Chain(cfg, max_frames=B) for _ in range(nh)]
    per = chains[0].iq_per_frame
    streams = [torch.cuda.Stream() for _ in range(nh)]
    ts = []
    for h in range(nh):
        t, base = ts_for_frames(cfg, h * B, B)
        ts.append((torch.from_numpy(t).cuda(), base, len(t), h * B))
    iq = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(nh)]

    def step(s):
        h = s % nh
        t, base, n, first = ts[h]
        chains[h].run_device(t.data_ptr(), base, n, first, B, iq[h].data_ptr(), streams[h].cuda_stream)

    for s in range(warm * nh):
        step(s)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for s in range(steps):
        step(s)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return steps * B * per / dt / 1e6


for nh, B in ((1, 64), (2, 64), (2, 32), (3, 64), (4, 32), (1, 128)):
    print("handles %d frames/step %3d: %.0f Msps" % (nh, B, run(nh, B)), flush=True)
