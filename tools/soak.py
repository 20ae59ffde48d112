#!/usr/bin/env python3
"""Long-run check of the pipelined chain (the bench's shape): STEPS steps of B cfg3 frames on 3 slots / streams
(two resident TS batches, as bench.py), and every CHECK-th step one frame of its IQ compared bit for bit with
the same frame encoded alone by a second handle; the TS sync-error counter must stay 0.  Prints one JSON line.

    python tools/soak.py [--steps 300] [--frames 1280] [--check 25]"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--frames", type=int, default=1280)
    ap.add_argument("--check", type=int, default=25)
    ap.add_argument("--config", default="cfg3")
    a = ap.parse_args()
    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames
    cfg = CONFIGS[a.config]
    B, S = a.frames, 3
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    ch.set_slots(S)
    one = dvbt2ll.Chain(cfg, max_frames=1)
    per = ch.iq_per_frame
    batches = []
    for r in range(2):
        ts, base = ts_for_frames(cfg, r * B, B)
        batches.append((torch.from_numpy(ts).cuda(), base, len(ts), r * B))
    iq = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(S)]
    streams = [torch.cuda.Stream() for _ in range(S)]
    rng = np.random.default_rng(7)
    checked, mismatches = 0, []
    t0 = time.perf_counter()
    for s in range(a.steps):
        ts_d, base, n, first = batches[s % 2]
        ch.run_device(ts_d.data_ptr(), base, n, first, B, iq[s % S].data_ptr(), streams[s % S].cuda_stream)
        if a.check and s % a.check == a.check - 1:
            k = int(rng.integers(0, B))
            streams[s % S].synchronize()
            got = iq[s % S][k * per:(k + 1) * per].cpu().numpy()
            want = one.run(first + k, 1)   # the same synthetic TS (seed 1), encoded alone
            checked += 1
            if not np.array_equal(got.view(np.uint32).reshape(-1), np.ascontiguousarray(want).view(np.uint32).reshape(-1)):
                mismatches.append((s, first + k))
        if s % 50 == 49:
            print("step %d / %d" % (s + 1, a.steps), file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    out = {"config": a.config, "steps": a.steps, "frames_per_step": B, "slots": S, "frames_checked": checked,
           "mismatches": mismatches, "sync_errors": ch.sync_errors(), "seconds": dt,
           "frames_encoded": a.steps * B, "airtime_hours": a.steps * B * per / 9142857.142857143 / 3600}
    print(json.dumps(out))
    return 0 if not mismatches and out["sync_errors"] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
