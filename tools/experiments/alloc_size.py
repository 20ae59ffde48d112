"""Experiment: the bench's pipelined step (cfg3, 768 frames per step, 2 slots on 2 streams) with the IQ output
buffers and the handle's own buffers allocated larger than the step needs.  Bench r4fr measured OFDM 3.5 %
faster per frame at 1280 frames per step than at 768 or 1024; this separates the buffer sizes (page /
translation footprint) from the launch size.  One JSON line per (iq_alloc_frames, max_frames).
Usage: python tools/experiments/alloc_size.py [steps]"""
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gr-dvbt2ll_amd"))


def main():
    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    cfg = CONFIGS["cfg3"]
    B = 768
    torch.cuda.set_device(0)
    ts_all, base = ts_for_frames(cfg, 0, 2 * B)
    ts_dev = torch.from_numpy(np.ascontiguousarray(ts_all)).cuda()
    del ts_all
    streams = [torch.cuda.Stream() for _ in range(2)]
    for alloc, maxf in [(768, 768), (1280, 768), (768, 1280), (1280, 1280), (2048, 768), (768, 768)]:
        ch = dvbt2ll.Chain(cfg, max_frames=maxf)
        ch.set_slots(2)
        per = ch.iq_per_frame
        iq = [torch.empty((alloc * per, 2), dtype=torch.float32, device="cuda") for _ in range(2)]
        torch.cuda.synchronize()

        def step(s):
            first = (s % 2) * B
            ch.run_device(ts_dev.data_ptr(), base, ts_dev.numel(), first, B, iq[s % 2].data_ptr(),
                          streams[s % 2].cuda_stream)
        for s in range(4):
            step(s)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(K):
            step(s)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / K
        ch.set_timing(True)
        for s in range(K):
            first = (s % 2) * B
            ch.run_device(ts_dev.data_ptr(), base, ts_dev.numel(), first, B, iq[0].data_ptr(), streams[0].cuda_stream)
        torch.cuda.synchronize()
        ms, n = ch.timing()
        ch.set_timing(False)
        print(json.dumps({"iq_alloc_frames": alloc, "max_frames": maxf, "step_ms": round(el * 1e3, 4),
                          "G_IQ_per_s": round(B * per / el / 1e9, 1),
                          "serial_stage_ms": [round(m / max(1, c), 4) for m, c in zip(ms[:3], n[:3])],
                          "iq_ptrs": [hex(t.data_ptr()) for t in iq]}), flush=True)
        del iq, ch
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
