"""PCIe-inclusive rate of the host-buffer boundary (dvbt2ll_chain_run_host: H2D of the TS, the
three kernels, D2H of the IQ, synchronous) for cfg3, beside the HBM-resident rate bench.py
reports as `value`.  Run on the GPU box: python tools/pcie_rate.py [frames] [iters]"""
import sys
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402

cfg = CONFIGS["cfg3"]
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ch = dvbt2ll.Chain(cfg, max_frames=B)
ts, base = ts_for_frames(cfg, 0, B)
for fmt, name in ((dvbt2ll.IQ_CF32, "cf32"), (dvbt2ll.IQ_SC16, "sc16")):
    ch.set_output(1.0 if fmt == dvbt2ll.IQ_CF32 else 0.2, fmt)
    ch.run(0, B, ts, base)      # warm-up (allocates the staging buffers)
    t0 = time.perf_counter()
    for _ in range(iters):
        ch.run(0, B, ts, base)
    dt = (time.perf_counter() - t0) / iters
    n = B * ch.iq_per_frame
    print("%s: %d frames per call, %.2f ms per call, %.0f Msamples/s PCIe-inclusive (host TS in, host IQ out, "
          "pageable numpy buffers)" % (name, B, dt * 1e3, n / dt / 1e6))
