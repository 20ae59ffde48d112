"""Experiment: per-stage launch times of the cfg3 chain on a stream restricted to k CUs
(hipExtStreamCreateWithCUMask).  If the OFDM kernel's time on k CUs is below its 256-CU time x 256/k
(its store phases saturate the chip's write rate when ~70 CUs store at once), splitting the CUs
between OFDM and FEC + map on two streams beats the serial sum.  One JSON line per (mask, k).
Usage: python tools/experiments/cu_split.py [frames] [steps]"""
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "gr-dvbt2ll_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))


def main():
    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 192
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    cfg = CONFIGS["cfg3"]
    torch.cuda.set_device(0)
    hip = ctypes.CDLL("libamdhip64.so.7")
    ncu = torch.cuda.get_device_properties(0).multi_processor_count
    chain = dvbt2ll.Chain(cfg, max_frames=B)
    per = chain.iq_per_frame
    ts, base = ts_for_frames(cfg, 0, B, 1)
    ts_dev = torch.from_numpy(np.ascontiguousarray(ts)).cuda()
    iq = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()

    def balanced(k):
        # k CUs (a multiple of 32), the same count on every (XCD, shader engine) whether mask bit
        # i = 32 y + 8 m + x sits on (XCD x, SE m, CU y) or (XCD y, SE m, CU x): per SE m the (x, y)
        # with (x + y) % 8 < k / 32, a Latin square with equal row and column counts
        return [i for i in range(256) if ((i % 8) + i // 32) % 8 < k // 32]

    def masked_stream(bits):
        words = (ctypes.c_uint32 * ((ncu + 31) // 32))()
        for i in bits:
            words[i // 32] |= 1 << (i % 32)
        s = ctypes.c_void_p()
        rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), len(words), words)
        assert rc == 0, rc
        return s.value

    def run(stream):
        for _ in range(2):
            chain.run_device(ts_dev.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), stream)
        hip.hipStreamSynchronize(ctypes.c_void_p(stream))
        chain.set_timing(True)
        t0 = time.perf_counter()
        for _ in range(K):
            chain.run_device(ts_dev.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), stream)
        hip.hipStreamSynchronize(ctypes.c_void_p(stream))
        el = (time.perf_counter() - t0) / K * 1e3
        ms, n = chain.timing()
        chain.set_timing(False)
        return el, [m / max(1, c) for m, c in zip(ms[:3], n[:3])]

    ref = None
    assert ncu == 256, ncu
    for name, k in [("all", 256), ("ls", 224), ("ls", 192), ("ls", 160), ("ls", 128), ("ls", 96)]:
        bits = balanced(k)
        assert len(bits) == k and len(set(bits)) == k
        s = masked_stream(bits)
        el, st = run(s)
        if ref is None:
            ref = st
        print(json.dumps({"mask": name, "cus": k, "step_ms": round(el, 4), "fec_ms": round(st[0], 4),
                          "map_ms": round(st[1], 4), "ofdm_ms": round(st[2], 4),
                          "ofdm_x_k_over_all": round(st[2] * k / ncu / ref[2], 3),
                          "map_x_k_over_all": round(st[1] * k / ncu / ref[1], 3),
                          "fec_x_k_over_all": round(st[0] * k / ncu / ref[0], 3)}), flush=True)
        hip.hipStreamDestroy(ctypes.c_void_p(s))


if __name__ == "__main__":
    main()
