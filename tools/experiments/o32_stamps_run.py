"""Run the 32K OFDM phase-probe build (exp_build/libo32st.so, tools/experiments/o32_stamps.py) on a
cfg3 chain of 192 frames and print the median / p90 phase durations (us) over all workgroups.
    python tools/experiments/o32_stamps_run.py [LIB]"""
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
import dvbt2ll._lib as L  # noqa: E402

L.LIB_PATH = Path(sys.argv[1] if len(sys.argv) > 1 else ROOT / "exp_build" / "libo32st.so")
import torch  # noqa: E402
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402

cfg = CONFIGS["cfg3"]
B = 192
ch = dvbt2ll.Chain(cfg, max_frames=B)
ts, base = ts_for_frames(cfg, 0, B)
d = torch.from_numpy(ts).cuda()
per = ch.iq_per_frame
iq = torch.empty((B * per, 2), dtype=torch.float32, device="cuda")
for _ in range(4):
    ch.run_device(d.data_ptr(), base, len(ts), 0, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
torch.cuda.synchronize()
N, G, nsym = 32768, 2048, ch.info["num_symbols"]
w = iq.cpu().numpy().view(np.uint32).reshape(B, per * 2)
idx = 2 * (2048 + np.arange(nsym) * (N + G))
st = np.stack([w[:, i:i + 12] for i in idx], axis=1).reshape(-1, 12).astype(np.int64)   # (B*nsym, 12)
t = st[:, :10] - st[:, :1]
names = ["scatter0", "read0", "scatter1", "read1+dft", "exch1+twA", "stageB+exch2", "stageC", "store_issue",
         "store_drain"]
dur = np.diff(st[:, :10], axis=1) * 0.01   # 100 MHz -> us
out = {"workgroups": int(st.shape[0])}
for k, n in enumerate(names):
    out[n] = [round(float(np.median(dur[:, k])), 3), round(float(np.percentile(dur[:, k], 90)), 3)]
tot = (st[:, 9] - st[:, 0]) * 0.01
out["total"] = [round(float(np.median(tot)), 3), round(float(np.percentile(tot, 90)), 3)]
span = (st[:, 9].max() - st[:, 0].min()) * 0.01
out["kernel_span_us"] = round(float(span), 1)
hw = st[:, 11]
cu = (hw >> 8) & 0xF, (hw >> 13) & 0x7, (hw >> 16) & 0x3
out["distinct_hw_id"] = int(len(np.unique(hw & 0xFFFF00)))
# per-CU occupancy: sum of workgroup durations / span
out["busy_frac_mean"] = round(float(tot.sum() / (span * 256)), 3)
print(json.dumps(out))
