"""sha256 of the chain's IQ (cfg3, 192 frames; cfg1, 600 frames) with a given library build, for
same-box bit-exactness checks of experiment variants:  python tools/experiments/lib_iq_hash.py [LIB]"""
import hashlib
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))
import dvbt2ll._lib as L  # noqa: E402

if len(sys.argv) > 1:
    L.LIB_PATH = Path(sys.argv[1])
import torch  # noqa: E402
import dvbt2ll  # noqa: E402
from dvbt2ll.configs import CONFIGS, ts_for_frames  # noqa: E402

out = []
for name, B in (("cfg3", 192), ("cfg1", 600)):
    cfg = CONFIGS[name]
    ch = dvbt2ll.Chain(cfg, max_frames=B)
    ts, base = ts_for_frames(cfg, 3, B)
    d = torch.from_numpy(ts).cuda()
    iq = torch.zeros((B * ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
    ch.run_device(d.data_ptr(), base, len(ts), 3, B, iq.data_ptr(), torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    out.append("%s %s" % (name, hashlib.sha256(iq.cpu().numpy().tobytes()).hexdigest()[:16]))
print(" ".join(out))
