"""GPU: the RCCL side of the multi-GPU path on the one GPU a test box has (verdict r5, "multi-GPU correctness rests
on gloo alone"): torch.distributed's nccl backend (RCCL) initialised with device_id, the frame-sharded encode and
the ordered gather (dvbt2ll.distributed.encode_sharded / gather_frames) at world size 1, checked bit for bit
against a direct run.  The send / recv legs need a second GPU; they are covered by the gloo tests
(test_cpu_distributed.py) and run on the driver's 8-GPU node."""
import datetime
import socket

import numpy as np
import pytest
import torch

import dvbt2ll
from dvbt2ll.configs import CONFIGS
from dvbt2ll.distributed import encode_sharded

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("name,nframes", [("cfg1", 3), ("cfg3", 2)])
def test_rccl_world1_sharded_encode_and_gather(gpu, name, nframes):
    import torch.distributed as dist
    assert not dist.is_initialized()
    dist.init_process_group("nccl", init_method="tcp://127.0.0.1:%d" % _free_port(), rank=0, world_size=1,
                            device_id=torch.device("cuda", 0), timeout=datetime.timedelta(seconds=120))
    try:
        assert dist.get_backend() == "nccl"
        x = torch.arange(8, dtype=torch.float32, device="cuda")
        dist.all_reduce(x)
        torch.testing.assert_close(x, torch.arange(8, dtype=torch.float32, device="cuda"))
        cfg = CONFIGS[name]
        ch = dvbt2ll.Chain(cfg, max_frames=nframes)
        iq = encode_sharded(ch, 0, nframes, gather=True)
        torch.cuda.synchronize()
        got = iq.cpu().numpy().view(np.complex64).reshape(-1)
        want = dvbt2ll.Chain(cfg, max_frames=nframes).run(0, nframes)
        np.testing.assert_array_equal(got.view(np.uint32), np.ascontiguousarray(want).view(np.uint32))
    finally:
        dist.destroy_process_group()
