"""CPU, world_size 2 (gloo): frame sharding covers every frame exactly once, each shard's TS
slice equals the corresponding slice of the global stream, and the ordered gather reassembles
the frames in stream order.  Per-frame payload = the oracle chain's carriers for that frame."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from dvbt2ll import distributed as D
from dvbt2ll.configs import CONFIGS, ts_for_frames, ts_packets


def test_frame_range_partition():
    for total in (0, 1, 5, 16, 17):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                f, c = D.frame_range(total, r, world, first_frame=100)
                seen += list(range(f, f + c))
            assert seen == list(range(100, 100 + total))


def _oracle_frames(cfg, nframes):
    import oracle_lib as O
    ts, _ = ts_for_frames(cfg, 0, nframes)
    F = cfg.fecblocks
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args())
    off, out = 0, []
    for _ in range(nframes):
        bits, cons = bb.work(ts[off:], F)
        off += cons
        out.append(fm.work(im.work(ld.work(bits, F), F)))
    return np.stack(out)


def _worker(rank, world, port, total, q):
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(__file__)),
                    os.path.join(os.path.dirname(__file__), "..", "gr-dvbt2ll_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        cfg = CONFIGS["cfg1"]
        first, count = D.frame_range(total, rank, world)
        # the shard's TS slice is exactly the global stream's bytes
        ts, base = ts_for_frames(cfg, first, count)
        full = ts_packets(0, (base + len(ts)) // 188)
        assert np.array_equal(full[base:], ts)
        ref = _oracle_frames(cfg, first + count)[first:]            # this rank's frames
        per = ref.shape[1]
        local = torch.from_numpy(ref.reshape(-1).view(np.float32).reshape(-1, 2).copy())
        got = D.gather_frames(local, total, per)
        if rank != 0:
            assert got is None           # only the root receives (point-to-point, not all_gather)
        if rank == 0:
            want = _oracle_frames(cfg, total).reshape(-1).view(np.float32).reshape(-1, 2)
            q.put(bool(np.array_equal(got.numpy(), want)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,world", [(4, 2), (5, 2), (2, 3)])
def test_gloo_ordered_gather(total, world):
    """world_size 2 (even and ragged shards) and 3 with one empty shard"""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get(timeout=5)


def _if_worker(rank, world, port, total, q):
    """TIME_IL_TYPE 1 sharding: each rank encodes its whole launch units (interleaving frames of P_I = 2 T2
    frames) from scratch -- its PLPs' TS slices and the oracle framemapper seeked to its first frame -- and
    the ordered gather equals the sequential run"""
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(__file__)),
                    os.path.join(os.path.dirname(__file__), "..", "gr-dvbt2ll_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_lib as O
        from dvbt2ll.configs import IF_CONFIGS
        m = IF_CONFIGS["mix_4k"]
        u = m.unit_frames
        first, count = D.frame_range(total, rank, world, unit=u)
        fm = O.FMM(m)
        fm.seek(first)
        cells, _, _ = O.mplp_cells(m, first, count)
        mine = np.stack([fm.work(c) for c in cells]) if count else np.zeros((0, fm.mapped_items), np.complex64)
        per = fm.mapped_items
        local = torch.from_numpy(mine.reshape(-1).view(np.float32).reshape(-1, 2).copy())
        got = D.gather_frames(local, total, per, unit=u)
        if rank == 0:
            seq = O.FMM(m)
            want = np.stack([seq.work(c) for c in O.mplp_cells(m, 0, total)[0]])
            q.put(bool(np.array_equal(got.numpy(), want.reshape(-1).view(np.float32).reshape(-1, 2))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("total,world", [(6, 2), (4, 3)])
def test_gloo_if_sharded_equals_sequential(total, world):
    """mix_4k (a P_I = 2 Type-2 PLP beside two type-0 PLPs): shards of whole interleaving frames, ragged
    (6 frames over 2 ranks: 4 + 2) and with an empty shard (4 frames over 3 ranks)"""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_if_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get(timeout=5)


class _FakeChain:
    """stands in for dvbt2ll.Chain on the CPU (no HIP): run_device writes placeholder frames (frame k's samples
    all hold k) through the IQ pointer, after checking that the TS slice it was handed is exactly the global
    stream's bytes for its frames"""
    def __init__(self, cfg, max_frames, per=64):
        self.cfg, self.max_frames, self.iq_per_frame, self.unit_frames = cfg, max_frames, per, 1
        self.calls = []

    def run_device(self, ts_ptr, base, n, first, count, iq_ptr, stream):
        import ctypes
        ts = np.ctypeslib.as_array((ctypes.c_uint8 * n).from_address(ts_ptr))
        assert np.array_equal(ts, ts_for_frames(self.cfg, first, count)[0])
        frames = np.repeat(np.arange(first, first + count, dtype=np.float32), self.iq_per_frame * 2)
        ctypes.memmove(iq_ptr, frames.ctypes.data, frames.nbytes)
        self.calls.append((first, count))


def _enc_worker(rank, world, port, total, q):
    import sys
    sys.path[:0] = [os.path.join(os.path.dirname(__file__)),
                    os.path.join(os.path.dirname(__file__), "..", "gr-dvbt2ll_amd")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ch = _FakeChain(CONFIGS["cfg1"], max_frames=total)
        got = D.encode_sharded(ch, 0, total, device="cpu")
        first, count = D.frame_range(total, rank, world)
        assert ch.calls == ([(first, count)] if count else [])   # empty shards launch nothing
        if rank == 0:
            want = np.repeat(np.arange(total, dtype=np.float32), ch.iq_per_frame * 2).reshape(-1, 2)
            q.put(bool(np.array_equal(got.numpy(), want)))
        else:
            assert got is None
    finally:
        dist.destroy_process_group()


def test_gloo_encode_sharded_more_ranks_than_frames():
    """encode_sharded with 3 ranks and 2 frames: rank 2's shard is empty (no launch, no send), the ordered
    gather still delivers both frames to rank 0"""
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_enc_worker, args=(r, 3, port, 2, q)) for r in range(3)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(180)
        assert p.exitcode == 0
    assert q.get(timeout=5)
