"""Frame sharding across GPUs (one process per GPU, torch.distributed over RCCL).

The chain encodes T2 frame k from closed-form stream state (the absolute FEC-block index fixes
the BBHEADER, the scrambler restarts per BBFRAME, the previous packet's CRC-8 is recomputed from
the TS bytes one packet before the frame), so a contiguous run of frames splits across ranks
with no data-path collective: each rank encodes its own frames from its own slice of the TS.
The only collective is the optional ordered gather of the IQ to one rank (for a sink that
wants the whole stream); the benchmark does not use it.
"""
import torch
import torch.distributed as dist

from .configs import ts_for_frames


def frame_range(total_frames, rank, world, first_frame=0, unit=1):
    """contiguous, ragged-safe split of [first_frame, first_frame + total_frames): (first, count).  unit:
    the chain's launch unit (dvbt2ll_chain_unit_frames: the least common multiple of its PLPs' interleaving-
    frame lengths; a TIME_IL_TYPE 1 PLP's interleaving frame spans P_I T2 frames); every shard is whole units,
    so first_frame and total_frames must be multiples of it"""
    unit = int(unit)
    if total_frames % unit or first_frame % unit:
        raise ValueError("frames [%d, +%d) are not whole launch units of %d T2 frames"
                         % (first_frame, total_frames, unit))
    base, extra = divmod(int(total_frames) // unit, int(world))
    count = base + (1 if rank < extra else 0)
    first = first_frame // unit + rank * base + min(rank, extra)
    return first * unit, count * unit


def gather_frames(local, total_frames, per_frame, group=None, dst=0, unit=1):
    """ordered gather of per-rank frame shards (local: [count * per_frame, ...] tensor) to rank dst,
    the chain's one exchange step: RCCL has no gather primitive, so every other rank
    sends its shard point-to-point (one grouped batch of isend / irecv, ncclGroupStart/End under the
    nccl backend) straight into its place in dst's output.  dst receives world - 1 shards, the
    other ranks receive nothing.  Returns the [total_frames * per_frame, ...] tensor on dst, None
    elsewhere; empty shards (more ranks than frames) send nothing (verified under gloo; the RCCL
    empty-shard case has not run on a multi-GPU node)."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    counts = [frame_range(total_frames, r, world, unit=unit)[1] for r in range(world)]
    firsts = [frame_range(total_frames, r, world, unit=unit)[0] for r in range(world)]
    assert local.shape[0] == counts[rank] * per_frame, "shard size mismatch"
    # every rank joins one collective first: under RCCL a grouped send/recv that is the group's
    # first operation and leaves some ranks out (empty shards) is undefined
    sync = torch.zeros(1, dtype=torch.int32, device=local.device)
    dist.all_reduce(sync, group=group)

    def peer(r):
        return dist.get_global_rank(group, r) if group is not None else r

    if rank != dst:
        if counts[rank]:
            for req in dist.batch_isend_irecv([dist.P2POp(dist.isend, local.contiguous(), peer(dst), group)]):
                req.wait()
        return None
    out = torch.empty((total_frames * per_frame,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    out[firsts[rank] * per_frame:(firsts[rank] + counts[rank]) * per_frame] = local
    ops = [dist.P2POp(dist.irecv, out[firsts[r] * per_frame:(firsts[r] + counts[r]) * per_frame], peer(r), group)
           for r in range(world) if r != dst and counts[r]]
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()
    return out


def encode_sharded(chain, first_frame, total_frames, group=None, gather=True, seed=1, device="cuda"):
    """each rank encodes its contiguous share of the frames -- whole launch units (interleaving frames) --
    on its own GPU (synthetic TS slice generated for exactly those frames; a multi-PLP chain's PLP k uses
    seed + k); optional ordered gather of the IQ to rank 0."""
    from .configs import MplpConfig
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    unit = getattr(chain, "unit_frames", 1)
    first, count = frame_range(total_frames, rank, world, first_frame, unit)
    per = chain.iq_per_frame
    iq = torch.zeros((count * per, 2), dtype=torch.float32, device=device)
    if count:
        if count > chain.max_frames:
            raise ValueError("shard of %d frames exceeds chain max_frames %d" % (count, chain.max_frames))
        st = torch.cuda.current_stream().cuda_stream if device != "cpu" else 0
        if isinstance(chain.cfg, MplpConfig):
            tss = [ts_for_frames(p, first, count, seed + k) for k, p in enumerate(chain.cfg.plps)]
            bufs = [torch.from_numpy(ts).to(device) for ts, _ in tss]
            chain.run_plps([b.data_ptr() for b in bufs], [b for _, b in tss], [len(t) for t, _ in tss], first, count,
                           iq.data_ptr(), st)
        else:
            ts, base = ts_for_frames(chain.cfg, first, count, seed)
            ts_d = torch.from_numpy(ts).to(device)
            chain.run_device(ts_d.data_ptr(), base, len(ts), first, count, iq.data_ptr(), st)
    if not gather:
        return iq
    return gather_frames(iq, total_frames, per, group, unit=unit)
