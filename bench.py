#!/usr/bin/env python3
"""DVB-T2 transmit-chain benchmark on MI355X (BASELINE.json metric: IQ Msamples/s for the whole
node + FEC blocks/s, 32K-FFT 256-QAM 3/5 = cfg3).

One "step" = the whole hot path (TS bytes -> BBFRAME/BCH/LDPC -> bit interleave/QAM/cell
interleave -> time/frame/frequency interleave + pilots + IFFT + GI + P1) over a batch of
--frames T2 frames per GPU, TS input already resident in HBM, IQ written to HBM.

Multi-GPU: frame-sharded, one process per GPU (torchrun); each rank encodes its own
disjoint T2 frames with closed-form stream state, no data-path collective ("weak" scaling).
Rank 0 prints one JSON line.  Synthetic data: splitmix64 TS packets (dvbt2ll.configs).

Steps are pipelined: the chain handle holds --slots intermediate buffer sets and step s is
issued on HIP stream s % slots (dvbt2ll_chain_set_slots), so consecutive steps overlap on the GPU.

Extra fields: roofline (dominant kernel, HIP-event timed on the launch stream inside a serial
timed pass of the same K steps on one stream -- per-kernel event durations mean nothing under
cross-stream overlap; traffic from rocprofv3 PMC passes run as child processes BEFORE this
process touches the GPU), serial_1_stream (that pass's rate) and cpu_baseline (the oracle C
restatement, single thread, bounded sample).
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import tempfile
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "gr-dvbt2ll_amd"))

RT_SPS = 8e6 * 8 / 7          # real-time IQ rate of the 8 MHz channel (apps/vv009-4kshort.grc:143)
HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
METRIC = "IQ Msamples/sec (whole node) + FEC blocks/sec, 32K-FFT 256-QAM 3/5"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--frames", type=int, default=64, help="T2 frames per step per GPU")
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sc16", action="store_true", help="skip the secondary sc16-output timing")
    ap.add_argument("--no-latency", action="store_true", help="skip the one-frame latency calls")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--shard", choices=("frames", "streams"), default="frames",
                    help="frames: one TS stream, disjoint frame ranges per rank; streams: an independent "
                         "TS stream per rank (seed = rank + 1), SURVEY 8(e)'s two modes")
    ap.add_argument("--slots", type=int, default=2,
                    help="chain buffer slots = HIP streams the steps alternate over (1 = serial)")
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def algorithmic_bytes(cfg, info):
    """SURVEY.md section 8(d) per-frame algorithmic bytes of each stage."""
    from dvbt2ll.configs import KBCH
    F = info["fec_blocks_per_frame"]
    nldpc = 64800 if cfg.framesize == 1 else 16200
    kbch = KBCH[(cfg.framesize, cfg.rate)]
    cs, S, M, IQ = info["cell_size"], info["stream_items"], info["mapped_items"], info["iq_samples_per_frame"]
    s1 = F * ((kbch - 80) // 8 + nldpc // 8)
    s2 = F * (nldpc // 8 + 8 * cs)
    s3 = 8 * S + 8 * M
    s4 = 8 * M + 8 * IQ
    # kernel stages: fec = S1 (+ LDPC), map = S2, ofdm = S3 + S4 (fused)
    return {"fec": s1, "map": s2, "ofdm": s3 + s4}


def pmc_passes(args):
    """rocprofv3 FETCH_SIZE / WRITE_SIZE of the ofdm kernel, one counter set per pass, run as child
    processes before this process initialises the GPU.  Returns per-launch corrected bytes or None."""
    import shutil
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    res = {}
    for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
        d = tempfile.mkdtemp(prefix="t2pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = [rp, "--pmc", ctr, "--kernel-include-regex", "ofdm_kernel", "-T", "-f", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, str(ROOT / "bench.py"), "--pmc-child", "--config", args.config,
               "--frames", str(args.frames), "--steps", "2", "--warmup", "1"]
        try:
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except Exception as e:  # noqa: BLE001
            return None, "rocprofv3 %s pass failed: %s" % (ctr, e)
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        vals = []
        for fn in files:
            import csv
            with open(fn) as fh:
                for row in csv.DictReader(fh):
                    if row.get("Counter_Name") == ctr and "ofdm_kernel" in row.get("Kernel_Name", ""):
                        vals.append(float(row["Counter_Value"]))
        if not vals:
            return None, "no %s rows" % ctr
        res[ctr] = sum(vals) / len(vals)
    # FETCH_SIZE / WRITE_SIZE are in KiB; gfx950 FETCH_SIZE reads half of the streamed bytes
    # (MI355X_MICROARCH.md, HBM section) -> x2 on the read side
    fetch = res["FETCH_SIZE"] * 1024 * 2
    write = res["WRITE_SIZE"] * 1024
    return {"fetch_bytes": fetch, "write_bytes": write, "total": fetch + write}, None


def _oracle_stream(cfg, seconds, max_frames, seed=1):
    """one oracle replica: the five blocks over consecutive T2 frames of one TS stream until the
    time or frame bound; returns (frames, IQ samples, seconds)"""
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    from dvbt2ll.configs import ts_for_frames
    F = cfg.fecblocks
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args()); pg = O.PG(*cfg.pg_args())
    ts, _ = ts_for_frames(cfg, 0, max_frames, seed)
    off, frames, samples = 0, 0, 0
    t0 = time.perf_counter()
    while True:
        bits, cons = bb.work(ts[off:], F)
        off += cons
        cells = im.work(ld.work(bits, F), F)
        iq = pg.work(fm.work(cells))
        frames += 1
        samples += len(iq)
        dt = time.perf_counter() - t0
        if dt >= seconds or frames >= max_frames:
            return frames, samples, dt


def cpu_host_replicas(cfg, seconds, threads):
    """SURVEY 8(d) whole-host figure: `threads` independent oracle stream replicas (one per host
    thread; the oracle's C calls release the GIL), aggregate IQ rate over a common window"""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(threads) as ex:
        t0 = time.perf_counter()
        res = list(ex.map(lambda k: _oracle_stream(cfg, seconds, 64, seed=k + 1), range(threads)))
        dt = time.perf_counter() - t0
    frames = sum(r[0] for r in res)
    rate = sum(r[1] / r[2] for r in res)     # concurrent replicas, each timed over its own frames
    return {"value": rate / 1e6, "unit": "Msamples/s", "cores": threads, "kind": "port",
            "sample": "%d independent %s streams, %d T2 frames in total through the oracle C restatement "
                      "(one replica per thread, each timed over its own frames), %.1f s wall" % (threads, cfg.name, frames, dt),
            "fec_blocks_per_sec": sum(r[0] / r[2] for r in res) * cfg.fecblocks}


def cpu_baseline(cfg, seconds):
    """Oracle C restatement (single thread) over a bounded sample of the same workload."""
    frames, samples, dt = _oracle_stream(cfg, seconds, 64)
    F = cfg.fecblocks
    return {"value": samples / dt / 1e6, "unit": "Msamples/s", "cores": 1, "kind": "port",
            "sample": "%d %s T2 frames (%d FEC blocks) through the oracle C restatement of all five "
                      "blocks, one thread, own radix-2 float IFFT (FFTW unavailable), %.1f s"
                      % (frames, cfg.name, frames * F, dt),
            "fec_blocks_per_sec": frames * F / dt}


def one_frame_latency(chain, ts_dev, ts_meta, iq, streams, per):
    """per-frame latency (the reference's stated aim, README:21-29): one T2 frame per call, TS
    resident in HBM, from the call to the frame's IQ complete in HBM; median / p90 of 20 calls,
    direct launches and hipGraph mode"""
    import torch
    lat = []
    first, base, n = ts_meta[0]
    for k in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        chain.run_device(ts_dev[0].data_ptr(), base, n, first, 1, iq[0].data_ptr(), streams[0].cuda_stream)
        streams[0].synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
    lat = sorted(lat[5:])
    latency = {"median_ms": lat[len(lat) // 2], "p90_ms": lat[int(len(lat) * 0.9)],
               "frame_airtime_ms": per / RT_SPS * 1e3,
               "note": "one T2 frame per run_device call (TS resident, IQ to HBM, host-synchronised); "
                       "not `value`"}
    chain.set_graph(True)          # the same calls as one hipGraph launch each
    lat = []
    for k in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        chain.run_device(ts_dev[0].data_ptr(), base, n, first, 1, iq[0].data_ptr(), streams[0].cuda_stream)
        streams[0].synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
    chain.set_graph(False)
    lat = sorted(lat[5:])
    latency["graph_median_ms"] = lat[len(lat) // 2]
    latency["graph_p90_ms"] = lat[int(len(lat) * 0.9)]
    return latency


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    traffic, pmc_note = None, "skipped"
    if world == 1 and not args.pmc_child and not args.no_pmc:
        traffic, pmc_note = pmc_passes(args)          # before any GPU initialisation here

    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames

    cfg = CONFIGS[args.config]
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    B = args.frames
    chain = dvbt2ll.Chain(cfg, max_frames=B, device=local_rank)
    info = chain.info
    per = chain.iq_per_frame
    # R distinct resident batches per rank; frames split contiguously across ranks
    # (dvbt2ll.distributed.frame_range), disjoint across ranks and batches
    from dvbt2ll.distributed import frame_range
    R = 2
    rank_first, _ = frame_range(world * R * B, rank, world)
    seed = 1
    if args.shard == "streams":
        rank_first, seed = 0, rank + 1
    ts_dev, ts_meta = [], []
    for r in range(R):
        first = rank_first + r * B
        ts, base = ts_for_frames(cfg, first, B, seed)
        ts_dev.append(torch.from_numpy(ts).cuda())
        ts_meta.append((first, base, len(ts)))
    # pipelined steps: the handle holds `slots` intermediate buffer sets and step s is issued on
    # stream s % slots into its own IQ buffer, so one step's kernels fill the CUs the previous
    # step's kernel tails leave idle (dvbt2ll_chain_set_slots); every step still does all the work
    S = max(1, args.slots)
    chain.set_slots(S)
    iq = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(S)]
    streams = [torch.cuda.Stream() for _ in range(S)]
    torch.cuda.synchronize()

    def step(s, serial=False):
        first, base, n = ts_meta[s % R]
        st = streams[0] if serial else streams[s % S]
        chain.run_device(ts_dev[s % R].data_ptr(), base, n, first, B, out[0][s % S].data_ptr(), st.cuda_stream)

    out = [iq]
    for s in range(args.warmup):
        step(s)
    torch.cuda.synchronize()
    if args.pmc_child:
        for s in range(args.steps):
            step(s, serial=True)
        torch.cuda.synchronize()
        return

    def timed(serial=False, timing=False):
        """K steps between barrier + synchronize on both sides; max over ranks"""
        if timing:
            chain.set_timing(True)
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s in range(args.steps):
            step(s, serial)
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        e = time.perf_counter() - t0
        st = None
        if timing:
            st = chain.timing()
            chain.set_timing(False)
        if dist:
            t = torch.tensor([e], dtype=torch.float64, device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            e = float(t.item())
        return e, st

    # the headline: pipelined steps over S streams.  Per-kernel HIP-event durations are only
    # meaningful without cross-stream overlap, so the roofline comes from a serial pass of the same
    # K steps (all on one stream) right after it
    if S > 1:
        elapsed, _ = timed()
        serial_elapsed, (stage_ms, launches) = timed(serial=True, timing=True)
    else:
        elapsed, (stage_ms, launches) = timed(timing=True)
        serial_elapsed = elapsed
    # secondary line (not `value`): the same chain with the flowgraph's output step fused into the
    # IQ store (x0.2 gain, sc16 wire format: 4 B per sample instead of 8)
    sc16 = None
    if not args.no_sc16:
        torch.cuda.synchronize()
        out[0] = [torch.empty((B * per, 2), dtype=torch.int16, device="cuda") for _ in range(S)]
        chain.set_output(0.2, dvbt2ll.IQ_SC16)
        for s in range(S):
            step(s)
        e16, _ = timed()
        _, (ms16, n16) = timed(serial=True, timing=True)
        chain.set_output(1.0, dvbt2ll.IQ_CF32)
        out[0] = iq
        sc16 = {"ms_per_step": e16 / args.steps * 1e3, "elapsed": e16,
                "ofdm_avg_launch_ms": ms16[2] / max(1, n16[2])}
    latency = None
    if not args.no_latency:
        latency = one_frame_latency(chain, ts_dev, ts_meta, iq, streams, per)
    frames_total = B * args.steps * world
    samples_total = frames_total * per
    fec_total = frames_total * info["fec_blocks_per_frame"]
    msps = samples_total / elapsed / 1e6
    if rank == 0:
        ab = algorithmic_bytes(cfg, info)
        stages = {}
        for k, name in enumerate(("fec", "map", "ofdm")):
            avg_ms = stage_ms[k] / max(1, launches[k])
            bytes_launch = ab[name] * B
            stages[name] = {"avg_launch_ms": avg_ms, "algorithmic_bytes_per_launch": bytes_launch,
                            "achieved_GBs": bytes_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else None}
        dom = max(stages, key=lambda n: stages[n]["avg_launch_ms"])
        st = stages[dom]
        roof = {"kernel": dom + "_kernel", "bound": "hbm", "achieved": st["achieved_GBs"], "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": st["achieved_GBs"] / HBM_PEAK_GBS if st["achieved_GBs"] else None,
                "traffic": (traffic["total"] if (traffic and dom == "ofdm") else None),
                "traffic_note": pmc_note if traffic is None else
                "rocprofv3 PMC passes (FETCH_SIZE x1024 x2 gfx950 read correction + WRITE_SIZE x1024), "
                "ofdm_kernel per launch",
                "algorithmic_bytes_per_launch": st["algorithmic_bytes_per_launch"],
                "avg_launch_ms": st["avg_launch_ms"]}
        if roof["traffic"]:
            # what HBM actually carried: the fused kernel never writes or re-reads the cells as
            # complex64 (SURVEY 8(d)'s S3 + S4 stage figures), so its measured traffic is far below
            # the algorithmic bytes and `achieved` can approach or pass the HBM peak
            tgbs = roof["traffic"] / (st["avg_launch_ms"] * 1e-3) / 1e9
            roof["traffic_GBs"] = tgbs
            roof["traffic_frac"] = tgbs / HBM_PEAK_GBS
            roof["note"] = ("achieved = SURVEY 8(d) stage bytes of the unfused S3+S4 pipeline / kernel time, i.e. "
                            "the fused kernel's speed as a fraction of an ideal unfused pipeline at HBM peak; "
                            "traffic_frac = measured HBM bytes / time / peak (the kernel is LDS/VALU-latency "
                            "bound at one 138 KB workgroup per CU, not HBM-bound)")
        out = {
            "metric": METRIC, "value": msps, "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "%s: TS->IQ full DVB-T2 chain, %d T2 frames per step per GPU "
                                   "(%d FEC blocks, %d IQ samples per frame)"
                                   % (cfg.name, B, info["fec_blocks_per_frame"], per),
                       "frames_per_step_per_gpu": B, "slots_streams_per_gpu": S,
                       "parallelism": "%s x%d (no data-path collective)"
                                      % ("frame-sharded" if args.shard == "frames" else "independent streams", world)},
            "fec_blocks_per_sec": fec_total / elapsed,
            "serial_1_stream": {"value": samples_total / serial_elapsed / 1e6,
                                "ms_per_step": serial_elapsed / args.steps * 1e3,
                                "note": "same K steps issued on one stream (no cross-step overlap); the "
                                        "stage timings and roofline come from this pass"},
            "x_realtime": msps * 1e6 / RT_SPS,
            "stages": stages,
            "roofline": roof,
        }
        if sc16:
            out["iq_sc16_x0.2"] = {
                "value": samples_total / sc16["elapsed"] / 1e6, "unit": "Msamples/s",
                "ms_per_step": sc16["ms_per_step"], "ofdm_avg_launch_ms": sc16["ofdm_avg_launch_ms"],
                "note": "secondary: same chain, output gain 0.2 + int16 I/Q store (the flowgraph's "
                        "multiply_const and SDR wire format fused into the IQ store); not `value`"}
        if latency:
            out["latency_1_frame"] = latency
        if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only (host cores are shared)
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
            # the box's CPU share is 16 threads (os.cpu_count() reports the whole machine)
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"]["whole_host"] = cpu_host_replicas(cfg, args.cpu_seconds / 2, threads)
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
