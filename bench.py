#!/usr/bin/env python3
"""DVB-T2 transmit-chain benchmark on MI355X (BASELINE.json metric: IQ Msamples/s for the whole
node + FEC blocks/s, 32K-FFT 256-QAM 3/5 = cfg3).

One "step" = the whole hot path (TS bytes -> BBFRAME/BCH/LDPC -> bit interleave/QAM/cell
interleave -> time/frame/frequency interleave + pilots + IFFT + GI + P1) over a batch of
--frames T2 frames per GPU, TS input already resident in HBM, IQ written to HBM.

Multi-GPU: frame-sharded, one process per GPU; each rank encodes its own disjoint T2 frames with
closed-form stream state, no data-path collective ("weak" scaling).  `--gpus N` under torchrun
(WORLD_SIZE set) checks WORLD_SIZE == N; without it, this process spawns the N rank processes
itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set, after its PMC passes and before anything
touches the GPU) and relays rank 0's line.  `--dry-run` (gloo, no HIP) exercises the same spawn ->
frame_range -> barrier -> all_reduce -> gather_frames path on CPU.  Rank 0 prints one JSON line.
Synthetic data: splitmix64 TS packets (dvbt2ll.configs).

Steps are pipelined: the chain handle holds --slots intermediate buffer sets and step s is
issued on HIP stream s % slots (dvbt2ll_chain_set_slots), so consecutive steps overlap on the GPU.

Extra fields: roofline (dominant kernel, HIP-event timed on the launch stream inside a serial
timed pass of the same K steps on one stream -- per-kernel event durations mean nothing under
cross-stream overlap; traffic from rocprofv3 PMC passes run as child processes BEFORE this
process touches the GPU), serial_1_stream (that pass's rate) and cpu_baseline (the oracle C
restatement, single thread, bounded sample).
"""
import argparse
import datetime
import glob
import json
import os
import re
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
    ap.add_argument("--frames", type=int, default=1280,
                    help="T2 frames per step per GPU (1280 cfg3 frames = 293 s of airtime; at most 1359 per cfg3 "
                         "launch; 640 / 768 / 896 / 1152 / 1280 / 1344 frames per step measured 218.6 / 223.6 / "
                         "223.6 / 227.6 / 227.4 / 227.7 G IQ samples/s on one box, profiles/r4_frames_sweep.txt)")
    ap.add_argument("--config", default="cfg3")
    ap.add_argument("--no-pmc", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sc16", action="store_true", help="skip the secondary sc16-output timing")
    ap.add_argument("--no-latency", action="store_true", help="skip the one-frame latency calls")
    ap.add_argument("--no-blocks", action="store_true", help="skip the per-block general_work timing")
    ap.add_argument("--no-mplp", action="store_true", help="skip the secondary multi-PLP (2-PLP 32K frame) timing")
    ap.add_argument("--no-host", action="store_true", help="skip the secondary host-delivered (streaming host path) "
                                                           "timing")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--shard", choices=("frames", "streams"), default="frames",
                    help="frames: one TS stream, disjoint frame ranges per rank; streams: an independent "
                         "TS stream per rank (seed = rank + 1), SURVEY 8(e)'s two modes")
    ap.add_argument("--slots", type=int, default=3,
                    help="chain buffer slots = HIP streams the steps alternate over (1 = serial); at 1280 frames "
                         "per step 3 slots measured +1.5 %% over 2 (profiles/r4_frames_sweep.txt)")
    ap.add_argument("--streams", type=int, default=1,
                    help="independent TS streams per launch (seeds 1..S, dvbt2ll_chain_run_streams; BASELINE cfg4 "
                         "x4 / cfg5 x8): each step encodes --frames // S frames of every stream")
    ap.add_argument("--dry-run", action="store_true",
                    help="no HIP: exercise the multi-rank spawn / frame sharding / barrier / all_reduce / "
                         "ordered gather path with placeholder frames (CPU tensors, gloo)")
    ap.add_argument("--backend", default=None, help="torch.distributed backend (default nccl = RCCL; gloo for "
                                                    "--dry-run)")
    ap.add_argument("--rank-timeout", type=float, default=1500.0,
                    help="spawned ranks: seconds before the parent ends a run that has not finished")
    ap.add_argument("--init-timeout", type=float, default=600.0,
                    help="seconds init_process_group and the first barrier may take")
    ap.add_argument("--fail-rank", type=int, default=-1, help=argparse.SUPPRESS)   # tests: this rank exits at init
    ap.add_argument("--pmc-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


def algorithmic_bytes(cfg, info):
    """SURVEY.md section 8(d) per-frame algorithmic bytes of each stage (the standalone-pass HBM
    traffic of an unfused S1..S4 pipeline; the fused kernels report against these as a second,
    separately named figure)."""
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


def minimal_bytes(cfg, info, iq_bytes=8):
    """per-frame bytes each kernel stage of the fused chain must move through HBM at least:
    fec (the fused BB + BCH pass) reads the TS payload and writes the BBFRAMEs and their BCH parity;
    map (the LDPC + map kernel) reads those and writes one 2-byte constellation index pair per cell;
    ofdm reads the pairs and writes the IQ samples (per-symbol tables are shared by every frame of a
    launch and are not counted)"""
    from dvbt2ll.configs import KBCH
    F = info["fec_blocks_per_frame"]
    nldpc = 64800 if cfg.framesize == 1 else 16200
    kbch = KBCH[(cfg.framesize, cfg.rate)]
    cs, S, IQ = info["cell_size"], info["stream_items"], info["iq_samples_per_frame"]
    # BCH parity bits: 168 (short), 160 (normal 2/3, 5/6), 192 (the other normal codes)
    nbch = kbch + (168 if cfg.framesize == 0 else 160 if cfg.rate in (2, 5) else 192)
    return {"fec": F * ((kbch - 80) // 8 + nbch // 8), "map": F * (nbch // 8 + 2 * cs),
            "ofdm": 2 * S + iq_bytes * IQ}


KERNELS = ("fec", "map", "ofdm")
# the kernels each stage launches per step: fec = the fused BB + BCH pass (BBFRAME from the TS, BCH parity on the
# matrix cores), map = the LDPC + map kernel (LDPC parity, bit interleaver, cell + time interleaver; with the
# frames' L1-post workgroups)
STAGE_KERNELS = {"fec": ("bbch",), "map": ("ldpc_map",), "ofdm": ("ofdm",)}
# rocprofv3 FETCH_SIZE / WRITE_SIZE (KiB) -> bytes.  gfx950 tallies 128-B read requests at 64 B
# (MI355X_MICROARCH.md, HBM): x2 on the read side, calibrated per access width by tools/fetch_calib
# (profiles/r2_fetch_calib.json); the kernels' dominant access widths: fec 16-B TS staging / BBFRAME
# loads and 16-B BBFRAME stores, map 16-B BBFRAME loads and 8-B index-pair quad stores, ofdm 16-B
# data-slot loads and 16-B IQ stores (two samples per lane)
LOAD_WIDTH = {"fec": 16, "map": 16, "ofdm": 16}
STORE_WIDTH = {"fec": 16, "map": 8, "ofdm": 16}


def _calibration():
    f = ROOT / "profiles" / "r2_fetch_calib.json"
    try:
        return json.loads(f.read_text())
    except Exception:  # noqa: BLE001
        return {}


def pmc_passes(args):
    """rocprofv3 passes (one counter set each, run as child processes before this process initialises
    the GPU): FETCH_SIZE, WRITE_SIZE and the SQ instruction counts of the three kernels.  Returns
    ({kernel: {counter: mean per launch}}, note)."""
    import shutil
    import csv
    rp = shutil.which("rocprofv3")
    if rp is None:
        return None, "rocprofv3 not found"
    res = {k: {} for k in KERNELS}
    names = set()
    for ctrs in (["FETCH_SIZE"], ["WRITE_SIZE"], ["SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_LDS"]):
        d = tempfile.mkdtemp(prefix="t2pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        # (no --kernel-include-regex: with it rocprofv3 7.2 dropped ofdm32_kernel's dispatches; kernels are
        # matched by name below)
        cmd = [rp, "--pmc", *ctrs, "-T", "-f", "csv", "-d", d,
               "-o", "pmc", "--", sys.executable, str(ROOT / "bench.py"), "--pmc-child", "--config", args.config,
               "--frames", str(args.frames), "--streams", str(args.streams), "--steps", "2", "--warmup", "1"]
        try:
            subprocess.run(cmd, check=True, timeout=240, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        except Exception as e:  # noqa: BLE001
            return None, "rocprofv3 %s pass failed: %s" % (ctrs, e)
        vals = {}
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as fh:
                for row in csv.DictReader(fh):
                    kn = row.get("Kernel_Name", "")
                    names.add(kn[:60])
                    m = re.search(r"\b(bbch|ldpc_map|fec|map|ofdm)(32)?_kernel", kn)
                    if m and row.get("Counter_Name") in ctrs:
                        vals.setdefault((m.group(1), row["Counter_Name"]), []).append(float(row["Counter_Value"]))
        # per-launch means (a stage with several kernels adds their means)
        for (kn, c), v in vals.items():
            k = next((st for st, kns in STAGE_KERNELS.items() if kn in kns), kn)
            res[k][c] = res[k].get(c, 0.0) + sum(v) / len(v)
        shutil.rmtree(d, ignore_errors=True)
    cal = _calibration()
    for k in KERNELS:
        r = res[k]
        if "FETCH_SIZE" not in r or "WRITE_SIZE" not in r:
            r["kernel_names_seen"] = sorted(names)   # diagnostic: what the PMC pass recorded
        if "FETCH_SIZE" in r and "WRITE_SIZE" in r:
            fr = cal.get("FETCH_SIZE rd %dB" % LOAD_WIDTH[k], 0.5)
            wr = cal.get("WRITE_SIZE wr %dB" % STORE_WIDTH[k], 1.0)
            r["fetch_bytes"] = r["FETCH_SIZE"] * 1024 / fr
            r["write_bytes"] = r["WRITE_SIZE"] * 1024 / wr
            r["hbm_bytes"] = r["fetch_bytes"] + r["write_bytes"]
            r["fetch_write_bytes"] = [r["fetch_bytes"], r["write_bytes"]]
            r["calibration"] = {"fetch_counter_per_byte": fr, "write_counter_per_byte": wr,
                                "source": "profiles/r2_fetch_calib.json" if cal else "MI355X_MICROARCH.md default"}
    return res, None


VALU_ISSUE_PEAK = 256 * 4 * 2.4e9 / 2   # wave-instructions/s: 256 CUs x 4 SIMDs, one wave64 VALU op per 2 cycles


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


def cpu_stage_times(cfg, seconds, max_frames=64, seed=1):
    """per-frame time of each reference block restated in the oracle (bbheaderbch, ldpc,
    interleavermod, framemapperfint, pilotgenp1insert), one thread, over consecutive frames of one
    stream until the time bound; plus the FFTW-class variant of the pilotgen stage: its carrier
    fill (oracle) + numpy's single-precision pocketfft IFFT, scale and guard interval instead of
    the oracle's radix-2 IFFT (FFTW is absent)"""
    import numpy as np
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    from dvbt2ll.configs import ts_for_frames
    F = cfg.fecblocks
    bb = O.BB(*cfg.bb_args()); ld = O.LDPC(cfg.framesize, cfg.rate); im = O.IM(*cfg.im_args())
    fm = O.FM(*cfg.fm_args()); pg = O.PG(*cfg.pg_args())
    N, G, nrm = pg.vlength, pg.guard, np.float32(pg.normalization)
    ts, _ = ts_for_frames(cfg, 0, max_frames, seed)
    tot = dict.fromkeys(("bbheaderbch", "ldpc", "interleavermod", "framemapperfint", "pilotgenp1insert",
                         "pilotgen_fill", "pocketfft_ifft_gi"), 0.0)
    off, frames, samples = 0, 0, 0
    t_start = time.perf_counter()
    while True:
        t0 = time.perf_counter()
        bits, cons = bb.work(ts[off:], F)
        t1 = time.perf_counter()
        cw = ld.work(bits, F)
        t2 = time.perf_counter()
        cells = im.work(cw, F)
        t3 = time.perf_counter()
        mapped = fm.work(cells)
        t4 = time.perf_counter()
        iq = pg.work(mapped)
        t5 = time.perf_counter()
        car = pg.carriers(mapped)
        t6 = time.perf_counter()
        x = np.fft.ifft(np.fft.ifftshift(car, axes=1), axis=1) * np.float32(N) * nrm
        out = np.concatenate([x[:, N - G:], x], axis=1)
        t7 = time.perf_counter()
        assert out.dtype == np.complex64
        off += cons
        for k, dt in zip(tot, (t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5, t7 - t6)):
            tot[k] += dt
        frames += 1
        samples += len(iq)
        if time.perf_counter() - t_start >= seconds or frames >= max_frames:
            break
    per = {k: v / frames for k, v in tot.items()}
    return per, frames, samples // frames


def cpu_config_figures(cfg, seconds):
    """SURVEY 8(d)'s CPU figures for one config: single-thread sequential chain (sum of the block
    times), GR-style pipelined (one thread per block, throughput = 1 / slowest block), each with the
    oracle's radix-2 IFFT and with the FFTW-class pocketfft IFFT; Msamples/s, FEC blocks/s, x RT"""
    per, frames, iq = cpu_stage_times(cfg, seconds)
    blocks = ("bbheaderbch", "ldpc", "interleavermod", "framemapperfint", "pilotgenp1insert")
    fast = dict(per)
    fast["pilotgenp1insert"] = per["pilotgen_fill"] + per["pocketfft_ifft_gi"]

    def fig(times, pipelined):
        t = max(times[b] for b in blocks) if pipelined else sum(times[b] for b in blocks)
        return {"msps": iq / t / 1e6, "fec_blocks_per_sec": cfg.fecblocks / t, "x_realtime": iq / t / RT_SPS}
    return {"frames": frames, "stage_ms_per_frame": {k: v * 1e3 for k, v in per.items()},
            "sequential_radix2": fig(per, False), "sequential_pocketfft": fig(fast, False),
            "gr_pipelined_5_threads_radix2": fig(per, True), "gr_pipelined_5_threads_pocketfft": fig(fast, True)}


def cpu_baseline(cfg, seconds, all_configs=True):
    """Oracle C restatement (single thread) over a bounded sample of the same workload; per-config
    figures for every BASELINE config beside it."""
    from dvbt2ll.configs import CONFIGS
    main = cpu_config_figures(cfg, seconds)
    seq = main["sequential_radix2"]
    out = {"value": seq["msps"], "unit": "Msamples/s", "cores": 1, "kind": "port",
           "sample": "%d %s T2 frames (%d FEC blocks) through the oracle C restatement of all five "
                     "blocks, one thread, own radix-2 float IFFT (FFTW unavailable)"
                     % (main["frames"], cfg.name, main["frames"] * cfg.fecblocks),
           "fec_blocks_per_sec": seq["fec_blocks_per_sec"], "x_realtime": seq["x_realtime"],
           "figures": main}
    if all_configs:
        out["per_config"] = {n: cpu_config_figures(c, 2.0) for n, c in CONFIGS.items() if c is not cfg}
    return out


def iq_accuracy(names):
    """IQ error of one T2 frame per config against a float64 IFFT of the oracle's carriers, for the
    GPU chain, the oracle's own float32 radix-2 IFFT (its restatement of pilotgen's FFTW path) and numpy's float32
    pocketfft (an FFTW-class float FFT); max and mean over the frame's symbols of ||y - x|| / ||x||.  Runs only
    with the CPU baseline (the oracle is the checker here, never the measured path)."""
    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames
    sys.path.insert(0, str(ROOT / "tests"))
    import oracle_lib as O
    import iq_check
    res = {}
    for name in names:
        cfg = CONFIGS[name]
        ch = dvbt2ll.Chain(cfg, max_frames=1)
        ts, base = ts_for_frames(cfg, 0, 1)
        ts_d = torch.from_numpy(ts).cuda()
        iq_d = torch.empty((ch.iq_per_frame, 2), dtype=torch.float32, device="cuda")
        ch.run_device(ts_d.data_ptr(), base, len(ts), 0, 1, iq_d.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        iq = iq_d.cpu().numpy().view(np.complex64).reshape(-1)
        F = cfg.fecblocks
        bits, _ = O.BB(*cfg.bb_args()).work(ts, F)
        cells = O.IM(*cfg.im_args()).work(O.LDPC(cfg.framesize, cfg.rate).work(bits, F), F)
        pg = O.PG(*cfg.pg_args())
        mapped = O.FM(*cfg.fm_args()).work(cells)
        car, oiq = pg.carriers(mapped), pg.work(mapped)
        N, G, norm = pg.vlength, pg.guard, pg.normalization
        g, o, f = [], [], []
        for j in range(car.shape[0]):
            lo, hi = 2048 + j * (N + G), 2048 + (j + 1) * (N + G)
            want = iq_check.symbol_reference(car[j], N, G, norm)
            g.append(iq_check.errors(iq[lo:hi], want)[0])
            o.append(iq_check.errors(oiq[lo:hi], want)[0])
            f.append(iq_check.f32_reference_errors(car[j], N, G, norm, want)[0])
        res[name] = {"fft_size": N, "symbols": len(g), "gpu_rel_rms_max": max(g), "gpu_rel_rms_mean": sum(g) / len(g),
                     "oracle_f32_radix2_rel_rms_max": max(o), "oracle_f32_radix2_rel_rms_mean": sum(o) / len(o),
                     "pocketfft_f32_rel_rms_max": max(f), "pocketfft_f32_rel_rms_mean": sum(f) / len(f),
                     "gpu_over_pocketfft_mean": (sum(g) / len(g)) / (sum(f) / len(f))}
        del ch
    return {"per_config": res,
            "note": "rel RMS error of one T2 frame's symbols against a float64 IFFT of the oracle's carriers: the GPU "
                    "chain, the oracle's own float32 radix-2 IFFT and numpy's float32 pocketfft (SURVEY 8(c) bound "
                    "1e-6)"}


def per_block_rate(cfg, frames=6, pinned=False):
    """the drop-in path GNU Radio would drive: the five blocks' C-ABI general_work calls on host
    buffers (pageable numpy, or page-locked with `pinned`: the DMA then reads / writes the caller's
    buffers directly), one T2 frame per framemapper / pilotgen call, each call synchronous
    (H2D + kernels + D2H); secondary figure, not `value`"""
    import numpy as np
    import dvbt2ll
    from dvbt2ll.configs import ts_for_frames
    F = cfg.fecblocks
    bb = dvbt2ll.bbheaderbch_bb(*cfg.bb_args()); ld = dvbt2ll.ldpc_bb(cfg.framesize, cfg.rate)
    im = dvbt2ll.interleavermod_bc(*cfg.im_args()); fm = dvbt2ll.framemapperfint_cc(*cfg.fm_args())
    pg = dvbt2ll.pilotgenp1insert_cc(*cfg.pg_args())
    nbch, nldpc, cs = bb.output_multiple(), ld.output_multiple(), im.output_multiple()

    def host(n, dt):
        if not pinned:
            return np.zeros(n, dt)
        import torch
        tdt = {np.uint8: torch.uint8, np.complex64: torch.complex64}[dt]
        return torch.zeros(n, dtype=tdt).pin_memory().numpy()
    bits = host(F * nbch, np.uint8); cw = host(F * nldpc, np.uint8)
    cells = host(F * cs, np.complex64); mapped = host(fm.output_multiple(), np.complex64)
    iq = host(pg.output_multiple(), np.complex64)
    ts, _ = ts_for_frames(cfg, 0, frames + 1)
    if pinned:
        tsp = host(len(ts), np.uint8)
        tsp[:] = ts
        ts = tsp
    off = 0
    names = ("bbheaderbch", "ldpc", "interleavermod", "framemapperfint", "pilotgenp1insert")
    tot = dict.fromkeys(names, 0.0)
    t_all = 0.0
    for k in range(frames + 1):
        t = [time.perf_counter()]
        bb.general_work([ts[off:]], [bits]); off += bb.last_consumed; t.append(time.perf_counter())
        ld.general_work([bits], [cw]); t.append(time.perf_counter())
        im.general_work([cw], [cells]); t.append(time.perf_counter())
        fm.general_work([cells], [mapped]); t.append(time.perf_counter())
        pg.general_work([mapped], [iq]); t.append(time.perf_counter())
        if k:                               # frame 0 is the warm-up
            for i, n in enumerate(names):
                tot[n] += t[i + 1] - t[i]
            t_all += t[-1] - t[0]
    per = len(iq)
    hbytes = (len(ts) // (frames + 1) + 2 * bits.nbytes + 2 * cw.nbytes + 2 * cells.nbytes + 2 * mapped.nbytes
              + iq.nbytes)
    return {"value": frames * per / t_all / 1e6, "unit": "Msamples/s", "frames": frames,
            "ms_per_frame": {n: v / frames * 1e3 for n, v in tot.items()},
            "x_realtime": frames * per / t_all / RT_SPS,
            "host_bytes_per_frame": hbytes, "pcie_GBs": hbytes * frames / t_all / 1e9,
            "host_buffers": "pinned" if pinned else "pageable",
            "note": "secondary: the per-block drop-in path (bbheaderbch -> ldpc -> interleavermod -> "
                    "framemapperfint -> pilotgenp1insert general_work through the C ABI on %s host "
                    "buffers, synchronous per call, one stream); PCIe-bound (the blocks exchange unpacked "
                    "bits and complex64 cells, as the reference's streams do), not `value`"
                    % ("page-locked" if pinned else "pageable")}


def one_frame_latency(chain, ts_dev, ts_meta, iq, streams, per):
    """per-frame latency (the reference's stated aim, README:21-29): one T2 frame per call, TS
    resident in HBM, from the call to the frame's IQ complete in HBM; median / p90 of 20 calls,
    direct launches and hipGraph mode"""
    import torch
    lat = []
    first, base, n, _ = ts_meta[0]
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
    lat = sorted(lat[5:])
    latency["graph_median_ms"] = lat[len(lat) // 2]
    latency["graph_p90_ms"] = lat[int(len(lat) * 0.9)]
    # a different frame each call: the graph's kernel arguments change, so every call rewrites its nodes
    # (hipGraphExecKernelNodeSetParams); the calls above repeat one frame and skip that
    lat = []
    for k in range(25):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        chain.run_device(ts_dev[0].data_ptr(), base, n, first + k, 1, iq[0].data_ptr(), streams[0].cuda_stream)
        streams[0].synchronize()
        lat.append((time.perf_counter() - t0) * 1e3)
    chain.set_graph(False)
    lat = sorted(lat[5:])
    latency["graph_new_args_median_ms"] = lat[len(lat) // 2]
    return latency


def mplp_rate(frames, steps, warmup, name="mplp2_32k"):
    """secondary (not `value`): a T2 frame carrying two Type-1 data PLPs of cfg3's
    frame geometry -- 100 FEC blocks of 256-QAM 3/5 rotated + 70 of 64-QAM 2/3, each PLP its own TS --
    through the fused chain (dvbt2ll_chain_run_plps), TS resident in HBM, K steps on one stream"""
    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import MPLP_CONFIGS, ts_for_frames
    m = MPLP_CONFIGS[name]
    ch = dvbt2ll.Chain(m, max_frames=frames)
    per = ch.iq_per_frame
    bufs, bases, lens = [], [], []
    for k, p in enumerate(m.plps):
        ts, base = ts_for_frames(p, 0, frames, seed=k + 1)
        bufs.append(torch.from_numpy(ts).cuda())
        bases.append(base)
        lens.append(len(ts))
    iq = torch.empty((frames * per, 2), dtype=torch.float32, device="cuda")
    st = torch.cuda.Stream()
    ptrs = [b.data_ptr() for b in bufs]

    def step():
        ch.run_plps(ptrs, bases, lens, 0, frames, iq.data_ptr(), st.cuda_stream)
    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    ch.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ms, n = ch.timing()
    ch.set_timing(False)
    fec = frames * sum(p.fecblocks for p in m.plps) * steps
    return {"value": frames * per * steps / dt / 1e6, "unit": "Msamples/s", "ms_per_step": dt / steps * 1e3,
            "fec_blocks_per_sec": fec / dt, "frames_per_step": frames, "plps": m.nplp,
            "workload": m.name + ": %d T2 frames per step, PLPs %s" % (frames, [
                "%d FEC blocks %s" % (p.fecblocks, ("QPSK", "16QAM", "64QAM", "256QAM")[p.constellation])
                for p in m.plps]),
            "stage_avg_launch_ms": {k: ms[i] / max(1, n[i]) for i, k in enumerate(("fec", "map", "ofdm"))},
            "note": "secondary: multi-PLP frames (parity unpinned beyond one PLP: the reference carries one); "
                    "one stream, no cross-step overlap; not `value`"}


def pcie_peaks(nbytes=1 << 30, reps=5):
    """page-locked copy rates of this box (GB/s): device -> host, host -> device, and both at once on two
    streams (the denominators of host_delivered's fractions)"""
    import torch
    dev = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    host = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    dev2 = torch.empty(nbytes, dtype=torch.uint8, device="cuda")
    host2 = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()

    def rate(fn):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return reps * nbytes / (time.perf_counter() - t0) / 1e9

    def both():
        with torch.cuda.stream(s1):
            host.copy_(dev, non_blocking=True)
        with torch.cuda.stream(s2):
            dev2.copy_(host2, non_blocking=True)
    d2h = rate(lambda: host.copy_(dev, non_blocking=True))
    h2d = rate(lambda: dev.copy_(host, non_blocking=True))
    bidir = rate(both)
    del dev, dev2, host, host2
    return {"d2h_GBs": d2h, "h2d_GBs": h2d, "bidirectional_GBs_each_way": bidir,
            "note": "1 GiB page-locked copies, torch (hipMemcpyAsync), %d reps each" % reps}


def host_delivered(cfg, chunk, chunks, peaks):
    """secondary (not `value`): the streaming host path -- host TS in, host IQ out -- through
    dvbt2ll_chain_host_submit / _host_wait (a ring of DVBT2LL_HOST_RING submissions on copy-in / compute /
    copy-out streams), page-locked buffers, chunk frames per submission, the sink's ring of three host IQ
    buffers recycled as a sink would consume them; cf32 and sc16 (x0.2).  Rates are samples delivered
    into host memory per second of wall time, PCIe bytes moved per second, and their fraction of the box's
    page-locked D2H copy rate"""
    import torch
    import dvbt2ll
    from dvbt2ll.configs import ts_for_frames
    ch = dvbt2ll.Chain(cfg, max_frames=chunk)
    per = ch.iq_per_frame
    n = chunk * chunks
    ts, base = ts_for_frames(cfg, 0, n)
    ts_pin = torch.from_numpy(ts).pin_memory()
    out = {}
    for fmt, name in ((dvbt2ll.IQ_CF32, "cf32"), (dvbt2ll.IQ_SC16, "sc16_x0.2")):
        ch.set_output(0.2 if fmt == dvbt2ll.IQ_SC16 else 1.0, fmt)
        sb = 4 if fmt == dvbt2ll.IQ_SC16 else 8
        ring = [torch.empty(chunk * per * sb, dtype=torch.uint8).pin_memory() for _ in range(3)]

        def run(k0, k1):
            t = []
            for k in range(k0, k1):
                if k - k0 >= 3:
                    ch.host_wait(t[k - k0 - 3])             # the sink has taken that buffer
                t.append(ch.host_submit(ts_pin.data_ptr(), base, len(ts), k * chunk, chunk,
                                        ring[k % 3].data_ptr()))
            ch.host_wait(t[-1])
        run(0, 3)                                           # warm-up: buffers, first-touch
        t0 = time.perf_counter()
        run(0, chunks)
        dt = time.perf_counter() - t0
        samples = n * per
        d2h = samples * sb
        h2d = len(ts)
        out[name] = {"value": samples / dt / 1e6, "unit": "Msamples/s", "seconds": dt,
                     "d2h_GBs": d2h / dt / 1e9, "h2d_GBs": h2d / dt / 1e9,
                     "frac_of_d2h_peak": d2h / dt / 1e9 / peaks["d2h_GBs"] if peaks else None}
        del ring
    out.update({"frames": n, "frames_per_submission": chunk, "workload": cfg.name,
                "pcie_peaks": peaks,
                "note": "secondary: host TS -> host IQ through the streaming ring (page-locked buffers, overlapped "
                        "copy-in / kernels / copy-out); PCIe-bound, never `value`"})
    return out


def hbm_footprint(info, B, S, R, world, ts_len, sc16, gather_frames):
    """bytes the bench allocates in HBM per rank (rank 0 holds the gather's output too): the chain's S buffer
    slots (codewords, BCH partials, index pairs, L1 cells), S complex64 IQ buffers (+ S sc16 ones while the
    sc16 pass runs), R resident TS batches, and rank 0's gathered IQ"""
    F = info["fec_blocks_per_frame"]
    slot = F * B * (info["cw_stride_bytes"] + 32) + (info["stream_items"] + 8) * B * 2 + B * 8 * 2048
    iq = B * info["iq_samples_per_frame"] * 8
    total = S * slot + S * iq + R * ts_len
    if sc16:
        total += S * iq // 2
    if world > 1:
        total += world * gather_frames * info["iq_samples_per_frame"] * 8
    return total


HBM_BYTES = 288e9   # MI355X HBM3E per GPU


def metric_for(cfg_name):
    """BASELINE.json's metric string for cfg3 (the configuration it is quoted on); the same metric
    named by its configuration for the others"""
    if cfg_name == "cfg3":
        return METRIC
    from dvbt2ll.configs import CONFIGS
    return "IQ Msamples/sec (whole node) + FEC blocks/sec, " + CONFIGS[cfg_name].name


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def spawn_ranks(args):
    """`bench.py --gpus N` outside torchrun: the PMC passes (child processes on one GPU; per-launch
    traffic does not depend on N under weak scaling), then N rank processes of this script with
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT set -- started before this process
    touches the GPU (it never does) -- and rank 0's JSON line relayed.  Any rank failing fails the run."""
    n = args.gpus
    env0 = dict(os.environ)
    if not args.dry_run and not args.no_pmc:
        traffic, note = pmc_passes(args)
        fd, path = tempfile.mkstemp(prefix="t2pmc_", suffix=".json", dir=os.environ.get("TMPDIR", "/tmp"))
        with os.fdopen(fd, "w") as fh:
            json.dump({"traffic": traffic, "note": note}, fh)
        env0["DVBT2LL_BENCH_PMC_JSON"] = path
    port = _free_port()
    procs = []
    outs = [tempfile.TemporaryFile(mode="w+") for _ in range(n)]
    for r in range(n):
        env = dict(env0, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), DVBT2LL_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, str(ROOT / "bench.py")] + sys.argv[1:], env=env,
                                      stdout=outs[r], text=True))
    # poll every rank: the first one to exit non-zero ends the run (the survivors would otherwise sit
    # in init_process_group or a barrier until the backend timeout); this parent never touches the GPU,
    # so terminating its children is safe
    deadline = time.monotonic() + args.rank_timeout
    rcs = [None] * n
    while any(c is None for c in rcs):
        rcs = [p.poll() for p in procs]
        failed = [c for c in rcs if c not in (None, 0)]
        if failed or time.monotonic() > deadline:
            for p in procs:
                if p.poll() is None:
                    p.terminate()
            for p in procs:
                try:
                    p.wait(timeout=20)
                except subprocess.TimeoutExpired:
                    p.kill()
                    p.wait()
            rcs = [p.returncode for p in procs]
            if not failed:
                sys.stderr.write("bench.py: ranks still running after %.0f s (--rank-timeout)\n" % args.rank_timeout)
            break
        time.sleep(0.1)
    if env0.get("DVBT2LL_BENCH_PMC_JSON"):
        os.unlink(env0["DVBT2LL_BENCH_PMC_JSON"])
    outs[0].seek(0)
    out0 = outs[0].read()
    if any(rcs) or any(c is None for c in rcs):
        sys.stderr.write("bench.py: rank exit codes %s\n" % rcs)
        sys.stderr.write(out0[-2000:])
        return max([1] + [abs(c) for c in rcs if c])
    for line in out0.splitlines():        # rank 0's JSON line to stdout, its other output to stderr
        (sys.stdout if line.startswith("{") else sys.stderr).write(line + "\n")
    sys.stdout.flush()
    return 0


def shard_plan(shard, B, NS, R, rank, world):
    """each rank's R resident batches: (first frame, frames per stream, TS stream seeds).  shard "frames": one
    TS stream per launch slot k (seed k + 1), the frames split contiguously across ranks and batches
    (dvbt2ll.distributed.frame_range), disjoint; shard "streams": rank r encodes its own NS independent
    streams (seeds r NS + 1 .. r NS + NS) from frame 0 -- SURVEY 8(e)'s two modes.  NS > 1: one launch
    encodes B // NS frames of each of NS streams (dvbt2ll_chain_run_streams)"""
    from dvbt2ll.distributed import frame_range
    if B % NS:
        raise SystemExit("--frames must be a multiple of --streams")
    BS = B // NS
    if shard == "streams":
        first0, seed = 0, rank * NS + 1
    else:
        first0, seed = frame_range(world * R * BS, rank, world)[0], 1
    return [(first0 + r * BS, BS, list(range(seed, seed + NS))) for r in range(R)]


def dry_run(args, rank, world):
    """the multi-rank plumbing without HIP: placeholder frames (frame k's samples all hold k) are
    produced per rank from its frame_range shard, K steps are timed between barriers with the
    max over ranks by all_reduce, and the ordered gather to rank 0 is checked frame by frame"""
    import torch
    import torch.distributed as dist
    from dvbt2ll.distributed import frame_range, gather_frames
    if rank == args.fail_rank:
        raise SystemExit("bench.py: rank %d made to fail at init (--fail-rank)" % rank)
    if world > 1:
        dist.init_process_group(args.backend or "gloo", timeout=datetime.timedelta(seconds=args.init_timeout))
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    B, per = min(args.frames, 16), 1024
    NS = max(1, args.streams)
    if args.shard == "streams":
        # each rank its own NS streams (shard_plan), B // NS frames of each per step; placeholder frame
        # = seed * 1000 + frame
        plan = shard_plan("streams", B, NS, 1, rank, world)[0]
        first, count, seeds = plan[0], plan[1] * NS, plan[2]
        vals = torch.tensor([sd * 1000 + plan[0] + k for sd in seeds for k in range(plan[1])], dtype=torch.float32)
    else:
        first, count = frame_range(world * B, rank, world)
        seeds = [1]
        vals = torch.arange(first, first + count, dtype=torch.float32)
    buf = torch.empty((count * per, 2), dtype=torch.float32)

    def step():
        buf.view(count, per, 2)[:] = vals[:, None, None]
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    if world > 1:
        dist.barrier()
    e = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world > 1:
        dist.all_reduce(e, op=dist.ReduceOp.MAX)
    if args.shard == "streams":
        # every rank's stream set (no gather: independent streams are replicas)
        allseeds = [None] * world
        if world > 1:
            dist.all_gather_object(allseeds, seeds)
        else:
            allseeds = [seeds]
        ok = bool((buf.view(count, per, 2)[:, 0, 0] == vals).all())
        if rank == 0:
            flat = sorted(sd for ss in allseeds for sd in ss)
            print(json.dumps({"metric": "dry run: placeholder frames/s (no HIP)",
                              "value": world * count * args.steps / float(e), "unit": "frames/s", "n_gpus": world,
                              "steps": args.steps, "warmup": args.warmup, "dry_run": True, "shard": "streams",
                              "streams_per_rank": NS, "stream_seeds": allseeds,
                              "seeds_disjoint_complete": flat == list(range(1, world * NS + 1)),
                              "frames_ok": ok, "world_size_verified": world == args.gpus,
                              "launcher": "bench.py spawn" if os.environ.get("DVBT2LL_BENCH_SPAWNED") else
                                          ("external" if world > 1 else "single process")}))
        if world > 1:
            dist.destroy_process_group()
        return 0
    shards = [list(frame_range(world * B, r, world)) for r in range(world)]
    g = gather_frames(buf, world * B, per) if world > 1 else buf
    if rank == 0:
        got = g.view(world * B, per, 2)
        ok = bool((got == torch.arange(world * B, dtype=torch.float32)[:, None, None]).all())
        print(json.dumps({"metric": "dry run: placeholder frames/s (no HIP)", "value": world * B * args.steps / float(e),
                          "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                          "dry_run": True, "backend": args.backend or "gloo",
                          "world_size_verified": world == args.gpus, "shards": shards, "gather_in_order": ok,
                          "launcher": "bench.py spawn" if os.environ.get("DVBT2LL_BENCH_SPAWNED") else
                                      ("external" if world > 1 else "single process")}))
    if world > 1:
        dist.destroy_process_group()
    return 0


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not args.pmc_child:
        return spawn_ranks(args)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not args.pmc_child:
        raise SystemExit("bench.py: --gpus %d but WORLD_SIZE %d" % (args.gpus, world))
    if args.dry_run:
        return dry_run(args, rank, world)
    traffic, pmc_note = None, "skipped"
    if os.environ.get("DVBT2LL_BENCH_PMC_JSON"):        # measured by the spawning parent (spawn_ranks)
        with open(os.environ["DVBT2LL_BENCH_PMC_JSON"]) as fh:
            pm = json.load(fh)
        traffic, pmc_note = pm["traffic"], pm["note"]
    elif world == 1 and not args.pmc_child and not args.no_pmc:
        traffic, pmc_note = pmc_passes(args)          # before any GPU initialisation here
    elif world > 1:
        pmc_note = "not collected under an external launcher (bench.py --gpus N spawns its ranks after its PMC passes)"

    import numpy as np
    import torch
    import dvbt2ll
    from dvbt2ll.configs import CONFIGS, ts_for_frames

    cfg = CONFIGS[args.config]
    torch.cuda.set_device(local_rank)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if rank == args.fail_rank:
            raise SystemExit("bench.py: rank %d made to fail at init (--fail-rank)" % rank)
        dist.init_process_group(args.backend or "nccl", device_id=torch.device("cuda", local_rank),
                                timeout=datetime.timedelta(seconds=args.init_timeout))
        assert dist.get_world_size() == args.gpus, (dist.get_world_size(), args.gpus)
    B = args.frames
    chain = dvbt2ll.Chain(cfg, max_frames=B, device=local_rank)
    info = chain.info
    per = chain.iq_per_frame
    # R distinct resident batches per rank (shard_plan)
    R = 2
    NS = max(1, args.streams)
    plan = shard_plan(args.shard, B, NS, R, rank, world)
    BS = B // NS
    ts_dev, ts_meta = [], []
    for r, (first, _, seeds) in enumerate(plan):
        tss = [ts_for_frames(cfg, first, BS, sd) for sd in seeds]
        base, n = tss[0][1], len(tss[0][0])
        stride = (n + 255) // 256 * 256
        buf = np.zeros((NS, stride), np.uint8)
        for k, (ts, _) in enumerate(tss):
            buf[k, :n] = ts
        ts_dev.append(torch.from_numpy(buf.reshape(-1)).cuda())
        ts_meta.append((first, base, n, stride))
    # pipelined steps: the handle holds `slots` intermediate buffer sets and step s is issued on
    # stream s % slots into its own IQ buffer, so one step's kernels fill the CUs the previous
    # step's kernel tails leave idle (dvbt2ll_chain_set_slots); every step still does all the work
    S = max(1, args.slots)
    # the default shapes must fit HBM at N = 8 too (rank 0 also holds the ordered gather's output)
    G = min(B, 512)
    need = hbm_footprint(info, B, S, R, world, max(m[2] for m in ts_meta), not args.no_sc16, G)
    if need > 0.9 * HBM_BYTES:
        raise SystemExit("bench.py: %.1f GB of HBM needed per rank, more than 90 %% of %.0f GB" % (need / 1e9,
                                                                                              HBM_BYTES / 1e9))
    chain.set_slots(S)
    iq = [torch.empty((B * per, 2), dtype=torch.float32, device="cuda") for _ in range(S)]
    streams = [torch.cuda.Stream() for _ in range(S)]
    torch.cuda.synchronize()

    def step(s, serial=False):
        first, base, n, stride = ts_meta[s % R]
        st = streams[0] if serial else streams[s % S]
        if NS > 1:
            chain.run_streams(ts_dev[s % R].data_ptr(), stride, NS, base, n, first, BS, out[0][s % S].data_ptr(),
                              st.cuda_stream)
        else:
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
    # (with one slot too: the headline pass never records the per-stage timing events, which cost ~3 % of a step)
    elapsed, _ = timed()
    serial_elapsed, (stage_ms, launches) = timed(serial=True, timing=True)
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
    if not args.no_latency and NS == 1:
        latency = one_frame_latency(chain, ts_dev, ts_meta, iq, streams, per)
    blocks = None
    if not args.no_blocks and world == 1 and rank == 0:
        blocks = per_block_rate(cfg)
        blocks["pinned"] = per_block_rate(cfg, pinned=True)
    mplp = None
    if not args.no_mplp and world == 1 and rank == 0 and args.config == "cfg3":
        mplp = mplp_rate(B, args.steps, args.warmup)
    host = None
    if not args.no_host and world == 1 and rank == 0:
        host = host_delivered(cfg, 32 if info["fft_size"] == 32768 else 128, 24, pcie_peaks())
    gathered = None
    if dist and args.shard == "frames" and NS == 1:
        # secondary (not `value`): each step followed by the ordered IQ gather to rank 0, the
        # chain's one exchange step (point-to-point sends to the root over RCCL / xGMI)
        from dvbt2ll.distributed import gather_frames
        kg = min(args.steps, 3)
        # at most G = 512 frames per rank gathered per step: the root's output tensor (N x G frames of
        # complex64 IQ, 68 GB at N = 8) beside the chain's slots and IQ buffers (hbm_footprint, checked
        # against 288 GB before anything is allocated; the multi-PLP chain is not built under N > 1)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for s_ in range(kg):
            step(s_, serial=True)
            torch.cuda.current_stream().wait_stream(streams[0])
            gather_frames(iq[s_ % S][:G * per], world * G, per)
        torch.cuda.synchronize()
        dist.barrier()
        eg = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device="cuda")
        dist.all_reduce(eg, op=dist.ReduceOp.MAX)
        eg = float(eg.item())
        gathered = {"value": world * B * kg * per / eg / 1e6, "unit": "Msamples/s", "steps": kg,
                    "ms_per_step": eg / kg * 1e3, "gathered_frames_per_rank": G,
                    "bytes_to_root_per_step": (world - 1) * G * per * 8,
                    "note": "secondary: every step (all B frames encoded) followed by the ordered gather of its "
                            "first G frames' complex64 IQ per rank to rank 0 (dvbt2ll.distributed.gather_frames, "
                            "grouped send/recv); not `value`"}
    frames_total = B * args.steps * world
    samples_total = frames_total * per
    fec_total = frames_total * info["fec_blocks_per_frame"]
    msps = samples_total / elapsed / 1e6
    if rank == 0:
        ab = algorithmic_bytes(cfg, info)
        mb = minimal_bytes(cfg, info)
        stages, rooflines = {}, {}
        for k, name in enumerate(KERNELS):
            avg_ms = stage_ms[k] / max(1, launches[k])
            t = avg_ms * 1e-3
            stages[name] = {"avg_launch_ms": avg_ms, "algorithmic_bytes_per_launch": ab[name] * B,
                            "achieved_GBs": ab[name] * B / t / 1e9 if t > 0 else None}
            kname = ("ofdm32_kernel" if name == "ofdm" and info["fft_size"] == 32768 else
                     "bbch_kernel (BB + BCH)" if name == "fec" else
                     "ldpc_map_kernel (+ L1-post workgroups)" if name == "map" else name + "_kernel")
            e = {"kernel": kname, "bound": "hbm", "avg_launch_ms": avg_ms, "peak": HBM_PEAK_GBS,
                 "unit": "GB/s", "min_bytes_per_launch": mb[name] * B,
                 "achieved": mb[name] * B / t / 1e9 if t > 0 else None,
                 "stage_bytes_per_launch": ab[name] * B,
                 "stage_bytes_frac": ab[name] * B / t / 1e9 / HBM_PEAK_GBS if t > 0 else None}
            e["frac"] = e["achieved"] / HBM_PEAK_GBS if e["achieved"] else None
            pm = (traffic or {}).get(name, {})
            e["traffic"] = pm.get("hbm_bytes")
            if traffic is not None and e["traffic"] is None:
                e["pmc_missing"] = {"counters": sorted(c for c in pm if c.isupper()),
                                    "kernel_names_seen": pm.get("kernel_names_seen")}
            if e["traffic"] and t > 0:
                e["traffic_GBs"] = e["traffic"] / t / 1e9
                e["traffic_frac"] = e["traffic_GBs"] / HBM_PEAK_GBS
                e["traffic_over_min"] = e["traffic"] / (mb[name] * B)
                e["traffic_fetch_write"] = pm.get("fetch_write_bytes")
                e["calibration"] = pm.get("calibration")
            if name in ("fec", "map"):
                nb = info["fec_blocks_per_frame"] * B
                e["fec_blocks_per_s"] = nb / t if t > 0 else None
                e["note"] = ("BB pass + BCH as a GF(2) product on the matrix cores (two kernels; traffic and "
                             "instruction counts are their sums)" if name == "fec" else
                             "LDPC parity + bit interleaver + cell / time interleaver of each FEC block in one "
                             "kernel (the codeword stays in LDS), plus the frames' L1-post workgroups") + (
                             ": integer codec work, latency/issue-bound, not HBM-bound (SURVEY 8(d)); frac is "
                             "the minimal HBM bytes / time / peak")
                if "SQ_INSTS_VALU" in pm and t > 0:
                    e["valu_wave_instr_per_block"] = pm["SQ_INSTS_VALU"] / nb
                    e["salu_wave_instr_per_block"] = pm.get("SQ_INSTS_SALU", 0) / nb
                    e["valu_issue_frac"] = pm["SQ_INSTS_VALU"] / t / VALU_ISSUE_PEAK
            rooflines[name] = e
        dom = max((n for n in stages if n in KERNELS), key=lambda n: stages[n]["avg_launch_ms"])
        roof = dict(rooflines[dom])
        roof["note"] = ("frac = the kernel's minimal HBM bytes (DESIGN.md 5) / its HIP-event launch time / 8 TB/s; "
                        "traffic = calibrated rocprofv3 FETCH_SIZE + WRITE_SIZE per launch; stage_bytes_frac = "
                        "SURVEY 8(d)'s unfused stage bytes over the same time (not an HBM utilisation)")
        if traffic is None:
            roof["traffic_note"] = pmc_note
        out = {
            "metric": metric_for(args.config), "value": msps, "unit": "Msamples/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f32", "data": "synthetic",
            "config": {"workload": "%s: TS->IQ full DVB-T2 chain, %d T2 frames per step per GPU%s "
                                   "(%d FEC blocks, %d IQ samples per frame)"
                                   % (cfg.name, B, " (%d independent TS streams x %d frames, one launch)" % (NS, BS)
                                      if NS > 1 else "", info["fec_blocks_per_frame"], per),
                       "frames_per_step_per_gpu": B, "slots_streams_per_gpu": S,
                       "symbols_per_frame": info["num_symbols"], "fft_size": info["fft_size"],
                       "guard_samples": info["guard_interval"],
                       "ts_streams_per_launch": NS,
                       "parallelism": "%s x%d (no data-path collective)"
                                      % ("frame-sharded" if args.shard == "frames" else "independent streams", world),
                       "launcher": "bench.py spawn" if os.environ.get("DVBT2LL_BENCH_SPAWNED") else
                                   ("external" if world > 1 else "single process")},
            "fec_blocks_per_sec": fec_total / elapsed,
            "serial_1_stream": {"value": samples_total / serial_elapsed / 1e6,
                                "ms_per_step": serial_elapsed / args.steps * 1e3,
                                "note": "same K steps issued on one stream (no cross-step overlap); the "
                                        "stage timings and roofline come from this pass"},
            "x_realtime": msps * 1e6 / RT_SPS,
            "stages": stages,
            "roofline": roof,
            "rooflines": rooflines,
        }
        # chain level (per GPU): the bytes the step cannot avoid (TS payload in, IQ out) and the bytes the PMC
        # passes counted (each stage's calibrated FETCH + WRITE per launch x its launches per step), over the
        # pipelined step time; the serial kernel sum beside the pipelined step is what the slots overlap
        from dvbt2ll.configs import KBCH
        ts_in = info["fec_blocks_per_frame"] * ((KBCH[(cfg.framesize, cfg.rate)] - 80) // 8)
        mand = B * (ts_in + 8 * per)
        t_step = elapsed / args.steps
        chain_f = {"mandatory_bytes_per_step": mand,
                   "mandatory_bytes_frac": mand / t_step / 1e9 / HBM_PEAK_GBS,
                   "serial_kernel_ms_per_step": sum(stage_ms) / args.steps,
                   "pipelined_ms_per_step": t_step * 1e3,
                   "overlap_ms_per_step": sum(stage_ms) / args.steps - t_step * 1e3,
                   "note": "per GPU: mandatory = TS payload in + complex64 IQ out per step; pmc = calibrated "
                           "FETCH_SIZE + WRITE_SIZE of every kernel launch of a step; fracs over ms_per_step and "
                           "8 TB/s; overlap = serial kernel sum - pipelined step (profiles/r6_overlap_trace.txt)"}
        if traffic is not None and all(rooflines[k].get("traffic") for k in KERNELS):
            pb = sum(rooflines[k]["traffic"] * launches[i] / args.steps for i, k in enumerate(KERNELS))
            chain_f["pmc_bytes_per_step"] = pb
            chain_f["pmc_bytes_frac"] = pb / t_step / 1e9 / HBM_PEAK_GBS
        else:
            chain_f["pmc_bytes_per_step"] = None
        out["chain"] = chain_f
        if sc16:
            out["iq_sc16_x0.2"] = {
                "value": samples_total / sc16["elapsed"] / 1e6, "unit": "Msamples/s",
                "ms_per_step": sc16["ms_per_step"], "ofdm_avg_launch_ms": sc16["ofdm_avg_launch_ms"],
                "note": "secondary: same chain, output gain 0.2 + int16 I/Q store (the flowgraph's "
                        "multiply_const and SDR wire format fused into the IQ store); not `value`"}
        if latency:
            out["latency_1_frame"] = latency
        if gathered:
            out["gather_to_rank0"] = gathered
        if mplp:
            out["mplp_2plp_32k"] = mplp
        if host:
            out["host_delivered"] = host
        if blocks:
            out["per_block_general_work"] = blocks
        if not args.no_cpu_baseline and world == 1:   # rank 0 at N=1 only (host cores are shared)
            out["cpu_baseline"] = cpu_baseline(cfg, args.cpu_seconds)
            # the box's CPU share is 16 threads (os.cpu_count() reports the whole machine)
            threads = min(16, os.cpu_count() or 1)
            out["cpu_baseline"]["whole_host"] = cpu_host_replicas(cfg, args.cpu_seconds / 2, threads)
            out["iq_accuracy"] = iq_accuracy(sorted({args.config, "cfg1", "cfg4"}))
        print(json.dumps(out))
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
