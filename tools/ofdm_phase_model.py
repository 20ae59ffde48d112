#!/usr/bin/env python3
"""Per-symbol resource model of the 32K OFDM kernel from one session's counters and the measured
store rate:

    python tools/ofdm_phase_model.py PMC.txt BENCH.json [STORE_RATE.jsonl]

One 16-wave workgroup per CU holds one symbol (the symbol fills the register file), with barriers
between the kernel's phases.  Per symbol, on its CU:

    T_valu  = SQ_INSTS_VALU / symbols x 2 cycles (a wave64 VALU instruction issues over 2 cycles,
              MI355X_MICROARCH.md) / 4 SIMDs
    T_lds   = SQ_LDS_IDX_ACTIVE / symbols (LDS-array cycles, bank conflicts included)
    T_store = the symbol's IQ bytes at the measured per-CU store rate of tools/store_rate.hip (one
              workgroup storing alone: the CU's own write path, no contention; profiles/r4_store_rate.jsonl)

in cycles at the launch's clock: GRBM_GUI_ACTIVE per XCD (cycles of the profiled launch, counted in the
PMC run) over that launch's duration (the bench's HIP-event average of the same kernel, a separate run
on the same box: the clock is an estimate, and the per-symbol cycles carry its error).  Each
of the three alone is a lower bound on the symbol's time (the CU cannot run its LDS, its SIMDs or
its write path faster), and so is the chip-wide one, all IQ bytes at the measured all-CU store rate.
Their sum, the serial-sum model, is NOT a bound: VALU and LDS work of different waves overlap inside
a phase.  It is the time the symbol would take if its phases ran back to back, each at its busiest
resource's rate with nothing else in the way; measured / serial sum > 1 is what latency (barrier
waits, the first loads of each scatter half, the store drain under contention) adds on top.
The round-3 version priced the store at a fair 1/256 share of 8 TB/s and called the sum a bound;
the measured per-CU store rate (74 GB/s, about 3.8 us per symbol against 10.6 us at the fair share)
shows that share was not a property of the hardware."""
import json
import pathlib
import sys

CUS, XCDS, HBM = 256, 8, 8.0e12
ROOT = pathlib.Path(__file__).resolve().parents[1]


def counters(path, kernel="ofdm32_kernel"):
    out = {}
    for line in open(path):
        f = line.split()
        if len(f) == 3 and f[0] == kernel:
            out[f[1]] = float(f[2])
    return out


def store_rates(path):
    """(per-CU bytes/s of one workgroup storing alone, chip bytes/s of the all-CU grid case)"""
    lone = grid = None
    for line in open(path):
        r = json.loads(line)
        if r.get("nontemporal", 1) != 1:
            continue
        if r["case"] == "lone" and r["workgroups"] == 1:
            lone = r["GBs_per_cu"] * 1e9
        if r["case"] == "grid":
            grid = r["GBs_total"] * 1e9
    return lone, grid


def model(pmc, bench, rates):
    st, cf = bench["stages"]["ofdm"], bench["config"]
    # symbols per frame from the bench line (round 4 on); older lines are cfg3: 2091008 IQ samples per
    # frame = P1 (2048) + 60 symbols x (32768 + 2048 GI)
    nsym = cf.get("symbols_per_frame", 60) * cf["frames_per_step_per_gpu"]
    N, G = cf.get("fft_size", 32768), cf.get("guard_samples", 2048)
    launch_s = st["avg_launch_ms"] * 1e-3
    cycles = pmc["GRBM_GUI_ACTIVE"] / XCDS           # GPU cycles of the (profiled) launch
    clock = cycles / launch_s
    per_cu = nsym / CUS
    t_meas = cycles / per_cu
    iq_bytes = 8 * (N + G)
    lone, grid = rates
    t_valu = pmc["SQ_INSTS_VALU"] / nsym * 2 / 4
    t_lds = pmc["SQ_LDS_IDX_ACTIVE"] / nsym
    t_store = iq_bytes / lone * clock
    t_fair = bench["roofline"]["min_bytes_per_launch"] / nsym / (HBM / CUS) * clock
    chip_store_s = iq_bytes * nsym / grid
    serial = t_valu + t_lds + t_store
    return {"symbols": nsym, "clock_GHz": round(clock / 1e9, 3), "cycles_per_symbol": round(t_meas),
            "valu": round(t_valu), "lds": round(t_lds), "store_lone_cu": round(t_store),
            "store_fair_share_r3": round(t_fair),
            "largest_single_resource_bound": round(max(t_valu, t_lds, t_store)),
            "measured_over_largest_bound": round(t_meas / max(t_valu, t_lds, t_store), 3),
            "chip_store_bound_ms": round(chip_store_s * 1e3, 4), "launch_ms": round(launch_s * 1e3, 4),
            "serial_sum": round(serial), "measured_over_serial_sum": round(t_meas / serial, 3),
            "latency_cycles_per_symbol": round(t_meas - serial)}


def main():
    pmc, bench = counters(sys.argv[1]), json.load(open(sys.argv[2]))
    rates = store_rates(sys.argv[3] if len(sys.argv) > 3 else ROOT / "profiles" / "r4_store_rate.jsonl")
    print(json.dumps(model(pmc, bench, rates)))


if __name__ == "__main__":
    main()
