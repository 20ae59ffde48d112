#!/usr/bin/env python3
"""Extract the DVB-T2 constant tables (ETSI EN 302 755 / EN 302 307 data) that the
reference blocks carry as C arrays, and write them as one generated C header.

Run once in the development container (the reference tree does not exist on the
GPU box):

    python tools/extract_tables.py /root/reference gr-dvbt2ll_amd/csrc/gen/dvbt2_std_tables.h

Only numeric table *data* is taken (LDPC parity-address tables, BCH minimal
polynomials, bit-interleaver column twists / demux permutations, frequency
interleaver bit permutations, L1 puncture / padding orders, continual-pilot and
PAPR carrier lists, P1 carrier list and S1/S2 patterns, the PN sequence) plus the
per-(FFT, pilot-pattern) C_DATA / N_FC / C_FC counts and the *structure* of the
reference's continual-pilot selection (which list, how many entries, which modulus,
whether MISO TX2 inversion applies, whether it is extended-carrier-only).  All code
that uses these tables is written from scratch in csrc/ and oracle/.

Source locations (reference file:line):
  LDPC tables         lib/bbheaderbch_bb_impl.cc:744-1764, L1 codes lib/framemapperfint_cc_impl.cc:2153-2188
  BCH polynomials     lib/bbheaderbch_bb_impl.cc:428-453
  twist / mux         lib/interleavermod_bc_impl.cc:706-804
  L1 tables, bitperm  lib/framemapperfint_cc_impl.cc:2190-2288
  C_DATA/N_FC/C_FC    lib/framemapperfint_cc_impl.cc:425-897
  pilot tables        lib/pilotgenp1insert_cc_impl.cc:2909-3505
  CP selection logic  lib/pilotgenp1insert_cc_impl.cc:1285-2705
"""
import re
import sys
from pathlib import Path


def arrays(text):
    """name -> flat list of ints for every `const <type> <cls>::<name>[...] = { ... };`"""
    out = {}
    for m in re.finditer(r"const\s+(?:unsigned\s+char|int)\s+\w+::(\w+)((?:\[[^\]]*\])+)\s*=\s*\{", text):
        name = m.group(1)
        start = m.end()
        depth = 1
        i = start
        while depth:
            if text[i] == "{":
                depth += 1
            elif text[i] == "}":
                depth -= 1
            i += 1
        body = text[start:i - 1]
        dims = [int(d) for d in re.findall(r"\[(\d+)\]", m.group(2))]
        num = r"0x[0-9A-Fa-f]+|\d+"
        if len(dims) == 2:
            # 2-D: one brace group per row; short rows are zero-filled as C would do
            vals = []
            for row in re.findall(r"\{([^{}]*)\}", body):
                r = [int(v, 0) for v in re.findall(num, row)]
                vals.extend(r + [0] * (dims[1] - len(r)))
            assert len(vals) == dims[0] * dims[1], (name, len(vals), dims)
        else:
            vals = [int(v, 0) for v in re.findall(num, body)]
        out[name] = vals
        out[name + "__dims"] = dims
    return out


def local_arrays(text):
    """local `const int polyXX[]={...};` arrays"""
    return {m.group(1): [int(v) for v in m.group(2).split(",")]
            for m in re.finditer(r"const int (poly[ns]\d\d)\[\]=\{([0-9,]+)\};", text)}


FFT_ENUM = {"FFTSIZE_1K": 1024, "FFTSIZE_2K": 2048, "FFTSIZE_4K": 4096, "FFTSIZE_8K": 8192,
            "FFTSIZE_16K": 16384, "FFTSIZE_32K": 32768}


def data_counts(fm_text):
    """Parse the C_DATA/N_FC/C_FC switch of the framemapper ctor (lines 425-897)."""
    lines = fm_text.splitlines()[424:897]
    fft = None
    ext = 0
    pp = None
    res = {}
    for ln in lines:
        m = re.search(r"case (FFTSIZE_\w+):", ln)
        if m and m.group(1) in FFT_ENUM:
            fft = FFT_ENUM[m.group(1)]
            ext = 0
            continue
        if "carriermode == CARRIERS_NORMAL" in ln:
            ext = 0
            continue
        if re.match(r"\s*else\s*\{", ln) and fft is not None and fft >= 8192:
            ext = 1
            continue
        m = re.search(r"case PILOT_PP(\d):", ln)
        if m:
            pp = int(m.group(1))
            continue
        for key in ("C_DATA", "N_FC", "C_FC"):
            m = re.search(key + r" = (\d+);", ln)
            if m:
                res.setdefault((fft, ext, pp), {})[key] = int(m.group(1))
    for fft in (1024, 2048, 4096):   # no extended mode below 8K: same numbers
        for pp in range(1, 9):
            res[(fft, 1, pp)] = dict(res[(fft, 0, pp)])
    return res


def cp_structure(pg_text):
    """Walk init_pilots (lines 1285-2705) and record every continual-pilot list it applies."""
    lines = pg_text.splitlines()[1284:2705]
    fft = None
    pp = None
    ext_only = False
    ext_depth = None
    depth = 0
    pending = None
    recs = {}
    for ln in lines:
        m = re.search(r"case (FFTSIZE_\w+):", ln)
        if m and m.group(1) in FFT_ENUM:
            fft = FFT_ENUM[m.group(1)]
        m = re.search(r"case PILOT_PP(\d):", ln)
        if m:
            pp = int(m.group(1))
        if "carrier_mode == CARRIERS_EXTENDED" in ln:
            ext_only = True
            ext_depth = depth
        m = re.search(r"for \(int i = 0; i < (\d+); i\+\+\)", ln)
        if m:
            pending = {"count": int(m.group(1)), "miso": False, "table": None, "mod": 0,
                       "ext": ext_only}
            recs.setdefault((fft, pp), []).append(pending)
        if pending is not None:
            if "miso_group == MISO_TX2" in ln:
                pending["miso"] = True
            m = re.search(r"data_carrier_map\[(pp\d_(?:cp\d|\d+k))\[i\](?: % (\d+))?\]", ln)
            if m and pending["table"] is None:
                pending["table"] = m.group(1)
                pending["mod"] = int(m.group(2)) if m.group(2) else 0
        depth += ln.count("{") - ln.count("}")
        if ext_only and ext_depth is not None and depth <= ext_depth:
            ext_only = False
            ext_depth = None
    return recs


def fmt_list(vals, per=16):
    rows = []
    for i in range(0, len(vals), per):
        rows.append("  " + ", ".join(str(v) for v in vals[i:i + per]) + ",")
    return "\n".join(rows)


def main():
    ref = Path(sys.argv[1])
    out_path = Path(sys.argv[2])
    bb = (ref / "lib/bbheaderbch_bb_impl.cc").read_text()
    im = (ref / "lib/interleavermod_bc_impl.cc").read_text()
    fm = (ref / "lib/framemapperfint_cc_impl.cc").read_text()
    pg = (ref / "lib/pilotgenp1insert_cc_impl.cc").read_text()
    A = {}
    A.update({"bb_" + k: v for k, v in arrays(bb).items()})
    A.update({"im_" + k: v for k, v in arrays(im).items()})
    A.update({"fm_" + k: v for k, v in arrays(fm).items()})
    A.update({"pg_" + k: v for k, v in arrays(pg).items()})
    polys = local_arrays(bb)

    o = []
    o.append("/* GENERATED by tools/extract_tables.py -- do not edit.\n"
             " * DVB-T2 constant tables (ETSI EN 302 755 V1.3.1 annexes; LDPC tables shared with\n"
             " * EN 302 307) as carried by the reference gr-dvbt2ll blocks.  Data only; every\n"
             " * algorithm using them is written independently in csrc/ and oracle/.  Layouts\n"
             " * here are flattened (CSR-style) and differ from the reference's arrays. */\n")
    o.append("#ifndef DVBT2_STD_TABLES_H\n#define DVBT2_STD_TABLES_H\n#include <stdint.h>\n")

    # ---------------- LDPC --------------------------------------------------------
    # (framesize: 1 normal / 0 short, rate enum, table name, q)
    codes = [
        (1, 0, "ldpc_tab_1_2N", 90), (1, 1, "ldpc_tab_3_5N", 72), (1, 2, "ldpc_tab_2_3N_DVBT2", 60),
        (1, 3, "ldpc_tab_3_4N", 45), (1, 4, "ldpc_tab_4_5N", 36), (1, 5, "ldpc_tab_5_6N", 30),
        (0, 6, "ldpc_tab_1_3S", 30), (0, 7, "ldpc_tab_2_5S", 27), (0, 0, "ldpc_tab_1_2S", 25),
        (0, 1, "ldpc_tab_3_5S_DVBT2", 18), (0, 2, "ldpc_tab_2_3S", 15), (0, 3, "ldpc_tab_3_4S", 12),
        (0, 4, "ldpc_tab_4_5S", 10), (0, 5, "ldpc_tab_5_6S", 8),
    ]
    rowlen, ents, desc = [], [], []

    def add_code(fs, rate, flat, dims, q, tag):
        nrows, ncols = dims
        row_off, ent_off = len(rowlen), len(ents)
        for r in range(nrows):
            row = flat[r * ncols:(r + 1) * ncols]
            rowlen.append(row[0])
            ents.extend(row[1:1 + row[0]])
        desc.append((fs, rate, nrows, q, row_off, ent_off, len(ents) - ent_off, tag))

    for fs, rate, name, q in codes:
        add_code(fs, rate, A["bb_" + name], A["bb_" + name + "__dims"], q, name)
    # L1 signalling codes (framemapper): 1/4 short (L1-pre) and 1/2 short (L1-post)
    add_code(0, 100, A["fm_ldpc_tab_1_4S"], A["fm_ldpc_tab_1_4S__dims"], 36, "l1pre_1_4S")
    add_code(0, 101, A["fm_ldpc_tab_1_2S"], A["fm_ldpc_tab_1_2S__dims"], 25, "l1post_1_2S")
    o.append("/* LDPC parity-address tables: per code, nrows info groups of 360 bits; row r has\n"
             " * T2_LDPC_ROWLEN[row_off + r] addresses stored consecutively in T2_LDPC_ADDR. */")
    o.append("typedef struct { int framesize_normal, rate, nrows, q, row_off, addr_off, naddr; } t2_ldpc_code_t;")
    o.append("static const t2_ldpc_code_t T2_LDPC_CODES[] = {")
    for d in desc:
        o.append("  {%d, %d, %d, %d, %d, %d, %d}, /* %s */" % (d[0], d[1], d[2], d[3], d[4], d[5], d[6], d[7]))
    o.append("};\n#define T2_LDPC_NCODES %d" % len(desc))
    o.append("static const uint8_t T2_LDPC_ROWLEN[] = {\n" + fmt_list(rowlen, 24) + "\n};")
    o.append("static const uint16_t T2_LDPC_ADDR[] = {\n" + fmt_list(ents, 14) + "\n};\n")

    # ---------------- BCH minimal polynomials --------------------------------------
    o.append("/* BCH minimal polynomials, coefficient lists lowest power first (17 / 15 terms). */")
    o.append("static const uint8_t T2_BCH_MINPOLY_NORMAL[12][17] = {")
    for i in range(1, 13):
        o.append("  {" + ",".join(map(str, polys["polyn%02d" % i])) + "},")
    o.append("};")
    o.append("static const uint8_t T2_BCH_MINPOLY_SHORT[12][15] = {")
    for i in range(1, 13):
        o.append("  {" + ",".join(map(str, polys["polys%02d" % i])) + "},")
    o.append("};\n")

    # ---------------- bit interleaver ----------------------------------------------
    o.append("/* Bit interleaver: column twist (per constellation / frame size) and demux bit\n"
             " * permutations, EN 302 755 tables 8 and 13. */")
    for nm in ["twist16n", "twist64n", "twist256n", "twist16s", "twist64s", "twist256s",
               "mux16", "mux64", "mux256", "mux16_35", "mux16_13", "mux16_25", "mux64_35",
               "mux64_13", "mux64_25", "mux256_35", "mux256_23", "mux256s", "mux256s_13",
               "mux256s_25"]:
        v = A["im_" + nm]
        o.append("static const uint8_t T2_BI_%s[%d] = {%s};" % (nm.upper(), len(v), ", ".join(map(str, v))))
    o.append("")

    # ---------------- L1 signalling tables -----------------------------------------
    o.append("/* L1 signalling: puncturing / shortening group orders, L1 16/64QAM demux. */")
    for nm in ["pre_puncture", "post_padding_bqpsk", "post_padding_16qam", "post_padding_64qam",
               "post_puncture_bqpsk", "post_puncture_16qam", "post_puncture_64qam", "mux16", "mux64"]:
        v = A["fm_" + nm]
        o.append("static const uint8_t T2_L1_%s[%d] = {%s};" % (nm.upper(), len(v), ", ".join(map(str, v))))
    o.append("")
    o.append("/* Frequency interleaver bit permutations (EN 302 755 9.4.1), index = FFT size order. */")
    for nm in ["bitperm1keven", "bitperm1kodd", "bitperm2keven", "bitperm2kodd", "bitperm4keven",
               "bitperm4kodd", "bitperm8keven", "bitperm8kodd", "bitperm16keven", "bitperm16kodd",
               "bitperm32k"]:
        v = A["fm_" + nm]
        o.append("static const uint8_t T2_FI_%s[%d] = {%s};" % (nm.upper(), len(v), ", ".join(map(str, v))))
    o.append("")

    # ---------------- C_DATA / N_FC / C_FC -----------------------------------------
    dc = data_counts(fm)
    o.append("/* Active cells per symbol: {fft, extended, pp(1-8), C_DATA, N_FC, C_FC} before any\n"
             " * PAPR-TR reduction or the SISO GI/PP N_FC=0 exceptions. */")
    o.append("typedef struct { int fft, ext, pp, c_data, n_fc, c_fc; } t2_cell_counts_t;")
    o.append("static const t2_cell_counts_t T2_CELL_COUNTS[] = {")
    keys = sorted(dc)
    for k in keys:
        v = dc[k]
        o.append("  {%d, %d, %d, %d, %d, %d}," % (k[0], k[1], k[2], v["C_DATA"], v["N_FC"], v["C_FC"]))
    o.append("};\n#define T2_NCELL_COUNTS %d\n" % len(keys))

    # ---------------- pilots ----------------------------------------------------------
    pg_names = [k[3:] for k in A if k.startswith("pg_") and not k.endswith("__dims")]
    list_names = [n for n in pg_names if re.match(r"pp\d_(cp\d|\d+k)$", n)]
    list_names.sort()
    o.append("/* Continual-pilot carrier lists and extended-carrier additions (EN 302 755 annex G). */")
    flat, offs = [], {}
    for n in list_names:
        offs[n] = (len(flat), len(A["pg_" + n]))
        flat.extend(A["pg_" + n])
    o.append("static const uint16_t T2_CP_LIST[] = {\n" + fmt_list(flat, 14) + "\n};")
    o.append("/* list id -> (offset, length) into T2_CP_LIST */")
    o.append("static const int T2_CP_LIST_SPAN[][2] = {")
    ids = {}
    for i, n in enumerate(list_names):
        ids[n] = i
        o.append("  {%d, %d}, /* %d: %s */" % (offs[n][0], offs[n][1], i, n))
    o.append("};")
    st = cp_structure(pg)
    o.append("/* Continual-pilot selection steps: {fft, pp, list id, count, modulus (0 = none),\n"
             " * miso_tx2_inversion, extended_carriers_only}.  Applied in order. */")
    o.append("typedef struct { int fft, pp, list, count, modulus, miso_inv, ext_only; } t2_cp_step_t;")
    o.append("static const t2_cp_step_t T2_CP_STEPS[] = {")
    nsteps = 0
    for (fft, pp) in sorted(st):
        for r in st[(fft, pp)]:
            assert r["table"] is not None, (fft, pp, r)
            assert r["count"] <= offs[r["table"]][1], (fft, pp, r)
            o.append("  {%d, %d, %d, %d, %d, %d, %d}, /* %s */" % (fft, pp, ids[r["table"]], r["count"],
                     r["mod"], int(r["miso"]), int(r["ext"]), r["table"]))
            nsteps += 1
    o.append("};\n#define T2_NCP_STEPS %d\n" % nsteps)

    for nm in ["p2_papr_map_1k", "p2_papr_map_2k", "p2_papr_map_4k", "p2_papr_map_8k",
               "p2_papr_map_16k", "p2_papr_map_32k", "tr_papr_map_1k", "tr_papr_map_2k",
               "tr_papr_map_4k", "tr_papr_map_8k", "tr_papr_map_16k", "tr_papr_map_32k"]:
        v = A["pg_" + nm]
        o.append("static const uint16_t T2_%s[%d] = {\n%s\n};" % (nm.upper(), len(v), fmt_list(v, 14)))
    v = A["pg_pn_sequence_table"]
    o.append("/* P2/data-symbol PN sequence (2624 chips, MSB first). */")
    o.append("static const uint8_t T2_PN_SEQ_BYTES[%d] = {\n%s\n};" % (len(v), fmt_list(["0x%02X" % x for x in v], 16)))
    v = A["pg_p1_active_carriers"]
    o.append("static const uint16_t T2_P1_CARRIERS[%d] = {\n%s\n};" % (len(v), fmt_list(v, 16)))
    v = A["pg_s1_modulation_patterns"]
    o.append("static const uint8_t T2_P1_S1[8][8] = {")
    for r in range(8):
        o.append("  {" + ", ".join("0x%02X" % x for x in v[r * 8:(r + 1) * 8]) + "},")
    o.append("};")
    v = A["pg_s2_modulation_patterns"]
    o.append("static const uint8_t T2_P1_S2[16][32] = {")
    for r in range(16):
        o.append("  {" + ", ".join("0x%02X" % x for x in v[r * 32:(r + 1) * 32]) + "},")
    o.append("};\n")
    o.append("#endif /* DVBT2_STD_TABLES_H */\n")
    out_path.write_text("\n".join(o))
    print("wrote", out_path, "codes", len(desc), "cp steps", nsteps, "count keys", len(keys))


if __name__ == "__main__":
    main()
