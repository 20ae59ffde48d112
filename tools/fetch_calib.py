#!/usr/bin/env python3
"""Summarise tools/fetch_calib runs under rocprofv3 --pmc: counter bytes / true bytes per kernel.

    python tools/fetch_calib.py DIR [DIR ...]   (rocprofv3 -d DIR of a FETCH_SIZE or WRITE_SIZE pass)

FETCH_SIZE and WRITE_SIZE are in KiB.  Every calibration kernel moves exactly 1 GiB."""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

TRUE_BYTES = 1 << 30
WIDTH = {"unsigned short": 2, "unsigned int": 4, "uint2": 8, "HIP_vector_type<unsigned int, 2u>": 8, "W16": 16}


def width_of(name):
    m = re.search(r"(rd|wr)_kernel<(.+?)>\(", name)
    if not m:
        return None, None
    return m.group(1), WIDTH.get(m.group(2), m.group(2))


ORDER = [("rd", 2), ("rd", 4), ("rd", 8), ("rd", 16), ("wr", 2), ("wr", 4), ("wr", 8), ("wr", 16)]


def from_db(d, rows):
    """rocpd (sqlite) output: kernel names are truncated (-T), so the launch order of
    tools/fetch_calib.hip (rd 2/4/8/16 B, wr 2/4/8/16 B, twice) identifies each dispatch"""
    import sqlite3
    for fn in glob.glob(os.path.join(d, "**", "*.db"), recursive=True):
        c = sqlite3.connect(fn)
        k = 0
        for name, ctr, val in c.execute("select kernel_name, counter_name, value from counters_collection "
                                        "order by dispatch_id"):
            if not (name.startswith("rd_kernel") or name.startswith("wr_kernel")):
                continue
            kind, w = ORDER[k % len(ORDER)]
            assert name.startswith(kind), (name, kind)
            rows[(ctr, kind, w)].append(float(val))
            k += 1


def main(dirs):
    rows = defaultdict(list)
    for d in dirs:
        from_db(d, rows)
        for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(fn) as fh:
                for r in csv.DictReader(fh):
                    kind, w = width_of(r.get("Kernel_Name", ""))
                    if kind:
                        rows[(r["Counter_Name"], kind, w)].append(float(r["Counter_Value"]))
    out = {}
    for (ctr, kind, w), vals in sorted(rows.items(), key=lambda kv: str(kv[0])):
        ratio = sum(vals) / len(vals) * 1024 / TRUE_BYTES
        out["%s %s %sB" % (ctr, kind, w)] = round(ratio, 4)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1:])
