#!/usr/bin/env python3
"""Aggregate rocprofv3 PMC passes into per-kernel HBM traffic (profiles/pmc_summary.json).

Collection (on the GPU box; one counter group per rocprofv3 run, kernel-trace only —
never combined with sys/runtime traces), e.g.:
    rocprofv3 --pmc FETCH_SIZE  -d OUT/fetch --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE  -d OUT/write --output-format csv -- python3 bench.py ...
    rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d OUT/hit --output-format csv -- ...
then:  python tools/pmc_traffic.py OUT [BATCHES] > profiles/pmc_summary.json
BATCHES = encode batches the profiled command ran (bench.py --warmup 1 --steps 1 --kt-steps 1
--no-serial-pass with every leg off: 3); with it every kernel also gets "bytes_per_batch"
(its summed HBM bytes / BATCHES), which bench.py adds up over the sort-stream kernels.

Corrections (MI355X_MICROARCH.md §HBM): FETCH_SIZE and WRITE_SIZE are in KiB;
on gfx950 FETCH_SIZE reports half the bytes of wide coalesced streaming reads, so the
read side is doubled ("fetch_bytes_x2"); WRITE_SIZE is exact for 16-B-per-lane stores.
Both raw and corrected numbers are kept; ratios between variants are unaffected.
Per-launch values are averaged over the dispatches of the kernel; families follow
include/kolm.h KOLM_KT_*.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

FAMILY = [
    ("k_classify", "classify"), ("k_keygen", "keygen"), ("k_msd_", "msd"), ("k_copy_back", "msd"),
    ("k_small_sort", "small_sort"), ("k_single", "small_sort"), ("k_finalize_eq", "small_sort"),
    ("k_lsd_", "lsd"), ("k_r0_", "lsd"), ("k_lz_local", "lz_parse"), ("k_lz_stitch", "lz_parse"),
    ("k_duval", "lyndon_gather"), ("k_prevc", "lyndon_gather"), ("k_keypos", "keygen"),
    ("k_mtf", "mtf"), ("k_sizes", "sizes"), ("k_mdl", "sizes"), ("k_offsets", "sizes"),
    ("k_emit", "emit"), ("k_rice", "emit"), ("k_simple", "emit"), ("k_lz_emit", "emit"),
    ("k_tile", "lyndon_gather"), ("k_lyn", "lyndon_gather"), ("k_fed", "lyndon_gather"),
    ("k_bbwt_gather", "lyndon_gather"), ("k_prev3", "lyndon_gather"),
]


def family(name):
    for key, fam in FAMILY:
        if key in name:
            return fam
    return None


def short(name):
    name = name.replace("(anonymous namespace)::", "").replace("kolm::", "")
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0]


def load(outdir):
    per = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values per dispatch]
    for f in glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            k = short(row.get("Kernel_Name", ""))
            per[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    return per


def main():
    outdir = sys.argv[1]
    batches = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    per = load(outdir)
    kernels = {}
    fams = defaultdict(lambda: {"fetch_kib": 0.0, "write_kib": 0.0, "dispatches": 0})
    for k, cs in per.items():
        ent = {}
        for c, vals in cs.items():
            ent[c + "_avg"] = sum(vals) / len(vals)
            ent["dispatches"] = max(ent.get("dispatches", 0), len(vals))
        if "FETCH_SIZE_avg" in ent or "WRITE_SIZE_avg" in ent:
            fb = ent.get("FETCH_SIZE_avg", 0.0) * 1024
            wb = ent.get("WRITE_SIZE_avg", 0.0) * 1024
            ent["fetch_bytes_raw"] = fb
            ent["fetch_bytes_x2"] = 2 * fb
            ent["write_bytes"] = wb
            ent["hbm_bytes_per_launch"] = 2 * fb + wb
            if batches:
                ent["bytes_per_batch"] = (2 * fb + wb) * ent["dispatches"] / batches
        if "TCC_HIT_sum_avg" in ent and "TCC_MISS_sum_avg" in ent:
            h, m = ent["TCC_HIT_sum_avg"], ent["TCC_MISS_sum_avg"]
            ent["l2_hit_rate"] = h / (h + m) if h + m else None
        kernels[k] = ent
        fam = family(k)
        if fam:
            d = ent.get("dispatches", 0)
            fams[fam]["fetch_kib"] += ent.get("FETCH_SIZE_avg", 0.0) * d
            fams[fam]["write_kib"] += ent.get("WRITE_SIZE_avg", 0.0) * d
            fams[fam]["dispatches"] += d
    fam_out = {}
    for fam, v in fams.items():
        fam_out[fam] = {"fetch_bytes_x2_total": 2 * v["fetch_kib"] * 1024, "write_bytes_total": v["write_kib"] * 1024,
                        "dispatches": v["dispatches"]}
    print(json.dumps({"source": os.path.abspath(outdir), "batches": batches,
                      "note": __doc__.split("Corrections")[1].strip(),
                      "kernels": kernels, "families_total": fam_out}, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
