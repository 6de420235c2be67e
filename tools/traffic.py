"""Turn the rocprofv3 PMC passes into profiles/traffic.json (HBM bytes per launch of
the dominant kernel), with the gfx950 FETCH_SIZE correction calibrated on a kernel
of known byte count (MI355X_MICROARCH.md §HBM: FETCH_SIZE reads 1/2 of a wide
coalesced stream). Usage: python tools/traffic.py <profile dir> <arena_blocks>"""
import csv
import json
import os
import sys

KERNEL = "k_xxh64_glds_skew<16, 2, false, 8, 8, true>"  # rocprofv3 name of the dominant kernel


def rows(path):
    return list(csv.DictReader(open(path)))


def main(d, arena):
    fetch = [r for r in rows(os.path.join(d, "pmc_fetch_size.csv")) if KERNEL in r["Kernel_Name"]]
    write = [r for r in rows(os.path.join(d, "pmc_write_size.csv")) if KERNEL in r["Kernel_Name"]]
    calib = [r for r in rows(os.path.join(d, "pmc_fetch_calibration_probe.csv")) if "k_readpeak" in r["Kernel_Name"]]
    probe_bytes = 8 << 30  # tools/probe 8: every read-peak launch reads 8 GiB exactly once
    corr = probe_bytes / (sum(float(r["Counter_Value"]) for r in calib) / len(calib) * 1024)
    fk = sum(float(r["Counter_Value"]) for r in fetch) / len(fetch)
    wk = sum(float(r["Counter_Value"]) for r in write) / len(write)
    hbm = fk * 1024 * corr + wk * 1024
    alg = arena * (32768 + 8)
    out = {"kernel": "k_xxh64_glds_skew<16,nt,8w,4KiB>", "arena_blocks": arena, "fetch_size_kb": fk, "write_size_kb": wk,
           "fetch_correction": round(corr, 4), "hbm_bytes_per_launch": int(hbm),
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round(hbm / alg, 4),
           "source": os.path.relpath(d, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))}
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "traffic.json")
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]))
