"""Collect one rocprofv3 evidence session (tools/profile.sh <tag>, run on the GPU box)
into profiles/<tag>/ and write profiles/traffic.json for bench.py.

From gpurun_out/prof_<tag>/:
  trace/**/*kernel_stats.csv         -> kernel_stats.csv (kernel trace + stats of bench.py)
  trace.log (its JSON line)          -> bench_under_rocprof.json (the bench line of THAT process)
  fetch/**/*counter_collection.csv   -> pmc_fetch_size.csv   (separate --pmc FETCH_SIZE pass)
  write/**/*counter_collection.csv   -> pmc_write_size.csv   (separate --pmc WRITE_SIZE pass)
  calib/**/*counter_collection.csv   -> pmc_fetch_calibration_probe.csv
  gather_{trace,fetch,write}/...     -> gather_*.csv, gather_traffic.json (the gather
                                        workload: hash kernel + locality-order kernels)

traffic.json (per launch of the dominant kernel, one 2M-block arena pass):
  hbm_bytes_per_launch = FETCH_SIZE x 1024 x correction + WRITE_SIZE x 1024, where the
  gfx950 FETCH_SIZE correction is calibrated on a read-peak kernel of known byte count
  (MI355X_MICROARCH.md, HBM / rocprofv3 section: FETCH_SIZE counts half of a wide
  coalesced stream);
  profile_avg_launch_ms = the kernel-trace average of that kernel in the same session,
  and profile_frac = algorithmic bytes / that average / 8 TB/s, so the bench line's
  roofline.frac can be recomputed from the committed profile.

    python tools/collect_profile.py <tag> [arena_blocks]
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "k_xxh64_glds_skew<16, 2, false, 8, 8, true>"  # rocprofv3 name of the dominant kernel
BLOCK = 32768
PEAK = 8e12


def one(pattern):
    hits = sorted(glob.glob(pattern, recursive=True))
    if not hits:
        raise SystemExit(f"no file matches {pattern}")
    return hits[0]


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def main(tag, arena):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    files = {
        "kernel_stats.csv": one(os.path.join(src, "trace", "**", "*kernel_stats.csv")),
        "pmc_fetch_size.csv": one(os.path.join(src, "fetch", "**", "*counter_collection.csv")),
        "pmc_write_size.csv": one(os.path.join(src, "write", "**", "*counter_collection.csv")),
        "pmc_fetch_calibration_probe.csv": one(os.path.join(src, "calib", "**", "*counter_collection.csv")),
    }
    for name, path in files.items():
        shutil.copy(path, os.path.join(dst, name))
    bench_line = None
    with open(os.path.join(src, "trace.log")) as f:
        for line in f:
            if line.startswith("{"):
                bench_line = json.loads(line)
    with open(os.path.join(dst, "bench_under_rocprof.json"), "w") as f:
        json.dump(bench_line, f, indent=1)

    fetch = [r for r in rows(files["pmc_fetch_size.csv"]) if KERNEL in r["Kernel_Name"]]
    write = [r for r in rows(files["pmc_write_size.csv"]) if KERNEL in r["Kernel_Name"]]
    calib = [r for r in rows(files["pmc_fetch_calibration_probe.csv"]) if "k_readpeak" in r["Kernel_Name"]]
    probe_bytes = 8 << 30  # tools/probe 8: every read-peak launch reads 8 GiB exactly once
    corr = probe_bytes / (sum(float(r["Counter_Value"]) for r in calib) / len(calib) * 1024)
    fk = sum(float(r["Counter_Value"]) for r in fetch) / len(fetch)
    wk = sum(float(r["Counter_Value"]) for r in write) / len(write)
    hbm = fk * 1024 * corr + wk * 1024
    alg = arena * (BLOCK + 8)
    stats = [r for r in rows(files["kernel_stats.csv"]) if KERNEL in r["Name"]]
    avg_ns = float(stats[0]["AverageNs"])
    # the bench's timed launches in the same trace: the last launch_ms.n dispatches of the
    # dominant kernel (settle and warmup launches come first), to compare with the HIP
    # events the bench line's frac comes from
    trace_csv = glob.glob(os.path.join(src, "trace", "**", "*kernel_trace.csv"), recursive=True)
    timed = None
    if trace_csv and bench_line:
        shutil.copy(trace_csv[0], os.path.join(dst, "kernel_trace.csv"))
        disp = [r for r in rows(trace_csv[0]) if KERNEL in r["Kernel_Name"]]
        disp.sort(key=lambda r: int(r["Start_Timestamp"]))
        k = bench_line["roofline"]["launch_ms"]["n"]
        last = disp[-k:]
        t_ms = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in last) / len(last) * 1e-6
        timed = {"launches": len(last), "avg_launch_ms": round(t_ms, 4),
                 "frac": round(arena * (BLOCK + 8) / (t_ms * 1e-3) / PEAK, 4),
                 "bench_hip_event_avg_ms": bench_line["roofline"]["avg_launch_ms"],
                 "agreement": round(t_ms / bench_line["roofline"]["avg_launch_ms"], 4)}
    # the spread over fresh processes of the same session (placement), if collected
    spread = None
    plain = sorted(glob.glob(os.path.join(src, "plain_*.log")))
    fr = []
    for f in plain:
        ln = [x for x in open(f) if x.startswith("{")]
        if ln:
            fr.append(json.loads(ln[-1])["roofline"]["frac"])
            shutil.copy(f, os.path.join(dst, os.path.basename(f)))
    if fr:
        fr_all = sorted(fr + ([bench_line["roofline"]["frac"]] if bench_line else []))
        spread = {"processes": len(fr_all), "median": fr_all[len(fr_all) // 2], "min": fr_all[0], "max": fr_all[-1],
                  "fracs": fr_all, "what": "bench.py c3 frac in fresh processes of one session (plain and the "
                                           "profiled one): the spread the arena's HBM placement gives"}
    out = {"kernel": "k_xxh64_glds_skew<16,nt,8w,4KiB>", "arena_blocks": arena, "fetch_size_kb": fk,
           "write_size_kb": wk, "fetch_correction": round(corr, 4), "hbm_bytes_per_launch": int(hbm),
           "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round(hbm / alg, 4),
           "profile_calls": int(stats[0]["Calls"]), "profile_avg_launch_ms": round(avg_ns * 1e-6, 4),
           "profile_min_launch_ms": round(float(stats[0]["MinNs"]) * 1e-6, 4),
           "profile_max_launch_ms": round(float(stats[0]["MaxNs"]) * 1e-6, 4),
           "profile_frac": round(alg / (avg_ns * 1e-9) / PEAK, 4),
           "profile_timed_launches": timed, "placement_spread": spread,
           "bench_under_rocprof": {"frac": bench_line["roofline"]["frac"] if bench_line else None,
                                   "avg_launch_ms": bench_line["roofline"]["avg_launch_ms"] if bench_line else None},
           "source": os.path.relpath(dst, ROOT)}
    with open(os.path.join(ROOT, "profiles", "traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))
    if os.path.isdir(os.path.join(src, "gather_trace")):
        gather(src, dst, corr)


GATHER_KERNEL = "k_xxh64_glds_var<16, 2, false, 8, 8, true, true, true"  # a prefix: later template arguments vary


def last_json(path):
    line = None
    with open(path) as f:
        for x in f:
            if x.startswith("{"):
                line = json.loads(x)
    return line


def gather(src, dst, corr):
    """The gather workload's session: per launch of the hash kernel, HBM bytes from the
    FETCH_SIZE / WRITE_SIZE passes against the algorithmic bytes of the bench line, and
    the locality-order kernels' share of the launch."""
    files = {
        "gather_kernel_stats.csv": one(os.path.join(src, "gather_trace", "**", "*kernel_stats.csv")),
        "gather_pmc_fetch_size.csv": one(os.path.join(src, "gather_fetch", "**", "*counter_collection.csv")),
        "gather_pmc_write_size.csv": one(os.path.join(src, "gather_write", "**", "*counter_collection.csv")),
    }
    for name, path in files.items():
        shutil.copy(path, os.path.join(dst, name))
    line = last_json(os.path.join(src, "gather_trace.log"))
    with open(os.path.join(dst, "gather_bench_under_rocprof.json"), "w") as f:
        json.dump(line, f, indent=1)
    alg = line["roofline"]["algorithmic_bytes_per_launch"]

    def per_kernel(path):
        acc = {}
        for r in rows(path):
            name = r["Kernel_Name"]
            acc.setdefault(name, []).append(float(r["Counter_Value"]))
        return {k: sum(v) / len(v) for k, v in acc.items()}

    fetch, write = per_kernel(files["gather_pmc_fetch_size.csv"]), per_kernel(files["gather_pmc_write_size.csv"])
    hk = [k for k in fetch if GATHER_KERNEL in k][0]
    hbm = fetch[hk] * 1024 * corr + write[[k for k in write if GATHER_KERNEL in k][0]] * 1024
    stats = {r["Name"]: r for r in rows(files["gather_kernel_stats.csv"])}
    hs = [v for k, v in stats.items() if GATHER_KERNEL in k][0]
    order_ns = sum(float(v["AverageNs"]) for k, v in stats.items() if "k_order_" in k)
    order_bytes = sum(fetch[k] * 1024 * corr for k in fetch if "k_order_" in k) + \
        sum(write[k] * 1024 for k in write if "k_order_" in k)
    out = {"kernel": "k_xxh64_glds_var<16,nt,8w,4KiB,lens,offs,ordered>",
           "workload": line["config"]["workload"], "algorithmic_bytes_per_launch": alg,
           "hbm_bytes_per_launch": int(hbm), "traffic_over_algorithmic": round(hbm / alg, 4),
           "profile_calls": int(hs["Calls"]), "profile_avg_launch_ms": round(float(hs["AverageNs"]) * 1e-6, 4),
           "profile_frac_hash_kernel": round(alg / (float(hs["AverageNs"]) * 1e-9) / PEAK, 4),
           "order_kernels_avg_us": round(order_ns * 1e-3, 1), "order_kernels_hbm_bytes": int(order_bytes),
           "bench_under_rocprof": {"frac": line["roofline"]["frac"], "avg_launch_ms": line["roofline"]["avg_launch_ms"],
                                   "note": "bench launch = order kernels + hash kernel"},
           "source": os.path.relpath(dst, ROOT)}
    with open(os.path.join(dst, "gather_traffic.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 2 << 20)
