"""One line per bench log of tools/gpu_placement.sh: shape, frac, launch min/max, the
arena's VA alignment, the live read peak, and (with a rocprofv3 session dir) the
kernel-trace average of the dominant kernel and the frac it implies."""
import csv
import glob
import json
import sys

log = sys.argv[1]
line = [ln for ln in open(log) if ln.startswith("{")]
if not line:
    print(log, "NO LINE")
    sys.exit(1)
d = json.loads(line[-1])
r = d["roofline"]
rp = r.get("measured_read_peak") or {}
out = {"log": log, "kernel": r["kernel"], "frac": r["frac"], "avg_ms": r["avg_launch_ms"],
       "min_ms": r["launch_ms"]["min"], "max_ms": r["launch_ms"]["max"],
       "va": d["config"]["arena"]["va"], "va_align": d["config"]["arena"]["va_alignment"],
       "alloc": d["config"]["arena"].get("mode", "plain"), "mapped_chunk": d["config"]["arena"].get("mapped_chunk"),
       "read_peak_frac": rp.get("frac"), "root_check": d["root_check"]}
if len(sys.argv) > 2:
    stats = glob.glob(sys.argv[2] + "/**/*kernel_stats.csv", recursive=True)
    for row in csv.DictReader(open(stats[0])):
        if "k_xxh64_glds_skew" in row["Name"] and "true" in row["Name"].split(",")[5]:
            avg = float(row["AverageNs"]) * 1e-6
            out["prof_avg_ms"] = round(avg, 4)
            out["prof_frac"] = round(d["config"]["arena_blocks"] * 32776 / (avg * 1e-3) / 8e12, 4)
            out["prof_calls"] = int(row["Calls"])
print(json.dumps(out))
