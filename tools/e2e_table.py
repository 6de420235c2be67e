"""Markdown tables from `bench.py --workload batch_e2e` / `commit_e2e` logs.

    python tools/e2e_table.py gpurun_out/<tag>/batch_e2e.log gpurun_out/<tag>/commit_e2e.log
"""
import json
import sys

BATCH = [("dev", "device, pageable"), ("dev_reg", "device, registered"), ("host_1", "host, 1 thread"),
         ("host_all", "host, 16 threads"), ("host_1_reg", "host, 1 thread, registered"),
         ("host_all_reg", "host, 16 threads, registered"), ("split", "split"), ("split_1", "split, 1 host thread"),
         ("routed_reg", "routed (leg)"), ("routed_reg_1", "routed, 1 thread (leg)")]
COMMIT = [("dev_inplace", "device in place"), ("dev_hbm", "device, HBM arena"), ("host_1", "host, 1 thread"),
          ("host_all", "host, 16 threads"), ("split", "split"), ("split_1", "split, 1 host thread"),
          ("routed", "routed (leg)"), ("routed_1", "routed, 1 thread (leg)")]


def rows(path):
    for line in open(path):
        line = line.strip()
        if line.startswith("{"):
            d = json.loads(line)
            if "table" not in d:
                yield d


def fmt(v):
    return f"{v:,.0f}" if v >= 100 else f"{v:.1f}"


def table(path):
    out = []
    first = True
    for d in rows(path):
        batch = "batch" in d
        cols = BATCH if batch else COMMIT
        if first:
            out.append("| " + ("batch" if batch else "forest") + " | MB | " + " | ".join(c[1] for c in cols) +
                       " | split gain | routed / best |")
            out.append("|---" * (len(cols) + 4) + "|")
            first = False
        cells = []
        for k, _ in cols:
            if k + "_us" not in d:  # sessions before the column existed
                cells.append("–")
                continue
            v = fmt(d[k + "_us"])
            if k.startswith("routed"):
                v += f" ({d.get(k + '_leg')})"
            if k.startswith("split"):
                v += f" [{d.get(k + '_dev_share', 0):.2f}]"
            cells.append(v)
        ob = d.get("routed_reg_over_best", d.get("routed_over_best"))
        ob1 = d.get("routed_reg_1_over_best", d.get("routed_1_over_best"))
        name = d.get("batch") or d.get("forest")
        out.append(f"| {name} | {d['hashed_bytes'] / 1e6:,.1f} | " + " | ".join(cells) +
                   f" | {d['split_gain']:.2f} | {ob:.2f} / {ob1:.2f} |")
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print(table(p))
        print()
