"""Condense rocprofv3 outputs of a bench run into the files committed under profiles/.

Usage (on the GPU box, after the prof / fetch / write steps of tools/session.sh):
    python tools/profile_summary.py --tag r01 [--prof gpurun_out/prof]
        [--fetch gpurun_out/pmc_fetch] [--write gpurun_out/pmc_write]

Writes
  profiles/<tag>_kernel_stats.csv  -- the --kernel-trace --stats table (our kernels
                                      first, then every other kernel of the run)
  profiles/<tag>_summary.json      -- per cbn kernel: calls, average duration, and
                                      the PMC per-dispatch averages with the
                                      MI355X_MICROARCH.md HBM-section corrections:
                                      FETCH_SIZE (KB) x 2 for 16-B/lane streaming
                                      reads, WRITE_SIZE (KB) as is.
bench.py reads <tag>_summary.json to fill roofline.traffic.
"""
from __future__ import annotations

import argparse
import csv
import glob
import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OURS = ("k_query_staged", "k_query_fast", "k_query_cols", "k_query<", "k_build_tables", "k_cpd_", "k_scale", "k_param")


def short_name(name: str) -> str:
    """'void (anonymous namespace)::k_query_fast<2, true, 2>(int, ...)' -> 'k_query_fast<2, true, 2>'."""
    n = name
    for prefix in ("void ", "(anonymous namespace)::"):
        if n.startswith(prefix):
            n = n[len(prefix):]
    depth = 0
    for i, ch in enumerate(n):
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            return n[:i]
    return n


def find(d: str, suffix: str) -> str | None:
    hits = sorted(glob.glob(os.path.join(d, "**", "*" + suffix), recursive=True))
    return hits[0] if hits else None


def read_stats(d: str):
    path = find(d, "kernel_stats.csv")
    if not path:
        return [], None
    with open(path) as fh:
        rows = list(csv.DictReader(fh))
    return rows, path


def timed_window(d: str, warmup: int, steps: int):
    """Per-kernel duration stats over the bench's timed region only: dispatches
    warmup .. warmup + steps - 1 of each kernel in the --kernel-trace CSV (the
    --stats table also averages the warm-up and the cold-table steps)."""
    path = find(d, "kernel_trace.csv") if d else None
    if not path:
        return {}
    per = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            per.setdefault(short_name(r["Kernel_Name"]), []).append(
                (int(r["Start_Timestamp"]), (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3))
    out = {}
    for k, v in per.items():
        v.sort()
        x = sorted(t for _, t in v[warmup:warmup + steps])
        if len(x) >= steps // 2 and x:
            out[k] = {"timed_dispatches": len(x), "timed_avg_us": round(sum(x) / len(x), 3),
                      "timed_median_us": x[len(x) // 2], "timed_min_us": x[0], "timed_max_us": x[-1]}
    return out


def pmc_avg(d: str, counter: str):
    """Per-kernel average of one counter over its dispatches (KB, rocprofv3 units)."""
    path = find(d, "counter_collection.csv") if d else None
    if not path:
        return {}
    acc = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if r["Counter_Name"] != counter:
                continue
            k = short_name(r["Kernel_Name"])
            s, n = acc.get(k, (0.0, 0))
            acc[k] = (s + float(r["Counter_Value"]), n + 1)
    return {k: (s / n, n) for k, (s, n) in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tag", required=True)
    ap.add_argument("--prof", default=os.path.join(ROOT, "gpurun_out", "prof"))
    ap.add_argument("--fetch", default=os.path.join(ROOT, "gpurun_out", "pmc_fetch"))
    ap.add_argument("--write", default=os.path.join(ROOT, "gpurun_out", "pmc_write"))
    ap.add_argument("--warmup", type=int, default=20, help="bench warm-up steps before the timed region")
    ap.add_argument("--steps", type=int, default=200, help="bench timed steps")
    ap.add_argument("--command", default="", help="the profiled command line (recorded in the summary)")
    a = ap.parse_args()

    rows, src = read_stats(a.prof)
    os.makedirs(os.path.join(ROOT, "profiles"), exist_ok=True)
    ours = [r for r in rows if any(o in r["Name"] for o in OURS)]
    rest = [r for r in rows if r not in ours]
    if rows:
        out_csv = os.path.join(ROOT, "profiles", f"{a.tag}_kernel_stats.csv")
        with open(out_csv, "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=list(rows[0].keys()))
            w.writeheader()
            for r in ours + rest:
                w.writerow(r)
        print("wrote", out_csv)

    timed = timed_window(a.prof, a.warmup, a.steps)
    fetch = pmc_avg(a.fetch, "FETCH_SIZE")
    write = pmc_avg(a.write, "WRITE_SIZE")
    kernels = {}
    for r in ours:
        k = short_name(r["Name"])
        e = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3,
             "min_us": float(r["MinNs"]) / 1e3, "max_us": float(r["MaxNs"]) / 1e3}
        if k in timed and k.startswith("k_query"):
            e.update(timed[k])
        if k in fetch:
            e["fetch_size_kb"] = fetch[k][0]
            e["fetch_dispatches"] = fetch[k][1]
        if k in write:
            e["write_size_kb"] = write[k][0]
            e["write_dispatches"] = write[k][1]
        if k in fetch and k in write:
            # guide (MI355X_MICROARCH.md, HBM): FETCH_SIZE counts half the bytes of
            # 16-B/lane streaming reads -> x2; WRITE_SIZE exact for 16-B/lane stores.
            e["traffic_bytes"] = int(round((2.0 * fetch[k][0] + write[k][0]) * 1024))
        kernels[k] = e
    summary = {"tag": a.tag, "command": a.command, "stats_source": os.path.relpath(src, ROOT) if src else None,
               "pmc_correction": "traffic = (2 x FETCH_SIZE + WRITE_SIZE) KB per dispatch; FETCH_SIZE "
                                 "includes Infinity-Cache hits (memory-side request counter)",
               "kernels": kernels}
    out_json = os.path.join(ROOT, "profiles", f"{a.tag}_summary.json")
    with open(out_json, "w") as fh:
        json.dump(summary, fh, indent=1)
    print("wrote", out_json)
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
