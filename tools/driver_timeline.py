"""Itemise the driver's bench command from its rocprofv3 kernel trace
(round 4): the k_query_staged<2> dispatches of bench.py
--steps K --warmup W in order -- W warmup launches, then the K timed ones,
then bench's back-to-back calibration launches -- with each dispatch's
duration and the GPU idle gap before it, plus the bench line's own timing
fields.  Usage: python tools/driver_timeline.py TRACE_DIR BENCH_JSON_LINE_FILE OUT.json"""
import csv
import glob
import json
import os
import sys


def main():
    trace_dir, bench_file, out = sys.argv[1:4]
    path = sorted(glob.glob(os.path.join(trace_dir, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = []
    with open(path) as fh:
        for r in csv.DictReader(fh):
            if "k_query_staged<2>" in r["Kernel_Name"]:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    rows.sort()
    line = json.loads([l for l in open(bench_file) if l.startswith("{")][-1])
    K, W = line["steps"], line["warmup"]
    dur = [(e - s) / 1e3 for s, e in rows]
    gap = [0.0] + [(rows[i][0] - rows[i - 1][1]) / 1e3 for i in range(1, len(rows))]
    timed = list(range(W, W + K))
    back = list(range(W + K + 4, len(rows)))  # bench.backlogged_launch_us: 4 host-timed, then the queued ones
    back = [i for i in back if i < W + K + 4 + max(K, 100)]
    avg = lambda xs: round(sum(xs) / len(xs), 3) if xs else None
    res = dict(command="rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps %d --warmup %d" % (K, W),
               dispatches=len(rows),
               timed=dict(duration_us=[round(dur[i], 2) for i in timed], gap_before_us=[round(gap[i], 2) for i in timed],
                          avg_duration_us=avg([dur[i] for i in timed]),
                          avg_gap_us=avg([gap[i] for i in timed[1:]]),
                          first_gap_us=round(gap[timed[0]], 2)),
               backlogged=dict(avg_duration_us=avg([dur[i] for i in back]), avg_gap_us=avg([gap[i] for i in back[1:]]),
                               n=len(back)),
               bench_line=dict(value=line["value"], ms_per_step=line["ms_per_step"], timing=line.get("timing"),
                               roofline_avg_us=line["roofline"]["avg_us"]))
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "bench_line"})[:1500])


if __name__ == "__main__":
    main()
