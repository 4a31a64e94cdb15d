"""Per-kernel averages of rocprofv3 outputs (run on the GPU box, then the raw
directories can be deleted so gpurun_out stays small).

    python tools/pmc_summary.py --kernel k_param_query --out gpurun_out/x.json DIR [DIR ...]

For every DIR: *_counter_collection.csv -> mean Counter_Value per dispatch of
the matching kernels; *_kernel_stats.csv -> the matching rows."""
import argparse
import csv
import glob
import json
import os
import re
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--kernel", default="k_param")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rx = re.compile(a.kernel)
    res = {"kernel_regex": a.kernel, "counters": {}, "stats": []}
    for d in a.dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            acc = defaultdict(list)
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    if rx.search(row.get("Kernel_Name", "")):
                        acc[(row["Kernel_Name"][:90], row["Counter_Name"])].append(float(row["Counter_Value"]))
            for (k, c), v in acc.items():
                res["counters"].setdefault(k, {})[c] = sum(v) / len(v)
        for path in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
            with open(path) as fh:
                for row in csv.DictReader(fh):
                    if rx.search(row.get("Name", "")):
                        res["stats"].append(row)
    with open(a.out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1)[:4000])


if __name__ == "__main__":
    main()
