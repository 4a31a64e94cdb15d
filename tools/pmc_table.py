"""Average per-dispatch PMC counters of the query kernels from rocprofv3 CSVs: python tools/pmc_table.py DIR..."""
import collections
import csv
import sys

for d in sys.argv[1:]:
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        if "k_query" in r["Kernel_Name"]:
            k = r["Kernel_Name"].replace("void (anonymous namespace)::", "").split("(")[0]
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d, k, {c: round(sum(x) / len(x)) for c, x in v.items()})
