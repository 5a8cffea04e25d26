"""Aggregate rocprofv3 counter_collection CSVs per kernel (mean per dispatch)."""
import csv
import glob
import json
import sys
from collections import defaultdict

root = sys.argv[1]
out = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            name = row.get("Kernel_Name", "")
            short = name.split("(")[0].replace("void ", "")[:60]
            out[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in out.items()}
print(json.dumps(res, indent=1))
