"""Aggregate rocprofv3 counter_collection CSVs per kernel: median (and mean) per dispatch of every counter,
plus `_dispatches` (how many dispatches of that kernel the run made, from the first counter
seen)."""
import csv
import re
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
            # drop the parameter list only (names in anonymous namespaces hold "(" too)
            short = re.sub(r"\([^()]*\)\s*$", "", name).replace("void ", "")[:80]
            out[short][row["Counter_Name"]].append(float(row["Counter_Value"]))
res = {}
for k, d in out.items():
    # the median per dispatch: the steady-state launch of a timed loop (a one-off dispatch of
    # the same kernel — e.g. the rank-0 table build at upload, one 25K-query search — would
    # otherwise skew the mean); the mean is kept beside it
    res[k] = {c: sorted(v)[len(v) // 2] for c, v in d.items()}
    res[k].update({c + "_mean": sum(v) / len(v) for c, v in d.items()})
    res[k]["_dispatches"] = max(len(v) for v in d.values())
print(json.dumps(res, indent=1))
