"""Average PMC counter values per dispatch, per kernel, over rocprofv3 --pmc csv dirs.
Usage: python tools/pmc_summary.py KERNEL_REGEX DIR [DIR ...]"""
import collections
import csv
import glob
import os
import re
import sys

pat = re.compile(sys.argv[1])
acc = collections.defaultdict(lambda: [0, 0.0])
for d in sys.argv[2:]:
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if not pat.search(r["Kernel_Name"]):
                continue
            k = (re.sub(r"_ZN12_GLOBAL__N_1\d+", "", r["Kernel_Name"])[:40], r["Counter_Name"])
            a = acc[k]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
for (kern, ctr), (n, s) in sorted(acc.items()):
    print(f"{kern:40s} {ctr:32s} {s / n:16.4g}  (n={n})")
