"""Where the waves of each kernel spend their cycles, from a rocprofv3 PMC pass of
`--pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU`
(MI355X_MICROARCH.md: WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~= WAVE_CYCLES, disjoint):
  wait      = SQ_WAIT_ANY / SQ_WAVE_CYCLES         parked on s_waitcnt / barrier (memory latency)
  issue     = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES    ready but not issued (pipe busy: MFMA/VALU/LDS)
  active    = SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES  issuing
  valu      = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES issuing VALU
Usage: python tools/sq_stall.py PMC_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import re
import sys


def main():
    d, out = sys.argv[1:3]
    acc = collections.defaultdict(lambda: collections.defaultdict(lambda: [0, 0.0]))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = re.sub(r"_ZN12_GLOBAL__N_1\d+", "", r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", ""))
            a = acc[name][r["Counter_Name"]]
            a[0] += 1
            a[1] += float(r["Counter_Value"])
    res = {}
    for name, ctr in acc.items():
        tot = {k: v[1] for k, v in ctr.items()}
        wc = tot.get("SQ_WAVE_CYCLES") or 0.0
        row = {"launches": max(v[0] for v in ctr.values()), **{k: round(v / ctr[k][0], 1) for k, v in tot.items()}}
        if wc:
            for key, c in (("wait", "SQ_WAIT_ANY"), ("issue", "SQ_WAIT_INST_ANY"), ("active", "SQ_ACTIVE_INST_ANY"),
                           ("valu", "SQ_ACTIVE_INST_VALU")):
                row[key] = round(tot.get(c, 0.0) / wc, 3)
        res[name] = row
    res = dict(sorted(res.items(), key=lambda kv: -(kv[1].get("SQ_WAVE_CYCLES", 0) * kv[1]["launches"])))
    json.dump({"fractions_of": "SQ_WAVE_CYCLES", "kernels": res}, open(out, "w"), indent=1)
    for name, v in list(res.items())[:10]:
        print(f"{name[:58]:58s} n {v['launches']:4d} wait {v.get('wait')} issue {v.get('issue')} "
              f"active {v.get('active')} valu {v.get('valu')}")


if __name__ == "__main__":
    main()
