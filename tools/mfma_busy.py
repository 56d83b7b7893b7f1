"""MFMA-busy fraction per kernel from a rocprofv3 PMC pass of
`--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE` (MI355X_MICROARCH.md §rocprofv3):
SQ_VALU_MFMA_BUSY_CYCLES counts MFMA cycles summed over the chip (= 32 x N_mfma for
v_mfma_f32_32x32x16_bf16) and GRBM_GUI_ACTIVE is the kernel's busy clock summed over the 8 XCDs,
so   mfma_busy = MFMA_BUSY / (1024 SIMDs x GRBM_GUI_ACTIVE / 8).
Usage: python tools/mfma_busy.py PMC_DIR OUT_JSON
"""
import collections
import csv
import glob
import json
import os
import re
import sys

SIMDS = 256 * 4


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
        avg = {k: v[1] / v[0] for k, v in ctr.items()}
        busy, grbm = avg.get("SQ_VALU_MFMA_BUSY_CYCLES"), avg.get("GRBM_GUI_ACTIVE")
        util = busy / (SIMDS * grbm / 8.0) if busy is not None and grbm else None
        res[name] = {"launches": max(v[0] for v in ctr.values()), **{k: round(v, 1) for k, v in avg.items()},
                     "mfma_busy": util}
    res = dict(sorted(res.items(), key=lambda kv: -(kv[1].get("GRBM_GUI_ACTIVE", 0) * kv[1]["launches"])))
    json.dump({"formula": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 * GRBM_GUI_ACTIVE / 8)", "kernels": res},
              open(out, "w"), indent=1)
    for name, v in list(res.items())[:12]:
        print(f"{name[:60]:60s} launches {v['launches']:5d}  mfma_busy {v['mfma_busy']}")


if __name__ == "__main__":
    main()
