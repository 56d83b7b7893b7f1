#!/bin/bash
# SQ counter passes of tools/e16_stamps.py (the 16-row-tile edge forward + backward at C3 level 0).
# usage: tools/e16_counters.sh TAG   (GPU box; writes gpurun_out/TAG_c*/ and gpurun_out/TAG_summary.json)
R=$PWD
TAG=${1:-e16}
cd /tmp && export TMPDIR=/tmp && cd "$R"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_RD SQ_LDS_IDX_ACTIVE" \
           "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --output-format csv -d gpurun_out/${TAG}_c$i -o m -- \
      python tools/e16_stamps.py --reps 2 > gpurun_out/${TAG}_c$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/${TAG}_c$i.log; exit 1; }
done
python tools/sq_stall.py gpurun_out gpurun_out/${TAG}_summary.json > /dev/null
python - "$TAG" << 'PY'
import collections, csv, glob, json, re, sys
tag = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/{tag}_c*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if "edge16" not in k:
            continue
        name = "fwd" if "fwd" in k else "bwd"
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {}
for n, c in acc.items():
    m = {k: sum(v) / len(v) for k, v in c.items()}
    wc = m.get("SQ_WAVE_CYCLES", 1.0)
    row = dict(m)
    for key, cc in (("wait", "SQ_WAIT_ANY"), ("issue_stall", "SQ_WAIT_INST_ANY"), ("active", "SQ_ACTIVE_INST_ANY"),
                    ("valu", "SQ_ACTIVE_INST_VALU"), ("lds_active", "SQ_ACTIVE_INST_LDS"), ("lds_issue_stall", "SQ_WAIT_INST_LDS"),
                    ("vmem_active", "SQ_ACTIVE_INST_VMEM")):
        if cc in m:
            row[key] = round(m[cc] / wc, 3)
    if "GRBM_GUI_ACTIVE" in m and "SQ_VALU_MFMA_BUSY_CYCLES" in m:
        row["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (1024 * m["GRBM_GUI_ACTIVE"] / 8), 3)
    out[n] = row
json.dump(out, open(f"gpurun_out/{tag}_e16.json", "w"), indent=1)
for n, r in out.items():
    print(n, {k: r[k] for k in r if k in ("wait", "issue_stall", "active", "valu", "lds_active", "lds_issue_stall", "vmem_active", "mfma_busy", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_LDS_IDX_ACTIVE")})
PY
