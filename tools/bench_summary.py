"""One line per bench log: value, ms/step and the kernels above 0.5 ms/step (ms/step, us/launch).

  python tools/bench_summary.py gpurun_out/*.log
"""
import json
import sys

for path in sys.argv[1:]:
    line = None
    for ln in open(path):
        if ln.startswith("{"):
            line = ln
    if line is None:
        print(f"{path}: no bench line")
        continue
    d = json.loads(line)
    ks = {n: (round(v["ms_per_step"], 2), round(v["avg_us"], 1)) for n, v in d.get("kernels", {}).items()
          if v.get("ms_per_step", 0) > 0.5}
    print(f"{path}: {d['value']} {d['unit']}  {d['ms_per_step']:.2f} ms/step  {ks}")
