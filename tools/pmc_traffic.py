"""Per-launch HBM traffic of the hot kernels from two rocprofv3 PMC passes.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT_JSON [STEPS]

FETCH_DIR / WRITE_DIR hold the `--pmc FETCH_SIZE` and `--pmc WRITE_SIZE` passes
(`--output-format csv`, separate runs: the two counters do not fit one TCC pass on gfx950).
Correction applied as MI355X_MICROARCH.md §HBM prescribes: FETCH_SIZE (KiB) reports half the
bytes of a wide 16-B/lane coalesced read on gfx950 -> x2; WRITE_SIZE (KiB) is exact for
16-B/lane stores.  Result: bytes per launch, averaged over every launch of the kernel, and with
STEPS (the train steps the profiled bench.py ran: warmup + timed + instrumented) the bytes per step
of every kernel the run launched (one-time setup launches included: host->device copies and
parameter init, well under 1 % of a step).
"""
import csv
import glob
import json
import os
import sys

# bench.py tag -> kernel-name prefix of the launch it times (bf16 H=128 C3 workload)
TAGS = {"edge_bwd": "mlp_bwd_res_kernel", "edge_fwd": "mlp_fwd_res_kernel", "wgrad": "wgrad_kernel",
        "segment_sum": "segment_sum_kernel", "gather_rows": "gather_rows_kernel",
        "edge_bwd_fused": "edge_bwd_fused_kernel"}


def _rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def _per_kernel(rows, counter):
    acc = {}
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        name = name.replace("void ", "")
        a = acc.setdefault(name, [0, 0.0])
        a[0] += 1
        a[1] += float(r["Counter_Value"])
    return acc


def main():
    fdir, wdir, out = sys.argv[1:4]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else None
    fetch = _per_kernel(_rows(fdir), "FETCH_SIZE")
    write = _per_kernel(_rows(wdir), "WRITE_SIZE")
    kern = {}
    for name in sorted(set(fetch) | set(write)):
        nf, sf = fetch.get(name, [0, 0.0])
        nw, sw = write.get(name, [0, 0.0])
        fb = 2.0 * 1024.0 * sf / nf if nf else None
        wb = 1024.0 * sw / nw if nw else None
        kern[name] = {"launches": max(nf, nw), "fetch_bytes": fb, "write_bytes": wb,
                      "bytes": (fb or 0.0) + (wb or 0.0)}
    tags = {}
    for tag, pre in TAGS.items():
        hit = [v for k, v in kern.items() if pre in k]
        if hit:
            n = sum(h["launches"] for h in hit)
            tags[tag] = sum(h["bytes"] * h["launches"] for h in hit) / n
    total = sum(v["bytes"] * v["launches"] for v in kern.values())
    json.dump({"per_launch_bytes": tags, "kernels": kern, "total_bytes": total, "steps": steps,
               "per_step_bytes": total / steps if steps else None,
               "correction": "FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM)"},
              open(out, "w"), indent=1)
    print(json.dumps(tags))


if __name__ == "__main__":
    main()
