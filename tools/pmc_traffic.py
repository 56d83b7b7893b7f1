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

# bench.py tag -> kernel names of the launch it times (bf16 H=128 C3 workload), first present wins:
# `edge_bwd` is the fused edge backward by default, the split path's resident backward otherwise
TAGS = {"edge_bwd": ("edge_bwd_fused_kernel", "mlp_bwd_res_kernel"), "edge_fwd": ("edge32_fwd_kernel", "mlp_fwd_res_kernel"),
        "wgrad": ("wgrad_kernel",), "segment_sum": ("segment_sum4_kernel", "segment_sum_kernel"),
        "gather_rows": ("gather_rows4_kernel", "gather_rows_kernel"),
        "node_fwd": ("node32_fwd_kernel", "mlp_fwd_kernelIDF16bLi4ELi0E"),
        "node_bwd": ("node32_bwd_kernel", "mlp_bwd_kernelIDF16bLi4ELi0E")}


def _rows(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def _per_kernel(rows, counter):
    """name -> [launches, summed value, per-dispatch values in dispatch order]"""
    acc = {}
    rows = sorted(rows, key=lambda r: int(r.get("Dispatch_Id", 0) or 0))
    for r in rows:
        if r.get("Counter_Name") != counter:
            continue
        name = r["Kernel_Name"].replace("(anonymous namespace)::", "")  # non-template kernels' demangled names
        name = name.split("(")[0].replace("void ", "")
        a = acc.setdefault(name, [0, 0.0, []])
        a[0] += 1
        a[1] += float(r["Counter_Value"])
        a[2].append(float(r["Counter_Value"]))
    return acc


def main():
    fdir, wdir, out = sys.argv[1:4]
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else None
    fetch = _per_kernel(_rows(fdir), "FETCH_SIZE")
    write = _per_kernel(_rows(wdir), "WRITE_SIZE")
    kern = {}
    for name in sorted(set(fetch) | set(write)):
        nf, sf, _ = fetch.get(name, [0, 0.0, []])
        nw, sw, _ = write.get(name, [0, 0.0, []])
        fb = 2.0 * 1024.0 * sf / nf if nf else None
        wb = 1024.0 * sw / nw if nw else None
        kern[name] = {"launches": max(nf, nw), "fetch_bytes": fb, "write_bytes": wb,
                      "bytes": (fb or 0.0) + (wb or 0.0)}
    tags, disp = {}, {}
    for tag, pres in TAGS.items():
        pre = next((p for p in pres if any(p in k for k in kern)), pres[0])
        hit = [v for k, v in kern.items() if pre in k]
        if hit:
            n = sum(h["launches"] for h in hit)
            tags[tag] = sum(h["bytes"] * h["launches"] for h in hit) / n
        # per-dispatch bytes (the two passes pair by dispatch order): a consumer that knows how many
        # of these launches carry its tag (e.g. the 15 edge-layer backwards among the encoders' on
        # the same kernel) can average just those
        names = [k for k in fetch if pre in k]
        if len(names) == 1 and names[0] in write and len(fetch[names[0]][2]) == len(write[names[0]][2]):
            disp[tag] = [2048.0 * f + 1024.0 * w for f, w in zip(fetch[names[0]][2], write[names[0]][2])]
    total = sum(v["bytes"] * v["launches"] for v in kern.values())
    json.dump({"per_launch_bytes": tags, "dispatch_bytes": disp, "kernels": kern, "total_bytes": total, "steps": steps,
               "per_step_bytes": total / steps if steps else None,
               "correction": "FETCH_SIZE*2*1024 + WRITE_SIZE*1024 (MI355X_MICROARCH.md §HBM)"},
              open(out, "w"), indent=1)
    print(json.dumps(tags))


if __name__ == "__main__":
    main()
