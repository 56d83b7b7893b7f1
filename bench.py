#!/usr/bin/env python3
"""Throughput benchmark: million edge-updates/s of the BSMS-MGN training step on MI355X.

Workload (BASELINE.json configs[2], "C3"): BiStridedMeshGraphNet, 4 scales, 2 layers per
scale, stride 2, processor_size 15, H=128, n_hid=2 everywhere, do_concat_trick=True, on a
synthetic 1,000,000-node / 5,996,000-edge ellipsoid aero surface mesh; bf16 activations,
fp32 master weights, Adam. One step = forward (incl. the per-forward pooling hierarchy
build, as the reference does) + MSE + backward + gradient all-reduce + Adam.
An edge-update is one directed edge processed by one MeshGraphNetLayer;
EU/step is counted from the actual hierarchy (82,432,142 for C3).

N GPUs (torchrun): every rank trains on its own mesh of the same size (rotation seed = rank),
one RCCL gradient all-reduce per step: weak scaling, value = total EU / max-rank time.

--config c4 (BASELINE.json configs[3]): a fixed global batch of 64 meshes of
ellipsoid(400,250) (rotation seed = mesh index) split contiguously over the ranks (64/N each),
PyG-collated into micro-batches of 8 meshes with gradient accumulation, one all-reduce per step:
strong scaling.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0         # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_PEAK = {"bf16": 2500.0, "f32": 157.3}   # dense TFLOP/s (spec; no sparsity)

CONFIGS = {
    # name: (nu, nv, num_scales, dtype)
    "c3": (1000, 1000, 4, torch.bfloat16),
    "c2": (400, 250, 1, torch.float32),
    "c5": (2500, 2000, 6, torch.bfloat16),
    "small": (200, 125, 4, torch.bfloat16),
    "c4": (400, 250, 4, torch.bfloat16),
}
BATCHED = {"c4": (64, 8)}  # config: (global batch of meshes, meshes per micro-batch)


def build_model(num_scales, dev):
    from models.bsms_mgn import BiStridedMeshGraphNet
    kw = dict(processor_size=15, activation_fn="relu", num_hidden_layers_node_processor=2,
              num_hidden_layers_edge_processor=2, hidden_dim_processor=128, num_hidden_layers_node_encoder=2,
              hidden_dim_node_encoder=128, num_hidden_layers_edge_encoder=2, hidden_dim_edge_encoder=128,
              aggregation="add", hidden_dim_decoder=128, num_hidden_layers_decoder=2, dropout=0.0,
              do_concat_trick=True, num_scales=num_scales, layers_per_scale=2, stride=2)
    torch.manual_seed(0)
    return BiStridedMeshGraphNet(6, 4, 4, **kw).to(dev), kw


def mesh_tensors(nu, nv, seed, dev, dtype):
    from aerognn.meshgen import ellipsoid
    m = ellipsoid(nu, nv, seed=seed)
    t = {k: torch.from_numpy(v).to(dev) for k, v in m.items()}
    for k in ("x", "edge_attr"):
        t[k] = t[k].to(dtype)
    return t


def batch_tensors(nu, nv, seeds, dev, dtype):
    """PyG-style collate (aerognn.meshgen.collate: concatenated rows, edge_index offset by the
    running node count, `batch` = mesh index per node) of one mesh per seed, on the device."""
    from aerognn.meshgen import collate, ellipsoid
    b = collate([ellipsoid(nu, nv, seed=s) for s in seeds])
    t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
    for k in ("x", "edge_attr"):
        t[k] = t[k].to(dtype)
    return t


def edge_updates(model, t):
    """EU per step = sum over processor layers of the edge count of the level it runs on."""
    level, pools = model._hierarchy(t["edge_index"], t.get("batch"), t["pos"], t["x"].shape[0])
    E = [level.E] + [p.coarse.E for p in pools]
    nd = len(model.down_layers)
    eu = sum(len(model.down_layers[s]) * E[s] for s in range(nd))
    eu += len(model.bottleneck_layers) * E[nd]
    eu += sum(len(model.up_layers[s]) * E[nd - 1 - s] for s in range(nd))
    return eu, E


def cpu_baseline(num_scales, seconds_hint=20.0):
    """Oracle (oracle/refcpu.py, op-for-op the reference's CPU path) timed on host cores:
    one fp32 training step (fwd + MSE + bwd) of the same model on a bounded sample mesh."""
    from aerognn.meshgen import ellipsoid
    from oracle import refcpu as R
    nthreads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(nthreads)
    nu, nv = 250, 200  # 50,000 nodes / 299,000 edges
    m = ellipsoid(nu, nv, seed=0)
    t = {k: torch.from_numpy(v) for k, v in m.items()}
    model, kw = build_model(num_scales, "cpu")
    p = {k: v.detach().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    cfg = R.cfg_from_kwargs(**kw)
    batch = torch.zeros(t["x"].shape[0], dtype=torch.long)
    # EU of the sample
    down, bott, up = R.bsms_schedule(cfg["processor_size"], cfg["num_scales"], cfg["layers_per_scale"])
    Es, ei, pos, b = [], t["edge_index"], t["pos"], batch
    Es.append(ei.shape[1])
    node = torch.zeros(t["x"].shape[0], 1)
    for _ in down:
        node, _e, ei, b, pos, _a = R.downsample(node, torch.zeros(ei.shape[1], 1), ei, b, pos, cfg["stride"], True)
        Es.append(ei.shape[1])
    eu = sum(c * Es[i] for i, c in enumerate(down)) + bott * Es[len(down)] + \
        sum(c * Es[len(down) - 1 - i] for i, c in enumerate(up))
    t0 = time.perf_counter()
    pred = R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], cfg, batch, t["pos"], stable=True)
    loss = torch.nn.functional.mse_loss(pred, t["y"])
    loss.backward()
    dt = time.perf_counter() - t0
    return {"value": eu / dt / 1e6, "unit": "M edge-updates/s", "cores": nthreads, "kind": "port",
            "sample": f"1 fp32 train step (fwd+MSE+bwd) of the same BSMS-{num_scales} model, oracle/refcpu.py "
                      f"(the reference's aten ops in order) on a {nu * nv}-node/{m['edge_index'].shape[1]}-edge "
                      f"ellipsoid, {eu} EU, {dt:.1f} s, torch threads={nthreads}"}


def setup_bsms_gnn(nu, nv, seed, dev, dtype, num_levels=3):
    """The stale BSMS-GNN design (BSMS_MeshGraphNet) on the same mesh: the BFS
    bi-stride hierarchy is built once per mesh (MultiScaleGraphPreprocessor, 'done once during
    data loading'), timed separately and reported as preprocess_ms."""
    from models.bsms_mgn import BSMS_MeshGraphNet, MultiScaleGraphPreprocessor
    t = mesh_tensors(nu, nv, seed=seed, dev=dev, dtype=dtype)

    class _D:
        pass
    d = _D()
    d.edge_index, d.pos, d.num_nodes = t["edge_index"], t["pos"], t["x"].shape[0]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    multi = MultiScaleGraphPreprocessor(num_levels).create_multiscale_graph(d)
    torch.cuda.synchronize()
    prep_ms = 1e3 * (time.perf_counter() - t0)
    torch.manual_seed(0)
    model = BSMS_MeshGraphNet(6, 4, 4, num_levels=num_levels, latent_dim=128, hidden_dim=128, pos_dim=3).to(dev)
    Es = [int(ei.shape[1]) for ei in multi["edge_indices"]]
    eu = sum(Es)  # one GMP per level on the way down (levels 0..L-1) + the bottom GMP (level L)
    return model, t, multi, eu, Es, prep_ms


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="train", choices=["train", "fwd"])
    ap.add_argument("--model", default="bsms_mgn", choices=["bsms_mgn", "bsms_gnn"],
                    help="bsms_mgn: BiStridedMeshGraphNet (the headline); bsms_gnn: the stale BSMS_MeshGraphNet")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles",
                                                      "r1e_pmc_traffic.json"),
                    help="tools/pmc_traffic.py output: PMC-derived HBM bytes per launch of the hot kernels")
    args = ap.parse_args()

    from aerognn import core, dist as D
    rank, ws = D.init_from_env()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local %= max(1, torch.cuda.device_count())  # ranks > GPUs only when rehearsing on one card
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    nu, nv, S, dtype = CONFIGS[args.config]

    extra = {}
    scaling = "weak"
    if args.model == "bsms_mgn" and args.config in BATCHED:
        gb, mb = BATCHED[args.config]
        if gb % ws:
            raise SystemExit(f"bench: global batch {gb} is not divisible by {ws} ranks")
        per = gb // ws
        seeds = list(range(rank * per, (rank + 1) * per))
        model, kw = build_model(S, dev)
        batches = [batch_tensors(nu, nv, seeds[i:i + mb], dev, dtype) for i in range(0, per, mb)]
        eus = [edge_updates(model, b) for b in batches]
        eu_step = sum(e for e, _ in eus)
        Es = eus[0][1]
        scaling = "strong"
        what = "train step (fwd+MSE+bwd+allreduce+Adam)" if args.mode == "train" else "forward (no_grad)"
        workload = (f"BSMS-MGN {S}-scale U-Net {what}, global batch {gb} meshes of {nu * nv} nodes / "
                    f"{batches[0]['edge_index'].shape[1] // min(mb, per)} edges, {per} per GPU in micro-batches "
                    f"of {min(mb, per)} (gradient accumulation)")
        model_name = "BiStridedMeshGraphNet(H=128, n_hid=2, processor_size=15, stride=2, concat_trick)"
        extra["global_batch_meshes"] = gb
    elif args.model == "bsms_mgn":
        model, kw = build_model(S, dev)
        t = mesh_tensors(nu, nv, seed=rank, dev=dev, dtype=dtype)
        batches = [t]
        eu_step, Es = edge_updates(model, t)
        what = "train step (fwd+MSE+bwd+allreduce+Adam)" if args.mode == "train" else "forward (no_grad)"
        workload = (f"BSMS-MGN {S}-scale U-Net {what}, "
                    f"{t['x'].shape[0]} nodes / {t['edge_index'].shape[1]} edges per GPU")
        model_name = "BiStridedMeshGraphNet(H=128, n_hid=2, processor_size=15, stride=2, concat_trick)"
    else:
        model, t, multi, eu_step, Es, prep_ms = setup_bsms_gnn(nu, nv, rank, dev, dtype)
        batches = [t]
        extra["preprocess_ms"] = round(prep_ms, 1)
        what = "train step (fwd+MSE+bwd+allreduce+Adam)" if args.mode == "train" else "forward (no_grad)"
        workload = (f"BSMS-GNN (stale design) 3-level {what}, "
                    f"{t['x'].shape[0]} nodes / {t['edge_index'].shape[1]} edges per GPU, BFS hierarchy prebuilt")
        model_name = "BSMS_MeshGraphNet(num_levels=3, latent=128, hidden=128, WeightedEdgeConv pooling)"

    def fwd(b):
        if args.model == "bsms_mgn":
            return model(b["x"], b["edge_attr"], b["edge_index"], batch=b.get("batch"), pos=b["pos"])
        return model(b["x"], b["edge_attr"], b["edge_index"], multi_data=multi)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    allreduce = D.GradAllReduce(model.parameters())
    n_glob = D.global_count(sum(b["y"].numel() for b in batches), dev)

    def step():
        if args.mode == "train":
            for b in batches:  # gradient accumulation over micro-batches (sum loss / global count)
                loss = D.mse_sum_loss(fwd(b), b["y"], n_glob)
                loss.backward()
            allreduce()
            opt.step()
            opt.zero_grad(set_to_none=True)
        else:
            with torch.no_grad():
                for b in batches:
                    fwd(b)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    core.PROF = []
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if ws > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    prof, core.PROF = core.PROF, None
    if ws > 1:
        e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        if D._host_staged():
            e = e.cpu()
        torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(e.item())

    # per-kernel device time from the HIP events recorded on the launch stream
    agg = {}
    for tag, cost, s, e in prof:
        ms = s.elapsed_time(e)
        a = agg.setdefault(tag, [0, 0.0, 0.0, 0.0])
        a[0] += 1
        a[1] += ms
        a[2] += cost[0] if cost else 0.0
        a[3] += cost[1] if cost else 0.0
    dom = max(agg.items(), key=lambda kv: kv[1][1]) if agg else None
    roof = None
    kernels = {}
    for tag, (n, ms, by, fl) in agg.items():
        kernels[tag] = {"launches": n, "avg_us": 1e3 * ms / n, "alg_GBs": by / (ms * 1e-3) / 1e9,
                        "alg_TFLOPs": fl / (ms * 1e-3) / 1e12, "share_of_step": ms / (1e3 * elapsed)}
    dname = "bf16" if dtype == torch.bfloat16 else "f32"
    if dom:
        tag, (n, ms, by, fl) = dom
        ach = by / n / (ms / n * 1e-3) / 1e9
        traffic = None
        if (args.traffic and os.path.exists(args.traffic) and args.config == "c3" and args.mode == "train"
                and args.model == "bsms_mgn"):
            traffic = json.load(open(args.traffic)).get("per_launch_bytes", {}).get(tag)
        roof = {"kernel": tag, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                "alg_bytes_per_launch": by / n, "avg_launch_us": 1e3 * ms / n,
                "mfma_tflops": round(fl / (ms * 1e-3) / 1e12, 2), "mfma_peak": MFMA_PEAK[dname]}

    value = eu_step * args.steps * ws / elapsed / 1e6
    out = {
        "metric": "million edge-updates/sec, 1M-node/6M-edge mesh, 1->8 MI355X",
        "value": round(value, 2),
        "unit": "M edge-updates/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * elapsed / args.steps, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": dname,
        "data": "synthetic ellipsoid aero surface mesh (aerognn.meshgen), random-init weights (seed 0)",
        "config": {"workload": workload, "model": model_name, **extra,
                   "mode": args.mode, "edge_updates_per_step_per_gpu": eu_step, "level_edges": Es,
                   "global_batch": extra.get("global_batch_meshes", ws), "parallelism": f"dp{ws}"},
        "roofline": roof,
        "kernels": kernels,
    }
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and args.model == "bsms_mgn":
        out["cpu_baseline"] = cpu_baseline(S)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if ws > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
