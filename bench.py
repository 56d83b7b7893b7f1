#!/usr/bin/env python3
"""Throughput benchmark: million edge-updates/s of the BSMS-MGN training step on MI355X.

Workload (BASELINE.json configs[2], "C3"): BiStridedMeshGraphNet, 4 scales, 2 layers per
scale, stride 2, processor_size 15, H=128, n_hid=2 everywhere, do_concat_trick=True, on a
synthetic 1,000,000-node / 5,996,000-edge ellipsoid aero surface mesh; bf16 activations,
fp32 master weights, Adam. One step = forward (incl. the per-forward pooling hierarchy
build, as the reference does) + MSE + backward + gradient all-reduce + Adam.
An edge-update is one directed edge processed by one MeshGraphNetLayer;
EU/step is counted from the actual hierarchy.

N GPUs: `bench.py --gpus N` starts N worker processes itself (one per GPU; or run it under
torchrun with N ranks, whose WORLD_SIZE must equal --gpus): every rank trains on its own mesh of the same size (rotation seed = rank),
one RCCL gradient all-reduce per step (bucketed, overlapped with the backward): weak scaling,
value = total EU / max-rank time. The same run also measures the north-star scaling case,
C4 strong scaling (BASELINE.json configs[3]: a fixed global batch of 64 ellipsoid(400,250)
meshes split over the ranks), and reports it under "c4_strong" (disable: --no-c4).

--config c4 makes C4 the headline instead; --config c5 --mode fwd is the HBM stress forward.

Timing: W untimed warm-up steps, then K steps with NO instrumentation, bracketed by barrier +
synchronize, max over ranks. A separate pass of --profile-steps steps (not timed for `value`)
records HIP events around every libaerognn launch for the per-kernel table and the roofline.

Prints ONE JSON line (rank 0).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import statistics
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
    "c4small": (40, 25, 4, torch.bfloat16),  # the C4 leg's shape at test size (tests/test_gpu_dist.py)
}
BATCHED = {"c4": (64, 8), "c4small": (4, 2)}  # config: (global batch of meshes, meshes per micro-batch)
MODEL_NAME = "BiStridedMeshGraphNet(H=128, n_hid=2, processor_size=15, stride=2, concat_trick)"


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
    running node count, `batch` = mesh index per node), moved to the device."""
    from aerognn.meshgen import collate, ellipsoid
    b = collate([ellipsoid(nu, nv, seed=s) for s in seeds])
    t = {k: torch.from_numpy(v).to(dev) for k, v in b.items()}
    for k in ("x", "edge_attr"):
        t[k] = t[k].to(dtype)
    return t


def level_sizes(model, t):
    """(N_l, E_l) of every level of the hierarchy actually built for this input."""
    level, pools = model._hierarchy(t["edge_index"], t.get("batch"), t["pos"], t["x"].shape[0])
    return [level.N] + [p.coarse.N for p in pools], [level.E] + [p.coarse.E for p in pools]


def layer_levels(model):
    """Level index of every processor layer, in execution order (bsms_mgn.py:126-215)."""
    nd = len(model.down_layers)
    lv = []
    for s in range(nd):
        lv += [s] * len(model.down_layers[s])
    lv += [nd] * len(model.bottleneck_layers)
    for s in range(nd):
        lv += [nd - 1 - s] * len(model.up_layers[s])
    return lv


def edge_updates(model, t):
    """EU per step = sum over processor layers of the edge count of the level it runs on."""
    _, E = level_sizes(model, t)
    return sum(E[l] for l in layer_levels(model)), E


def alg_step_cost(model, t, s, train, H=128, d_n=6, d_e=4, d_out=4):
    """SURVEY §8(d) algorithmic minimum of one step (fully fused): (bytes, flops).

    Per processor layer on level l: B = E(2sH + 8) + N(8sH), F = 8H^2 E + 14H^2 N.
    Pool l -> l+1: sH(N_l + E_l + N_l+1 + E_l+1) + 24 E_l + 12 N_l; unpool: sH(N_l+1 + 2 N_l) + 4 N_l.
    Encoders/decoder: read input + write latent; flops exact. Training = 3x forward."""
    N, E = level_sizes(model, t)
    B = F = 0.0
    for l in layer_levels(model):
        B += E[l] * (2 * s * H + 8) + N[l] * 8 * s * H
        F += 8 * H * H * E[l] + 14 * H * H * N[l]
    for l in range(len(N) - 1):
        B += s * H * (N[l] + E[l] + N[l + 1] + E[l + 1]) + 24 * E[l] + 12 * N[l]
        B += s * H * (N[l + 1] + 2 * N[l]) + 4 * N[l]
    B += N[0] * (d_n * s + s * H) + E[0] * (d_e * s + s * H) + N[0] * (s * H + d_out * s)
    F += E[0] * 2 * (d_e * H + 3 * H * H) + N[0] * 2 * (d_n * H + 3 * H * H) + N[0] * 2 * (3 * H * H + H * d_out)
    k = 3.0 if train else 1.0
    return k * B, k * F


def cpu_info():
    name = platform.processor() or "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                name = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return name


def host_threads():
    """Every core this process may run on: its CPU affinity set, bounded by a cgroup v2 CPU quota
    when one is set (a quota of Q CPUs makes more than Q threads slower, not faster)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (min(aff, quota) if quota else aff), {"affinity_cpus": aff, "cgroup_quota_cpus": quota}


def latest_profile(suffix):
    """The newest committed profiles/r<round>[e]_<suffix> (round names sort: r2_ < r2e_ < r3_)."""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_" + suffix)))
    return fs[-1] if fs else None


def latest_cpu_plan():
    """The newest committed profiles/r*_cpu_plan.json (bench.py --cpu-plan on the GPU box)."""
    f = latest_profile("cpu_plan.json")
    if not f:
        return None, None
    return os.path.basename(f), json.load(open(f))


def _median_time(fn, reps=3, label=None):
    """1 warm-up + median of `reps`; with a label, a progress line per run and a heartbeat every
    60 s on stderr (a multi-minute CPU row must not look hung to a job watchdog)."""
    import threading
    stop = threading.Event()
    if label:
        t_start = time.perf_counter()

        def beat():
            while not stop.wait(60):
                print(f"cpu-plan {label}: running, {time.perf_counter() - t_start:.0f} s", file=sys.stderr, flush=True)
        threading.Thread(target=beat, daemon=True).start()
    try:
        fn()  # warm-up
        ts = []
        for i in range(reps):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
            if label:
                print(f"cpu-plan {label}: run {i + 1}/{reps} {ts[-1]:.2f} s", file=sys.stderr, flush=True)
        return statistics.median(ts)
    finally:
        stop.set()


def cpu_baseline(num_scales, nu=250, nv=200):
    """The oracle (oracle/refcpu.py: the reference's aten ops in order, verified bitwise-equal to
    the imported reference in tools/make_goldens.py) timed on this box's host cores, BASELINE.md
    §3 protocol (1 warm-up, median of 3), fp32, on a bounded sample of the headline model: the
    same BSMS model's forward on a 50,000-node / 299,000-edge ellipsoid (~20 s of CPU work)."""
    from aerognn.meshgen import ellipsoid
    from oracle import refcpu as R
    nthreads, tinfo = host_threads()
    torch.set_num_threads(nthreads)
    m = ellipsoid(nu, nv, seed=0)
    t = {k: torch.from_numpy(v) for k, v in m.items()}
    model, kw = build_model(num_scales, "cpu")
    p = {k: v.detach().clone() for k, v in model.state_dict().items()}
    cfg = R.cfg_from_kwargs(**kw)
    batch = torch.zeros(t["x"].shape[0], dtype=torch.long)
    down, bott, up = R.bsms_schedule(cfg["processor_size"], cfg["num_scales"], cfg["layers_per_scale"])
    Es, ei, pos, b = [t["edge_index"].shape[1]], t["edge_index"], t["pos"], batch
    node = torch.zeros(t["x"].shape[0], 1)
    for _ in down:
        node, _e, ei, b, pos, _a = R.downsample(node, torch.zeros(ei.shape[1], 1), ei, b, pos, cfg["stride"], True)
        Es.append(ei.shape[1])
    eu = sum(c * Es[i] for i, c in enumerate(down)) + bott * Es[len(down)] + \
        sum(c * Es[len(down) - 1 - i] for i, c in enumerate(up))

    def fwd():
        with torch.no_grad():
            R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], cfg, batch, t["pos"], stable=True)
    dt = _median_time(fwd)
    out = {"value": eu / dt / 1e6, "unit": "M edge-updates/s", "cores": nthreads, "threads": tinfo, "kind": "port",
           "cpu": cpu_info(), "torch": torch.__version__, "dtype": "f32",
           "sample": f"fp32 forward (no_grad) of the same BSMS-{num_scales} model, oracle/refcpu.py, on a "
                     f"{nu * nv}-node/{m['edge_index'].shape[1]}-edge ellipsoid ({eu} EU); 1 warm-up, median of 3 "
                     f"= {dt:.2f} s; torch threads={nthreads} (every CPU of the affinity set, bounded by the cgroup "
                     f"quota). The full-size C3 forward (minutes of CPU work) is c3_forward, from bench.py --cpu-plan"}
    name, plan = latest_cpu_plan()
    if plan:
        row = next((r for r in plan["rows"] if r["config"] == "C3" and r["mode"] == "fwd"), None)
        if row:
            out["c3_forward"] = {"value": row["M_EU_per_s"], "unit": "M edge-updates/s", "seconds": row["seconds"],
                                 "cores": plan["cores"], "nodes": row["nodes"], "edges": row["edges"],
                                 "source": f"profiles/{name} (bench.py --cpu-plan on this box type, "
                                           f"{plan['protocol']})"}
    return out


def cpu_plan():
    """BASELINE.md §3 in full: forward at C1/C2/C3 and train step at C1/C2, 1 warm-up + median
    of 3, fp32, oracle/refcpu.py on host cores (minutes of CPU work; run once, results committed)."""
    from aerognn.meshgen import ellipsoid
    from oracle import refcpu as R
    nthreads, tinfo = host_threads()
    torch.set_num_threads(nthreads)
    out = {"cpu": cpu_info(), "cores": nthreads, "threads": tinfo, "torch": torch.__version__, "dtype": "f32",
           "protocol": "1 warm-up, median of 3", "rows": []}
    for name, (nu, nv), S, modes in (("C1", (40, 25), 1, ("fwd", "train")), ("C2", (400, 250), 1, ("fwd", "train")),
                                     ("C3", (1000, 1000), 4, ("fwd",))):
        m = ellipsoid(nu, nv, seed=0)
        t = {k: torch.from_numpy(v) for k, v in m.items()}
        model, kw = build_model(S, "cpu")
        cfg = R.cfg_from_kwargs(**kw)
        batch = torch.zeros(t["x"].shape[0], dtype=torch.long)
        # the bench model family at every config (BSMS-MGN; num_scales=1 is the single-level MGN-15)
        eu = 15 * t["edge_index"].shape[1] if S == 1 else None
        run = lambda p: R.bsms_forward(p, t["x"], t["edge_attr"], t["edge_index"], cfg, batch,  # noqa: E731
                                       t["pos"], stable=True)
        if eu is None:
            down, bott, up = R.bsms_schedule(cfg["processor_size"], cfg["num_scales"], cfg["layers_per_scale"])
            Es, ei, pos, b = [t["edge_index"].shape[1]], t["edge_index"], t["pos"], batch
            node = torch.zeros(t["x"].shape[0], 1)
            for _ in down:
                node, _e, ei, b, pos, _a = R.downsample(node, torch.zeros(ei.shape[1], 1), ei, b, pos, 2, True)
                Es.append(ei.shape[1])
            eu = sum(c * Es[i] for i, c in enumerate(down)) + bott * Es[len(down)] + \
                sum(c * Es[len(down) - 1 - i] for i, c in enumerate(up))
        p0 = {k: v.detach().clone() for k, v in model.state_dict().items()}
        for mode in modes:
            if mode == "fwd":
                def fn():
                    with torch.no_grad():
                        run(p0)
            else:
                pt = {k: v.clone().requires_grad_(True) for k, v in p0.items()}
                opt = torch.optim.Adam(list(pt.values()), lr=1e-3)

                def fn():
                    torch.nn.functional.mse_loss(run(pt), t["y"]).backward()
                    opt.step()
                    opt.zero_grad(set_to_none=True)
            dt = _median_time(fn, label=f"{name} {mode}")
            out["rows"].append({"config": name, "mode": mode, "nodes": int(t["x"].shape[0]),
                                "edges": int(t["edge_index"].shape[1]), "eu": int(eu), "seconds": dt,
                                "M_EU_per_s": eu / dt / 1e6})
            print(json.dumps(out["rows"][-1]), flush=True)
    return out


def kernel_table(prof, steps, elapsed_step_s):
    agg = {}
    for tag, cost, s, e in prof:
        ms = s.elapsed_time(e)
        a = agg.setdefault(tag, [0, 0.0, 0.0, 0.0, 0.0, False])
        a[0] += 1
        a[1] += ms
        if cost:
            a[2] += cost[0]
            a[3] += cost[1]
            a[4] += cost[2] if len(cost) > 2 else cost[0]
            a[5] = True
    tab = {}
    for tag, (n, ms, by, fl, impl, has) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        sec = ms * 1e-3
        tab[tag] = {"launches_per_step": n / steps, "avg_us": 1e3 * ms / n, "ms_per_step": ms / steps,
                    "share_of_step": (ms / steps) / (1e3 * elapsed_step_s),
                    "alg_GBs": (by / sec / 1e9) if has else None, "impl_GBs": (impl / sec / 1e9) if has else None,
                    "alg_TFLOPs": (fl / sec / 1e12) if has else None,
                    "_sum": (n, ms, by, fl, impl, has)}
    return tab


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def rank_envs(n, port, base=None):
    """The environment of each of n worker ranks on this node (torchrun's variables, rendezvous on
    127.0.0.1): rank r drives GPU r (LOCAL_RANK), HSA_ENABLE_IPC_MODE_LEGACY=0 kept (dmabuf IPC)."""
    base = dict(os.environ if base is None else base)
    base.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return [dict(base, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                 GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)) for r in range(n)]


def launch_ranks(n, argv):
    """`bench.py --gpus N` started without torchrun: start N fresh worker processes of this script
    (one per GPU, each a child process — nothing here has touched the GPU, and no exec), wait for
    all of them and return the worst exit status. Rank 0 prints the JSON line. If a rank fails,
    the others (the exact processes started here) are terminated so no rank waits forever in a
    collective."""
    import subprocess
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env)
             for env in rank_envs(n, port)]
    rc = 0
    try:
        pending = list(procs)
        while pending:
            for p in list(pending):
                r = p.poll()
                if r is None:
                    continue
                pending.remove(p)
                if r != 0:
                    rc = rc or r
                    for q in pending:
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
                p.wait()
    return rc if rc >= 0 else 128 - rc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--mode", default="train", choices=["train", "fwd"])
    ap.add_argument("--model", default="bsms_mgn", choices=["bsms_mgn", "bsms_gnn"],
                    help="bsms_mgn: BiStridedMeshGraphNet (the headline); bsms_gnn: the stale BSMS_MeshGraphNet")
    ap.add_argument("--profile-steps", type=int, default=1, help="extra instrumented steps for the kernel table")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-c4", action="store_true", help="skip the secondary C4 strong-scaling measurement")
    ap.add_argument("--strong-config", default=None, choices=sorted(BATCHED),
                    help="run the strong-scaling leg on this batched config (default: c4 after a c3 train run)")
    ap.add_argument("--cpu-plan", action="store_true", help="run BASELINE.md §3's full CPU plan and exit")
    ap.add_argument("--traffic", default=latest_profile("pmc_traffic.json"),
                    help="tools/pmc_traffic.py output: PMC-derived HBM bytes per launch of the hot kernels "
                         "and per step (default: the newest profiles/r*_pmc_traffic.json)")
    args = ap.parse_args()
    if args.cpu_plan:
        print(json.dumps(cpu_plan()))
        return
    if args.gpus < 1:
        raise SystemExit("bench: --gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one process per GPU, started here (the same run torchrun would make)
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        raise SystemExit(f"bench: --gpus {args.gpus} but WORLD_SIZE={os.environ.get('WORLD_SIZE')} "
                         f"(the launcher's rank count must equal --gpus)")

    from aerognn import core, dist as D
    rank, ws = D.init_from_env()
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local %= max(1, torch.cuda.device_count())  # ranks > GPUs only when rehearsing on one card
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    nu, nv, S, dtype = CONFIGS[args.config]
    dname = "bf16" if dtype == torch.bfloat16 else "f32"
    s_el = 2 if dtype == torch.bfloat16 else 4
    what = "train step (fwd+MSE+bwd+allreduce+Adam)" if args.mode == "train" else "forward (no_grad)"

    def setup(config):
        """(model, batches, eu_step, level_edges, workload, scaling, extra) for one config."""
        nu, nv, S, _ = CONFIGS[config]
        extra = {}
        if args.model == "bsms_mgn" and config in BATCHED:
            gb, mb = BATCHED[config]
            if gb % ws:
                raise SystemExit(f"bench: global batch {gb} is not divisible by {ws} ranks")
            per = gb // ws
            seeds = list(range(rank * per, (rank + 1) * per))
            model, _ = build_model(S, dev)
            batches = [batch_tensors(nu, nv, seeds[i:i + mb], dev, dtype) for i in range(0, per, mb)]
            eus = [edge_updates(model, b) for b in batches]
            workload = (f"BSMS-MGN {S}-scale U-Net {what}, global batch {gb} meshes of {nu * nv} nodes / "
                        f"{batches[0]['edge_index'].shape[1] // min(mb, per)} edges, {per} per GPU in micro-batches "
                        f"of {min(mb, per)} (gradient accumulation)")
            extra["global_batch_meshes"] = gb
            return model, batches, sum(e for e, _ in eus), eus[0][1], workload, "strong", extra
        if args.model == "bsms_mgn":
            model, _ = build_model(S, dev)
            t = mesh_tensors(nu, nv, seed=rank, dev=dev, dtype=dtype)
            eu, Es = edge_updates(model, t)
            workload = (f"BSMS-MGN {S}-scale U-Net {what}, {t['x'].shape[0]} nodes / {t['edge_index'].shape[1]} "
                        f"edges per GPU")
            return model, [t], eu, Es, workload, "weak", extra
        from models.bsms_mgn import BSMS_MeshGraphNet, MultiScaleGraphPreprocessor
        t = mesh_tensors(nu, nv, seed=rank, dev=dev, dtype=dtype)
        d = type("D", (), {})()
        d.edge_index, d.pos, d.num_nodes = t["edge_index"], t["pos"], t["x"].shape[0]
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        multi = MultiScaleGraphPreprocessor(3).create_multiscale_graph(d)
        torch.cuda.synchronize()
        extra["preprocess_ms"] = round(1e3 * (time.perf_counter() - t0), 1)
        extra["multi"] = multi
        torch.manual_seed(0)
        model = BSMS_MeshGraphNet(6, 4, 4, num_levels=3, latent_dim=128, hidden_dim=128, pos_dim=3).to(dev)
        Es = [int(ei.shape[1]) for ei in multi["edge_indices"]]
        workload = (f"BSMS-GNN (stale design) 3-level {what}, {t['x'].shape[0]} nodes / {t['edge_index'].shape[1]} "
                    f"edges per GPU, BFS hierarchy prebuilt")
        return model, [t], sum(Es), Es, workload, "weak", extra

    allreduce_ref = []  # the headline step's GradAllReduce (for the line's collective record)

    def make_step(model, batches, extra):
        multi = extra.pop("multi", None)

        def fwd(b):
            if multi is None:
                return model(b["x"], b["edge_attr"], b["edge_index"], batch=b.get("batch"), pos=b["pos"])
            return model(b["x"], b["edge_attr"], b["edge_index"], multi_data=multi)
        opt = torch.optim.Adam(model.parameters(), lr=1e-3)
        allreduce = D.GradAllReduce(model.parameters())
        allreduce_ref[:] = [allreduce]
        n_glob = D.global_count(sum(b["y"].numel() for b in batches), dev)

        def step():
            if args.mode == "train":
                for i, b in enumerate(batches):  # gradient accumulation over micro-batches
                    if i == len(batches) - 1:
                        allreduce.arm()  # buckets all-reduce as their grads land (overlaps the backward)
                    D.mse_sum_loss(fwd(b), b["y"], n_glob).backward()
                allreduce()
                opt.step()
                opt.zero_grad(set_to_none=True)
            else:
                with torch.no_grad():
                    for b in batches:
                        fwd(b)
        return step

    def timed_run(step, steps, warmup, per_rank=None):
        """Wall time of `steps` steps bracketed by barrier + synchronize, the MAX over ranks; with
        per_rank a dict, also each rank's own time (min / max over ranks)."""
        for _ in range(warmup):
            step()
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if ws > 1:
            torch.distributed.barrier()
        elapsed = time.perf_counter() - t0
        own = elapsed
        if ws > 1:
            e = torch.tensor([elapsed], dtype=torch.float64, device=dev)
            if D._host_staged():
                e = e.cpu()
            torch.distributed.all_reduce(e, op=torch.distributed.ReduceOp.MAX)
            elapsed = float(e.item())
        if per_rank is not None:
            lo = own
            if ws > 1:
                m = torch.tensor([own], dtype=torch.float64, device=dev)
                if D._host_staged():
                    m = m.cpu()
                torch.distributed.all_reduce(m, op=torch.distributed.ReduceOp.MIN)
                lo = float(m.item())
            per_rank.update(rank_ms_min=1e3 * lo / steps, rank_ms_max=1e3 * elapsed / steps)
        return elapsed

    model, batches, eu_step, Es, workload, scaling, extra = setup(args.config)
    step = make_step(model, batches, extra)
    elapsed = timed_run(step, args.steps, args.warmup)
    step_s = elapsed / args.steps
    eu_all = eu_step * ws
    if ws > 1:  # every rank's own hierarchy (its mesh seed differs): sum the counts, not rank 0's x N
        t_eu = torch.tensor([float(eu_step)], dtype=torch.float64, device=dev)
        if D._host_staged():
            t_eu = t_eu.cpu()
        torch.distributed.all_reduce(t_eu)
        eu_all = int(t_eu.item())
    value = eu_all * args.steps / elapsed / 1e6

    # instrumented pass (not part of `value`): HIP events around every libaerognn launch
    kernels, roof = {}, None
    if args.profile_steps > 0:
        core.PROF = []
        torch.cuda.synchronize()
        for _ in range(args.profile_steps):
            step()
        torch.cuda.synchronize()
        prof, core.PROF = core.PROF, None
        kernels = kernel_table(prof, args.profile_steps, step_s)
    if args.model == "bsms_mgn":
        B, F = 0.0, 0.0
        for b in batches:
            bb, ff = alg_step_cost(model, b, s_el, args.mode == "train")
            B, F = B + bb, F + ff
        t_hbm, t_mfma = B / (HBM_PEAK_GBS * 1e9), F / (MFMA_PEAK[dname] * 1e12)
        t_roof = max(t_hbm, t_mfma)
        step_roof = {"alg_bytes": B, "alg_flops": F, "t_roof_ms": 1e3 * t_roof, "t_measured_ms": 1e3 * step_s,
                     "bound": "hbm" if t_hbm >= t_mfma else "mfma", "frac": t_roof / step_s,
                     "achieved_GBs": B / step_s / 1e9, "achieved_TFLOPs": F / step_s / 1e12,
                     "basis": "SURVEY §8(d) fully-fused minimum: per layer E(2sH+8)+N(8sH) bytes, 8H^2E+14H^2N "
                              "flops, + pool/unpool/encoders/decoder; x3 for training"}
    else:
        step_roof = None
    pmc = None
    if args.traffic and os.path.exists(args.traffic) and args.config == "c3" and args.mode == "train" \
            and args.model == "bsms_mgn":
        pmc = json.load(open(args.traffic))
    if step_roof is not None and pmc and pmc.get("per_step_bytes"):
        step_roof["traffic_bytes"] = pmc["per_step_bytes"]
        step_roof["traffic_over_alg8d"] = pmc["per_step_bytes"] / step_roof["alg_bytes"]
        step_roof["traffic_source"] = os.path.relpath(args.traffic, ROOT) + " (PMC FETCH_SIZE/WRITE_SIZE passes)"
    if kernels:
        def kroof(tag, basis_bytes, basis):
            n, ms, by, fl, impl, has = kernels[tag]["_sum"]
            ach = basis_bytes / (ms * 1e-3) / 1e9
            traffic = (pmc or {}).get("per_launch_bytes", {}).get(tag)
            disp = (pmc or {}).get("dispatch_bytes", {}).get(tag)
            steps_pmc = (pmc or {}).get("steps")
            if disp and steps_pmc:  # the tag's own launches: the largest n/step x steps dispatches
                k = int(round(n / args.profile_steps)) * steps_pmc
                if 0 < k <= len(disp):
                    traffic = sum(sorted(disp)[-k:]) / k
            return {"kernel": tag, "bound": "hbm", "achieved": round(ach, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBS, 4), "traffic": traffic,
                    "alg_bytes_per_launch": basis_bytes / n,
                    "traffic_over_alg": (traffic / (basis_bytes / n)) if traffic else None,
                    "avg_launch_us": 1e3 * ms / n, "launches_per_step": n / args.profile_steps,
                    "share_of_step": kernels[tag]["share_of_step"],
                    "mfma_tflops": round(fl / (ms * 1e-3) / 1e12, 2), "mfma_peak": MFMA_PEAK[dname],
                    "alg_basis": basis}
        # the headline roofline: the kernel with the most device time among those that HAVE a §8(d)
        # share (wgrad has none: a fused backward never re-reads G and X)
        k8 = [t for t, v in kernels.items() if v["_sum"][5] and v["_sum"][2] > 0]
        if k8:
            roof = kroof(k8[0], kernels[k8[0]]["_sum"][2], "SURVEY §8(d) share of the fused layer (DESIGN.md §5)")
        top = next(iter(kernels))
        if top != (k8[0] if k8 else None) and kernels[top]["_sum"][5]:
            # the top kernel has no §8(d) share: its own operator I/O (G and X read once, dW/db
            # written) prices it, in a separately named object
            oio = kroof(top, kernels[top]["_sum"][4], "operator I/O (G and X read once, dW/db written); "
                                                      "its §8(d) fused share is 0 bytes")
            if roof is not None:
                roof["top_kernel_operator_io"] = oio
        if roof is not None:
            roof["step"] = step_roof
        for v in kernels.values():
            v.pop("_sum")
    if roof is None and step_roof:
        roof = {"kernel": None, "bound": step_roof["bound"], "achieved": step_roof["achieved_GBs"],
                "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": step_roof["frac"], "traffic": None, "step": step_roof}

    out = {
        "metric": "million edge-updates/sec, 1M-node/6M-edge mesh, 1->8 MI355X",
        "value": round(value, 2),
        "unit": "M edge-updates/s",
        "n_gpus": ws,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(1e3 * step_s, 3),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": dname,
        "data": "synthetic ellipsoid aero surface mesh (aerognn.meshgen), random-init weights (seed 0)",
        "config": {"workload": workload, "model": MODEL_NAME if args.model == "bsms_mgn" else "BSMS_MeshGraphNet",
                   **{k: v for k, v in extra.items() if k != "multi"}, "mode": args.mode,
                   "edge_updates_per_step_per_gpu": eu_step, "edge_updates_per_step_all_ranks": eu_all,
                   "level_edges": Es,
                   "global_batch": extra.get("global_batch_meshes", ws), "parallelism": f"dp{ws}"},
        "roofline": roof,
        "kernels": kernels,
    }
    if D.active():
        out["collective"] = {"backend": torch.distributed.get_backend(), "world_size": ws,
                             "buckets": len(allreduce_ref[0].buckets) if allreduce_ref else None,
                             "launched_in_hooks": allreduce_ref[0].launched_in_hooks if allreduce_ref else None}
    strong = args.strong_config or ("c4" if args.config == "c3" else None)
    if args.model == "bsms_mgn" and strong and args.mode == "train" and not args.no_c4:
        del model, batches, step
        torch.cuda.empty_cache()
        m4, b4, eu4, _, wl4, _, ex4 = setup(strong)
        st4 = make_step(m4, b4, ex4)
        k4 = min(args.steps, 5)
        ar4 = allreduce_ref[0]
        ar4.exposed_events = [] if D.active() else None
        pr4 = {}
        el4 = timed_run(st4, k4, 1, per_rank=pr4)
        exposed = None
        if ar4.exposed_events:  # the timed steps' brackets (the warm-up's first one dropped)
            torch.cuda.synchronize()
            evs = ar4.exposed_events[-k4:]
            exposed = sum(a.elapsed_time(b) for a, b in evs) / len(evs)
        ar4.exposed_events = None
        eu4_all = eu4 * ws
        if ws > 1:
            t4 = torch.tensor([float(eu4)], dtype=torch.float64, device=dev)
            if D._host_staged():
                t4 = t4.cpu()
            torch.distributed.all_reduce(t4)
            eu4_all = int(t4.item())
        out["c4_strong"] = {"value": round(eu4_all * k4 / el4 / 1e6, 2), "unit": "M edge-updates/s",
                            "ms_per_step": round(1e3 * el4 / k4, 3), "steps": k4, "warmup": 1, "scaling": "strong",
                            "workload": wl4, "edge_updates_per_step_per_gpu": eu4,
                            "rank_ms_min": round(pr4["rank_ms_min"], 3), "rank_ms_max": round(pr4["rank_ms_max"], 3),
                            "allreduce_exposed_ms": round(exposed, 3) if exposed is not None else None,
                            "allreduce_note": "rank 0's all-reduce work left after the backward (remaining bucket "
                                              "launches, waits, unpack), HIP events on the compute stream; "
                                              "null at world size 1 (no collective)",
                            "note": "BASELINE.json configs[3] / north_star's 1->8 scaling case (fixed global batch)"}
    # the persistent hand-off kernels' device fault word (agn_fault_status): a bounded LDS-ring wait
    # that gave up anywhere in this run means wrong dW; the line carries it and the run fails
    from aerognn import _lib as L
    fault = L.fault_status(reset=False)
    out["fault_word"] = fault
    if rank == 0 and ws == 1 and not args.no_cpu_baseline and args.model == "bsms_mgn":
        out["cpu_baseline"] = cpu_baseline(S)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if D.active():
        torch.distributed.destroy_process_group()
    if fault:
        raise SystemExit(f"bench: device fault word {fault:#x} (an LDS-ring wait of the fused edge backward gave up)")


if __name__ == "__main__":
    main()
