"""Data-parallel semantics on CPU (gloo, world_size 2): the N>1 path of bench.py / train step.

Each rank runs the oracle BSMS forward/backward (oracle/refcpu.py, test-only checker) on its OWN
mesh, back-propagates aerognn.dist.mse_sum_loss with the all-reduced global element count, and
all-reduces gradients with aerognn.dist.GradAllReduce. The result must equal the gradient of
the reference's single-process MSELoss over the PyG-collated union batch (utils.py:171-196,
SURVEY §8e) — independent meshes, different sizes per rank. float64 keeps the comparison tight.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

MESHES = [(12, 8, 0), (10, 6, 1)]  # (nu, nv, seed) per rank: different node counts


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _setup():
    from models.bsms_mgn import BiStridedMeshGraphNet
    from oracle import refcpu as R
    kw = dict(processor_size=5, activation_fn="relu", num_hidden_layers_node_processor=1,
              num_hidden_layers_edge_processor=1, hidden_dim_processor=16, num_hidden_layers_node_encoder=1,
              hidden_dim_node_encoder=16, num_hidden_layers_edge_encoder=1, hidden_dim_edge_encoder=16,
              aggregation="add", hidden_dim_decoder=16, num_hidden_layers_decoder=1, dropout=0.0,
              do_concat_trick=True, num_scales=2, layers_per_scale=1, stride=2)
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, **kw)
    params = {k: v.detach().double().clone().requires_grad_(True) for k, v in model.state_dict().items()}
    return params, R.cfg_from_kwargs(**kw)


def _mesh(nu, nv, seed):
    from aerognn.meshgen import ellipsoid
    m = ellipsoid(nu, nv, seed=seed)
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in m.items()}


def _worker(rank, ws, port, out, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(ws))
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "aero-gnn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.set_num_threads(1)
    from aerognn import dist as D
    from oracle import refcpu as R
    r, w = D.init_from_env(backend="gloo")
    assert (r, w) == (rank, ws)
    params, cfg = _setup()
    t = _mesh(*MESHES[rank])
    n_glob = D.global_count(t["y"].numel(), "cpu")
    batch = torch.zeros(t["x"].shape[0], dtype=torch.long)
    pred = R.bsms_forward(params, t["x"].double(), t["edge_attr"].double(), t["edge_index"], cfg, batch,
                          t["pos"].double(), stable=True)
    loss = D.mse_sum_loss(pred, t["y"].double(), n_glob)
    ar = D.GradAllReduce(params.values(), bucket_bytes=16 << 10)  # several buckets
    if overlap:  # buckets launch from post-accumulate-grad hooks during the backward
        ar.arm()
    loss.backward()
    if overlap:
        assert len(ar._works) == len(ar.buckets)  # every bucket fired inside the backward
    ar()
    if rank == 0:
        torch.save({k: v.grad for k, v in params.items()}, out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
def test_dp_gradients_equal_union_batch(tmp_path, overlap):
    from aerognn.meshgen import collate, ellipsoid
    from oracle import refcpu as R
    out = str(tmp_path / "g.pt")
    mp.start_processes(_worker, args=(2, _free_port(), out, overlap), nprocs=2, join=True, start_method="spawn")
    g_dp = torch.load(out, weights_only=True)

    params, cfg = _setup()
    u = collate([ellipsoid(*m[:2], seed=m[2]) for m in MESHES])
    u = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in u.items()}
    pred = R.bsms_forward(params, u["x"].double(), u["edge_attr"].double(), u["edge_index"], cfg, u["batch"],
                          u["pos"].double(), stable=True)
    torch.nn.functional.mse_loss(pred, u["y"].double()).backward()
    worst = 0.0
    for k, p in params.items():
        ref = p.grad
        err = (g_dp[k] - ref).norm() / max(ref.norm(), 1e-300)
        worst = max(worst, float(err))
    assert worst <= 1e-10, worst


def test_single_rank_is_noop():
    """world_size 1: init is skipped and the all-reduce leaves gradients untouched."""
    from aerognn import dist as D
    assert D.world() == (0, 1)
    p = torch.nn.Parameter(torch.ones(3))
    p.grad = torch.full((3,), 2.0)
    D.GradAllReduce([p])()
    assert torch.equal(p.grad, torch.full((3,), 2.0))
    assert D.global_count(7, "cpu") == 7.0


def _forced_one_worker(rank, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      AEROGNN_DIST_FORCE="1")
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for p in (root, os.path.join(root, "aero-gnn_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    torch.set_num_threads(1)
    from aerognn import dist as D
    assert D.init_from_env(backend="gloo") == (0, 1) and D.active()
    params = [torch.nn.Parameter(torch.randn(n, dtype=torch.float64)) for n in (5000, 3000, 7)]
    loss = sum((p ** 2).sum() for p in params)
    ar = D.GradAllReduce(params, bucket_bytes=16 << 10)
    ar.arm()
    loss.backward()
    fired = ar.launched_in_hooks
    ar()
    ok = all(torch.equal(p.grad, 2 * p.detach()) for p in params)
    torch.save({"fired": fired, "buckets": len(ar.buckets), "ok": ok}, out)
    dist.destroy_process_group()


def test_forced_world_of_one_runs_collective_path(tmp_path):
    """AEROGNN_DIST_FORCE=1: a single process still builds a process group, and GradAllReduce's
    armed path (hooks -> bucket pack -> async all-reduce -> wait -> unpack) runs and is an
    identity (the GPU suite runs the same path on RCCL)."""
    out = str(tmp_path / "f.pt")
    mp.start_processes(_forced_one_worker, args=(_free_port(), out), nprocs=1, join=True, start_method="spawn")
    r = torch.load(out, weights_only=True)
    assert r["ok"] and r["buckets"] >= 2 and r["fired"] == r["buckets"], r


def test_bench_rank_envs_and_world_size_check():
    """bench.py --gpus N without torchrun starts N ranks itself (bench.launch_ranks): each rank gets
    torchrun's variables with a 127.0.0.1 rendezvous; under a launcher WORLD_SIZE must equal --gpus
    (checked before anything touches a GPU)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import bench
    envs = bench.rank_envs(4, 29999, base={"PATH": "/usr/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"] and [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert all(e["WORLD_SIZE"] == "4" and e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29999"
               and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0" for e in envs)
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "1"], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE=1" in r.stderr, r.stderr[-2000:]
