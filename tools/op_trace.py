"""Which Python call sites launch the small torch kernels (fills, copies) in one training step.
Runs bench.py's model on the 'small' config under torch.profiler and prints the aten ops
grouped by their Python stack."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "aero-gnn_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402
from aerognn import dist as D  # noqa: E402

dev = torch.device("cuda", 0)
model, _ = bench.build_model(4, dev)
t = bench.mesh_tensors(200, 125, 0, dev, torch.bfloat16)
opt = torch.optim.Adam(model.parameters(), lr=1e-3)
ar = D.GradAllReduce(model.parameters())
n = t["y"].numel()


def step():
    pred = model(t["x"], t["edge_attr"], t["edge_index"], pos=t["pos"])
    D.mse_sum_loss(pred, t["y"], n).backward()
    ar()
    opt.step()
    opt.zero_grad(set_to_none=True)


for _ in range(2):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], with_stack=True) as p:
    step()
    torch.cuda.synchronize()
want = sys.argv[1:] or ["aten::fill_", "aten::zero_", "aten::copy_", "aten::zeros", "aten::cat"]
tab = p.key_averages(group_by_stack_n=6)
for ev in sorted(tab, key=lambda e: -e.count):
    if ev.key in want:
        print(f"{ev.key:14s} x{ev.count}")
        for fr in ev.stack[:6]:
            print("     ", fr)
