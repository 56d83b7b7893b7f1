"""A/B bitwise check of two builds of libaerognn (diagnostics, GPU). Usage:
  AEROGNN_LIB=<lib.so> python tools/ab_outputs.py save OUT.pt   # C3-size BSMS-4 bf16 step
  python tools/ab_outputs.py cmp A.pt B.pt
Saves the forward output, the input gradients and every parameter gradient of one training
step (bf16 activations, fp32 master weights, seed 0) on the 1M-node C3 mesh, plus an fp32 step on
a 100k-node mesh."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "aero-gnn_amd")]
os.environ.setdefault("AEROGNN_MEMLOG", "0")
import numpy as np  # noqa: E402
import torch  # noqa: E402


def step(nu, nv, dtype):
    from aerognn.meshgen import ellipsoid
    from models.bsms_mgn import BiStridedMeshGraphNet
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).cuda() for k, v in ellipsoid(nu, nv, seed=0).items()}
    torch.manual_seed(0)
    model = BiStridedMeshGraphNet(6, 4, 4, processor_size=15, num_hidden_layers_node_processor=2,
                                  num_hidden_layers_edge_processor=2, num_hidden_layers_node_encoder=2,
                                  num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
                                  do_concat_trick=True, num_scales=4, layers_per_scale=2, stride=2).cuda()
    x = t["x"].to(dtype).requires_grad_(True)
    ea = t["edge_attr"].to(dtype).requires_grad_(True)
    pred = model(x, ea, t["edge_index"], batch=None, pos=t["pos"])
    torch.nn.functional.mse_loss(pred.float(), t["y"]).backward()
    torch.cuda.synchronize()
    out = {"pred": pred.detach().cpu(), "gx": x.grad.cpu(), "gea": ea.grad.cpu()}
    out.update({"g:" + n: p.grad.cpu() for n, p in model.named_parameters()})
    return out


def main():
    if sys.argv[1] == "save":
        res = {f"bf16/{k}": v for k, v in step(1000, 1000, torch.bfloat16).items()}
        res.update({f"f32/{k}": v for k, v in step(400, 250, torch.float32).items()})
        torch.save(res, sys.argv[2])
        print("saved", len(res), "tensors from", os.environ.get("AEROGNN_LIB", "libaerognn.so"))
        return
    a = torch.load(sys.argv[2], weights_only=True)
    b = torch.load(sys.argv[3], weights_only=True)
    diff = [k for k in a if not torch.equal(a[k], b[k])]
    print(f"{len(a) - len(diff)} of {len(a)} tensors bitwise equal")
    for k in diff[:20]:
        d = (a[k].double() - b[k].double())
        print(f"  {k}: max |diff| {float(d.abs().max()):.3e}, rel-L2 {float(d.norm() / b[k].double().norm()):.3e}")
    sys.exit(1 if diff else 0)


if __name__ == "__main__":
    main()
