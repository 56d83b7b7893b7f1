"""Helpers to read tests/golden/*.npz (written by tools/make_goldens.py from the reference)."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    z = np.load(os.path.join(GOLDEN, f"{name}.npz"))  # allow_pickle=False (default)
    d = {k: torch.from_numpy(np.array(z[k])) for k in z.files if k != "meta"}
    meta = json.loads(str(z["meta"]))
    return d, meta


def params(d, prefix="p:"):
    return {k[len(prefix):]: v for k, v in d.items() if k.startswith(prefix)}


def rel_l2(a, b):
    a = a.detach().double()
    b = b.detach().double()
    n = b.norm()
    return float((a - b).norm() / (n if n > 0 else 1.0))


def max_rel(a, b):
    a = a.detach().double()
    b = b.detach().double()
    m = b.abs().max()
    return float((a - b).abs().max() / (m if m > 0 else 1.0))
