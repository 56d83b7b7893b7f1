"""Synthetic aero surface meshes (host-side, numpy) for benchmarks and parity tests.

The reference trains on pyvista-read CFD surface meshes (`dataset.py:39-106`,
`utils.py:15-130`); those files are not available here, so every workload in this
repo uses a closed-form lat-long ellipsoid surface with the SAME feature layout:

* node features  x         = [pos(3), unit normal(3)]      (`dataset.py:66-106`)
* edge features  edge_attr = [pos[dst]-pos[src], |.|]        (`dataset.py:39-64`)
* targets        y         = N(0,1), 4 channels (ahmed layout [p, tau(3)], `utils.py:121-128`)
* edge_index is undirected (both directions), coalesced and row-sorted, as PyG
  `to_undirected` leaves it (`utils.py:39-40`).

x-coordinates are made strictly unique (F4 in SURVEY.md: the reference's unstable
`argsort(pos[:,0])` is only reproducible on tie-free x) by nudging duplicates up by
whole ulps in sorted order.

Sizes: E = 2 * (nu*nv + 2*nu*(nv-1)); ellipsoid(40,25) -> 1,000 / 5,840;
ellipsoid(400,250) -> 100,000 / 598,400; ellipsoid(1000,1000) -> 1,000,000 / 5,996,000.
"""
from __future__ import annotations

import numpy as np

__all__ = ["ellipsoid", "collate", "num_edges"]


def num_edges(nu: int, nv: int) -> int:
    return 2 * (nu * nv + 2 * nu * (nv - 1))


def _f32_to_key(x: np.ndarray) -> np.ndarray:
    s = x.astype(np.float32).view(np.int32).astype(np.int64)
    return np.where(s >= 0, s, -(s & 0x7FFFFFFF))


def _key_to_f32(k: np.ndarray) -> np.ndarray:
    s = np.where(k >= 0, k, (-k) | 0x80000000).astype(np.int64)
    return (s & 0xFFFFFFFF).astype(np.uint32).view(np.float32)


def make_unique_x(x: np.ndarray) -> np.ndarray:
    """Return fp32 x with every duplicate nudged up (in sorted order) to the next free value."""
    order = np.argsort(x, kind="stable")
    keys = _f32_to_key(x[order])
    i = np.arange(keys.size, dtype=np.int64)
    keys = np.maximum.accumulate(keys - i) + i  # strictly increasing
    out = np.empty_like(x, dtype=np.float32)
    out[order] = _key_to_f32(keys)
    assert np.unique(out).size == out.size
    return out


def _rot(az: float, ay: float) -> np.ndarray:
    cz, sz = np.cos(az), np.sin(az)
    cy, sy = np.cos(ay), np.sin(ay)
    rz = np.array([[cz, -sz, 0.0], [sz, cz, 0.0], [0.0, 0.0, 1.0]])
    ry = np.array([[cy, 0.0, sy], [0.0, 1.0, 0.0], [-sy, 0.0, cy]])
    return ry @ rz


def ellipsoid(nu: int, nv: int, a: float = 4.0, b: float = 1.0, c: float = 1.0,
              seed: int = 0, unique_x: bool = True, dtype=np.float32) -> dict:
    """Triangulated ellipsoid surface, nu points around (periodic) x nv rings (no poles).

    `seed` selects the rotation (seed 0 = (0.3137 rad about z, 0.2718 about y)) and the
    target noise, so a batch of meshes with seeds 0..B-1 are distinct but equal-sized.
    Returns numpy arrays: pos, normals, x, edge_attr, y, edge_index (int64 [2,E]).
    """
    i = np.arange(nu)
    j = np.arange(nv)
    u = 2.0 * np.pi * i / nu
    v = np.pi * (j + 0.5) / nv
    U, V = np.meshgrid(u, v)                      # [nv, nu]; node id = j*nu + i
    X = a * np.cos(V)
    Y = b * np.sin(V) * np.cos(U)
    Z = c * np.sin(V) * np.sin(U)
    pos = np.stack([X, Y, Z], -1).reshape(-1, 3)
    nrm = pos / np.array([a * a, b * b, c * c])
    nrm /= np.linalg.norm(nrm, axis=1, keepdims=True)
    R = _rot(0.3137 + 0.0191 * seed, 0.2718 + 0.0317 * seed)
    pos = pos @ R.T
    nrm = nrm @ R.T
    pos = pos.astype(np.float32)
    if unique_x:
        pos[:, 0] = make_unique_x(pos[:, 0])
    nrm = nrm.astype(np.float32)

    nid = (j[:, None] * nu + i[None, :])          # [nv, nu]
    right = (j[:, None] * nu + (i[None, :] + 1) % nu)
    a_ = [nid.ravel(), nid[:-1].ravel(), nid[:-1].ravel()]
    b_ = [right.ravel(), nid[1:].ravel(), right[1:].ravel()]
    s = np.concatenate(a_)
    d = np.concatenate(b_)
    N = nu * nv
    row = np.concatenate([s, d]).astype(np.int64)
    col = np.concatenate([d, s]).astype(np.int64)
    key = np.unique(row * N + col)                # coalesce + row-major sort (to_undirected)
    ei = np.stack([key // N, key % N]).astype(np.int64)
    assert ei.shape[1] == num_edges(nu, nv)

    ev = pos[ei[1]] - pos[ei[0]]
    el = np.sqrt((ev.astype(np.float32) ** 2).sum(1, keepdims=True, dtype=np.float32))
    edge_attr = np.concatenate([ev, el], 1).astype(dtype)
    x = np.concatenate([pos, nrm], 1).astype(dtype)
    rng = np.random.default_rng(seed)
    y = rng.standard_normal((N, 4)).astype(dtype)
    return dict(pos=pos.astype(dtype), normals=nrm.astype(dtype), x=x, edge_attr=edge_attr,
                y=y, edge_index=ei)


def collate(meshes: list[dict]) -> dict:
    """PyG-style batch collation: concat rows, offset edge_index, build `batch`."""
    out = {k: np.concatenate([m[k] for m in meshes], 0) for k in ("pos", "x", "edge_attr", "y")}
    offs = np.cumsum([0] + [m["x"].shape[0] for m in meshes[:-1]])
    out["edge_index"] = np.concatenate([m["edge_index"] + o for m, o in zip(meshes, offs)], 1)
    out["batch"] = np.concatenate([np.full(m["x"].shape[0], g, np.int64)
                                   for g, m in enumerate(meshes)])
    return out
