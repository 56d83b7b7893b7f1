"""CPU-only checks of the drop-in boundary: the C-ABI library loads and exports every symbol
include/aerognn.h declares (no compute without a GPU), ctypes structs match the C layout,
the mirrored modules keep the reference's class names / state_dict keys / parameter counts,
and the product path refuses to run on CPU (no silent fallback)."""
import ctypes

import pytest
import torch

from golden_util import load, params


def test_library_exports_header_symbols():
    from aerognn import _lib
    lib = _lib.lib()
    names = _lib.exported_symbols()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    assert lib.agn_version() >= 1
    assert lib.agn_packed_bytes(128, 128, _lib.BF16) == 4 * 8 * 1024
    assert lib.agn_packed_bytes(128, 128, _lib.F32) == 2 * 4 * 8 * 1024
    assert lib.agn_error_string(-4) == b"unsupported shape"


def test_struct_layouts_match_c(tmp_path):
    """ctypes mirrors (aerognn/_lib.py) agree with the C compiler's layout of include/aerognn.h."""
    import os
    import subprocess
    from aerognn import _lib as L
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    fields = {"agn_seg": (L.Seg, ["kind", "k", "ld", "ptr", "index", "store"]),
              "agn_pack_desc": (L.PackDesc, ["src", "dst", "rows", "trans", "row_off", "dst_cols"]),
              "agn_mlp_fwd_args": (L.MlpFwdArgs, ["seg", "wpk", "bias", "ln_g", "proj", "resid", "act", "stats", "mask"]),
              "agn_mlp_bwd_args": (L.MlpBwdArgs, ["wtpk", "act", "g", "gidx", "gpre", "din_nseg", "din_k", "din",
                                                 "din_resid", "ln_partial"]),
              "agn_wgrad_desc": (L.WgradDesc, ["g", "x", "rows", "ldw", "dw_partial", "db", "nsplit", "xidx"]),
              "agn_wgrad_batch": (L.WgradBatch, ["n", "d"]),
              "agn_wec_args": (L.WecArgs, [f for f, _ in L.WecArgs._fields_ if not f.startswith("_")]),
              "agn_edge_bwd_args": (L.EdgeBwdArgs, [f for f, _ in L.EdgeBwdArgs._fields_]),
              "agn_edge_fwd_args": (L.EdgeFwdArgs, [f for f, _ in L.EdgeFwdArgs._fields_]),
              "agn_f64_seg": (L.F64Seg, [f for f, _ in L.F64Seg._fields_]),
              "agn_f64_gemm_args": (L.F64GemmArgs, [f for f, _ in L.F64GemmArgs._fields_ if not f.startswith("_")]),
              "agn_f64_wgrad_args": (L.F64WgradArgs, [f for f, _ in L.F64WgradArgs._fields_
                                                      if not f.startswith("_")])}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "aerognn.h"', 'int main(void){']
    for st, (_, fs) in fields.items():
        lines.append(f'printf("{st} size %zu\\n", sizeof({st}));')
        for f in fs:
            lines.append(f'printf("{st} {f} %zu\\n", offsetof({st}, {f}));')
    lines.append("return 0;}")
    src = tmp_path / "abi.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "abi"
    subprocess.check_call(["gcc", "-I", os.path.join(root, "include"), str(src), "-o", str(exe)])
    out = subprocess.check_output([str(exe)]).decode().split("\n")
    for line in out:
        if not line:
            continue
        st, f, v = line.split()
        cls = fields[st][0]
        want = int(v)
        got = ctypes.sizeof(cls) if f == "size" else getattr(cls, f).offset
        assert got == want, (st, f, got, want)


@pytest.mark.parametrize("name,ctor", [
    ("layer_sum_h32", "layer"), ("layer_cat_h32", "layer"), ("mgn5_f32", "mgn"), ("bsms_s4", "bsms"),
    ("bsms_s2_st3", "bsms")])
def test_state_dict_schema(name, ctor):
    """Reference checkpoints load unchanged; same key set and shapes."""
    d, m = load(name)
    ref = params(d)
    if ctor == "layer":
        from models.mgnLayer import MeshGraphNetLayer
        H, nh = m["H"], m["n_hid"]
        model = MeshGraphNetLayer(H, H, H, nh, nh, "relu", True, m["aggregation"], m["trick"])
    elif ctor == "mgn":
        from models.mgn import MeshGraphNet
        model = MeshGraphNet(*m["dims"], **m["kwargs"])
    else:
        from models.bsms_mgn import BiStridedMeshGraphNet
        model = BiStridedMeshGraphNet(*m["dims"], **m["kwargs"])
    sd = model.state_dict()
    assert set(sd) == set(ref)
    for k in sd:
        assert sd[k].shape == ref[k].shape, k
    model.load_state_dict(ref)


def test_same_init_as_reference():
    """Module tree + init order mirror the reference: same seed, same initial weights."""
    from models.bsms_mgn import BiStridedMeshGraphNet
    d, m = load("bsms_s4")
    torch.manual_seed(4)  # tools/make_goldens.py:case_bsms seeds 4 before building the mesh
    from aerognn.meshgen import ellipsoid  # noqa: F401  (mesh built before the model, no torch RNG)
    model = BiStridedMeshGraphNet(*m["dims"], **m["kwargs"])
    for k, v in model.state_dict().items():
        assert torch.equal(v, params(d)[k]), k


def test_param_count_c3():
    from models.bsms_mgn import BiStridedMeshGraphNet
    m = BiStridedMeshGraphNet(6, 4, 4, processor_size=15, num_hidden_layers_node_processor=2,
                              num_hidden_layers_edge_processor=2, num_hidden_layers_node_encoder=2,
                              num_hidden_layers_edge_encoder=2, num_hidden_layers_decoder=2,
                              do_concat_trick=True, num_scales=4)
    assert sum(p.numel() for p in m.parameters()) == 2877572
    assert m.__class__.__name__ == "BiStridedMeshGraphNet"    # utils.py:178-189 dispatch


def test_config_errors_match_reference():
    from models.bsms_mgn import BiStridedMeshGraphNet
    with pytest.raises(ValueError):
        BiStridedMeshGraphNet(6, 4, 4, num_scales=0)
    with pytest.raises(ValueError):
        BiStridedMeshGraphNet(6, 4, 4, stride=0)
    with pytest.raises(ValueError):
        BiStridedMeshGraphNet(6, 4, 4, num_scales=3, layers_per_scale=[1, 2, 3])


def test_cpu_tensors_fail_loudly():
    from models.mgnLayer import MeshGraphNetLayer
    layer = MeshGraphNetLayer(32, 32, 32, 2, 2, "relu", True, "add", True)
    x = torch.randn(10, 32)
    e = torch.randn(20, 32)
    ei = torch.randint(0, 10, (2, 20))
    with pytest.raises(RuntimeError):
        layer(x, e, ei)


def test_poolmgn_state_dict_and_errors():
    """poolMGN keeps the reference's module tree (state_dict keys of the golden, generated from
    /root/reference/models/poolmgn.py) and its ValueError for an unknown pooling method."""
    from golden_util import load as _load
    from models.poolmgn import poolMGN
    d, m = _load("poolmgn_mean")
    model = poolMGN(*m["dims"], **m["kwargs"])
    ref_keys = sorted(k[2:] for k in d if k.startswith("p:"))
    assert sorted(model.state_dict().keys()) == ref_keys
    model.load_state_dict(params(d))
    with pytest.raises(ValueError):
        poolMGN(6, 4, 4, global_pool_method="median")


def test_pack_rejects_float64_and_mixed_dtypes():
    """a float64 model (or a float64 weight in a 16/32-bit pack) raises on the host
    instead of being packed as float bits (agn_pack reads descriptors from device memory)."""
    import torch
    from aerognn.core import Pack
    w = torch.randn(128, 128, dtype=torch.float64)
    p = Pack()
    p.matrix("W", 128, 128, [(w, 0, 0, False)])
    with pytest.raises(NotImplementedError):
        p.update(torch.float64, torch.device("cpu"))
    with pytest.raises(TypeError):
        p.update(torch.float32, torch.device("cpu"))
