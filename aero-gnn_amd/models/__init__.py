"""Drop-in replacements for the reference's models package (cudagu/aero-gnn models/*.py).

Same module paths, class names, constructor arguments, forward signatures and state_dict
keys; the compute runs in libaerognn (HIP, gfx950). Put `aero-gnn_amd/` on sys.path ahead of
the reference and `from models.bsms_mgn import BiStridedMeshGraphNet` resolves here.
"""
