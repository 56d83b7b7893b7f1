"""aerognn — MI355X (gfx950) runtime for the bi-stride multi-scale MeshGraphNet hot path.

libaerognn.so (csrc/, C-ABI in include/aerognn.h) holds the HIP kernels; this package holds
the ctypes binding (_lib), launch wrappers (core), device graph levels / pooling maps
(graph), autograd Functions (functions), data-parallel helpers (dist) and the synthetic
mesh generator (meshgen). The drop-in reference modules live in ../models.
"""
__version__ = "0.1.0"
