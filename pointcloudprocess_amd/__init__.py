"""pointcloudprocess_amd: MI355X (gfx950) implementation of the kNN-driven geometry hot path
of RioWong/PointCloudProcess (kd_tree / kd_tree_lod search, voxel_grid downsample,
calculate_feature normals, ICP correspondence/transform loop) behind the C-ABI in
include/pcp.h.  See DESIGN.md.
"""
from ._lib import LIB_PATH, PcpError, load  # noqa: F401

__all__ = ["LIB_PATH", "PcpError", "load"]
