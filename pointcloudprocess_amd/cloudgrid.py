"""CloudGrid, the map cache of ICP targets (cloud_grid.h:37-88), on the GPU (libpcp pcp_grid_*).

Clouds are (n, 48) uint8 device tensors of PointXYZRGBA records (ops.cloud_to_device).
  add_cloud_internal(cloud)             cloud_grid.cpp:34-78 (sequential 4 cm de-duplication per 1 m cell)
  get_cloud_with_pos(min_xyz, max_xyz)  :110-131 (cells i in [(int)min.x, max.x), j likewise)
  get_cloud_with_pos_rot(rot, dis=60)   :84-108 (cells around ((int)rot[0,3], (int)rot[1,3]))
  get_grid_cloud()                      :150-158 (key order)
  get_grid_cloud_match(src, dis)        :160-216 -> (src_out, dst)
"""
import ctypes as C
import math

import numpy as np
import torch

from . import _lib


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _trunc(v):
    """C's (int) conversion of a double (toward zero)."""
    return int(math.trunc(v))


class CloudGrid:
    MAX_DIS = 60  # cloud_grid.h:60

    def __init__(self, ctx):
        self.ctx = ctx
        h = C.c_void_p()
        ctx.check(ctx.lib.pcp_grid_create(ctx.h, C.byref(h)))
        self.h = h

    def clear(self):
        self.ctx.check(self.ctx.lib.pcp_grid_clear(self.ctx.h, self.h))

    def add_cloud_internal(self, cloud):
        assert cloud.dtype == torch.uint8 and cloud.shape[1] == 48 and cloud.is_contiguous()
        self.ctx.check(self.ctx.lib.pcp_grid_add_cloud(self.ctx.h, self.h, _ptr(cloud), cloud.shape[0]))

    @property
    def size(self):
        return int(self.ctx.lib.pcp_grid_size(self.h))

    @property
    def cells(self):
        return int(self.ctx.lib.pcp_grid_cells(self.h))

    def get_grid_cloud(self):
        n = C.c_int64()
        out = torch.empty((max(self.size, 1), 48), dtype=torch.uint8, device=self.ctx.device)
        self.ctx.check(self.ctx.lib.pcp_grid_points(self.ctx.h, self.h, _ptr(out), out.shape[0], C.byref(n)))
        return out[:n.value]

    def box(self, i0, i1, j0, j1):
        n = C.c_int64()
        lib, ctx = self.ctx.lib, self.ctx
        ctx.check(lib.pcp_grid_box(ctx.h, self.h, int(i0), int(i1), int(j0), int(j1), None, 0, C.byref(n)))
        out = torch.empty((max(n.value, 1), 48), dtype=torch.uint8, device=ctx.device)
        ctx.check(lib.pcp_grid_box(ctx.h, self.h, int(i0), int(i1), int(j0), int(j1), _ptr(out), n.value,
                                   C.byref(n)))
        return out[:n.value]

    def get_cloud_with_pos(self, min_xyz, max_xyz):
        """for (int i = min.x; i < max.x; i++) for (int j = min.y; j < max.y; j++) (:118-119)"""
        return self.box(_trunc(min_xyz[0]), math.ceil(max_xyz[0]), _trunc(min_xyz[1]), math.ceil(max_xyz[1]))

    def get_cloud_with_pos_rot(self, rot, dis=MAX_DIS):
        """int irow = curRot(0, 3) (float pose, :90-91); cells [irow - dis, irow + dis)"""
        irow = _trunc(float(np.float32(rot[0][3])))
        icol = _trunc(float(np.float32(rot[1][3])))
        return self.box(irow - dis, irow + dis, icol - dis, icol + dis)

    def get_grid_cloud_match(self, src, dis):
        lib, ctx = self.ctx.lib, self.ctx
        n = src.shape[0]
        src_out = torch.empty((max(n, 1), 48), dtype=torch.uint8, device=ctx.device)
        dst = torch.empty((max(self.size, 1), 48), dtype=torch.uint8, device=ctx.device)
        ns, nd = C.c_int64(), C.c_int64()
        ctx.check(lib.pcp_grid_match(ctx.h, self.h, _ptr(src), n, float(dis), _ptr(src_out), C.byref(ns), _ptr(dst),
                                     dst.shape[0], C.byref(nd)))
        return src_out[:ns.value], dst[:nd.value]

    def close(self):
        if getattr(self, "h", None):
            self.ctx.lib.pcp_grid_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()
