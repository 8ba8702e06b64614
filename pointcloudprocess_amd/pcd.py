"""PCD v0.7 I/O of PointXYZRGBA clouds (libpcp pcp_pcd_* / pcp_lzf_*, host-only).

  load_pcd(path, pinned=False)          io::loadPCDFile (pcd_helper.h:1374): ascii / binary /
                                        binary_compressed -> (n,) POINT48 numpy array (or a pinned
                                        (n, 48) uint8 tensor ready for one host-to-device copy)
  load_pcd_ex(path, pinned=False)       the same + the cloud's is_dense, width, height as the
                                        reference's PCDReader sets them (pcd_helper.cpp:863,
                                        1124-1179)
  save_pcd(path, cloud, compressed=False)
                                        io::savePCDFile / savePCDFileBinary (writeBinary) or
                                        PCDWriter::writeBinaryCompressed (LZF)
  lzf_compress / lzf_decompress         lzf.cpp:86-415
"""
import ctypes as C
import os

import numpy as np

from . import _lib
from .ops import POINT48


def _path(p):
    return os.fsencode(os.fspath(p))


def load_pcd_ex(path, pinned=False):
    """(cloud, is_dense, width, height): is_dense is False when a binary / binary_compressed
    field value is non-finite (PCDReader, pcd_helper.cpp:1124-1179); ascii files stay dense."""
    lib = _lib.load()
    n, w, h, dense = C.c_int64(), C.c_int64(), C.c_int64(), C.c_int()
    _lib.check(lib.pcp_pcd_read_ex(_path(path), None, 0, C.byref(n), None, None, None))
    if pinned:
        import torch
        buf = torch.empty((max(n.value, 1), 48), dtype=torch.uint8).pin_memory()
        _lib.check(lib.pcp_pcd_read_ex(_path(path), C.c_void_p(buf.data_ptr()), n.value, C.byref(n), C.byref(w),
                                       C.byref(h), C.byref(dense)))
        return buf[:n.value], bool(dense.value), w.value, h.value
    out = np.zeros(max(n.value, 1), dtype=POINT48)
    _lib.check(lib.pcp_pcd_read_ex(_path(path), out.ctypes.data, n.value, C.byref(n), C.byref(w), C.byref(h),
                                   C.byref(dense)))
    return out[:n.value], bool(dense.value), w.value, h.value


def load_pcd(path, pinned=False):
    return load_pcd_ex(path, pinned)[0]


def save_pcd(path, cloud, compressed=False, width=0, height=0):
    a = np.ascontiguousarray(cloud)
    if a.dtype != POINT48:
        a = a.view(POINT48).reshape(-1)
    _lib.check(_lib.load().pcp_pcd_write(_path(path), a.ctypes.data, len(a), int(width), int(height),
                                         int(bool(compressed))))


def lzf_compress(data, out_len=None):
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    cap = int(len(b) * 1.5) + 16 if out_len is None else int(out_len)
    out = np.zeros(max(cap, 1), dtype=np.uint8)
    m = _lib.load().pcp_lzf_compress(b.ctypes.data, len(b), out.ctypes.data, cap)
    return bytes(out[:m]) if m else None


def lzf_decompress(data, out_len):
    b = np.frombuffer(bytes(data), dtype=np.uint8)
    out = np.zeros(max(int(out_len), 1), dtype=np.uint8)
    m = _lib.load().pcp_lzf_decompress(b.ctypes.data, len(b), out.ctypes.data, int(out_len))
    return bytes(out[:m]) if m else None
