"""PCD / LZF on the GPU box: file -> pinned host memory -> HBM -> the hot path -> file.

The reader and writer are host code (pcd.cpp, pcd_helper.h:487-760, lzf.cpp:86-284 in the
reference); this test runs them where the hot path runs.  Every file written is byte-compared
with the pure-Python restatement of the reference's writer (oracle/pcd_oracle.py), the records
staged through pinned memory into HBM are byte-compared with the file's, and the VoxelGrid
output computed on the device from them is byte-compared with the oracle's, then written back
and byte-compared again (binary and binary_compressed).
"""
import os
import sys

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle_ctypes as ora  # noqa: E402
import pcd_oracle as po  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from pointcloudprocess_amd import ops
    return ops.Context(0)


def _cloud(n, seed):
    rng = np.random.default_rng(seed)
    xyz = np.round(rng.uniform(-30, 30, (n, 3)), 3)  # quantised like a voxelised map (compressible)
    xyz[: n // 4] = np.round(xyz[: n // 4], 1)
    return ora.make_cloud(xyz, rgba=rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32),
                          stamp=(np.arange(n) // 131).astype(np.uint32))


@pytest.mark.parametrize("compressed", [False, True])
def test_pcd_pinned_device_round_trip_bytes(ctx, tmp_path, compressed):
    from pointcloudprocess_amd import ops, pcd
    c = _cloud(300_000, 4 + int(compressed))
    src = tmp_path / "src.pcd"
    pcd.save_pcd(src, c, compressed=compressed)
    assert src.read_bytes() == po.pcd_bytes(c, compressed)

    # file -> pinned host -> HBM; the device copy holds the file's records byte for byte
    buf, dense, w, h = pcd.load_pcd_ex(src, pinned=True)
    assert buf.is_pinned() and dense and (w, h) == (len(c), 1)
    dev = buf.to(ctx.device, non_blocking=True)
    torch.cuda.synchronize()
    assert dev.cpu().numpy().tobytes() == c.tobytes()

    # the hot path on the staged records (VoxelGrid leaf 0.1), against the oracle on the file's
    out = ops.cloud_to_host(ops.voxel_filter(ctx, dev, 0.1))
    eo, _ = ora.voxel_filter(pcd.load_pcd(src), 0.1)
    assert out.tobytes() == eo.tobytes()

    # device result -> file, byte-identical to the reference writer's bytes of the oracle result
    dst = tmp_path / "dst.pcd"
    pcd.save_pcd(dst, out, compressed=compressed)
    assert dst.read_bytes() == po.pcd_bytes(eo, compressed)
