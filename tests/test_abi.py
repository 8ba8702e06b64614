"""CPU-only checks of the drop-in boundary: libpcp.so loads (no GPU needed) and exports
exactly the C-ABI declared in include/pcp.h; host-side pieces of the ABI (the ICP solve)
are checked against the oracle."""
import os
import re
import subprocess

import numpy as np

import oracle_ctypes as ora

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "pcp.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(pcp_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_header():
    from pointcloudprocess_amd import _lib
    lib = _lib.load()  # binds every symbol in _lib.SIGNATURES
    assert lib.pcp_abi_version() == 1
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = set(re.findall(r" T (pcp_[a-z0-9_]+)$", out, flags=re.M))
    declared = header_functions()
    assert declared, "no functions parsed from include/pcp.h"
    missing = [f for f in declared if f not in exported]
    assert not missing, f"declared but not exported: {missing}"
    bound = {name for name, _, _ in _lib.SIGNATURES}
    assert set(declared) == bound, (set(declared) ^ bound)


def test_null_handles_rejected():
    from pointcloudprocess_amd import _lib
    lib = _lib.load()
    assert lib.pcp_index_destroy(None) == -1
    assert lib.pcp_icp_destroy(None) == -1
    assert lib.pcp_ctx_destroy(None) == -1
    assert lib.pcp_index_size(None) == -1


def test_solve_vs_oracle():
    # host solvers: libpcp (SVD) vs oracle (Horn quaternion) on the same accumulators
    from pointcloudprocess_amd import ops, synth
    rng = np.random.default_rng(0)
    p = rng.normal(size=(5000, 3)) * [30, 30, 3]
    T = synth.rigid(3.0, 1.0, -2.0, (0.5, -0.2, 0.1))
    q = (p - T[:3, 3]) @ T[:3, :3]
    acc = np.zeros(24)
    acc[0] = len(p)
    acc[1:4] = q.sum(0)
    acc[4:7] = p.sum(0)
    acc[7:16] = (q[:, :, None] * p[:, None, :]).sum(0).reshape(9)
    qq = q[:, :, None] * q[:, None, :]
    acc[16:22] = [qq[:, 0, 0].sum(), qq[:, 0, 1].sum(), qq[:, 0, 2].sum(), qq[:, 1, 1].sum(),
                  qq[:, 1, 2].sum(), qq[:, 2, 2].sum()]
    for scale in (False, True):
        rc, dT = ops.icp_solve(acc, scale)
        erc, edT = ora.icp_solve(acc, scale)
        assert rc == 0 and erc == 0
        assert np.abs(dT - edT).max() < 1e-9
        assert np.abs(dT - T).max() < 1e-9


def test_icp_size_guard():
    """ld16's 32-bit record offsets (icp.hip): targets of >= 2^28 - 1 points are rejected
    with PCP_ERR_CAPACITY instead of wrapping; queries are limited to < 2^31."""
    from pointcloudprocess_amd import _lib
    lib = _lib.load()
    assert lib.pcp_icp_check_sizes(50_000_000, 50_000_000) == 0
    assert lib.pcp_icp_check_sizes((1 << 28) - 2, 1) == 0
    assert lib.pcp_icp_check_sizes((1 << 28) - 1, 1) == -7
    assert lib.pcp_icp_check_sizes(1 << 30, 1) == -7
    assert lib.pcp_icp_check_sizes(10, 1 << 31) == -1
    assert lib.pcp_icp_check_sizes(-1, 1) == -1
