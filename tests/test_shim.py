"""The drop-in C++ shim (include/pcp_pcl.hpp): builds against the C-ABI on any host, and on
a GPU its parity driver (tests/cpp/shim_test.cpp -- the reference's main_test.cpp KAT bodies
plus randomised cross-checks against the oracle) passes."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CPP = os.path.join(HERE, "cpp")
ROOT = os.path.dirname(HERE)


def _build():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
    lib = os.path.join(ROOT, "pointcloudprocess_amd", "libpcp.so")
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-s", "-j8", "-C", os.path.join(ROOT, "pointcloudprocess_amd", "csrc")])
    subprocess.check_call(["make", "-s", "-C", CPP])
    return os.path.join(CPP, "_build", "shim_test")


def test_shim_builds():
    exe = _build()
    assert os.access(exe, os.X_OK)


@pytest.mark.gpu
def test_shim_parity_driver():
    exe = _build()
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600)
    print(r.stdout[-4000:], r.stderr[-2000:])
    assert r.returncode == 0 and "all checks passed" in r.stdout


def test_shim_request_combiner_host():
    """The combiner that merges concurrent per-point searches (host logic, no GPU)."""
    subprocess.check_call(["make", "-s", "-C", CPP, "_build/combiner_test"])
    r = subprocess.run([os.path.join(CPP, "_build", "combiner_test")], capture_output=True, text=True, timeout=300)
    print(r.stdout, r.stderr)
    assert r.returncode == 0 and "all checks passed" in r.stdout
