"""Build provenance: the libpcp.so a run loads reports (pcp_build_id) the SHA-1 of the sources
it was built from; it must equal the hash of the sources in this tree (the Makefile's rule:
every csrc *.hip / *.cpp / *.hpp, include/pcp.h and the Makefile, concatenated in sorted name
order).  On the GPU box the same check runs in the GPU suite, so a stale pushed library fails
there rather than silently testing old code."""
import glob
import hashlib
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
CSRC = os.path.join(ROOT, "pointcloudprocess_amd", "csrc")


def source_sha():
    names = [os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hip"))]
    names += [os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.cpp"))]
    names += [os.path.basename(p) for p in glob.glob(os.path.join(CSRC, "*.hpp"))]
    names += ["../../include/pcp.h", "Makefile"]
    h = hashlib.sha1()
    for n in sorted(names):
        with open(os.path.join(CSRC, n), "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def _check():
    from pointcloudprocess_amd import _lib
    got = _lib.load().pcp_build_id().decode()
    assert got == source_sha(), (f"libpcp.so was built from other sources ({got}); rebuild with "
                                 "`python -c 'import __graft_entry__ as g; g.build()'`")


def test_build_id_matches_sources():
    _check()


@pytest.mark.gpu
def test_build_id_matches_sources_on_gpu_box():
    _check()
