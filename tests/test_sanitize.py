"""SURVEY.md §5 "ASan/UBSan on the CPU oracle": oracle/sanitize_check.c drives every oracle
entry point (empty / tiny / non-finite / duplicate inputs, several OpenMP threads) in a build
with -fsanitize=address,undefined and -fno-sanitize-recover, so any report fails this test.
CPU only (host code; GPU sanitizers are not available on the GPU pool)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_asan_ubsan_clean():
    r = subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "check-asan"], capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "sanitize_check: clean" in r.stdout
