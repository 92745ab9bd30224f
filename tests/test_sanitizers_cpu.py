"""The host code under sanitizers (CPU suite): `make -C diamond-ppo_amd tsan asan` builds
tests/native/host_stress.cpp with csrc/perm.cpp (permutation draws, swap pool, producer ring,
chained async drafts waited on another thread -- the learn() look-ahead protocol) and
csrc/loop_sync.h (the loopback group barrier: generations, a member leaving, a timeout), under
ThreadSanitizer and under AddressSanitizer + UBSan, and runs them; any report fails the run."""
import os
import shutil
import subprocess

import pytest

from conftest import PKG

CLANG = "/opt/rocm/lib/llvm/bin/clang++"


@pytest.mark.skipif(not os.path.exists(CLANG) or shutil.which("make") is None,
                    reason="needs ROCm's clang++ (sanitizer runtimes) and make")
@pytest.mark.parametrize("target", ["tsan", "asan"])
def test_host_code_clean_under_sanitizer(target):
    r = subprocess.run(["make", "-C", PKG, target], capture_output=True, text=True, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert "OK:" in out and "0 failures" in out
    assert "WARNING: ThreadSanitizer" not in out and "ERROR: AddressSanitizer" not in out
