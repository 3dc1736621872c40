"""Host AddressSanitizer + UBSan over the native layer's CPU simulator path.

Builds ``build/asan/_native*.so`` (host code instrumented, device code untouched) and runs the
native-vs-oracle differential tests in a subprocess with the clang ASan runtime preloaded."""
import os
import shutil
import subprocess

import pytest

from tests.conftest import ROOT


@pytest.mark.skipif(not os.path.exists(os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")), reason="needs hipcc")
def test_native_host_path_under_asan_ubsan():
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "asan_check.sh"), "-k",
                        "native_matches_oracle_per_step or episode_reset or syn200"],
                       capture_output=True, text=True, timeout=1500)
    tail = (r.stdout + r.stderr)[-3000:]
    assert r.returncode == 0, tail
    assert "AddressSanitizer" not in tail and "runtime error" not in tail, tail
    assert " passed" in tail
