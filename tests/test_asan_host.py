"""The C-ABI host code under AddressSanitizer (SURVEY §5 "sanitizers"): runs the driver that
`make -C vision_transformer_detector_amd/csrc asan` builds (tests/asan/abi_host_check.cpp,
linked against ASan-instrumented host objects of every source file; ~5 min to build, so the
build is not part of this test) when it is present.  No GPU is touched."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "build", "asan", "abi_host_check")


@pytest.mark.skipif(not os.path.exists(EXE), reason="ASan build absent (make ... asan)")
def test_abi_host_code_is_asan_clean():
    r = subprocess.run([EXE], capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1:halt_on_error=1"))
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok: 0 failure(s)" in r.stdout
    assert "AddressSanitizer" not in r.stderr
