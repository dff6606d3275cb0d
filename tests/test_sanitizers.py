"""Host C++ under sanitizers: builds csrc/tests/native_tests.cpp with ASAN+UBSAN (ring
kernels, parser, graph passes, scheduler, mailbox, TCP networking) and TSAN (the
concurrent parts) and runs it (scripts/sanitize.sh).  SURVEY §5 "race detection /
sanitizers"; the reference has no sanitizer configuration."""
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
@pytest.mark.parametrize("variant", ["asan", "tsan"])
def test_native_tests_under_sanitizers(variant):
    r = subprocess.run(["bash", os.path.join(REPO, "scripts", "sanitize.sh"), variant],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-4000:]
    assert "0 failed" in r.stderr
