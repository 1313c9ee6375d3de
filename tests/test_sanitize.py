"""Host code of librevel_wal under AddressSanitizer + UndefinedBehaviorSanitizer
(tools/sanitize): writer, host-walk reader, files, framing layout, error
paths.  Host only -- the gfx950 kernels are linked uninstrumented."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_host_code_under_asan_ubsan():
    b = subprocess.run(["make", "-C", os.path.join(ROOT, "tools", "sanitize")], capture_output=True, text=True,
                       timeout=600)
    assert b.returncode == 0, b.stdout[-2000:] + b.stderr[-2000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ROOT, "build", "sanitize", "host_sanitize_test")], capture_output=True,
                       text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "all checks passed" in r.stdout
