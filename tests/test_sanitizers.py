"""Host sanitizer runs (SURVEY.md §5 race detection): the native test runner,
the C/C++ examples and the benchmark CLI's host path (every exchange type, two
transforms) built with AddressSanitizer + UndefinedBehaviorSanitizer and with
ThreadSanitizer (thread pool, in-process rank groups) — tools/sanitize.py.

CPU only; the first run compiles an instrumented build under build/san-*."""
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(1800)
@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_host_sanitizers(kind):
    r = subprocess.run([sys.executable, os.path.join(REPO, "tools", "sanitize.py"), kind],
                       cwd=REPO, capture_output=True, text=True, timeout=1800)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-6000:]
    assert out.count("clean") == 4, out[-6000:]
