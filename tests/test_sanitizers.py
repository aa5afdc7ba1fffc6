"""CPU sanitizer runs (the CPU code under ASAN / TSAN).

`make -C oracle asan tsan` builds oracle/san_main.cc against the oracle's
pthread pool and libme_hip's host-only C++ (me_plan.cpp: stripe planner and
candidate counts; me_io.cpp: the YUV and MEMV readers fed truncated, corrupt
and hostile files) under AddressSanitizer + UBSan and under ThreadSanitizer;
both runs must finish clean."""
import os
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE = os.path.join(REPO, "oracle")


@pytest.mark.parametrize("kind", ["asan", "tsan"])
def test_sanitizer_run_is_clean(kind, tmp_path):
    subprocess.run(["make", "-s", "-C", ORACLE, kind], check=True, timeout=300)
    env = dict(os.environ, TMPDIR=str(tmp_path),
               ASAN_OPTIONS="detect_leaks=1:abort_on_error=0:exitcode=23",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:exitcode=23")
    r = subprocess.run([os.path.join(ORACLE, "_san", f"san_{kind}")], capture_output=True,
                       text=True, timeout=300, env=env)
    assert r.returncode == 0 and "san ok" in r.stdout, r.stdout[-2000:] + r.stderr[-4000:]
    assert "WARNING: ThreadSanitizer" not in r.stderr
    assert "runtime error" not in r.stderr
