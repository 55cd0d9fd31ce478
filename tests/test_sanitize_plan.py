"""The LBA host planning path under ThreadSanitizer and AddressSanitizer + UBSan (CPU only: the
sanitizers instrument the host code of orb-slam3-noted_amd/csrc/lba.hip; no HIP call is made).

tests/cpp/plan_stress.cpp drives slamhot_lba_plan_stress: six threads, each with the PlanPool and
arena one solver handle owns, plan {4, 8, 128, 1, 16}-window calls for several rounds, so every pool
gains worker threads between calls while the other five plan too -- the concurrency bench.py's LBA
leg (six solvers in flight) puts on the library.  Every thread's plan must equal the others' byte for
byte, and the sanitizers must report nothing."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

pytestmark = pytest.mark.skipif(shutil.which("make") is None or not Path("/opt/rocm/bin/hipcc").exists(),
                                reason="needs make and hipcc")


@pytest.fixture(scope="module")
def built():
    r = subprocess.run(["make", "-s", "sanitize-plan"], cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("kind", ["tsan", "asan"])
def test_plan_pools_under_sanitizer(built, kind):
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66", ASAN_OPTIONS="halt_on_error=1 exitcode=66",
               UBSAN_OPTIONS="halt_on_error=1 exitcode=66 print_stacktrace=1")
    r = subprocess.run([str(ROOT / "tests" / "cpp" / f"plan_stress_{kind}"), "6", "3"], capture_output=True,
                       text=True, timeout=300, env=env)
    err = "\n".join(x for x in r.stderr.splitlines() if not x.startswith("fill sections"))
    assert r.returncode == 0, err[-4000:]
    assert "plan_stress ok" in r.stdout
    assert "Sanitizer" not in err and "runtime error" not in err, err[-4000:]
