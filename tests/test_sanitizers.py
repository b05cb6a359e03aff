"""ASan/UBSan run of the C oracle (race detection / sanitizers).

``make -C oracle sanitize`` builds oracle/sanitize_main.c with the whole
restatement under -fsanitize=address,undefined (no recovery) and runs the FD
worker (partial and odd blocks, resize both ways, block sizes 1..16, literal
Suzuki path) and the OF worker (direct and sliding box sums). Any
out-of-bounds access, leak or undefined behaviour fails the run.
"""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE = os.path.join(os.path.dirname(HERE), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_oracle_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", ORACLE, "sanitize"], check=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ORACLE, "_san", "sanitize_main")], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitized run ok" in r.stdout
