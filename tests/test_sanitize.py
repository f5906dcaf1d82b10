"""Host sanitizers over the CPU oracle (the parity checker): `make -C oracle sanitize` builds
it with AddressSanitizer + UndefinedBehaviorSanitizer (-fno-sanitize-recover=all) and a
driver over its entry points (oracle/sanitize_main.c: traced rollouts at 2-4 players,
threaded rollouts, MCTS with root noise, symmetries, self-play episodes with examples).
Any sanitizer report aborts the run. GPU code has no sanitizer on this pool."""
import os
import shutil
import subprocess

import pytest

ORACLE = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_oracle_clean_under_asan_ubsan():
    subprocess.check_call(["make", "-s", "-C", ORACLE, "sanitize"])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([os.path.join(ORACLE, "sanitize_oracle")], capture_output=True, text=True, timeout=300,
                       env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "sanitize ok" in r.stdout
    assert "runtime error" not in r.stderr, r.stderr
