"""the CPU oracle under AddressSanitizer + UndefinedBehaviorSanitizer.
Every parity verdict rests on the oracle's bounds arithmetic over malformed
input, so its own tests and the adversarial corpora run once more against
oracle/libhonu_oracle_san.so (oracle/Makefile `sanitize`, -fsanitize=address,
undefined -fno-sanitize-recover=all) in a child process with the ASan runtime
preloaded; any report aborts the child and fails this test."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SAN = os.path.join(ROOT, "oracle", "libhonu_oracle_san.so")


def _asan_runtime():
    try:
        p = subprocess.run(["gcc", "-print-file-name=libasan.so"], capture_output=True,
                           text=True, check=True).stdout.strip()
    except Exception:
        return None
    return p if os.path.isabs(p) and os.path.exists(p) else None


def test_oracle_under_asan_ubsan():
    rt = _asan_runtime()
    if rt is None:
        pytest.skip("no gcc ASan runtime")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True)
    env = dict(os.environ, LD_PRELOAD=rt, HONU_ORACLE_LIB=SAN,
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    probe = ("import sys; sys.path.insert(0, 'tests'); from oracle import oracle; oracle.load(); "
             "maps = open('/proc/self/maps').read(); "
             "print(oracle.LIB_PATH, 'libasan' in maps)")
    r = subprocess.run([sys.executable, "-c", probe], cwd=ROOT, env=env, capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.split() == [SAN, "True"]
    files = ["tests/test_oracle_golden.py", "tests/test_oracle_generated.py",
             "tests/test_oracle_corpora.py", "tests/test_golden_batches.py",
             "tests/test_system.py"]
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-m", "not gpu",
                        "-p", "no:cacheprovider"] + files, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    assert " passed" in r.stdout
