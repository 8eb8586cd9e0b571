"""The C oracle under AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY §5:
sanitizers on the CPU restatement): the oracle's golden and conv tests re-run in
a child process against `make -C oracle san`'s build, with libasan preloaded
(a sanitized shared library loaded into an unsanitized python needs the
runtime first). Any heap overflow, use-after-free or undefined behaviour
aborts the child."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.mark.skipif(_runtime("libasan.so") is None, reason="no libasan runtime")
def test_oracle_tests_pass_under_asan_ubsan():
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "san"], check=True)
    env = dict(os.environ, SHPL_ORACLE_LIB=os.path.join(ROOT, "oracle", "build", "libshpl_oracle_san.so"),
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1")
    pre = [_runtime("libasan.so"), _runtime("libubsan.so")]
    env["LD_PRELOAD"] = " ".join([p for p in pre if p] + ([os.environ["LD_PRELOAD"]] if os.environ.get("LD_PRELOAD")
                                                            else []))
    p = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(ROOT, "tests", "test_oracle_golden.py"),
                        os.path.join(ROOT, "tests", "test_oracle_conv.py"),
                        os.path.join(ROOT, "tests", "test_dist_gloo.py") + "::test_two_rank_strong_partition_matches_one_process"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "passed" in p.stdout
