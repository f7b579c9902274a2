"""The CPU restatement and the synthetic generator under the compiler's sanitizers (CPU).

SURVEY.md §5 asks for sanitizer builds of the host code. tests/sanitize/oracle_driver.c drives
oracle/ngs_oracle.c, oracle/ngs_oracle_g.c and stringsearchlib_amd/csrc/synth.c through builds,
searches (every threshold/limit shape, the wildcard, short and full-library-scan queries,
setValidChar, NULL words, zero/negative/large weights) and the pthread batches. Built three
ways with gcc: plain, ASan+UBSan (any report aborts), TSan (the batch workers share the index
and the work counter). All three must print the same checksum.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRCS = [os.path.join(ROOT, "tests", "sanitize", "oracle_driver.c"), os.path.join(ROOT, "oracle", "ngs_oracle.c"),
        os.path.join(ROOT, "oracle", "ngs_oracle_g.c"), os.path.join(ROOT, "stringsearchlib_amd", "csrc", "synth.c")]
BASE = ["gcc", "-std=gnu11", "-O1", "-g", "-fno-omit-frame-pointer", "-ffp-contract=off",
        "-I", os.path.join(ROOT, "oracle")]
MODES = {
    "plain": [],
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=all"],
    "tsan": ["-fsanitize=thread"],
}


def _build_and_run(mode, tmp_path):
    exe = str(tmp_path / f"driver_{mode}")
    subprocess.run(BASE + MODES[mode] + SRCS + ["-o", exe, "-lpthread"], check=True, capture_output=True, text=True)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
               TSAN_OPTIONS="halt_on_error=1:second_deadlock_stack=1")
    p = subprocess.run([exe, "4"], capture_output=True, text=True, env=env, timeout=600)
    assert p.returncode == 0, f"{mode}: rc {p.returncode}\n{p.stderr[-4000:]}"
    assert "runtime error" not in p.stderr and "WARNING: ThreadSanitizer" not in p.stderr, p.stderr[-4000:]
    out = p.stdout.strip().splitlines()[-1]
    assert out.startswith("ok "), out
    return out


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc absent")
def test_oracle_under_sanitizers(tmp_path):
    sums = {m: _build_and_run(m, tmp_path) for m in MODES}
    assert len(set(sums.values())) == 1, sums
