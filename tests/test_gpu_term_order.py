"""The opt-in key-rank term order (NGS_TERM_ORDER=rank, ngs_build.h): host and GPU builds agree,
the index reports term ids in key-rank order (DevIndex.tk_monotone) on a corpus of one term per
key, and tier 1b's tie-driven count threshold (raised_cmin) keeps every answer exact against the
oracle at thresholds 0 and 0.2. The build reads the variable once per process, so the checks run
in a child process (tests/term_order_child.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_rank_term_order_parity():
    env = dict(os.environ, NGS_TERM_ORDER="rank")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "term_order_child.py")
    p = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert not r["fails"], "\n".join(r["fails"])
    assert r["checked"] >= 2000
    assert r["flags"][0] & 4, f"unweighted synthetic corpus should be in key-rank order: flags {r['flags']}"
