"""The heavy list's term-id slices (lean_query, SearchParams.hslices) forced on small libraries.

By default a heavy query is sliced only on indexes of long lists (C3: ~4 slices per 8-character
query) and by its own postings, so the small corpora of the parity tests run mostly unsliced. Here
a child process (tests/heavy_slices_child.py, NGS_HEAVY_SLICES read once per process) forces 8 and
3 slices per query and reruns the heavy-list parity cases exactly against the oracle: cmin-2 spills
and hand-overs, threshold-0 rank lists, cmin-1 part_ones queries (which run whole in slice 0), and
promotion beside large weights."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("slices", [8, 3])
def test_heavy_slices_forced(slices):
    env = dict(os.environ, NGS_HEAVY_SLICES=str(slices))
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "heavy_slices_child.py")
    p = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, (p.stdout[-2000:], p.stderr[-4000:])
    assert p.stdout.strip().splitlines()[-1] == "ok"
