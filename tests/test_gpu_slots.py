"""Tier 1a's survivor slots grow with the workload. A query whose survivors overflow its HBM slots
(SearchParams.ecap) is handed to tier 1b; the call counts those queries (ngs_stats.
slot_full_queries) and, when they are more than 1/64 of the batch, the context's later calls run
with twice the slots (ensure_queries / emit_cap_max). Every call's answer stays exact: the
hand-over path and the grown slots both give the oracle's results (nGramSearch.hpp:278-341). The
starting slot count is read once per process (NGS_ECAP_INIT), so the calls run in a child process
(tests/slots_child.py)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_slots_grow_and_stay_exact():
    env = dict(os.environ, NGS_ECAP_INIT="256")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "slots_child.py")
    p = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert not r["fails"], "\n".join(r["fails"])
    slots, full = r["slots"], r["slot_full"]
    assert slots[0] == 256 and full[0] > 0, r  # the first call fills 256 slots and hands those over
    assert slots[:6] == sorted(slots[:6]) and slots[5] > 256, r  # later calls have more
    assert full[5] < full[0], r
    assert max(r["bytes"]) <= 16 << 30, r  # the budget holds after a large batch
    calm = r["calm_slots"]
    assert calm[-1] < calm[0], r  # grown slots went back after calls that filled none
