"""The batch-wide survivor arena (SearchParams.at): tier 1a's main launch writes a query's survivors
to its slots and, past them, to blocks of an arena shared by the call, chained per query; k_emit
reads them back in order (nGramSearch.hpp:310-341 over every survivor). Slots are 256 per query here
and the arena starts at 256 blocks of 1,024 (NGS_ECAP_INIT, NGS_ARENA_INIT, read once per process:
tests/arena_child.py runs in a child process), so queries of ~1,900 survivors live mostly in the
arena. Checked: answers exact against the oracle on
every call; the first call runs the arena out (its queries are handed to tier 1b, still exact) and
the arena grows instead of the slots; later calls fit."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu


def test_arena_holds_survivors_past_the_slots():
    env = dict(os.environ, NGS_ECAP_INIT="256", NGS_ARENA_INIT="256")
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "arena_child.py")
    p = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert not r["fails"], "\n".join(r["fails"])
    s = r["stats"]
    assert all(x["survivor_slots"] == 256 for x in s[:3]), s  # the slots never grew
    assert s[0]["heavy_queries"] == 0 and s[0]["fast_queries"] > 0, s  # the main launch's queries
    assert s[0]["arena_used"] > s[0]["arena_blocks"] and s[0]["slot_full_queries"] > 0, s  # ran out, handed over
    assert s[1]["arena_blocks"] > s[0]["arena_blocks"], s  # ... and grew
    assert s[2]["arena_used"] > 0 and s[2]["arena_used"] <= s[2]["arena_blocks"], s
    assert s[2]["slot_full_queries"] == 0, s
    assert s[3]["arena_used"] > 0 and s[3]["slot_full_queries"] == 0, s
    assert r["promoted"] == r["exact"], r  # every exact-key query answered with its key promoted to 100


def test_arena_allocation_failure_leaves_the_context_working():
    """An arena too large to allocate (NGS_ARENA_INIT of 2^30 blocks, 5 TB) is not an error of the call
    (ADVICE r5): the calls run without one, the queries past their slots go to tier 1b, every answer
    stays exact, and later calls on the same context keep working."""
    env = dict(os.environ, NGS_ECAP_INIT="256", NGS_ARENA_INIT=str(1 << 30))
    child = os.path.join(os.path.dirname(os.path.abspath(__file__)), "arena_child.py")
    p = subprocess.run([sys.executable, child], env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert not r["fails"], "\n".join(r["fails"])
    s = r["stats"]
    assert all(x["arena_blocks"] == 0 for x in s[:3]), s
    assert s[0]["slot_full_queries"] > 0, s  # the overflowing queries went to tier 1b
    assert r["promoted"] == r["exact"], r
