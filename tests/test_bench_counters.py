"""bench.py refuses a roofline computed from wrong work counters (CPU: the check itself).

The roofline's algorithmic ops come from the kernel's counters (Mandelbulb bodies and bailouts
are data dependent, fragment.wgsl:245-249), and the golden frame hash cannot see them: the
summed counters of a fixed workload must be `frames` x the oracle's counters of its golden frame.
"""
import json
import os

import bench

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "fullsize.json")


def _gold(key):
    with open(GOLDEN) as fh:
        return [int(v) for v in json.load(fh)[key]["counters"]]


def test_exact_counters_accepted():
    g = _gold("HEADLINE_P1")
    got = [20 * v for v in g]
    cc = bench.counters_check(got, "HEADLINE", "P1", 20)
    assert cc["counters_ok"] is True
    assert "counters_mismatch" not in cc


def test_round3_body_undercount_rejected():
    # the round-3 persistent kernel subtracted every bailout from the body count a second time
    g = _gold("HEADLINE_P1")
    got = [20 * v for v in g]
    got[5] -= got[6]
    cc = bench.counters_check(got, "HEADLINE", "P1", 20)
    assert cc["counters_ok"] is False
    assert set(cc["counters_mismatch"]) == {"fractal_bodies"}
    assert cc["counters_mismatch"]["fractal_bodies"]["want"] == 20 * g[5]


def test_any_single_counter_off_by_one_rejected():
    g = _gold("C3_P1")
    for i, name in enumerate(bench.COUNTER_NAMES):
        got = [3 * v for v in g]
        got[i] += 1
        cc = bench.counters_check(got, "C3", "P1", 3)
        assert cc["counters_ok"] is False and set(cc["counters_mismatch"]) == {name}


def test_no_golden_means_no_check():
    assert bench.counters_check([0] * 8, "C1", "P1", 5) is None
    assert bench.counters_check([0] * 8, "HEADLINE", "P1", 5, golden_path="/nonexistent") is None
