"""fedlesscan_amd.metrics.aggregate_metrics against the reference's own
FLStrategy.aggregate_metrics (fl_strategy.py:24-44), recorded by
tests/golden/make_golden_dropin.py: float64 bits, value lists, exception types."""
import json
import os

import numpy as np
import pytest

from fedlesscan_amd.common.models import TestMetrics
from fedlesscan_amd.metrics import aggregate_metrics

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "dropin.json")) as f:
    DROPIN = json.load(f)


@pytest.mark.parametrize("entry", DROPIN["metrics"], ids=lambda e: e["name"])
def test_aggregate_metrics_matches_reference(entry):
    tms = [TestMetrics(cardinality=c, metrics=m) for c, m in entry["metrics"]]
    if "raises" in entry:
        with pytest.raises(Exception) as ei:
            aggregate_metrics(tms, entry["names"])
        assert type(ei.value).__name__ == entry["raises"]
        return
    got = aggregate_metrics(tms, entry["names"])
    assert sorted(got) == sorted(entry["result"])
    for k, exp in entry["result"].items():
        if k.startswith("all_"):
            assert got[k] == exp["list"] and [type(x) for x in got[k]] == [type(x) for x in exp["list"]], k
        else:
            assert type(got[k]).__name__ == exp["type"], k
            assert float(got[k]).hex() == exp["hex"], k


def test_handler_swap_recorded_equal():
    """The reference handler with the drop-in strategies swapped in
     matched the unmodified handler in every
    scenario when the fixtures were made (the script asserts it)."""
    hs = DROPIN["handler_swap"]
    assert len(hs) >= 10 and all(v["same_as_reference"] for v in hs.values())
