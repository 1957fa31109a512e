"""Cardinality-weighted averaging of client test metrics on the round boundary.

Mirrors FLStrategy.aggregate_metrics (fedless/controller/strategies/fl_strategy.py:24-44):
for every requested metric name, the np.average of the clients' values weighted
by their test-set cardinality, the list of all values and their median.  These
are a handful of scalars per round, so this stays on the host.

Pinned to the reference itself (tests/golden/dropin.json "metrics", written by
tests/golden/make_golden_dropin.py): the same float64 bits, the same value
lists, and the same exceptions -- ValueError for an empty list (the
reference's `zip(*())` unpacking, fl_strategy.py:30-32), ZeroDivisionError when
the cardinalities sum to zero (np.average), KeyError for a missing name.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np

from .common.models import TestMetrics


def aggregate_metrics(metrics: Sequence[TestMetrics], metric_names: Optional[List[str]] = None) -> Dict:
    names = metric_names if metric_names is not None else ["loss"]
    # unpacked the way the reference does: an empty list raises ValueError here
    cards, values = zip(*((m.cardinality, m.metrics) for m in metrics))
    out: Dict = {}
    for name in names:
        v = [d[name] for d in values]
        out.update({f"mean_{name}": np.average(v, weights=cards), f"all_{name}": v,
                    f"median_{name}": np.median(v)})
    return out
