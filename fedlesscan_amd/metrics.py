"""Cardinality-weighted averaging of client test metrics on the round boundary.

Mirrors FLStrategy.aggregate_metrics (fedless/controller/strategies/fl_strategy.py:24-44):
for every requested metric name, the np.average of the clients' values weighted
by their test-set cardinality, the list of all values and their median.  These
are a handful of scalars per round, so this stays on the host.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence

import numpy as np

from .common.models import TestMetrics


def aggregate_metrics(metrics: Sequence[TestMetrics], metric_names: Optional[List[str]] = None) -> Dict:
    names = metric_names if metric_names is not None else ["loss"]
    cards = [m.cardinality for m in metrics]
    values = [m.metrics for m in metrics]
    out: Dict = {}
    for name in names:
        v = [d[name] for d in values]
        out[f"mean_{name}"] = np.average(v, weights=cards)
        out[f"all_{name}"] = v
        out[f"median_{name}"] = np.median(v)
    return out
