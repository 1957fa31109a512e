"""ORACLE — CPU restatement of the reference FedAvg / FedLesScan aggregation.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import this module, and only as the
checker or as the timed CPU baseline.  The product path
(``fedlesscan_amd``) never imports it: it runs the HIP kernels or fails.

Parity status: PINNED.  ``tests/golden/`` holds vectors produced by the
reference itself (``/root/reference`` imported under the shims of SURVEY.md
App. B by ``tests/golden/make_golden.py``) plus the reference's own unit-test
fixture (``test/test_aggregation.py:23-86``); ``tests/test_oracle_golden.py``
checks this module bit-for-bit against every one of them.

Each function cites the reference file:line it restates (paths relative to
the reference repo root).  The arithmetic is numpy's: ``np.multiply``,
``np.add`` and ``np.true_divide`` on arrays with *Python* scalar operands,
which numpy treats as weak scalars (NEP 50; value-based casting in numpy 1.x
gives the same dtype for these cases).  So for float32 updates:

    a_i = fl32(n_i), s_i = fl32((r_i + 1) / (R + 1))       (double divide, then round)
    t_i = fl32(fl32(x_i * a_i) * s_i)                       (two separate roundings)
    acc = t_0; acc = fl32(acc + t_i) for i = 1..N-1         (strict left fold)
    out = fl32(acc / fl32(sum(n_i)))                        (IEEE divide)
"""
from __future__ import annotations

import io
import base64
from functools import reduce
from typing import Iterable, List, Optional, Sequence

import numpy as np

UNKNOWN_CARDINALITY = -2   # tf.data.UNKNOWN_CARDINALITY (fed_avg_aggregator.py:73-76)
INFINITE_CARDINALITY = -1  # tf.data.INFINITE_CARDINALITY


class OracleUnknownCardinality(Exception):
    """Mirrors fedless.aggregator.exceptions.UnknownCardinalityError (exceptions.py:9)."""


# --------------------------------------------------------------------------
# scores: stall_aware_aggregation.py:34-40
# --------------------------------------------------------------------------
def score_clients(client_feats: Sequence[dict], current_round: int) -> List[float]:
    """s_i = (round_i + 1) / (R + 1) as Python floats (double division)."""
    out = []
    for feat in client_feats:
        out.append((feat["round_id"] + 1) / (current_round + 1))
    return out


# --------------------------------------------------------------------------
# literal restatements of the two _aggregate() hot loops
# --------------------------------------------------------------------------
def fedavg_literal(parameters: Sequence[Sequence[np.ndarray]], weights: Sequence) -> List[np.ndarray]:
    """fed_avg_aggregator.py:24-42.

    Total is a Python-level sum (exact for ints).  Every client's layers are
    scaled into a product temporary first, then each layer is folded
    left-to-right with np.add and divided once.  zip() truncation of both the
    client list and the per-client layer lists is kept.
    """
    total = sum(weights)
    products = []
    for client_layers, n in zip(parameters, weights):
        products.append([np.multiply(layer, n) for layer in client_layers])
    result = []
    for per_layer in zip(*products):
        acc = reduce(np.add, per_layer)
        result.append(np.true_divide(acc, total))
    return result


def stall_aware_literal(client_feats: Sequence[dict], current_round: int,
                        parameters: Sequence[Sequence[np.ndarray]], weights: Sequence) -> List[np.ndarray]:
    """stall_aware_aggregation.py:42-67.

    Product is ``(layer * n_i) * s_i`` (two roundings, left-to-right operator
    evaluation), divisor is sum(n_i) -- NOT sum(n_i * s_i).
    """
    total = sum(weights)
    scores = score_clients(client_feats, current_round)
    products = []
    for client_layers, n, s in zip(parameters, weights, scores):
        products.append([np.multiply(np.multiply(layer, n), s) for layer in client_layers])
    result = []
    for per_layer in zip(*products):
        acc = reduce(np.add, per_layer)
        result.append(np.true_divide(acc, total))
    return result


# --------------------------------------------------------------------------
# lean form on a stacked [N, P] matrix: one temporary, bit-identical
# --------------------------------------------------------------------------
def fedavg_stacked(X: np.ndarray, weights: Sequence, scores: Optional[Sequence[float]] = None,
                   total=None) -> np.ndarray:
    """Same op order as fedavg_literal on a row-stacked matrix, O(P) temporaries.

    Columns are independent, so flattening the layers of each client into one
    row changes no arithmetic.  ``total`` defaults to sum(weights).
    """
    if total is None:
        total = sum(weights)
    n_rows = X.shape[0]
    tmp = np.empty(X.shape[1:], dtype=np.result_type(X.dtype, *weights))
    acc = None
    for i in range(n_rows):
        np.multiply(X[i], weights[i], out=tmp)
        if scores is not None:
            np.multiply(tmp, scores[i], out=tmp)
        if acc is None:
            acc = tmp.copy()
        else:
            np.add(acc, tmp, out=acc)
    return np.true_divide(acc, total)


def fedavg_stacked_bf16(Xbits: np.ndarray, weights: Sequence, scores=None, total=None):
    """bf16 extension (no reference path; SURVEY 8c "bf16: parity unpinned").

    Defined as: upcast each bf16 element exactly to float32, then run the
    float32 reference algorithm.  Returns (out_f32, out_bf16_bits_RNE).
    """
    import fedlesscan_amd.synth as synth  # generator helpers only
    X = synth.bf16_bits_to_f32(Xbits)
    out = fedavg_stacked(X, weights, scores, total)
    return out, synth.f32_to_bf16_bits(out)


# --------------------------------------------------------------------------
# NPZ decode: serialization.py:80-93, 280-306
# --------------------------------------------------------------------------
def deserialize_npz(blob, string_format: str = "none") -> List[np.ndarray]:
    if string_format == "base64":
        blob = base64.b64decode(blob)
    with io.BytesIO(blob) as f:
        npz = np.load(f)
        return list(npz.values())


def _checked_cardinality(card, default_cardinality):
    """fed_avg_aggregator.py:73-82: -1/-2 -> default or error; `if not default` quirk kept."""
    if card in (UNKNOWN_CARDINALITY, INFINITE_CARDINALITY):
        if not default_cardinality:
            raise OracleUnknownCardinality("Cardinality for client result invalid. ")
        return default_cardinality
    return card


def aggregate_fedavg(results: Iterable[dict], default_cardinality=None):
    """fed_avg_aggregator.py:57-92 on plain dicts {blob, string_format, cardinality, test_metrics}."""
    params, cards, metrics = [], [], []
    for r in results:
        params.append(deserialize_npz(r["blob"], r.get("string_format", "none")))
        cards.append(_checked_cardinality(r["cardinality"], default_cardinality))
        if r.get("test_metrics"):
            metrics.append(r["test_metrics"])
    return fedavg_literal(params, cards), (metrics or None)


def aggregate_stall_aware(results: Iterable[dict], client_feats, current_round, default_cardinality=None):
    """stall_aware_aggregation.py:82-117."""
    params, cards, metrics = [], [], []
    for r in results:
        params.append(deserialize_npz(r["blob"], r.get("string_format", "none")))
        cards.append(_checked_cardinality(r["cardinality"], default_cardinality))
        if r.get("test_metrics"):
            metrics.append(r["test_metrics"])
    return stall_aware_literal(client_feats, current_round, params, cards), (metrics or None)


def _chunks(items, n):
    """fed_avg_aggregator.py:99-109 (a chunk of exactly n, then the remainder)."""
    buf = []
    for el in items:
        if len(buf) < n:
            buf.append(el)
        if len(buf) == n:
            yield buf
            buf = []
    if buf:
        yield buf


def aggregate_stream_fedavg(results, chunk_size=25, default_cardinality=None):
    """fed_avg_aggregator.py:111-153: g <- _aggregate([g, *chunk], [W, *n_chunk])."""
    g, w_sum, metrics = None, 0, []
    for chunk in _chunks(results, chunk_size):
        p_buf, c_buf = [], []
        for r in chunk:
            p_buf.append(deserialize_npz(r["blob"], r.get("string_format", "none")))
            c_buf.append(_checked_cardinality(r["cardinality"], default_cardinality))
            if r.get("test_metrics"):
                metrics.append(r["test_metrics"])
        if g is None:
            g = fedavg_literal(p_buf, c_buf)
        else:
            g = fedavg_literal([g, *p_buf], [w_sum, *c_buf])
        w_sum += sum(c_buf)
    return g, (metrics or None)


def aggregate_stream_stall_aware(results, client_feats, current_round, chunk_size=25,
                                 default_cardinality=None):
    """stall_aware_aggregation.py:142-187, including the score misalignment of App. C.2:
    every chunk re-scores client_feats from index 0."""
    g, w_sum, metrics = None, 0, []
    for chunk in _chunks(results, chunk_size):
        p_buf, c_buf = [], []
        for r in chunk:
            p_buf.append(deserialize_npz(r["blob"], r.get("string_format", "none")))
            c_buf.append(_checked_cardinality(r["cardinality"], default_cardinality))
            if r.get("test_metrics"):
                metrics.append(r["test_metrics"])
        if g is None:
            g = stall_aware_literal(client_feats, current_round, p_buf, c_buf)
        else:
            g = stall_aware_literal(client_feats, current_round, [g, *p_buf], [w_sum, *c_buf])
        w_sum += sum(c_buf)
    return g, (metrics or None)


def weighted_metrics(metrics: Sequence[dict], metric_names=None) -> dict:
    """fl_strategy.py:24-44: np.average weighted by test cardinality, plus median."""
    if metric_names is None:
        metric_names = ["loss"]
    cards = [m["cardinality"] for m in metrics]
    vals = [m["metrics"] for m in metrics]
    out = {}
    for name in metric_names:
        v = [d[name] for d in vals]
        out[f"mean_{name}"] = np.average(v, weights=cards)
        out[f"all_{name}"] = v
        out[f"median_{name}"] = np.median(v)
    return out
