"""Handler-level parity: fedlesscan_amd.handler.default_aggregation_handler against
the reference's own default_aggregation_handler (aggregation.py:45-167), run by
tests/golden/make_golden.py::case_handler over an in-memory Mongo/GridFS.

Each scenario re-creates the same stored documents (same order, sessions,
rounds, client ids, NPZ blobs, cardinalities, test metrics) in the in-memory
store and checks everything the reference handler returned or left behind:
new_round_id, num_clients (bit-exact integers), test_results, the model saved at
round R+1 (bit-for-bit), which results were deleted, and the reference's own
exceptions.  The empty rounds pin that InsufficientClientResults is never raised
at selection (the reference checks a generator's truthiness,
fed_avg_aggregator.py:51-54 / client_daos.py:125,161).

CPU tests take the fold from the oracle (bookkeeping is what they check); the
-m gpu tests run the real HIP fold through the same handler.
"""
from functools import reduce

import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import engine, synth
from fedlesscan_amd.common.models import (AggregationHyperParams, AggregationStrategy, ClientResult,
                                          NpzWeightsSerializerConfig, SerializedParameters, TestMetrics,
                                          WeightsSerializerConfig)
from fedlesscan_amd.common.serialization import NpzWeightsSerializer
from fedlesscan_amd.store import InMemoryClientResultStore, InMemoryParameterStore
from oracle import fedavg_oracle as O

CASE = "handler"
SER = WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())


def _scenarios():
    return sorted(G.manifest()[CASE]["scenarios"])


def _build_store(entry):
    m = G.manifest()[CASE]
    X = synth.clients_f32(m["seed"], m["rows"], 0, m["P"])
    st = InMemoryClientResultStore()
    for d in entry["docs"]:
        sess, rnd, cid, row, card = d[:5]
        tm = TestMetrics(cardinality=d[5][0], metrics=d[5][1]) if len(d) > 5 else None
        blob = NpzWeightsSerializer().serialize(G._split(X[row], m["shapes"]))
        st.save(sess, rnd, cid, ClientResult(parameters=SerializedParameters(blob=blob, serializer=SER),
                                             cardinality=card, test_metrics=tm))
    return st


def _run(entry, device=None, devices=None):
    from fedlesscan_amd.handler import default_aggregation_handler
    st, ps = _build_store(entry), InMemoryParameterStore()
    res = default_aggregation_handler("s", entry["round_id"], st, ps, SER, None, entry["delete"],
                                      AggregationStrategy(entry["strategy"]),
                                      AggregationHyperParams(**entry["hyperparams"]), device=device,
                                      devices=devices)
    return res, st, ps


def _check(name, entry, res, st, ps):
    R = entry["round_id"]
    assert res.new_round_id == entry["new_round_id"]
    assert type(res.num_clients) is int and res.num_clients == entry["num_clients"]
    got_tr = None if res.test_results is None else [t.model_dump() for t in res.test_results]
    assert got_tr == entry["test_results"]
    assert res.global_test_results is None
    assert sorted(r for (s, r) in ps._params if s == "s") == entry["saved_round_ids"]
    saved = ps.load("s", R + 1)
    outs = NpzWeightsSerializer().deserialize(saved.blob)
    exp = G.expected(CASE, name)
    assert len(outs) == len(exp)
    for o, e in zip(outs, exp):
        assert G.same_bits(o, e), name
    if entry["saved_blob_sha256"] is not None:  # the empty model: byte-identical NPZ
        import hashlib
        assert len(saved.blob) == entry["saved_blob_len"]
        assert hashlib.sha256(saved.blob).hexdigest() == entry["saved_blob_sha256"]
    left = sorted([d["session_id"], d["round_id"], d["client_id"]] for d in st._docs)
    assert left == entry["remaining_results"]
    assert len(st._files) == entry["remaining_files"]


@pytest.fixture
def oracle_fold(monkeypatch):
    def fake(parameters, weights, scores=None, device=None, devices=None):
        n = min(len(parameters), len(weights), len(scores) if scores is not None else len(weights))
        if scores is None:
            return O.fedavg_literal(parameters[:n], list(weights))
        total = sum(weights)
        prods = [[np.multiply(np.multiply(l, w), s) for l in p] for p, w, s in zip(parameters, weights, scores)]
        return [reduce(np.add, ls) / total for ls in zip(*prods)]

    def fake_decoded(items, scores=None, device=None, devices=None, expected_rows=0):
        rows, ws = [], []
        for layers, w in items:
            rows.append(layers)
            ws.append(w)
        return fake(rows, ws, scores) if rows else []

    monkeypatch.setattr(engine, "aggregate_layers", fake)
    monkeypatch.setattr(engine, "aggregate_decoded", fake_decoded)


@pytest.mark.parametrize("name", _scenarios())
def test_handler_bookkeeping_vs_reference(name, oracle_fold):
    entry = G.manifest()[CASE]["scenarios"][name]
    if "raises" in entry:
        with pytest.raises(Exception) as ei:
            _run(entry)
        assert type(ei.value).__name__ == entry["raises"]
        return
    _check(name, entry, *_run(entry))


def test_empty_round_needs_no_gpu():
    """Zero results never reach a kernel: [] parameters, an empty NPZ at R+1,
    num_clients 0 -- with the real engine, on a machine without a GPU."""
    for name in ("empty_per_round", "empty_per_session"):
        entry = G.manifest()[CASE]["scenarios"][name]
        _check(name, entry, *_run(entry))


def test_empty_selection_does_not_raise():
    from fedlesscan_amd import FedAvgAggregator, StallAwareAggregator
    st = InMemoryClientResultStore()
    dicts, cands = FedAvgAggregator().select_aggregation_candidates(st, "s", 1)
    assert dicts == [] and list(cands) == []
    dicts, cands = StallAwareAggregator(1, AggregationHyperParams(tolerance=2)).select_aggregation_candidates(
        st, "s", 1)
    assert dicts == [] and list(cands) == []
    assert FedAvgAggregator().aggregate([], []) == ([], None)
    assert StallAwareAggregator(1, None).aggregate([], []) == ([], None)


@pytest.mark.gpu
@pytest.mark.parametrize("name", _scenarios())
def test_handler_on_gpu_vs_reference(name):
    import torch
    entry = G.manifest()[CASE]["scenarios"][name]
    dev = torch.device("cuda", 0)
    if "raises" in entry:
        with pytest.raises(Exception) as ei:
            _run(entry, dev)
        assert type(ei.value).__name__ == entry["raises"]
        return
    _check(name, entry, *_run(entry, dev))


@pytest.mark.gpu
@pytest.mark.parametrize("name", _scenarios())
def test_handler_on_two_gpu_buckets_vs_reference(name):
    """The same scenarios with the strategy folding one column bucket per GPU
    (devices=[0, 0]: two buckets on the one GPU of a test box)."""
    entry = G.manifest()[CASE]["scenarios"][name]
    if "raises" in entry:
        with pytest.raises(Exception) as ei:
            _run(entry, devices=[0, 0])
        assert type(ei.value).__name__ == entry["raises"]
        return
    _check(name, entry, *_run(entry, devices=[0, 0]))
