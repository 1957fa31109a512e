"""The strategies' select_aggregation_candidates keeps the reference's
signature (fed_avg_aggregator.py:44, stall_aware_aggregation.py:69):
`(mongo_client, session_id, round_id)`, positional or by keyword, so the
reference's handler (aggregation.py:76-78) calls it unchanged (VERDICT r5
next #5).  A result store is used as it is; a raw MongoClient is wrapped into
the reference's ClientResultDao when that is importable, else TypeError."""
import sys
import types

import pytest

from fedlesscan_amd.aggregator import FedAvgAggregator, StallAwareAggregator
from fedlesscan_amd.aggregator.exceptions import InsufficientClientResults
from fedlesscan_amd.common.models import AggregationHyperParams
from fedlesscan_amd.store import InMemoryClientResultStore


def _store():
    st = InMemoryClientResultStore()
    for rnd, cid in ((3, "a"), (3, "b"), (2, "c"), (0, "d")):
        st.save("s1", rnd, cid, {"client": cid})
    st.save("s2", 3, "x", {"client": "x"})
    return st


def _strategies():
    return [FedAvgAggregator(), StallAwareAggregator(3, AggregationHyperParams(tolerance=1))]


def test_positional_and_keyword_calls_agree():
    st = _store()
    for agg in _strategies():
        d1, c1 = agg.select_aggregation_candidates(st, "s1", 3)
        d2, c2 = agg.select_aggregation_candidates(mongo_client=st, session_id="s1", round_id=3)
        assert d1 == d2 and d1  # the generators read the documents lazily, as the reference's
    fed, stall = _strategies()
    assert [d["client_id"] for d in fed.select_aggregation_candidates(st, "s1", 3)[0]] == ["a", "b"]
    # tolerance 1: rounds >= 2 of the session
    assert [d["client_id"] for d in stall.select_aggregation_candidates(mongo_client=st, session_id="s1",
                                                                        round_id=3)[0]] == ["a", "b", "c"]


def test_raw_client_without_the_reference_dao_raises_type_error(monkeypatch):
    # the reference package is not importable: nothing to wrap a MongoClient in
    for m in ("fedless", "fedless.persistence", "fedless.persistence.client_daos"):
        monkeypatch.setitem(sys.modules, m, None)
    for agg in _strategies():
        with pytest.raises(TypeError, match=r"ClientResultDao\(mongo_client\).*INTEGRATION"):
            agg.select_aggregation_candidates(mongo_client=object(), session_id="s1", round_id=3)


def test_raw_client_is_wrapped_in_the_reference_dao(monkeypatch):
    """With the reference's persistence module in the caller's environment, a
    MongoClient goes through ClientResultDao(mongo_client), as the reference
    does: here a stand-in DAO module over the in-memory store."""
    st = _store()
    seen = []

    class ClientResultDao:
        def __init__(self, client):
            seen.append(client)
            self._st = st

        def load_results_for_round(self, **kw):
            return self._st.load_results_for_round(**kw)

        def load_results_for_session(self, **kw):
            return self._st.load_results_for_session(**kw)

    pkg, sub, mod = (types.ModuleType(n) for n in ("fedless", "fedless.persistence",
                                                    "fedless.persistence.client_daos"))
    mod.ClientResultDao = ClientResultDao
    pkg.persistence, sub.client_daos = sub, mod
    monkeypatch.setitem(sys.modules, "fedless", pkg)
    monkeypatch.setitem(sys.modules, "fedless.persistence", sub)
    monkeypatch.setitem(sys.modules, "fedless.persistence.client_daos", mod)
    client = object()  # a pymongo.MongoClient stand-in
    fed, stall = _strategies()
    assert [d["client_id"] for d in fed.select_aggregation_candidates(client, "s1", 3)[0]] == ["a", "b"]
    assert [d["client_id"] for d in stall.select_aggregation_candidates(mongo_client=client, session_id="s1",
                                                                        round_id=3)[0]] == ["a", "b", "c"]
    assert seen == [client, client]


def test_empty_round_is_not_an_error_but_an_empty_store_query_is_kept():
    """The reference's `if not round_candidates` tests a generator (always
    truthy): an unknown round returns empty dicts, no exception."""
    st = _store()
    dicts, cands = FedAvgAggregator().select_aggregation_candidates(mongo_client=st, session_id="s9", round_id=1)
    assert dicts == [] and list(cands) == []
    assert InsufficientClientResults  # the class stays importable under the reference's name
