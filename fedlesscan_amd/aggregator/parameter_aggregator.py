"""Strategy plugin API (mirrors fedless/aggregator/parameter_aggregator.py:11-25)."""
import abc
from typing import Iterator, List, Optional, Tuple

from ..common.models import ClientResult, Parameters, TestMetrics


RESULT_QUERIES = ("load_results_for_round", "load_results_for_session")


def result_store(mongo_client):
    """What select_aggregation_candidates reads client results through.

    The reference's strategies take a pymongo.MongoClient and wrap it into
    ClientResultDao(mongo_client) themselves (fed_avg_aggregator.py:44-45,
    stall_aware_aggregation.py:69-70).  Here the argument may be any object
    with the DAO's two query methods -- the reference's ClientResultDao, or
    fedlesscan_amd.store.InMemoryClientResultStore -- and is used as it is.
    Anything else (a raw MongoClient) is wrapped into the reference's own
    ClientResultDao when the caller's environment has it (the reference's
    handler then calls the drop-in unchanged, aggregation.py:76-78); without
    it, TypeError names INTEGRATION.md §1's one-line change."""
    if all(callable(getattr(mongo_client, m, None)) for m in RESULT_QUERIES):
        return mongo_client
    try:
        from fedless.persistence.client_daos import ClientResultDao  # the caller's environment, if any
    except ImportError:
        ClientResultDao = None
    if ClientResultDao is not None:
        return ClientResultDao(mongo_client)
    raise TypeError(
        f"select_aggregation_candidates needs a result store with {' / '.join(RESULT_QUERIES)} "
        f"(fedlesscan_amd.store.InMemoryClientResultStore, or the reference's ClientResultDao); got "
        f"{type(mongo_client).__name__}, and fedless.persistence.client_daos is not importable to wrap it: pass "
        "ClientResultDao(mongo_client) instead (INTEGRATION.md §1)")


class ParameterAggregator(abc.ABC):
    """Select the client results of a round, then aggregate them."""

    @abc.abstractmethod
    def select_aggregation_candidates(self, **kwargs) -> Iterator:
        pass

    @abc.abstractmethod
    def aggregate(self, client_results: Iterator[ClientResult], client_feats: List[dict]
                  ) -> Tuple[Parameters, Optional[List[TestMetrics]]]:
        pass
