"""The drop-in classes fed pydantic-v1 objects, as the reference hands them over.

INTEGRATION.md section 1 swaps fedlesscan_amd's strategy classes into the
reference's handler, so the results they receive are the reference's
pydantic-v1 models (ClientResult.parse_obj(bson.decode(...)),
client_daos.py:142), its v1 AggregationHyperParams and its own
BinaryStringFormat enum -- not fedlesscan_amd's v2 models.

tests/golden/make_golden_dropin.py fed the REFERENCE's own objects through these
classes (fold from the oracle) in the build container, asserted equality with
the reference strategies, and recorded the inputs and outputs
(tests/golden/dropin.json / dropin.npz).  The GPU box has no reference, so the
objects here come from a v1 model family with the reference's field set
(pydantic.v1, below: the same types, defaults and str enum), and the fold is
the HIP one.  Outputs must equal the recorded reference outputs bit for bit;
test metrics come back as the same v1 objects.
"""
import enum
import json
import os
from typing import Dict, Optional, Union

import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth

pytestmark = pytest.mark.gpu
pydantic_v1 = pytest.importorskip("pydantic.v1")

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "dropin.json")) as f:
    DROPIN = json.load(f)


# --- a pydantic-v1 model family with the reference's field set (models.py:32-193,
#     aggregation_models.py:19-22); test infrastructure only ---------------------
class V1BinaryStringFormat(str, enum.Enum):
    BASE64 = "base64"
    NONE = "none"


class V1NpzWeightsSerializerConfig(pydantic_v1.BaseModel):
    type: str = pydantic_v1.Field("npz", const=True)
    compressed: bool = False


class V1WeightsSerializerConfig(pydantic_v1.BaseModel):
    type: str
    params: V1NpzWeightsSerializerConfig


class V1SerializedParameters(pydantic_v1.BaseModel):
    blob: Union[pydantic_v1.StrictBytes, str]
    serializer: V1WeightsSerializerConfig
    string_format: V1BinaryStringFormat = V1BinaryStringFormat.NONE


class V1TestMetrics(pydantic_v1.BaseModel):
    cardinality: int
    metrics: Dict


class V1ClientResult(pydantic_v1.BaseModel):
    parameters: V1SerializedParameters
    history: Optional[Dict]
    test_metrics: Optional[V1TestMetrics]
    cardinality: int


class V1AggregationHyperParams(pydantic_v1.BaseModel):
    tolerance: int = 0
    aggregate_online: bool = False
    test_batch_size: int = 10


def _v1_results(entry):
    from fedlesscan_amd.common.serialization import Base64StringConverter, NpzWeightsSerializer
    meta = DROPIN["strategies_meta"]
    shapes = [tuple(s) for s in meta["shapes"]]
    X = synth.clients_f32(meta["seed"], meta["rows"], 0, sum(int(np.prod(s)) for s in shapes))
    cfg = V1WeightsSerializerConfig(type="npz", params=V1NpzWeightsSerializerConfig())
    out = []
    mets = entry["metrics"] or [None] * len(entry["rows"])
    for r, c, f, m in zip(entry["rows"], entry["cards"], entry["fmts"], mets):
        blob = NpzWeightsSerializer().serialize(G._split(X[r], shapes))
        fmt = V1BinaryStringFormat.NONE
        if f == "base64":
            blob, fmt = Base64StringConverter.to_str(blob), V1BinaryStringFormat.BASE64
        tm = None if m is None else V1TestMetrics(cardinality=m[0], metrics=m[1])
        out.append(V1ClientResult(parameters=V1SerializedParameters(blob=blob, serializer=cfg, string_format=fmt),
                                  cardinality=c, test_metrics=tm))
    return out


@pytest.mark.parametrize("name", sorted(DROPIN["strategies"]))
def test_dropin_classes_on_v1_objects_match_reference(name):
    import fedlesscan_amd.aggregator as A
    e = DROPIN["strategies"][name]
    hp = V1AggregationHyperParams(tolerance=e["tolerance"])
    kind = e["kind"]
    if kind == "fedavg":
        agg = A.FedAvgAggregator()
    elif kind == "stall":
        agg = A.StallAwareAggregator(e["current_round"], hp)
    elif kind == "stream_fedavg":
        agg = A.StreamFedAvgAggregator(chunk_size=e["chunk_size"])
    else:
        agg = A.StreamStallAwareAggregator(e["current_round"], hp, chunk_size=e["chunk_size"])
    results = _v1_results(e)
    if "raises" in e:
        with pytest.raises(Exception) as ei:
            agg.aggregate(results, e["feats"], e["default_cardinality"])
        assert type(ei.value).__name__ == e["raises"]
        return
    params, tms = agg.aggregate(results, e["feats"], e["default_cardinality"])
    with np.load(os.path.join(HERE, "golden", "dropin.npz"), allow_pickle=False) as z:
        exp = [z[f"{name}/{i}"] for i in range(e["n_layers"])]
    assert len(params) == len(exp)
    for a, b in zip(params, exp):
        assert a.shape == b.shape and a.dtype == b.dtype and G.same_bits(a, b), name
    if e["test_metrics"] is None:
        assert tms is None
    else:
        assert all(isinstance(t, V1TestMetrics) for t in tms)  # passed through untouched
        assert [t.dict() for t in tms] == e["test_metrics"]
    # the reference's `del client_result.parameters` (fed_avg_aggregator.py:69): the blobs are released
    assert all(r.parameters is None for r in results)
