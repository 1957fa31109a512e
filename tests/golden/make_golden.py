#!/usr/bin/env python3
"""Generate golden vectors by running the REFERENCE aggregators.

Run in the build container only (``/root/reference`` does not exist on the GPU
box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports ``fedless.aggregator.*`` unmodified from /root/reference under the
four sys.modules shims of SURVEY.md App. B (pydantic v1 API, a MagicMock
tensorflow exposing only tf.data.*_CARDINALITY, h5py mock, pymongo BSONError
alias), feeds in-memory ClientResult objects and writes the outputs -- never
any reference source -- to tests/golden/:

    cases.npz      inputs that are not regenerable + every expected output
    manifest.json  per-case metadata: weights, scores, seeds, shapes, sha256

Inputs of the larger cases come from fedlesscan_amd/synth.py (integer-exact
generator, so the tests regenerate them bit-identically); their sha256 is
recorded so a generator change is caught.
"""
import hashlib
import json
import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
from fedlesscan_amd import synth  # noqa: E402


def _import_reference():
    from unittest import mock
    import pydantic.v1
    import pydantic.v1.fields
    sys.modules["pydantic"] = pydantic.v1
    sys.modules["pydantic.fields"] = pydantic.v1.fields
    tf = mock.MagicMock(name="tensorflow")
    tf.data.UNKNOWN_CARDINALITY = -2
    tf.data.INFINITE_CARDINALITY = -1
    sys.modules["tensorflow"] = tf
    sys.modules["h5py"] = mock.MagicMock(name="h5py")
    import pymongo.errors
    import bson.errors
    pymongo.errors.BSONError = bson.errors.BSONError
    sys.path.insert(0, "/root/reference")
    import fedless.aggregator.fed_avg_aggregator as fa
    import fedless.aggregator.stall_aware_aggregation as sa
    import fedless.aggregator.exceptions as ex
    import fedless.common.models as models
    import fedless.common.serialization as ser
    return fa, sa, ex, models, ser


fa, sa, ex, models, ser = _import_reference()

ARRAYS = {}
MANIFEST = {}


def sha(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def put(case, name, arr):
    ARRAYS[f"{case}/{name}"] = np.asarray(arr)


def client_results(params_list, cards, base64_every_other=False, metrics=None):
    out = []
    for i, params in enumerate(params_list):
        blob = ser.NpzWeightsSerializer().serialize(params)
        fmt = models.BinaryStringFormat.NONE
        if base64_every_other and i % 2 == 0:
            blob = ser.Base64StringConverter.to_str(blob)
            fmt = models.BinaryStringFormat.BASE64
        tm = None
        if metrics is not None:
            tm = models.TestMetrics(cardinality=metrics[i][0], metrics=metrics[i][1])
        out.append(models.ClientResult(
            parameters=models.SerializedParameters(
                blob=blob,
                serializer=models.WeightsSerializerConfig(
                    type="npz", params=models.NpzWeightsSerializerConfig()),
                string_format=fmt),
            cardinality=cards[i], test_metrics=tm))
    return out


def split_layers(row: np.ndarray, shapes):
    out, off = [], 0
    for shp in shapes:
        n = int(np.prod(shp)) if len(shp) else 1
        out.append(row[off:off + n].reshape(shp).copy())
        off += n
    return out


def record_outputs(case, prefix, outs):
    MANIFEST[case].setdefault("outputs", {})[prefix] = {
        "n_layers": len(outs), "shapes": [list(o.shape) for o in outs],
        "dtypes": [str(o.dtype) for o in outs], "sha256": [sha(o) for o in outs]}
    for li, o in enumerate(outs):
        put(case, f"{prefix}/{li}", o)


# ---------------------------------------------------------------------------
# 1. the reference's own unit-test fixture (test/test_aggregation.py:23-86)
# ---------------------------------------------------------------------------
def case_ref_fixture():
    case = "ref_fixture"
    params = [
        [np.array([[[3.0, 0.0, 5.0], [1.0, -5.0, 2.0]]]), np.array([[[4.0, 0.0, 5.0], [9.0, -5.0, 2.0]]])],
        [np.array([[[4.0, 2.0, 5.0], [1.0, -8.0, -5.0]]]), np.array([[[-2.0, -5.0, 5.0], [1.0, -8.0, -20.0]]])],
        [np.array([[[7.0, 3.0, 9.0], [3.0, -123.0, -4.0]]]), np.array([[[7.0, 3.0, 9.0], [3.0, -123.0, -4.0]]])],
    ]
    cards = [1.0, 2.0, 0.0]
    MANIFEST[case] = {"kind": "literal", "weights": cards, "n_clients": 3,
                      "source": "reference test/test_aggregation.py:23-86 fixture"}
    for i, p in enumerate(params):
        for li, layer in enumerate(p):
            put(case, f"X/{i}/{li}", layer)
    record_outputs(case, "_aggregate", fa.FedAvgAggregator()._aggregate(parameters=params, weights=cards))
    res, _ = fa.FedAvgAggregator().aggregate(client_results(params, [1, 2, 0], True), None)
    record_outputs(case, "aggregate_intcards", res)
    # cardinality -1 without default -> UnknownCardinalityError; with default=1.0 -> recovers
    crs = client_results(params, [1, 2, 0], True)
    crs[0].cardinality = -1
    try:
        fa.FedAvgAggregator().aggregate(crs, None)
        raised = False
    except ex.UnknownCardinalityError:
        raised = True
    MANIFEST[case]["infinite_card_raises"] = raised
    crs = client_results(params, [1, 2, 0], True)
    crs[0].cardinality = -1
    res, _ = fa.FedAvgAggregator().aggregate(crs, None, default_cardinality=1.0)
    record_outputs(case, "aggregate_default_card", res)
    for cs in (1, 2, 10, 50):
        res, _ = fa.StreamFedAvgAggregator(chunk_size=cs).aggregate(client_results(params, [1, 2, 0], True), None)
        record_outputs(case, f"stream_c{cs}", res)


# ---------------------------------------------------------------------------
# 2. small f32, three layers, explicit cardinalities incl. 0
# ---------------------------------------------------------------------------
SHAPES_SMALL = [(3, 5), (17,), (2, 2, 2)]


def case_f32_small():
    case = "f32_small"
    seed, N = 11, 7
    P = sum(int(np.prod(s)) for s in SHAPES_SMALL)
    X = synth.clients_f32(seed, N, 0, P)
    cards = [5, 0, 600, 1, 77, 300, 2]
    rounds = [10, 9, 8, 10, 8, 9, 10]
    R = 10
    params = [split_layers(X[i], SHAPES_SMALL) for i in range(N)]
    feats = [{"round_id": r, "client_id": f"c{i}", "session_id": "s"} for i, r in enumerate(rounds)]
    MANIFEST[case] = {"kind": "synth_layers", "seed": seed, "n_clients": N, "P": P, "shapes": [list(s) for s in SHAPES_SMALL],
                      "weights": cards, "round_ids": rounds, "current_round": R, "X_sha256": sha(X)}
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate(params, cards))
    hp = models.AggregationHyperParams(tolerance=2)
    record_outputs(case, "stall", sa.StallAwareAggregator(R, hp)._aggregate(feats, params, cards))
    MANIFEST[case]["scores_f64"] = sa.StallAwareAggregator(R, hp)._score_clients(feats)


# ---------------------------------------------------------------------------
# 3. stacked f32 cases (single layer), incl. aggregate() and both stream forms
# ---------------------------------------------------------------------------
def case_stacked(case, seed, N, P, R=10, tol=2, streams=False, card_hi=600):
    X = synth.clients_f32(seed, N, 0, P)
    cards = synth.cardinalities(seed, N, 1, card_hi)
    rounds = synth.round_ids(seed, N, R, tol)
    feats = [{"round_id": r, "client_id": f"c{i}", "session_id": "s"} for i, r in enumerate(rounds)]
    params = [[X[i].copy()] for i in range(N)]
    MANIFEST[case] = {"kind": "synth_stacked", "seed": seed, "n_clients": N, "P": P, "weights": cards,
                      "round_ids": rounds, "current_round": R, "tolerance": tol, "X_sha256": sha(X)}
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate(params, cards))
    hp = models.AggregationHyperParams(tolerance=tol)
    record_outputs(case, "stall", sa.StallAwareAggregator(R, hp)._aggregate(feats, params, cards))
    if streams:
        res, _ = fa.FedAvgAggregator().aggregate(client_results(params, cards), feats)
        record_outputs(case, "aggregate", res)
        res, _ = sa.StallAwareAggregator(R, hp).aggregate(client_results(params, cards), feats)
        record_outputs(case, "aggregate_stall", res)
        res, _ = fa.StreamFedAvgAggregator(chunk_size=25).aggregate(client_results(params, cards), feats)
        record_outputs(case, "stream_c25", res)
        res, _ = sa.StreamStallAwareAggregator(R, hp, chunk_size=25).aggregate(client_results(params, cards), feats)
        record_outputs(case, "stream_stall_c25", res)


# ---------------------------------------------------------------------------
# 4. config 1: 10 clients x MNIST CNN, n_i = 6000
# ---------------------------------------------------------------------------
MNIST_SHAPES = [(5, 5, 1, 32), (32,), (5, 5, 32, 64), (64,), (1024, 512), (512,), (512, 10), (10,)]


def case_mnist_c1():
    case = "mnist_c1"
    seed, N = 1, 10
    P = sum(int(np.prod(s)) for s in MNIST_SHAPES)
    X = synth.clients_f32(seed, N, 0, P)
    cards = [6000] * N
    params = [split_layers(X[i], MNIST_SHAPES) for i in range(N)]
    R, tol = 10, 2
    rounds = synth.round_ids(seed, N, R, tol)
    feats = [{"round_id": r, "client_id": f"c{i}", "session_id": "s"} for i, r in enumerate(rounds)]
    MANIFEST[case] = {"kind": "synth_layers", "seed": seed, "n_clients": N, "P": P,
                      "shapes": [list(s) for s in MNIST_SHAPES], "weights": cards, "round_ids": rounds,
                      "current_round": R, "X_sha256": sha(X), "sampled": True}
    for prefix, outs in (("fedavg", fa.FedAvgAggregator()._aggregate(params, cards)),
                         ("stall", sa.StallAwareAggregator(R, models.AggregationHyperParams(tolerance=tol))
                          ._aggregate(feats, params, cards))):
        flat = np.concatenate([o.ravel() for o in outs])
        MANIFEST[case].setdefault("outputs", {})[prefix] = {
            "n_layers": len(outs), "shapes": [list(o.shape) for o in outs],
            "dtypes": [str(o.dtype) for o in outs], "sha256": [sha(o) for o in outs],
            "flat_sha256": sha(flat), "sample_stride": 97}
        put(case, f"{prefix}/sample", flat[::97])


# ---------------------------------------------------------------------------
# 5. edge cases
# ---------------------------------------------------------------------------
def case_edges():
    # zero total cardinality -> NaN (0/0)
    case = "zero_total"
    X = synth.clients_f32(21, 3, 0, 64)
    MANIFEST[case] = {"kind": "literal", "weights": [0, 0, 0], "n_clients": 3}
    for i in range(3):
        put(case, f"X/{i}/0", X[i])
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[X[i]] for i in range(3)], [0, 0, 0]))

    # float (non-integer) weights: a_i = fl32(w), divisor = fl32(python float sum)
    case = "float_weights"
    X = synth.clients_f32(22, 5, 0, 257)
    w = [2.5, 1, 3, 0.1, 7.25]
    MANIFEST[case] = {"kind": "literal", "weights": w, "n_clients": 5}
    for i in range(5):
        put(case, f"X/{i}/0", X[i])
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[X[i]] for i in range(5)], w))

    # integer arrays -> float64 (true divide)
    case = "int64_inputs"
    rng = np.random.default_rng(23)
    Xi = [rng.integers(-1000, 1000, size=(4, 5)).astype(np.int64) for _ in range(3)]
    MANIFEST[case] = {"kind": "literal", "weights": [1, 2, 3], "n_clients": 3}
    for i in range(3):
        put(case, f"X/{i}/0", Xi[i])
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[x] for x in Xi], [1, 2, 3]))

    case = "int32_inputs"
    Xi = [rng.integers(-1000, 1000, size=(33,)).astype(np.int32) for _ in range(4)]
    MANIFEST[case] = {"kind": "literal", "weights": [7, 1, 0, 5], "n_clients": 4}
    for i in range(4):
        put(case, f"X/{i}/0", Xi[i])
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[x] for x in Xi], [7, 1, 0, 5]))

    # one client
    case = "n1"
    X = synth.clients_f32(24, 1, 0, 1000)
    MANIFEST[case] = {"kind": "literal", "weights": [37], "n_clients": 1}
    put(case, "X/0/0", X[0])
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[X[0]]], [37]))

    # float64 updates, FedAvg + stall-aware
    case = "f64_n40"
    Xf = synth.clients_f32(25, 40, 0, 1000).astype(np.float64) * (1.0 + 1.0 / 3.0)
    cards = synth.cardinalities(25, 40)
    rounds = synth.round_ids(25, 40, 10, 2)
    feats = [{"round_id": r} for r in rounds]
    MANIFEST[case] = {"kind": "literal", "weights": cards, "round_ids": rounds, "current_round": 10, "n_clients": 40}
    for i in range(40):
        put(case, f"X/{i}/0", Xf[i])
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[Xf[i]] for i in range(40)], cards))
    record_outputs(case, "stall", sa.StallAwareAggregator(10, models.AggregationHyperParams(tolerance=2))
                   ._aggregate(feats, [[Xf[i]] for i in range(40)], cards))

    # special values: inf, -inf, nan, -0.0, subnormals, large magnitudes
    case = "specials"
    sp = np.array([0.0, -0.0, np.inf, -np.inf, np.nan, 1e-45, -1e-45, 1.17e-38, 3.4e38, -3.4e38,
                   1.0, -1.0, 1e-40, 5e-39, 65504.0, 0.1], dtype=np.float32)
    Xs = [np.roll(sp, k) for k in range(4)]
    w = [1, 2, 3, 4]
    MANIFEST[case] = {"kind": "literal", "weights": w, "n_clients": 4, "nan_positions_only": True}
    for i in range(4):
        put(case, f"X/{i}/0", Xs[i])
    with np.errstate(all="ignore"):
        record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[x] for x in Xs], w))

    # FedAvg with all s_i == 1 equals stall-aware bit-for-bit (rounds all == R)
    case = "stall_all_current"
    X = synth.clients_f32(26, 9, 0, 300)
    cards = synth.cardinalities(26, 9)
    feats = [{"round_id": 10}] * 9
    MANIFEST[case] = {"kind": "literal", "weights": cards, "round_ids": [10] * 9, "current_round": 10, "n_clients": 9}
    for i in range(9):
        put(case, f"X/{i}/0", X[i])
    record_outputs(case, "stall", sa.StallAwareAggregator(10, models.AggregationHyperParams(tolerance=2))
                   ._aggregate(feats, [[X[i]] for i in range(9)], cards))
    record_outputs(case, "fedavg", fa.FedAvgAggregator()._aggregate([[X[i]] for i in range(9)], cards))


# ---------------------------------------------------------------------------
# 6. the reference's whole default_aggregation_handler (aggregation.py:45-167)
#    over an in-memory stand-in for MongoDB + GridFS: selection order, the
#    `$gte R-tol` filter, counts, delete-after, the saved round R+1 model, and
#    the empty round (the `if not round_candidates` check never fires, because
#    round_candidates is a generator: fed_avg_aggregator.py:51, client_daos.py:125)
# ---------------------------------------------------------------------------
def _match(doc, flt):
    for k, v in (flt or {}).items():
        if isinstance(v, dict):
            if set(v) != {"$gte"}:
                raise NotImplementedError(v)
            if not (k in doc and doc[k] >= v["$gte"]):
                return False
        elif doc.get(k) != v:
            return False
    return True


class _FakeCollection:
    """The pymongo Collection calls client_daos.py makes, in insertion order."""

    def __init__(self):
        self.docs = []

    def find(self, filter=None, **kw):
        return iter([dict(d) for d in self.docs if _match(d, filter)])

    def find_one(self, filter=None, **kw):
        return next(self.find(filter), None)

    def replace_one(self, flt, doc, upsert=False):
        for i, d in enumerate(self.docs):
            if _match(d, flt):
                self.docs[i] = dict(doc)
                return
        if upsert:
            self.docs.append(dict(doc))

    def delete_many(self, filter):
        self.docs = [d for d in self.docs if not _match(d, filter)]

    def count_documents(self, filter):
        return sum(1 for d in self.docs if _match(d, filter))


class _FakeDb(dict):
    def __init__(self):
        super().__init__()
        self.files = {}

    def __missing__(self, name):
        c = self[name] = _FakeCollection()
        return c


class _FakeClient:
    def __init__(self):
        self.dbs = {}

    def __getitem__(self, name):
        return self.dbs.setdefault(name, _FakeDb())

    def close(self):
        pass


class _FakeFile:
    def __init__(self, data):
        self.data = data

    def read(self):
        return self.data

    def close(self):
        pass


class _FakeGridFS:
    def __init__(self, db):
        self.files = db.files

    def put(self, data, **kw):
        fid = f"f{len(self.files)}"
        self.files[fid] = bytes(data)
        return fid

    def find_one(self, q):
        d = self.files.get(q["_id"])
        return None if d is None else _FakeFile(d)

    def delete(self, file_id):
        self.files.pop(file_id, None)


def _import_handler():
    from unittest import mock
    # benchmark_configurator pulls in tf.keras model builders; the handler uses it
    # only for global evaluation (test_data), which these cases leave at None
    sys.modules.setdefault("fedless.datasets.benchmark_configurator", mock.MagicMock(name="benchmark_configurator"))
    import fedless.aggregator.aggregation as agg
    import fedless.common.persistence.client_daos as cd
    return agg, cd


HANDLER_SHAPES = [(4, 6), (6,), (3, 1, 2)]


def case_handler():
    """Scenarios run through the unmodified reference handler.  Manifest entry per
    scenario: the stored documents (session, round, client, synth row, cardinality,
    optional metrics), the handler arguments and everything the handler returned or
    left behind."""
    from unittest import mock
    agg, cd = _import_handler()
    seed, rows = 31, 40
    P = sum(int(np.prod(s)) for s in HANDLER_SHAPES)
    X = synth.clients_f32(seed, rows, 0, P)
    cards = synth.cardinalities(seed, rows, 1, 600)
    docs_round = ([("s", 3, f"c{i}", i, cards[i]) for i in range(6)] +
                  [("s", 2, f"old{i}", 6 + i, cards[6 + i]) for i in range(2)] +
                  [("other", 3, "x0", 8, cards[8])])
    docs_session = ([("s", 7, "stale", 9, cards[9])] +
                    [("s", 8 + (i % 3), f"c{i}", 10 + i, cards[10 + i]) for i in range(7)] +
                    [("other", 10, "x0", 17, cards[17])])
    docs_online = [("s", 10 - (i % 3), f"c{i}", i, cards[i]) for i in range(30)]
    docs_metrics = [("s", 5, f"c{i}", 20 + i, cards[20 + i], (100 + i, {"loss": 0.5 + i, "accuracy": 0.25 * i}))
                    for i in range(3)] + [("s", 5, "c3", 23, cards[23])]
    scenarios = [
        ("per_round", docs_round, 3, "per_round", {}, True),
        ("per_round_keep", docs_round, 3, "per_round", {}, False),
        ("per_session_tol2", docs_session, 10, "per_session", {"tolerance": 2}, True),
        ("per_session_tol0", docs_session, 10, "per_session", {"tolerance": 0}, True),
        ("online_per_round", docs_online, 10, "per_round", {"aggregate_online": True}, True),
        ("online_per_session", docs_online, 10, "per_session", {"tolerance": 2, "aggregate_online": True}, True),
        ("metrics", docs_metrics, 5, "per_round", {}, True),
        ("empty_per_round", docs_round, 4, "per_round", {}, True),
        ("empty_per_session", [], 4, "per_session", {"tolerance": 2}, True),
        ("empty_online", [], 4, "per_round", {"aggregate_online": True}, True),
    ]
    case = "handler"
    MANIFEST[case] = {"kind": "handler", "seed": seed, "rows": rows, "P": P,
                      "shapes": [list(s) for s in HANDLER_SHAPES], "X_sha256": sha(X), "scenarios": {},
                      "source": "reference fedless/aggregator/aggregation.py:45-167 over an in-memory Mongo/GridFS"}
    ser_cfg = models.WeightsSerializerConfig(type="npz", params=models.NpzWeightsSerializerConfig())
    for name, docs, R, strategy, hp_kw, delete in scenarios:
        client = _FakeClient()
        with mock.patch.object(cd, "GridFS", _FakeGridFS):
            dao = cd.ClientResultDao(client)
            for d in docs:
                sess, rnd, cid, row, card = d[:5]
                tm = None if len(d) < 6 else models.TestMetrics(cardinality=d[5][0], metrics=d[5][1])
                blob = ser.NpzWeightsSerializer().serialize(split_layers(X[row], HANDLER_SHAPES))
                cr = models.ClientResult(parameters=models.SerializedParameters(blob=blob, serializer=ser_cfg),
                                         cardinality=card, test_metrics=tm)
                dao.save(session_id=sess, round_id=rnd, client_id=cid, result=cr)
            entry = {"docs": [list(d[:5]) + ([list(d[5])] if len(d) > 5 else []) for d in docs],
                     "round_id": R, "strategy": strategy, "hyperparams": hp_kw, "delete": delete}
            with mock.patch.object(agg.pymongo, "MongoClient", return_value=client):
                try:
                    res = agg.default_aggregation_handler(
                        "s", R, models.MongodbConnectionConfig(host="h", port=1, username="u", password="p"),
                        ser_cfg, None, delete, models.AggregationStrategy(strategy),
                        models.AggregationHyperParams(**hp_kw))
                except Exception as e:  # the reference's own failure, recorded as the expected outcome
                    entry["raises"] = type(e).__name__
                    MANIFEST[case]["scenarios"][name] = entry
                    continue
            saved = cd.ParameterDao(client).load(session_id="s", round_id=R + 1)
        outs = ser.NpzWeightsSerializer().deserialize(saved.blob)
        entry.update({
            "new_round_id": res.new_round_id, "num_clients": res.num_clients,
            "test_results": None if res.test_results is None else [t.dict() for t in res.test_results],
            "global_test_results": res.global_test_results,
            "saved_round_ids": sorted(d["round_id"] for d in client["fedless"]["parameters"].docs),
            "saved_blob_len": len(saved.blob),
            "saved_blob_sha256": hashlib.sha256(saved.blob).hexdigest() if not outs else None,
            "remaining_results": sorted([d["session_id"], d["round_id"], d["client_id"]]
                                        for d in client["fedless"]["results"].docs),
            "remaining_files": len(client["fedless"].files) - 1,  # minus the saved model
        })
        MANIFEST[case]["scenarios"][name] = entry
        record_outputs(case, name, outs)


def main():
    case_handler()
    case_ref_fixture()
    case_f32_small()
    case_stacked("f32_n60", 12, 60, 4096, streams=True)
    case_stacked("f32_n1024", 13, 1024, 512)
    case_stacked("f32_c5_shape", 5, 512, 96, card_hi=2000)
    case_mnist_c1()
    case_edges()
    np.savez_compressed(os.path.join(HERE, "cases.npz"), **ARRAYS)
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(MANIFEST, f, indent=1, sort_keys=True)
    print(f"wrote {len(ARRAYS)} arrays, {len(MANIFEST)} cases")


if __name__ == "__main__":
    main()
