#!/usr/bin/env python3
"""Drop-in fixtures from the REFERENCE's own objects and code.

Run in the build container only (/root/reference does not exist on the GPU
box), after make_golden.py:

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_dropin.py

It imports the reference under the same App. B shims as make_golden.py (by
importing that module) and writes tests/golden/dropin.json + dropin.npz:

 1. "strategies": the reference's pydantic-v1 ClientResult /
    SerializedParameters / WeightsSerializerConfig / BinaryStringFormat /
    TestMetrics / AggregationHyperParams objects, built the way
    ClientResultDao hands them over (client_daos.py:125-147), fed to
    fedlesscan_amd's strategy classes exactly as INTEGRATION.md section 1
    wires them in (FedAvg, stall-aware, both stream variants, base64 and raw
    blobs, cardinality -1 with and without a default).  The engine fold is
    replaced by the oracle (CPU; checker only).  The script asserts that every
    output and exception equals the reference strategy's own on identical
    objects, then records the reference outputs; tests/test_gpu_dropin.py
    replays the same inputs through the HIP fold.
 2. "handler_swap": the reference's own default_aggregation_handler
    (aggregation.py:45-167) over the in-memory Mongo/GridFS of make_golden.py,
    with its strategy classes replaced by fedlesscan_amd's and the one-line
    ClientResultDao change of INTEGRATION.md section 1: every scenario must
    return, save and delete exactly what the unmodified handler did
    (tests/golden manifest "handler").
 3. "metrics": FLStrategy.aggregate_metrics (fl_strategy.py:24-44) of the
    reference itself on TestMetrics lists (default names, several names, float
    and int values, one client, zero total weight, empty input), recorded with
    exact float64 bits (float.hex) or the exception type.
"""
import io
import json
import os
import sys
from functools import reduce

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import make_golden as MG  # noqa: E402  (applies the App. B shims, imports the reference)
import numpy as np  # noqa: E402
from fedlesscan_amd import synth  # noqa: E402

fa, sa, ex, models, ser = MG.fa, MG.sa, MG.ex, MG.models, MG.ser

OUT = {"strategies": {}, "handler_swap": {}, "metrics": []}
ARR = {}

SHAPES = [(5, 3), (7,), (2, 2, 2)]
SEED, ROWS = 41, 30


def _oracle_fold(monkeypatch_target):
    """Replace the engine's HIP entry points with the oracle (numpy, CPU)."""
    from oracle import fedavg_oracle as O
    import fedlesscan_amd.engine as E

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

    monkeypatch_target.append((E, "aggregate_layers", E.aggregate_layers))
    monkeypatch_target.append((E, "aggregate_decoded", E.aggregate_decoded))
    E.aggregate_layers = fake
    E.aggregate_decoded = fake_decoded


def ref_results(rows, cards, fmts, metrics=None):
    """Reference ClientResult objects, as ClientResultDao yields them."""
    X = synth.clients_f32(SEED, ROWS, 0, sum(int(np.prod(s)) for s in SHAPES))
    cfg = models.WeightsSerializerConfig(type="npz", params=models.NpzWeightsSerializerConfig())
    out = []
    for k, (r, c, f) in enumerate(zip(rows, cards, fmts)):
        blob = ser.NpzWeightsSerializer().serialize(MG.split_layers(X[r], SHAPES))
        fmt = models.BinaryStringFormat.NONE
        if f == "base64":
            blob, fmt = ser.Base64StringConverter.to_str(blob), models.BinaryStringFormat.BASE64
        tm = None
        if metrics is not None and metrics[k] is not None:
            tm = models.TestMetrics(cardinality=metrics[k][0], metrics=metrics[k][1])
        out.append(models.ClientResult(parameters=models.SerializedParameters(blob=blob, serializer=cfg,
                                                                              string_format=fmt),
                                       cardinality=c, test_metrics=tm))
    return out


def _run(obj, results, feats, default_cardinality):
    try:
        params, tms = obj.aggregate(results, feats, default_cardinality)
    except Exception as e:
        return {"raises": type(e).__name__}
    return {"params": [np.asarray(p) for p in params],
            "test_metrics": None if tms is None else [t.dict() for t in tms]}


def _same(a, b):
    if set(a) != set(b):
        return False
    if "raises" in a:
        return a["raises"] == b["raises"]
    if a["test_metrics"] != b["test_metrics"] or len(a["params"]) != len(b["params"]):
        return False
    return all(x.dtype == y.dtype and x.shape == y.shape and
               np.array_equal(x.view(np.uint8), y.view(np.uint8)) for x, y in zip(a["params"], b["params"]))


def case_strategies():
    import fedlesscan_amd.aggregator as A
    cards = synth.cardinalities(SEED, ROWS, 1, 600)
    rounds = synth.round_ids(SEED, ROWS, 10, 2)
    scen = {
        # name: (kind, rows, cards, fmts, R, tolerance, default_cardinality, chunk, metrics)
        "fedavg_raw": ("fedavg", list(range(12)), cards[:12], ["raw"] * 12, None, 0, None, None, None),
        "fedavg_b64_mixed": ("fedavg", list(range(9)), cards[:9], ["base64", "raw"] * 4 + ["base64"], None, 0,
                             None, None, None),
        "fedavg_default_card": ("fedavg", [0, 1, 2, 3], [-1, cards[1], -2, cards[3]], ["raw"] * 4, None, 0, 7.0,
                                None, None),
        "fedavg_unknown_card": ("fedavg", [0, 1, 2], [cards[0], -1, cards[2]], ["raw"] * 3, None, 0, None, None,
                                None),
        "fedavg_metrics": ("fedavg", [3, 4, 5, 6], cards[3:7], ["raw"] * 4, None, 0, None, None,
                           [(100, {"loss": 0.5, "accuracy": 0.75}), None, (50, {"loss": 1.5, "accuracy": 0.25}),
                            (7, {"loss": 2.0, "accuracy": 0.5})]),
        "stall_tol2": ("stall", list(range(20)), cards[:20], ["raw"] * 20, 10, 2, None, None, None),
        "stall_b64_default": ("stall", list(range(6)), [cards[0], -1] + cards[2:6], ["base64"] * 6, 10, 2, 3.0,
                              None, None),
        "stream_fedavg_c4": ("stream_fedavg", list(range(13)), cards[:13], ["raw"] * 13, None, 0, None, 4, None),
        "stream_stall_c5": ("stream_stall", list(range(17)), cards[:17], ["base64", "raw"] * 8 + ["raw"], 10, 2,
                            None, 5, None),
    }
    for name, (kind, rows, cs, fmts, R, tol, dflt, chunk, mets) in scen.items():
        feats = [{"round_id": rounds[r]} for r in rows]
        hp_ref = models.AggregationHyperParams(tolerance=tol)
        if kind == "fedavg":
            ref, mine = fa.FedAvgAggregator(), A.FedAvgAggregator()
        elif kind == "stall":
            ref, mine = sa.StallAwareAggregator(R, hp_ref), A.StallAwareAggregator(R, hp_ref)
        elif kind == "stream_fedavg":
            ref, mine = fa.StreamFedAvgAggregator(chunk_size=chunk), A.StreamFedAvgAggregator(chunk_size=chunk)
        else:
            ref = sa.StreamStallAwareAggregator(R, hp_ref, chunk_size=chunk)
            mine = A.StreamStallAwareAggregator(R, hp_ref, chunk_size=chunk)
        with np.errstate(all="ignore"):
            got_ref = _run(ref, ref_results(rows, cs, fmts, mets), feats, dflt)
            restore = []
            _oracle_fold(restore)
            try:
                got_mine = _run(mine, ref_results(rows, cs, fmts, mets), feats, dflt)
            finally:
                for mod, attr, val in restore:
                    setattr(mod, attr, val)
        assert _same(got_ref, got_mine), f"drop-in differs from the reference on its own objects: {name}"
        entry = {"kind": kind, "rows": rows, "cards": cs, "fmts": fmts, "current_round": R, "tolerance": tol,
                 "default_cardinality": dflt, "chunk_size": chunk, "feats": feats,
                 "metrics": None if mets is None else [None if m is None else [m[0], m[1]] for m in mets]}
        if "raises" in got_ref:
            entry["raises"] = got_ref["raises"]
        else:
            entry["test_metrics"] = got_ref["test_metrics"]
            entry["n_layers"] = len(got_ref["params"])
            for i, p in enumerate(got_ref["params"]):
                ARR[f"{name}/{i}"] = p
        OUT["strategies"][name] = entry
    OUT["strategies_meta"] = {"seed": SEED, "rows": ROWS, "shapes": [list(s) for s in SHAPES]}


def case_handler_swap():
    """INTEGRATION.md section 1 applied to the reference's own handler."""
    from unittest import mock
    import fedlesscan_amd.aggregator as A
    agg, cd = MG._import_handler()

    class _Dao:  # aggregation.py:76-78 after the one-line diff: the DAO instead of the client
        @staticmethod
        def wrap(cls):
            class Swapped(cls):
                def select_aggregation_candidates(self, mongo_client, session_id, round_id):
                    return super().select_aggregation_candidates(cd.ClientResultDao(mongo_client), session_id,
                                                                 round_id)
            Swapped.__name__ = cls.__name__
            return Swapped

    swapped = {n: _Dao.wrap(getattr(A, n)) for n in ("FedAvgAggregator", "StallAwareAggregator",
                                                      "StreamFedAvgAggregator", "StreamStallAwareAggregator")}
    manifest = json.load(open(os.path.join(HERE, "manifest.json")))
    hm = manifest["handler"]
    X = synth.clients_f32(hm["seed"], hm["rows"], 0, hm["P"])
    shapes = [tuple(s) for s in hm["shapes"]]
    with np.load(os.path.join(HERE, "cases.npz"), allow_pickle=False) as z:
        expected = {k: z[k] for k in z.files if k.startswith("handler/")}
    ser_cfg = models.WeightsSerializerConfig(type="npz", params=models.NpzWeightsSerializerConfig())
    for name, entry in sorted(hm["scenarios"].items()):
        client = MG._FakeClient()
        restore = []
        _oracle_fold(restore)
        try:
            with mock.patch.object(cd, "GridFS", MG._FakeGridFS), \
                    mock.patch.multiple(agg, **swapped), \
                    mock.patch.object(agg.pymongo, "MongoClient", return_value=client):
                dao = cd.ClientResultDao(client)
                for d in entry["docs"]:
                    sess, rnd, cid, row, card = d[:5]
                    tm = None if len(d) < 6 else models.TestMetrics(cardinality=d[5][0], metrics=d[5][1])
                    blob = ser.NpzWeightsSerializer().serialize(MG.split_layers(X[row], shapes))
                    dao.save(session_id=sess, round_id=rnd, client_id=cid,
                             result=models.ClientResult(parameters=models.SerializedParameters(
                                 blob=blob, serializer=ser_cfg), cardinality=card, test_metrics=tm))
                try:
                    res = agg.default_aggregation_handler(
                        "s", entry["round_id"], models.MongodbConnectionConfig(host="h", port=1, username="u",
                                                                               password="p"),
                        ser_cfg, None, entry["delete"], models.AggregationStrategy(entry["strategy"]),
                        models.AggregationHyperParams(**entry["hyperparams"]))
                except Exception as e:
                    assert entry.get("raises") == type(e).__name__, (name, e)
                    OUT["handler_swap"][name] = {"raises": type(e).__name__, "same_as_reference": True}
                    continue
                assert "raises" not in entry, name
                saved = cd.ParameterDao(client).load(session_id="s", round_id=entry["round_id"] + 1)
        finally:
            for mod, attr, val in restore:
                setattr(mod, attr, val)
        outs = ser.NpzWeightsSerializer().deserialize(saved.blob)
        exp = [expected[f"handler/{name}/{i}"] for i in range(len([k for k in expected
                                                                    if k.startswith(f"handler/{name}/")]))]
        same = (res.new_round_id == entry["new_round_id"] and res.num_clients == entry["num_clients"] and
                (None if res.test_results is None else [t.dict() for t in res.test_results]) ==
                entry["test_results"] and len(outs) == len(exp) and
                all(np.array_equal(o.view(np.uint8), e.view(np.uint8)) for o, e in zip(outs, exp)) and
                sorted([d["session_id"], d["round_id"], d["client_id"]]
                       for d in client["fedless"]["results"].docs) == entry["remaining_results"])
        assert same, f"handler with the drop-in strategies differs from the reference handler: {name}"
        OUT["handler_swap"][name] = {"num_clients": res.num_clients, "new_round_id": res.new_round_id,
                                     "same_as_reference": True}


def case_metrics():
    from fedless.controller.strategies.fl_strategy import FLStrategy
    cases = [
        ("default_names", [(10, {"loss": 0.5}), (30, {"loss": 1.25}), (7, {"loss": 0.1})], None),
        ("two_names", [(100, {"loss": 0.5, "accuracy": 0.9}), (50, {"loss": 1.5, "accuracy": 0.8}),
                       (25, {"loss": 0.3, "accuracy": 0.1}), (1, {"loss": 7.0, "accuracy": 1.0})],
         ["loss", "accuracy"]),
        ("int_values", [(3, {"loss": 2}), (4, {"loss": 5}), (5, {"loss": 11})], None),
        ("one_client", [(17, {"loss": 0.123456789})], ["loss"]),
        ("even_count_median", [(i + 1, {"loss": 0.1 * (i * i % 7)}) for i in range(10)], None),
        ("synthetic_60", [(int(c), {"loss": float(v), "accuracy": float(a)})
                          for c, v, a in zip(synth.cardinalities(5, 60, 1, 600),
                                             np.linspace(0.01, 3.0, 60) ** 1.5,
                                             np.linspace(0.99, 0.1, 60))], ["accuracy", "loss"]),
        ("zero_weights", [(0, {"loss": 1.0}), (0, {"loss": 2.0})], None),
        ("empty", [], None),
        ("missing_name", [(1, {"loss": 1.0})], ["accuracy"]),
    ]
    for name, rows, names in cases:
        tms = [models.TestMetrics(cardinality=c, metrics=m) for c, m in rows]
        entry = {"name": name, "metrics": [[c, m] for c, m in rows], "names": names}
        try:
            with np.errstate(all="raise"):
                res = FLStrategy.aggregate_metrics(None, tms, names)  # `self` is unused (fl_strategy.py:24-44)
        except Exception as e:
            entry["raises"] = type(e).__name__
        else:
            enc = {}
            for k, v in res.items():
                if k.startswith("all_"):
                    enc[k] = {"list": list(v)}
                else:
                    enc[k] = {"type": type(v).__name__, "hex": float(v).hex()}
            entry["result"] = enc
        OUT["metrics"].append(entry)


def main():
    case_strategies()
    case_handler_swap()
    case_metrics()
    buf = io.BytesIO()
    np.savez(buf, **ARR)
    with open(os.path.join(HERE, "dropin.npz"), "wb") as f:
        f.write(buf.getvalue())
    with open(os.path.join(HERE, "dropin.json"), "w") as f:
        json.dump(OUT, f, indent=1, sort_keys=True)
    print(f"strategies {len(OUT['strategies'])}, handler_swap {len(OUT['handler_swap'])}, "
          f"metrics {len(OUT['metrics'])}, arrays {len(ARR)}")


if __name__ == "__main__":
    main()
