"""Pin the oracle: every restatement must reproduce the reference-generated
golden vectors bit for bit (tests/golden/make_golden.py ran the reference)."""
import hashlib
import io

import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth
from oracle import fedavg_oracle as O
from oracle import oracle_lib as OL


def _sha(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def _npz(layers):
    f = io.BytesIO()
    np.savez(f, *layers)
    return f.getvalue()


def _results(params, cards):
    return [{"blob": _npz(p), "string_format": "none", "cardinality": c} for p, c in zip(params, cards)]


LITERAL_CASES = [(c, p) for c, m in G.manifest().items() if not m.get("sampled")
                 for p in m["outputs"] if p in ("fedavg", "_aggregate", "stall")]


def test_synth_inputs_match_recorded_hashes():
    for case, m in G.manifest().items():
        if "X_sha256" in m:
            assert _sha(G.stacked(case)) == m["X_sha256"], case


def test_reference_unit_test_expectation():
    # test/test_aggregation.py:79-99 -- the reference's own golden values
    expected = [np.array([[[3.6666666667, 1.33333333, 5.0], [1.0, -7.0, -2.66666666667]]]),
                np.array([[[0.0, -3.33333333333, 5.0], [3.66666666667, -7.0, -12.666666666667]]])]
    out = O.fedavg_literal(G.parameters("ref_fixture"), G.manifest()["ref_fixture"]["weights"])
    assert all(np.allclose(a, b) for a, b in zip(out, expected))


@pytest.mark.parametrize("case,prefix", LITERAL_CASES)
def test_literal_matches_golden(case, prefix):
    m = G.manifest()[case]
    params = G.parameters(case)
    with np.errstate(all="ignore"):
        if prefix == "stall":
            out = O.stall_aware_literal(G.feats(case), m["current_round"], params, m["weights"])
        else:
            out = O.fedavg_literal(params, m["weights"])
    exp = G.expected(case, prefix)
    assert len(out) == len(exp)
    for a, b in zip(out, exp):
        assert G.same_bits(a, b), (case, prefix)


def test_ref_fixture_aggregate_paths():
    m = G.manifest()["ref_fixture"]
    params = G.parameters("ref_fixture")
    res, _ = O.aggregate_fedavg(_results(params, [1, 2, 0]))
    assert all(G.same_bits(a, b) for a, b in zip(res, G.expected("ref_fixture", "aggregate_intcards")))
    bad = _results(params, [-1, 2, 0])
    with pytest.raises(O.OracleUnknownCardinality):
        O.aggregate_fedavg(bad)
    assert m["infinite_card_raises"] is True
    res, _ = O.aggregate_fedavg(bad, default_cardinality=1.0)
    assert all(G.same_bits(a, b) for a, b in zip(res, G.expected("ref_fixture", "aggregate_default_card")))
    for cs in (1, 2, 10, 50):
        res, _ = O.aggregate_stream_fedavg(_results(params, [1, 2, 0]), chunk_size=cs)
        assert all(G.same_bits(a, b) for a, b in zip(res, G.expected("ref_fixture", f"stream_c{cs}"))), cs


def test_n60_aggregate_and_stream_paths():
    case = "f32_n60"
    m = G.manifest()[case]
    params = G.parameters(case)
    feats = G.feats(case)
    R = m["current_round"]
    checks = {
        "aggregate": O.aggregate_fedavg(_results(params, m["weights"]))[0],
        "aggregate_stall": O.aggregate_stall_aware(_results(params, m["weights"]), feats, R)[0],
        "stream_c25": O.aggregate_stream_fedavg(_results(params, m["weights"]), 25)[0],
        "stream_stall_c25": O.aggregate_stream_stall_aware(_results(params, m["weights"]), feats, R, 25)[0],
    }
    for prefix, out in checks.items():
        exp = G.expected(case, prefix)
        assert all(G.same_bits(a, b) for a, b in zip(out, exp)), prefix


def test_stall_all_current_equals_fedavg():
    a = G.expected("stall_all_current", "stall")
    b = G.expected("stall_all_current", "fedavg")
    assert all(G.same_bits(x, y) for x, y in zip(a, b))


def test_mnist_c1_sampled():
    case = "mnist_c1"
    m = G.manifest()[case]
    params = G.parameters(case)
    out = O.fedavg_literal(params, m["weights"])
    flat = np.concatenate([o.ravel() for o in out])
    assert _sha(flat) == m["outputs"]["fedavg"]["flat_sha256"]
    out = O.stall_aware_literal(G.feats(case), m["current_round"], params, m["weights"])
    flat = np.concatenate([o.ravel() for o in out])
    assert _sha(flat) == m["outputs"]["stall"]["flat_sha256"]
    assert np.array_equal(flat[::97], G.arrays()[f"{case}/stall/sample"])


STACKED = [c for c, m in G.manifest().items() if m["kind"] == "synth_stacked"]


@pytest.mark.parametrize("case", STACKED)
def test_stacked_numpy_and_c_oracle_match_golden(case):
    m = G.manifest()[case]
    X = G.stacked(case)
    w = m["weights"]
    scores = O.score_clients(G.feats(case), m["current_round"])
    exp_f = G.expected(case, "fedavg")[0]
    exp_s = G.expected(case, "stall")[0]
    assert G.same_bits(O.fedavg_stacked(X, w), exp_f)
    assert G.same_bits(O.fedavg_stacked(X, w, scores), exp_s)
    a = np.array(w, dtype=np.float32)
    s = np.array(scores, dtype=np.float32)
    div = np.float32(sum(w))
    assert G.same_bits(OL.fedavg_f32(X, a, div), exp_f)
    assert G.same_bits(OL.fedavg_f32(X, a, div, s=s), exp_s)


def test_c_oracle_f64_matches_golden():
    case = "f64_n40"
    m = G.manifest()[case]
    X = np.stack([p[0] for p in G.parameters(case)])
    scores = O.score_clients(G.feats(case), m["current_round"])
    a = np.array(m["weights"], dtype=np.float64)
    assert G.same_bits(OL.fedavg_f64(X, a, float(sum(m["weights"]))), G.expected(case, "fedavg")[0])
    assert G.same_bits(OL.fedavg_f64(X, a, float(sum(m["weights"])), s=np.array(scores)),
                       G.expected(case, "stall")[0])


def test_c_oracle_specials_and_float_weights():
    for case in ("specials", "float_weights", "zero_total", "n1"):
        m = G.manifest()[case]
        X = np.stack([p[0] for p in G.parameters(case)])
        a = np.array([np.float32(w) for w in m["weights"]], dtype=np.float32)
        with np.errstate(all="ignore"):
            out = OL.fedavg_f32(X, a, np.float32(sum(m["weights"])))
        assert G.same_bits(out, G.expected(case, "fedavg")[0]), case


def test_bf16_definition_is_f32_upcast():
    # bf16 has no reference path: it is defined as exact upcast + f32 algorithm.
    Xb = synth.clients_bf16(4, 33, 0, 500)
    w = synth.cardinalities(4, 33)
    out, outb = OL.fedavg_bf16(Xb, np.array(w, np.float32), np.float32(sum(w)))
    ref = O.fedavg_stacked(synth.bf16_bits_to_f32(Xb), w)
    assert G.same_bits(out, ref)
    assert np.array_equal(outb, synth.f32_to_bf16_bits(ref))
    o2, b2 = O.fedavg_stacked_bf16(Xb, w)
    assert G.same_bits(o2, ref) and np.array_equal(b2, outb)


def test_c_synth_matches_numpy_synth():
    a = synth.clients_f32(99, 4, 12345, 777, row0=10)
    b = OL.synth_f32(99, 4, 777, row0=10, col0=12345)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    assert np.array_equal(synth.clients_bf16(99, 4, 5, 300), OL.synth_bf16(99, 4, 300, col0=5))


def test_weighted_metrics():
    ms = [{"cardinality": 10, "metrics": {"loss": 1.0, "accuracy": 0.5}},
          {"cardinality": 30, "metrics": {"loss": 3.0, "accuracy": 0.9}}]
    r = O.weighted_metrics(ms, ["loss", "accuracy"])
    assert r["mean_loss"] == pytest.approx(2.5)
    assert r["median_accuracy"] == pytest.approx(0.7)
