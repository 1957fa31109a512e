"""Single-process multi-GPU drop-in (fedlesscan_amd/multigpu.py) on the MI355X.

The reference calls the strategy in-process once per round (aggregation.py:
71-97); here the same strategy objects take devices=[...] and fold one column
bucket per GPU.  A one-GPU box lists cuda:0 several times: every bucket then
has its own pinned chunks, copy stream and fold on that GPU, and the peer
reassembly runs as a same-device hipMemcpyPeerAsync.  Everything is compared
bit for bit with the reference goldens / the oracle.  Tests that need a
second GPU (a fold on cuda:1 while the current device is 0) skip when only one
is visible.
"""
import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEVSETS = [[0, 0], [0, 0, 0], ["cuda:0"] * 8]


def _npz_results(params, cards):
    from fedlesscan_amd.common.models import (ClientResult, NpzWeightsSerializerConfig, SerializedParameters,
                                              WeightsSerializerConfig)
    from fedlesscan_amd.common.serialization import NpzWeightsSerializer
    return [ClientResult(parameters=SerializedParameters(
        blob=NpzWeightsSerializer().serialize(p),
        serializer=WeightsSerializerConfig(type="npz", params=NpzWeightsSerializerConfig())), cardinality=c)
        for p, c in zip(params, cards)]


@pytest.mark.parametrize("devices", DEVSETS)
def test_drop_in_devices_match_reference_goldens(devices):
    from fedlesscan_amd import (FedAvgAggregator, StallAwareAggregator, StreamFedAvgAggregator,
                                StreamStallAwareAggregator)
    from fedlesscan_amd.common.models import AggregationHyperParams
    case = "f32_n60"
    m = G.manifest()[case]
    params, w, feats, R = G.parameters(case), m["weights"], G.feats(case), m["current_round"]
    hp = AggregationHyperParams(tolerance=2)
    got = {
        "fedavg": FedAvgAggregator(devices=devices)._aggregate(params, w),
        "stall": StallAwareAggregator(R, hp, devices=devices)._aggregate(feats, params, w),
        "aggregate": FedAvgAggregator(devices=devices).aggregate(_npz_results(params, w), feats)[0],
        "aggregate_stall": StallAwareAggregator(R, hp, devices=devices).aggregate(_npz_results(params, w),
                                                                                   feats)[0],
        "stream_c25": StreamFedAvgAggregator(25, devices=devices).aggregate(_npz_results(params, w), feats)[0],
        "stream_stall_c25": StreamStallAwareAggregator(R, hp, 25, devices=devices).aggregate(
            _npz_results(params, w), feats)[0],
    }
    for prefix, out in got.items():
        exp = G.expected(case, prefix)
        assert len(out) == len(exp), prefix
        for a, b in zip(out, exp):
            assert a.shape == b.shape and a.dtype == b.dtype, prefix
            assert G.same_bits(a, b), prefix


@pytest.mark.parametrize("devices", DEVSETS[:2])
def test_drop_in_devices_all_golden_cases(devices):
    """Every literal golden case (odd shapes, 0-d layers, float64 / int layers,
    specials) through FedAvgAggregator(devices=...)._aggregate: the multi-GPU
    path takes the host float32 groups, the rest runs on the first GPU."""
    from fedlesscan_amd import FedAvgAggregator
    for case, m in G.manifest().items():
        if m.get("sampled") or "fedavg" not in m["outputs"]:
            continue
        out = FedAvgAggregator(devices=devices)._aggregate(G.parameters(case), m["weights"])
        exp = G.expected(case, "fedavg")
        assert len(out) == len(exp), case
        assert all(a.shape == b.shape and a.dtype == b.dtype and G.same_bits(a, b)
                   for a, b in zip(out, exp)), case


@pytest.mark.parametrize("P", [1, 63, 64, 1000, 65536 + 7, 1 << 20])
@pytest.mark.parametrize("ndev", [2, 3, 5])
def test_fold_stacked_multi_peer_reassembly(P, ndev):
    from fedlesscan_amd import multigpu
    from oracle import oracle_lib as OL
    N, seed = 33, 17
    Xh = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    parts = multigpu.scatter_columns(Xh, [0] * ndev)
    for scores in (None, sc):
        out = multigpu.fold_stacked_multi(parts, w, scores)
        exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)),
                            s=None if scores is None else np.array(scores, np.float32))
        assert out.shape == (P,)
        assert G.same_bits(out.cpu().numpy(), exp), (P, ndev, scores is None)


def test_multistreaming_fold_small_chunks():
    """Chunks of 1-3 rows per GPU bucket: the carried accumulator across many
    chunks on every GPU, stall-aware, bit-exact."""
    from fedlesscan_amd.multigpu import MultiStreamingFold
    from oracle import fedavg_oracle as O
    N, seed = 23, 4
    shapes = [(3, 5, 7), (11,), (), (1000, 3), (64,)]
    P = sum(int(np.prod(s)) for s in shapes)
    Xh = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(seed, N, 10, 2)]
    for chunk_bytes in (4 * 500, 4 * 3000, 64 << 20):
        sf = MultiStreamingFold(P, [0, 0, 0], chunk_bytes=chunk_bytes)
        for i in range(N):
            row, off = [], 0
            for s in shapes:
                n = int(np.prod(s))
                row.append(Xh[i, off:off + n].reshape(s))
                off += n
            sf.add(row, w[i], sc[i])
        got = sf.finish()
        exp = O.fedavg_stacked(Xh, w, sc)
        assert G.same_bits(got, exp), chunk_bytes


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two visible GPUs")
def test_fold_on_noncurrent_device():
    """Tensors on cuda:1 folded from a thread whose current device is 0: the
    library stages the factors and picks the kernel for the stream's GPU."""
    from fedlesscan_amd import engine
    from oracle import oracle_lib as OL
    N, P, seed = 64, 300_003, 9
    Xh = synth.clients_f32(seed, N, 0, P)
    w = synth.cardinalities(seed, N)
    torch.cuda.set_device(0)
    X1 = torch.from_numpy(Xh).to("cuda:1")
    out = engine.fold_stacked(X1, w)
    assert out.device.index == 1
    exp = OL.fedavg_f32(Xh, np.array(w, np.float32), np.float32(sum(w)))
    assert G.same_bits(out.cpu().numpy(), exp)
    from fedlesscan_amd import multigpu
    parts = multigpu.scatter_columns(Xh, [1, 0])
    assert G.same_bits(multigpu.fold_stacked_multi(parts, w, out_device="cuda:0").cpu().numpy(), exp)
