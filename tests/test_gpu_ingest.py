"""GPU: host-side ingest routes into the fold (fedlesscan_amd/ingest.py).

Rows whose layers sit in page-locked memory are DMA'd straight from the stored
document (fa_copy_h2d); other rows are packed (fa_pack) and copied in runs.
Whatever the route and the mix, the fold must be bit-identical to the batch
fold and to the reference-generated goldens."""
import numpy as np
import pytest

import golden_cases as G
from fedlesscan_amd import synth
from oracle import oracle_lib as OL  # checker

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")


@pytest.fixture(scope="module")
def dev():
    assert torch.cuda.is_available()
    return torch.device("cuda", 0)


def test_host_is_pinned(dev):
    from fedlesscan_amd.pinned import is_pinned, pinned_bytes
    t = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True)
    assert is_pinned(t.data_ptr(), t.numel())
    assert is_pinned(t.data_ptr() + 4096, 1000)
    a = np.zeros(1 << 20, np.uint8)  # pageable
    assert not is_pinned(a.ctypes.data, a.nbytes)
    v = pinned_bytes(12345)
    base = np.frombuffer(v, np.uint8).ctypes.data
    assert is_pinned(base, 12345) and not is_pinned(base, 1 << 30)
    v[:5] = b"hello"
    assert bytes(v[:5]) == b"hello"
    del v  # released with its last view


@pytest.mark.parametrize("chunk_rows", [1, 3, 16])
@pytest.mark.parametrize("pattern", ["all_pinned", "mixed", "none_pinned"])
@pytest.mark.parametrize("scored", [False, True])
def test_direct_and_packed_rows_mix(dev, chunk_rows, pattern, scored):
    from fedlesscan_amd.ingest import StreamingFold
    from fedlesscan_amd.pinned import pinned_bytes
    N, P = 23, 5003
    X = synth.clients_f32(97, N, 0, P)
    w = synth.cardinalities(97, N)
    sc = [(r + 1) / 11 for r in synth.round_ids(97, N, 10, 2)] if scored else None
    rows = []
    for i in range(N):
        pin = pattern == "all_pinned" or (pattern == "mixed" and i % 3 != 1)
        if pin:
            buf = np.frombuffer(pinned_bytes(P * 4), np.float32)
            buf[:] = X[i]
            rows.append(buf)
        else:
            rows.append(X[i].copy())
    before = dict(StreamingFold.stats)
    sf = StreamingFold(P, chunk_rows=chunk_rows, device=dev)
    sf.acc.fill_(float("nan"))
    for i in range(N):
        r = rows[i]
        sf.add([r[:1000].reshape(10, 100), r[1000:3000], r[3000:]], w[i], None if sc is None else sc[i])
    got = sf.finish().cpu().numpy()
    exp = OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w)),
                        s=None if sc is None else np.array(sc, np.float32))
    assert G.same_bits(got, exp)
    n_direct = {"all_pinned": N, "mixed": sum(1 for i in range(N) if i % 3 != 1), "none_pinned": 0}[pattern]
    assert sf.direct_rows == n_direct
    assert StreamingFold.stats["direct_rows"] - before["direct_rows"] == n_direct


def test_direct_off_packs_everything(dev):
    from fedlesscan_amd.ingest import StreamingFold
    from fedlesscan_amd.pinned import pinned_bytes
    N, P = 5, 777
    X = synth.clients_f32(5, N, 0, P)
    w = synth.cardinalities(5, N)
    sf = StreamingFold(P, chunk_rows=2, device=dev, direct=False)
    for i in range(N):
        buf = np.frombuffer(pinned_bytes(P * 4), np.float32)
        buf[:] = X[i]
        sf.add(buf, w[i])
    got = sf.finish().cpu().numpy()
    assert sf.direct_rows == 0
    assert G.same_bits(got, OL.fedavg_f32(X, np.array(w, np.float32), np.float32(sum(w))))


@pytest.mark.parametrize("strategy_name", ["fedlesscan", "fedavg"])
def test_config1_pinned_store_direct_route(dev, strategy_name):
    """BASELINE config 1 through a pinned result store: every client row takes
    the direct DMA route, and the round is bit-exact against the reference's
    golden output."""
    from fedlesscan_amd.ingest import StreamingFold
    from test_host import config1_round
    before = StreamingFold.stats["direct_rows"]
    res, shapes, sha, exp = config1_round(strategy_name, pinned=True)
    assert res.new_round_id == 11 and res.num_clients == 10
    assert [list(s) for s in shapes] == exp["shapes"]
    assert sha == exp["flat_sha256"]
    assert StreamingFold.stats["direct_rows"] - before == 10


def test_pinned_bson_documents_round_trip(dev):
    from fedlesscan_amd import bsondoc as B
    from fedlesscan_amd.pinned import is_pinned, pinned_bytes
    d = {"parameters": {"blob": bytes(range(256)) * 100, "string_format": "none"}, "cardinality": 7}
    v = B.encode_into(d, pinned_bytes)
    assert bytes(v) == B.encode(d)
    cr = B.decode(v, zero_copy=True)
    blob = cr["parameters"]["blob"]
    assert isinstance(blob, memoryview) and bytes(blob) == d["parameters"]["blob"]
    assert is_pinned(np.frombuffer(blob, np.uint8).ctypes.data, len(blob))
