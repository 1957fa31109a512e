#!/usr/bin/env python3
"""Pointer-list fold (fa_fedavg_f32_ptrs: N separately allocated client rows)
against the stacked fold on the same values.  All times are GPU-event spans
around the Python call, so they include its host work whenever the GPU waits
for it: ptrs_ms = a fresh list of rows per call, rowset_ms = an engine.RowSet
built once, views_ms = X[i] rows of one stacked tensor (equal-stride view).

    python tools/ptrs_bench.py [--clients N] [--params P]   (GPU box) -> one JSON line
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import _lib, engine, synth  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--clients", type=int, default=1024)
ap.add_argument("--params", type=int, default=1_000_000)
ap.add_argument("--reps", type=int, default=20)
ap.add_argument("--variants", action="store_true", help="also time the tuning library's pointer variants")
ap.add_argument("--scored", action="store_true", help="variants: the stall-aware fold (tolerance factors)")
args = ap.parse_args()
dev = torch.device("cuda", 0)
N, P = args.clients, args.params
L = _lib.load()
st = torch.cuda.current_stream(dev).cuda_stream
X = torch.empty((N, P), dtype=torch.float32, device=dev)
_lib.check(_lib.load_bench().fa_synth_f32(X.data_ptr(), N, P, P, 9, 0, 0, st), "synth", bench=True)
rows = [X[i].clone() for i in range(N)]  # separate allocations
# a table of X[i]: rows of one allocation in their natural order (16-B aligned only when P % 4 == 0)
ord_tab = torch.from_numpy(np.array([X[i].data_ptr() for i in range(N)], dtype=np.int64)).to(dev)
# the product entry for tables of X[i] rows: the aligned one only when they are
xrows_fold = L.fa_fedavg_f32_ptrs_aligned if P % 4 == 0 else L.fa_fedavg_f32_ptrs
w = synth.cardinalities(9, N)


def timed(fn):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(args.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    return sorted(ts)[len(ts) // 2]


t_rows = timed(lambda: engine.fold_rows(rows, w))  # a fresh list each call: validation + pointer table
rs = engine.RowSet(rows)  # prepared once, as a caller that keeps its client tensors would
t_rowset = timed(lambda: engine.fold_rows(rs, w))
views = [X[i] for i in range(N)]  # rows of one stacked tensor: the equal-stride view path
t_views = timed(lambda: engine.fold_rows(views, w))
rs_views = engine.RowSet(views)
t_views_rs = timed(lambda: engine.fold_rows(rs_views, w))
# the kernel alone: pointer table and factors built once, as a caller that
# keeps its client tensors would
ptr_tab = torch.from_numpy(np.array([r.data_ptr() for r in rows], dtype=np.int64)).to(dev)
a_dev = torch.tensor([float(np.float32(x)) for x in w], dtype=torch.float32, device=dev)
out = torch.empty(P, dtype=torch.float32, device=dev)
div = float(np.float32(sum(w)))
t_kern = timed(lambda: _lib.check(L.fa_fedavg_f32_ptrs_aligned(ptr_tab.data_ptr(), N, P, a_dev.data_ptr(), None,
                                                               div, out.data_ptr(), st), "ptrs"))
t_stack = timed(lambda: engine.fold_stacked(X, w))
# rows of ONE allocation in a shuffled order: the pointer-table kernel over the
# same memory as the stacked fold (tells the kernel apart from the placement
# of separately allocated rows)
perm = np.random.default_rng(5).permutation(N)
rs_shuf = engine.RowSet([X[int(i)] for i in perm])
w_shuf = [w[int(i)] for i in perm]
assert rs_shuf.view is None
t_shuf = timed(lambda: engine.fold_rows(rs_shuf, w_shuf))
shuf_tab = rs_shuf.ptrs
a_shuf = torch.tensor([float(np.float32(x)) for x in w_shuf], dtype=torch.float32, device=dev)
t_shuf_kern = timed(lambda: _lib.check(xrows_fold(shuf_tab.data_ptr(), N, P, a_shuf.data_ptr(),
                                                                    None, div, out.data_ptr(), st), "ptrs"))
t_ord_kern = timed(lambda: _lib.check(xrows_fold(ord_tab.data_ptr(), N, P, a_dev.data_ptr(),
                                                                  None, div, out.data_ptr(), st), "ptrs"))
# loader / tile variants of the LDS pointer fold (tuning library), kernel alone
var = {}
if args.variants:
    B = _lib.load_bench()
    sc = [(r + 1) / 11 for r in synth.round_ids(9, N, 10, 2)] if args.scored else None
    s_dev = torch.tensor(sc, dtype=torch.float32, device=dev) if sc else None
    s_ptr = s_dev.data_ptr() if sc else None
    ref_v = engine.fold_stacked(X, w, sc).view(torch.int32)
    for v in range(B.fa_num_ptrs_variants()):
        name = B.fa_ptrs_variant_name(v).decode()
        o2 = torch.empty(P, dtype=torch.float32, device=dev)
        fn = lambda: _lib.check(B.fa_fedavg_f32_ptrs_variant(ptr_tab.data_ptr(), N, P, a_dev.data_ptr(), s_ptr, div,
                                                             o2.data_ptr(), st, v), "ptrs variant", bench=True)
        var[name] = round(timed(fn), 4)
        assert torch.equal(o2.view(torch.int32), ref_v), name
        if name.startswith(("ptrs_dw", "ptrs_rows_scalar", "ptrs_generic")):
            # the same rows through a table of X[i] (16-B aligned only when P % 4 == 0)
            fu = lambda: _lib.check(B.fa_fedavg_f32_ptrs_variant(ord_tab.data_ptr(), N, P, a_dev.data_ptr(), s_ptr,
                                                                 div, o2.data_ptr(), st, v), "ptrs variant", bench=True)
            var[name + "@xrows"] = round(timed(fu), 4)
            assert torch.equal(o2.view(torch.int32), ref_v), name
same_shuf = torch.equal(engine.fold_rows(rs_shuf, w_shuf).view(torch.int32),
                        engine.fold_stacked(X[torch.from_numpy(perm).to(dev)], w_shuf).view(torch.int32))
ref = engine.fold_stacked(X, w).view(torch.int32)
same = all(torch.equal(engine.fold_rows(r, w).view(torch.int32), ref) for r in (rows, rs, views, rs_views))
gb = (N * P * 4 + P * 4) / 1e9
print(json.dumps({"clients": N, "params": P, "ptrs_ms": round(t_rows, 4), "ptrs_GBps": round(gb / t_rows * 1e3, 1),
                  "rowset_ms": round(t_rowset, 4), "views_ms": round(t_views, 4),
                  "views_rowset_ms": round(t_views_rs, 4), "shuffled_rowset_ms": round(t_shuf, 4),
                  "shuffled_kernel_ms": round(t_shuf_kern, 4), "inorder_table_kernel_ms": round(t_ord_kern, 4),
                  "ptrs_kernel_ms": round(t_kern, 4), "ptrs_kernel_GBps": round(gb / t_kern * 1e3, 1),
                  "stacked_ms": round(t_stack, 4), "stacked_GBps": round(gb / t_stack * 1e3, 1),
                  "bit_identical": bool(same and same_shuf), "scored_variants": bool(args.scored),
                  **({"variants_kernel_ms": var} if var else {})}))
