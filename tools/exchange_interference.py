#!/usr/bin/env python3
"""How much does a collective's traffic beside the fold slow the fold?  A proxy
for the 8-GPU exchange on a one-GPU box: one rank's step with the default slot
layout (sharding.overlap_layout) on the high-priority fold stream, and after
each round's fold, on a normal-priority stream, a copy kernel on a fixed
number of blocks moving the bytes that rank would receive in that round's
all-gather ((world - 1) x the round's slot).  An RCCL all-gather over xGMI
only WRITES those bytes into local HBM and runs its own kernels on a few CUs;
this copy reads and writes them, so it over-states the HBM side and roughly
matches the CU side.  Prints the fold time per step with and without it.

--copy sdma (round 5) moves each round's received bytes with hipMemcpyAsync
from page-locked host memory instead (fa_copy_h2d on the copy stream): the
copy engines (SDMA), no kernel and no CU -- the cost a kernel-free exchange
(each rank pulling its peers' slots with copy-engine peer copies) would put
on the fold.  --blocks then only says "with copies" (any nonzero entry).

    python tools/exchange_interference.py [--config c3|c4] [--world 8] [--blocks 16,32,64] [--copy kernel|sdma]
"""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import _lib, synth  # noqa: E402
from fedlesscan_amd.engine import Factors  # noqa: E402
from fedlesscan_amd.sharding import fold_stream, overlap_layout, pass_quantum  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="c3", choices=["c3", "c4"])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--blocks", default="16,32,64")
    ap.add_argument("--rounds", type=int, default=4, help="exchange rounds per step (overlap_layout)")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--host-src", action="store_true",
                    help="read the copied bytes from page-locked host memory (long-latency loads over PCIe, closer "
                         "to an all-gather's remote reads over xGMI than an HBM-to-HBM copy)")
    ap.add_argument("--scale", type=float, default=1.0, help="fraction of the received bytes to copy per round")
    ap.add_argument("--fold-free", type=int, default=0,
                    help="leave this many CUs (every (256/k)-th CU id) out of the fold stream's CU mask")
    ap.add_argument("--copy-on-free", action="store_true",
                    help="with --fold-free: the copy stream gets exactly the CUs the fold leaves (the ideal "
                         "placement); otherwise the copy stream has every CU, as RCCL's")
    ap.add_argument("--forms", default="", help="comma-separated fold forms (fa_f32_form_name / fa_bf16_form_name) "
                                              "to force instead of the product's tuned choice")
    ap.add_argument("--forced-rounds", default="all", choices=["all", "overlapped"],
                    help="rounds that run the forced form: all, or only those after round 0 (the rounds an "
                         "exchange overlaps; round 0 keeps the tuned form)")
    ap.add_argument("--step-forms", default="",
                    help="comma-separated step forms (fa_step_form_name; 'product' = fa_fedavg_*_rounds): the whole "
                         "step in ONE launch, each round's copy queued behind fa_*_rounds_wait on the copy stream")
    ap.add_argument("--quantum", default="0",
                    help="round slot widths in whole quanta of columns (SlotLayout quantum): a number, or 'pass' "
                         "(sharding.pass_quantum: one pass of the one-launch step's wide tiles), or 'half'")
    ap.add_argument("--copy", default="kernel", choices=["kernel", "sdma"],
                    help="kernel: fa_bench_copy_f32 on --blocks blocks; sdma: hipMemcpyAsync from page-locked "
                         "host memory on the copy stream (copy engines, no CUs)")
    ap.add_argument("--with-f32", action="store_true",
                    help="bf16: also store the fp32 result (round 5's steps); by default a bf16 step stores only the "
                         "RNE-bf16 copy it exchanges, as ShardedAggregator does (ABI 5)")
    args = ap.parse_args()
    if args.copy == "sdma":
        args.host_src = True
    dev = torch.device("cuda", 0)
    L, B = _lib.load(), _lib.load_bench()
    if args.config == "c3":
        N, P_rank, dt, esz, out_esz = 1024, 10_000_000, "f32", 4, 4
        P_total = P_rank * args.world
    else:
        N, P_total, dt, esz, out_esz = 256, 100_000_000, "bf16", 2, 2
    cus0 = torch.cuda.get_device_properties(dev).multi_processor_count
    q = (pass_quantum(cus0, dt) if args.quantum == "pass" else pass_quantum(cus0, dt) // 2 if args.quantum == "half"
         else int(args.quantum))
    lay = overlap_layout(P_total, args.world, dt, rounds=args.rounds, quantum=q)
    W = lay.local_width
    st0 = torch.cuda.current_stream(dev)
    X = torch.empty((N, W), dtype=torch.float32 if dt == "f32" else torch.bfloat16, device=dev)
    gen = B.fa_synth_f32 if dt == "f32" else B.fa_synth_bf16
    _lib.check(gen(X.data_ptr(), N, W, W, 11, 0, 0, st0.cuda_stream), "synth", bench=True)
    w = synth.cardinalities(11, N)
    a, _ = Factors(w, None, np.dtype(np.float32)).to(dev)
    div = float(np.float32(sum(w)))
    out = torch.empty(W, dtype=torch.float32, device=dev)
    outb = torch.empty(W, dtype=torch.bfloat16, device=dev) if dt == "bf16" else None
    f32_out = dt == "f32" or args.with_f32  # bf16 exchange steps store only the bf16 copy (ABI 5)

    def optr(off=0):
        return out.data_ptr() + off * 4 if f32_out else None
    recv = max(lay.widths) * (args.world - 1) * out_esz // 4 * 4  # floats moved per round, at most
    src = (torch.empty(recv // 4 * 4 + 4, dtype=torch.float32, pin_memory=True) if args.host_src else
           torch.empty(recv // 4 * 4 + 4, dtype=torch.float32, device=dev))
    dst = torch.empty(recv // 4 * 4 + 4, dtype=torch.float32, device=dev)
    import ctypes
    cus = torch.cuda.get_device_properties(dev).multi_processor_count
    handles = []

    def masked_stream(bits):
        words = (cus + 31) // 32
        arr = (ctypes.c_uint32 * words)(*[0] * words)
        for c in bits:
            arr[c // 32] |= 1 << (c % 32)
        h = ctypes.c_void_p()
        _lib.check(B.fa_bench_stream_cu_mask(0, arr, words, ctypes.byref(h)), "cu mask", bench=True)
        handles.append(h)
        return torch.cuda.ExternalStream(h.value, device=dev)

    if args.fold_free:
        step_ = max(1, cus // args.fold_free)
        free = [c for c in range(cus) if c % step_ == step_ - 1][:args.fold_free]
        fs = masked_stream([c for c in range(cus) if c not in free])
        xs = masked_stream(free) if args.copy_on_free else torch.cuda.Stream(device=dev)
    else:
        fs = fold_stream(dev)
        xs = torch.cuda.Stream(device=dev)  # normal priority, like RCCL's stream

    if dt == "f32":
        names = {B.fa_f32_form_name(i).decode(): i for i in range(B.fa_num_f32_forms())}
    else:
        names = {B.fa_bf16_form_name(i).decode(): i for i in range(B.fa_num_bf16_forms())}
    form = [None]

    def copy(k, blocks):
        """Round k's received bytes ((world - 1) x its slot, x --scale) onto the copy stream."""
        n = int(lay.width(k) * (args.world - 1) * out_esz * args.scale) // 16 * 4
        if args.copy == "sdma":
            _lib.check(L.fa_copy_h2d(dst.data_ptr(), src.data_ptr(), n * 4, xs.cuda_stream), "sdma copy")
        else:
            _lib.check(B.fa_bench_copy_f32(dst.data_ptr(), src.data_ptr(), n, blocks, xs.cuda_stream), "copy",
                       bench=True)

    def fold(k):
        off, width = lay.offset(k), lay.width(k)
        x = X.data_ptr() + off * esz
        forced = form[0] is not None and (args.forced_rounds == "all" or k > 0)
        if forced and dt == "f32":
            rc = B.fa_fedavg_f32_form(x, N, width, W, a.data_ptr(), None, div, out.data_ptr() + off * 4,
                                      fs.cuda_stream, form[0])
            _lib.check(rc, "form", bench=True)
            return
        if forced:
            rc = B.fa_fedavg_bf16_form(x, N, width, W, a.data_ptr(), None, div, optr(off),
                                       outb.data_ptr() + off * 2, fs.cuda_stream, form[0])
            _lib.check(rc, "form", bench=True)
            return
        if dt == "f32":
            rc = L.fa_fedavg_f32(x, N, width, W, a.data_ptr(), None, div, out.data_ptr() + off * 4, fs.cuda_stream)
        else:
            rc = L.fa_fedavg_bf16(x, N, width, W, a.data_ptr(), None, div, optr(off),
                                  outb.data_ptr() + off * 2, fs.cuda_stream)
        _lib.check(rc, "fold")

    def step(blocks, ev, end=None):
        for k in range(lay.rounds):
            ev[k][0].record(fs)
            fold(k)
            ev[k][1].record(fs)
            if blocks:
                xs.wait_event(ev[k][1])
                copy(k, blocks)
        fs.wait_stream(xs)
        if end is not None:
            end.record(fs)

    import ctypes as _ct
    offs = (_ct.c_int64 * (lay.rounds + 1))(*[lay.offset(k) for k in range(lay.rounds + 1)])
    step_names = {B.fa_step_form_name(i).decode(): i for i in range(B.fa_num_step_forms())}
    rs_bench = _ct.c_void_p()
    _lib.check(B.fa_bench_rounds_create(_ct.byref(rs_bench), 0), "rounds state", bench=True)
    rs_prod = _ct.c_void_p()
    _lib.check(L.fa_rounds_create(_ct.byref(rs_prod), 0), "rounds state")

    def step_one_launch(sform, blocks, ev, end=None):
        """The whole step in one launch; round k's copy behind a waiter for round k."""
        ev[0][0].record(fs)
        if sform == "product":
            if dt == "f32":
                rc = L.fa_fedavg_f32_rounds(rs_prod, X.data_ptr(), N, W, a.data_ptr(), None, div, out.data_ptr(),
                                            lay.rounds, offs, None, fs.cuda_stream)
            else:
                rc = L.fa_fedavg_bf16_rounds(rs_prod, X.data_ptr(), N, W, a.data_ptr(), None, div, optr(),
                                             outb.data_ptr(), lay.rounds, offs, None, fs.cuda_stream)
            _lib.check(rc, "rounds fold")
        else:
            rc = B.fa_fedavg_rounds_form(rs_bench, step_names[sform], X.data_ptr(), N, W, a.data_ptr(), None, div,
                                         optr(), None if outb is None else outb.data_ptr(), lay.rounds, offs,
                                         fs.cuda_stream)
            _lib.check(rc, "rounds form", bench=True)
        ev[0][1].record(fs)
        if blocks:
            for k in range(lay.rounds):
                if sform == "product":
                    _lib.check(L.fa_rounds_wait(rs_prod, k, xs.cuda_stream), "rounds wait")
                else:
                    _lib.check(B.fa_bench_rounds_wait(rs_bench, k, xs.cuda_stream), "rounds wait", bench=True)
                copy(k, blocks)
        fs.wait_stream(xs)
        if end is not None:
            end.record(fs)

    for _ in range(3):  # the tuner's first calls, warm-up
        step(0, [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                 for _ in range(lay.rounds)])
    torch.cuda.synchronize()
    print(f"{args.config} rank of {args.world}: widths {lay.widths}, fold CUs {cus - args.fold_free}"
          f"{' (copy on the others)' if args.copy_on_free else ''}, copy "
          f"{'hipMemcpyAsync (SDMA)' if args.copy == 'sdma' else 'kernel'} from "
          f"{'host (PCIe)' if args.host_src else 'HBM'}, {args.scale:g} of the received bytes")
    for sform in [f for f in args.step_forms.split(",") if f]:
        for _ in range(3):
            step_one_launch(sform, 0, [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))])
        torch.cuda.synchronize()
        for blocks in [0] + [int(b) for b in args.blocks.split(",") if b]:
            folds, steps = [], []
            for _ in range(args.steps):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))]
                end = torch.cuda.Event(enable_timing=True)
                step_one_launch(sform, blocks, ev, end)
                torch.cuda.synchronize()
                folds.append(ev[0][0].elapsed_time(ev[0][1]))
                steps.append(ev[0][0].elapsed_time(end))
            folds.sort()
            steps.sort()
            print(f"  {'one launch ' + sform:24s} copy blocks {blocks:3d}: fold per step median "
                  f"{folds[len(folds) // 2]:.4f} ms (min {folds[0]:.4f}), step (copies included) median "
                  f"{steps[len(steps) // 2]:.4f} ms", flush=True)
    tmo = L.fa_rounds_timeouts(rs_prod)
    if tmo:
        print(f"  WARNING: {tmo} round waits timed out", flush=True)
    for fname in [f for f in args.forms.split(",") if f] or [None]:
        form[0] = None if fname is None else names[fname]
        for _ in range(2):  # warm the forced form
            step(0, [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                     for _ in range(lay.rounds)])
        torch.cuda.synchronize()
        label = (fname or "tuned") + (" r1+" if fname and args.forced_rounds != "all" else "")
        for blocks in [0] + [int(b) for b in args.blocks.split(",") if b]:
            folds, spans, steps = [], [], []
            for _ in range(args.steps):
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                      for _ in range(lay.rounds)]
                end = torch.cuda.Event(enable_timing=True)
                step(blocks, ev, end)
                torch.cuda.synchronize()
                folds.append(sum(e0.elapsed_time(e1) for e0, e1 in ev))
                spans.append(ev[0][0].elapsed_time(ev[-1][1]))
                steps.append(ev[0][0].elapsed_time(end))
            folds.sort()
            spans.sort()
            steps.sort()
            # fold per step = the rounds' launches summed (gaps between them left out);
            # span = first launch's start to last launch's end on the fold stream, the
            # figure comparable with a one-launch step
            print(f"  {label:24s} copy blocks {blocks:3d}: fold per step median {folds[len(folds) // 2]:.4f} ms "
                  f"(min {folds[0]:.4f}), span median {spans[len(spans) // 2]:.4f} ms, step (copies included) "
                  f"median {steps[len(steps) // 2]:.4f} ms", flush=True)


if __name__ == "__main__":
    main()
