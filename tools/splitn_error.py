#!/usr/bin/env python3
"""Normwise error of the opt-in split-client fold (fa_fedavg_f32_splitn)
against the exact fp64 sum of the same fp32 products, next to the error of the
reference's own left fold (the exact, bit-identical path).

    python tools/splitn_error.py      (GPU box)   -> one JSON line per shape
"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fedlesscan_amd import engine, synth  # noqa: E402

dev = torch.device("cuda", 0)
for N, P in [(100, 16384), (1024, 16384), (1024, 67267), (1024, 582026)]:
    X = synth.clients_f32(77, N, 0, P)
    w = synth.cardinalities(77, N)
    a = np.array(w, np.float32).astype(np.float64)
    exact = (X.astype(np.float64) * a[:, None]).sum(axis=0) / float(np.float32(sum(w)))
    ldx = -(-P // 64) * 64  # 256-B row pitch, as the ingest lays rows out
    Xd = torch.zeros((N, ldx), dtype=torch.float32, device=dev)
    Xd[:, :P] = torch.from_numpy(X).to(dev)
    Xd = Xd[:, :P]
    left = engine.fold_stacked(Xd, w).cpu().numpy()
    split = engine.fold_stacked(Xd, w, exact=False).cpu().numpy()
    den = np.max(np.abs(exact))
    print(json.dumps({"clients": N, "params": P,
                      "left_fold_normwise_vs_fp64": float(np.max(np.abs(left - exact)) / den),
                      "split_normwise_vs_fp64": float(np.max(np.abs(split - exact)) / den),
                      "split_normwise_vs_left_fold": float(np.max(np.abs(split - left)) / den),
                      "split_elements_differing_from_left_fold": float(np.mean(split != left))}), flush=True)
