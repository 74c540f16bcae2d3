"""Timing probe (not a product path): the 6x128 B=128 train step (backward + clip/Adam
at a fixed step count) replayed from a captured HIP graph vs launched eagerly.  The
difference bounds what launch overhead and dispatch gaps cost the eager step.

    python scripts/train_graph_probe.py [--steps 50]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--batch", type=int, default=128)
    args = ap.parse_args()
    from network import PyTorchModel
    from synth import synth_encoded
    dev = torch.device("cuda", 0)
    B = args.batch
    rng = np.random.default_rng(5)
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=6, channels=128)
    m.net.train()
    eng = m.engine
    x = torch.from_numpy(synth_encoded(B, seed=5)).to(dev)
    pi = rng.random((B, 225)).astype(np.float32)
    pi /= pi.sum(1, keepdims=True)
    pi = torch.from_numpy(pi).to(dev)
    z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).to(dev)
    losses = torch.empty(3, device=dev)
    opt = m.optimizer
    opt._ensure_state()
    g = opt.param_groups[0]

    def step_raw():
        eng.lib.azg_pv_train_backward(eng.h, x.data_ptr(), pi.data_ptr(), z.data_ptr(), B, losses.data_ptr(),
                                      torch.cuda.current_stream().cuda_stream)
        eng.lib.azg_pv_train_apply(eng.h, opt.flat_exp_avg.data_ptr(), opt.flat_exp_avg_sq.data_ptr(), 5,
                                   float(g["lr"]), 0.9, 0.999, 1e-8, float(g["weight_decay"]), 3.0, None,
                                   torch.cuda.current_stream().cuda_stream)

    for _ in range(5):
        m.train_batch_device(x, pi, z, return_tensor=True)
        step_raw()
    torch.cuda.synchronize()
    res = {}
    for rnd in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            m.train_batch_device(x, pi, z, return_tensor=True)
        torch.cuda.synchronize()
        res.setdefault("eager_product_ms", []).append((time.perf_counter() - t0) / args.steps * 1e3)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step_raw()
        torch.cuda.synchronize()
        res.setdefault("eager_raw_ms", []).append((time.perf_counter() - t0) / args.steps * 1e3)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        step_raw()
    torch.cuda.current_stream().wait_stream(s)
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        step_raw()
    torch.cuda.synchronize()
    for rnd in range(3):
        t0 = time.perf_counter()
        for _ in range(args.steps):
            graph.replay()
        torch.cuda.synchronize()
        res.setdefault("graph_ms", []).append((time.perf_counter() - t0) / args.steps * 1e3)
    print(json.dumps({k: [round(v, 4) for v in vs] for k, vs in res.items()}), flush=True)


if __name__ == "__main__":
    main()
