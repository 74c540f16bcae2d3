"""Batch sweep of the 3x3 conv (6x128 forward): average conv launch time per batch
size and shape, from the engine's hipEvent instrumentation, to separate the
per-tile rate from launch-granularity (tail) effects.

    python scripts/conv_sweep.py [--batches 256,512,1024] [--shapes 5,8] [--steps 5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="128,256,384,448,512,576,640,768,1024,1536,2048,4096")
    ap.add_argument("--shapes", default="5,8")
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--channels", type=int, default=128)
    args = ap.parse_args()
    from network import PyTorchModel
    from synth import synth_encoded
    import _native

    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=6, channels=args.channels)
    eng = m.engine
    C = args.channels
    res = {}
    for B in map(int, args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=5)).cuda()
        probs = torch.empty((B, 225), device="cuda")
        values = torch.empty((B, 1), device="cuda")
        row = {}
        for s in map(int, args.shapes.split(",")):
            lib.azg_pv_set_tuning(0, s)
            eng.forward_into(x, probs, values)
            best = None
            for _ in range(3):
                eng.profile_enable(True)
                for _ in range(args.steps):
                    eng.forward_into(x, probs, values)
                ms, n = eng.profile_read()["conv3x3"]
                eng.profile_enable(False)
                us = ms / n * 1e3
                best = us if best is None else min(best, us)
            tf = 2 * 225 * C * 9 * C * B / (best * 1e-6) / 1e12
            row[f"s{s}"] = {"us": round(best, 2), "tflops": round(tf, 1), "frac": round(tf / 157.3, 4)}
        res[B] = row
        print(json.dumps({"batch": B, **row}), flush=True)
    lib.azg_pv_set_tuning(0, -1)


if __name__ == "__main__":
    main()
