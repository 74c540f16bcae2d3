"""A/B of per-layer conv tile shapes on the 6x128 eval forward (key 5 = 0: per-layer
launches, key 0: forced shape): outputs must be bitwise identical to the first shape;
conv3x3 hipEvent time per launch and MFMA fraction, interleaved rounds.

    python scripts/conv_shape_ab.py --shapes 8,13 --batches 512,1024,2048,4096
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="8,13")
    ap.add_argument("--batches", default="512,1024,2048,4096")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=6)
    args = ap.parse_args()
    import _native
    lib = _native.load_library()
    lib.azg_pv_set_tuning(5, 0)
    from network import PyTorchModel
    from synth import synth_encoded
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=args.blocks, channels=args.channels)
    m.net.eval()
    eng = m.engine
    # a variant is "SHAPE" or "SHAPE/KEY=VAL" (e.g. 8/21=0: shape 8 without the tail split)
    shapes = args.shapes.split(",")

    def select(v):
        lib.azg_pv_set_tuning(21, 1)
        sh, *kv = v.split("/")
        lib.azg_pv_set_tuning(0, int(sh))
        for item in kv:
            k, val = (int(a) for a in item.split("="))
            lib.azg_pv_set_tuning(k, val)
    C = args.channels
    for B in (int(b) for b in args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=B)).to(dev)
        probs = torch.empty((B, 225), device=dev)
        values = torch.empty((B, 1), device=dev)
        ref = None
        res = {s: [] for s in shapes}
        for s in shapes:   # bitwise check + warm-up
            select(s)
            eng.forward_into(x, probs, values)
            torch.cuda.synchronize()
            out = torch.cat([probs.reshape(-1), values.reshape(-1)]).cpu()
            if ref is None:
                ref = out
            elif not torch.equal(ref, out):
                print(json.dumps({"batch": B, "shape": s, "bitwise_equal": False}), flush=True)
                sys.exit(3)
        for _ in range(args.rounds):
            for s in shapes:
                select(s)
                eng.forward_into(x, probs, values)
                eng.profile_enable(True)
                for _ in range(args.steps):
                    eng.forward_into(x, probs, values)
                torch.cuda.synchronize()
                prof = eng.profile_read()
                eng.profile_enable(False)
                ms, n = prof["conv3x3"]
                res[s].append(ms / n)
        flop = 2 * 225 * C * 9 * C * B
        print(json.dumps({"batch": B, **{f"shape{s}": {"us": round(min(v) * 1e3, 1),
                                                        "frac": round(flop / (min(v) / 1e3) / 157.3e12, 4)}
                                          for s, v in res.items()}}), flush=True)
    lib.azg_pv_set_tuning(0, -1)


if __name__ == "__main__":
    main()
