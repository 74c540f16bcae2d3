"""Residual-tower time per forward vs batch: the persistent tower (key 5 = 1, shape 8)
against per-layer launches with the 64x64 (shape 5) and 128x64 (shape 8) tiles,
interleaved rounds, hipEvent totals of the 12 residual convs.  Informs the tuner's
preferred variant per batch bucket (pv_capi.hip tower_variant).

    python scripts/tower_vs_layer.py --batches 256,512,768,1024,1280,1536,2048,3072,4096
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
    ap.add_argument("--batches", default="256,512,768,1024,1280,1536,2048,3072,4096")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    import _native
    lib = _native.load_library()
    from network import PyTorchModel
    from synth import synth_encoded
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=6, channels=128)
    m.net.eval()
    eng = m.engine
    variants = {"tower8": ((5, 1), (6, 8), (0, -1)), "layer5": ((5, 0), (0, 5)), "layer8": ((5, 0), (0, 8))}
    for B in (int(b) for b in args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=B)).to(dev)
        probs = torch.empty((B, 225), device=dev)
        values = torch.empty((B, 1), device=dev)
        res = {k: [] for k in variants}
        for _ in range(args.rounds):
            for name, kv in variants.items():
                for k, v in kv:
                    lib.azg_pv_set_tuning(k, v)
                eng.forward_into(x, probs, values)
                eng.profile_enable(True)
                for _ in range(args.steps):
                    eng.forward_into(x, probs, values)
                torch.cuda.synchronize()
                prof = eng.profile_read()
                eng.profile_enable(False)
                ms = sum(prof.get(c, (0.0, 0))[0] for c in ("tower", "tower16", "conv3x3")) / args.steps
                res[name].append(ms)
        flop = 12 * 2 * 225 * 128 * 9 * 128 * B
        print(json.dumps({"batch": B, **{k: {"ms": round(min(v), 4), "frac": round(flop / (min(v) / 1e3) / 157.3e12, 4)}
                                         for k, v in res.items()}}), flush=True)
    lib.azg_pv_set_tuning(5, 2)
    lib.azg_pv_set_tuning(0, -1)


if __name__ == "__main__":
    main()
