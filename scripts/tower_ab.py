"""Per-layer conv launches vs the persistent residual tower (one launch), 6x128
eval forward: residual-tower device time per forward (hipEvents) and whole-forward
wall time, per batch size and tower tile shape.

    python scripts/tower_ab.py [--batches 128,512,4096] [--steps 10]
"""
import os as _os

# A/B study variants live only in the study build (make -C alphazero-gomoku_amd/csrc study)
_os.environ.setdefault("AZG_PV_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                   "alphazero-gomoku_amd", "libazg_pv_study.so"))
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="32,128,256,512,1024,4096")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--ablations", default="", help="comma list of tower ablation masks to time too")
    ap.add_argument("--shapes", default="", help="extra tower tile shapes")
    ap.add_argument("--vars", default="", help="tower tile-body variants (C=128, 128x64 tiles): 0..5")
    args = ap.parse_args()
    from network import PyTorchModel
    from synth import synth_encoded
    import _native

    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=args.blocks, channels=args.channels)
    eng = m.engine
    C = args.channels
    for B in map(int, args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=5)).cuda()
        probs = torch.empty((B, 225), device="cuda")
        values = torch.empty((B, 1), device="cuda")
        flop = 2 * 225 * C * 9 * C * B * 2 * args.blocks
        row = {"batch": B}
        variants = [("layers", 0, 5, 0, 0), ("tower64", 1, 5, 0, 0), ("tower128", 1, 8, 0, 0),
                    ("tower128_group", 1, 8, 0, 0)]
        variants += [(f"tower128_abl{a}", 1, 8, int(a), 0) for a in args.ablations.split(",") if a]
        variants += [(f"tower_s{t}", 1, int(t), 0, 0) for t in args.shapes.split(",") if t]
        variants += [(f"tower128_v{v}", 1, 8, 0, int(v)) for v in args.vars.split(",") if v]
        for name, mode, shape, abl, var in variants:
            lib.azg_pv_set_tuning(5, mode)
            lib.azg_pv_set_tuning(6, shape)
            lib.azg_pv_set_tuning(8, abl)
            lib.azg_pv_set_tuning(10, var)
            lib.azg_pv_set_tuning(17, 1 if name.endswith("_group") else 0)   # claim an M tile x all N tiles
            for _ in range(2):
                eng.forward_into(x, probs, values)
            best_dev, best_wall = None, None
            for _ in range(3):
                eng.profile_enable(True)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(args.steps):
                    eng.forward_into(x, probs, values)
                torch.cuda.synchronize()
                wall = (time.perf_counter() - t0) / args.steps
                prof = eng.profile_read()
                eng.profile_enable(False)
                dev = sum(prof.get(c, (0.0, 0))[0] for c in ("tower", "tower16", "conv3x3")) / args.steps
                best_dev = dev if best_dev is None else min(best_dev, dev)
                best_wall = wall if best_wall is None else min(best_wall, wall)
            row[name] = {"tower_ms": round(best_dev, 4), "frac": round(flop / (best_dev * 1e-3) / 157.3e12, 4),
                         "fwd_ms": round(best_wall * 1e3, 4), "boards_per_s": round(B / best_wall)}
        print(json.dumps(row), flush=True)
    lib.azg_pv_set_tuning(5, 2)
    lib.azg_pv_set_tuning(6, 8)
    lib.azg_pv_set_tuning(8, 0)
    lib.azg_pv_set_tuning(10, 0)


if __name__ == "__main__":
    main()
