"""In-process A/B of the persistent tower's dependency protocol (key 31): an
L2-invalidating acquire after each wait (0) vs agent-coherent halo / residual loads
(1); 6x128 eval forward at B = 512 / 1024, tower device time per forward (hipEvents
on the tower's stream, azg_pv_profile_*), interleaved rounds.

    python scripts/tower_coh_ab.py [--batches 512,1024] [--rounds 5 --steps 10]
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
    ap.add_argument("--batches", default="512,1024")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    args = ap.parse_args()
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=6, channels=128)
    eng = m.engine
    lib.azg_pv_set_tuning(5, 1)      # tower on
    lib.azg_pv_set_tuning(6, 8)      # 128x64 tiles
    for B in (int(b) for b in args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=B)).cuda()
        res = {0: [], 1: []}
        for r in range(args.rounds):
            for coh in (0, 1):
                lib.azg_pv_set_tuning(31, coh)
                for _ in range(2):
                    eng.forward(x)
                torch.cuda.synchronize()
                s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s.record()
                for _ in range(args.steps):
                    eng.forward(x)
                e.record()
                torch.cuda.synchronize()
                res[coh].append(s.elapsed_time(e) / args.steps)
        flop = 12 * 2 * 225 * 128 * 9 * 128 * B
        for coh, t in res.items():
            t = sorted(t)
            print(json.dumps({"batch": B, "key31": coh, "forward_ms_min": round(t[0], 4),
                              "forward_ms_median": round(t[len(t) // 2], 4),
                              "tower_frac_upper_bound": round(flop / (t[0] * 1e-3) / 157.3e12, 4)}), flush=True)


if __name__ == "__main__":
    main()
