"""Eval forward of the 6x128 net at one batch with the residual convs forced to
per-layer launches (key 5 = 0) or the persistent tower (key 5 = 1): the probe the
PMC passes for the self-play roofline's traffic run on (the self-play forwards are
dominated by per-layer conv3x3_halo<128,64,4,1,8> launches at B ~ 4096).

    python scripts/conv_probe.py --batch 4096 --tower 0 --steps 3
"""
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
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--tower", type=int, default=0)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--shape", type=int, default=-1, help="force the per-layer tile shape (key 0)")
    args = ap.parse_args()
    import _native
    lib = _native.load_library()
    lib.azg_pv_set_tuning(5, args.tower)
    lib.azg_pv_set_tuning(0, args.shape)
    from network import PyTorchModel
    from synth import synth_encoded
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=6, channels=128)
    m.net.eval()
    B = args.batch
    x = torch.from_numpy(synth_encoded(B, seed=3)).to(dev)
    probs = torch.empty((B, 225), device=dev)
    values = torch.empty((B, 1), device=dev)
    eng = m.engine
    eng.forward_into(x, probs, values)
    torch.cuda.synchronize()
    eng.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.forward_into(x, probs, values)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile_enable(False)
    eng.check_status()
    flop = 2 * 225 * 128 * 9 * 128 * B
    out = {"batch": B, "tower": args.tower, "ms_per_forward": round(dt / args.steps * 1e3, 3)}
    for k, (ms, n) in prof.items():
        out[k] = {"launches": n, "avg_us": round(ms / n * 1e3, 1)}
        if k in ("conv3x3", "tower"):
            per = flop * (12 if k == "tower" else 1)
            out[k]["mfma_frac"] = round(per / (ms / n / 1e3) / 157.3e12, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
