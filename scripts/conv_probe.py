"""Eval forward of the 6x128 (or --blocks x --channels) net at one batch with the
residual convs forced to per-layer launches (key 5 = 0) or the persistent tower
(key 5 = 1, tile shape --tower-shape: 10 = 16-wave 128x128, 8 = 128x64, 5 = 64x64):
the probe the PMC passes for the rooflines' traffic run on.

    python scripts/conv_probe.py --batch 3456 --tower 1 --tower-shape 10 --steps 3
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
    ap.add_argument("--tower-shape", type=int, default=8, help="persistent tower tile shape (key 6)")
    ap.add_argument("--var", type=int, default=0, help="study build: tower tile-body variant (key 10)")
    ap.add_argument("--coh", type=int, default=0, help="study build: round-2 sc1 tower hand-off at 2 WG/CU (key 31)")
    ap.add_argument("--abl", type=int, default=0, help="study build: tower ablation bits (key 8; 4 no weight loads, 8 no halo loads)")
    ap.add_argument("--group", type=int, default=1, help="tower claims (key 17: 0 tile, 1 M tile)")
    ap.add_argument("--board-abl", type=int, default=0, help="board tower timing ablations (key 51; results invalid)")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--check", action="store_true", help="compare the outputs bitwise with the 128x64 tower (shape 8)")
    args = ap.parse_args()
    import _native
    lib = _native.load_library()
    lib.azg_pv_set_tuning(5, args.tower)
    lib.azg_pv_set_tuning(6, args.tower_shape)
    lib.azg_pv_set_tuning(0, args.shape)
    lib.azg_pv_set_tuning(10, args.var)
    lib.azg_pv_set_tuning(31, args.coh)
    lib.azg_pv_set_tuning(8, args.abl)
    lib.azg_pv_set_tuning(17, args.group)
    if args.board_abl:
        lib.azg_pv_set_tuning(51, args.board_abl)
    from network import PyTorchModel
    from synth import synth_encoded
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=args.blocks, channels=args.channels)
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
    ch = args.channels
    flop = 2 * 225 * ch * 9 * ch * B
    out = {"net": f"{args.blocks}x{ch}", "batch": B, "tower": args.tower, "tower_shape": args.tower_shape,
           "ms_per_forward": round(dt / args.steps * 1e3, 3)}
    for k, (ms, n) in prof.items():
        out[k] = {"launches": n, "avg_us": round(ms / n * 1e3, 1)}
        if k in ("conv3x3", "tower", "tower16"):
            per = flop * (2 * args.blocks if k.startswith("tower") else 1)
            out[k]["mfma_frac"] = round(per / (ms / n / 1e3) / 157.3e12, 4)
    if args.check:
        lib.azg_pv_set_tuning(6, 8)
        lib.azg_pv_set_tuning(10, 0)
        p8, v8 = torch.empty_like(probs), torch.empty_like(values)
        eng.forward_into(x, p8, v8)
        torch.cuda.synchronize()
        eng.check_status()
        out["bitwise_vs_shape8"] = bool(torch.equal(p8, probs) and torch.equal(v8, values))
        out["max_abs_diff_vs_shape8"] = float(max((p8 - probs).abs().max(), (v8 - values).abs().max()))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
