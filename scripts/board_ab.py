"""In-process A/B of the split-fp16 eval towers (device time per forward, best of 4
interleaved rounds; bitwise check against per-layer launches): the 128x64 tile tower
(shape 8), h3_tile (12) and the board-resident towers (13; 14 on 16x16x32 products, its
own arithmetic class: max |d logit| instead of bitwise).

    python scripts/board_ab.py [--blocks 6] [--ch 128] [--batches 256,512,2048,3456]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--ch", type=int, default=128)
    ap.add_argument("--batches", default="256,512,1024,2048,3456,4096")
    ap.add_argument("--shapes", default="8,12,13")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import _native
    import bench
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device="cuda", n_res_blocks=args.blocks, channels=args.ch)
    bench.pretrain(m, m.engine.device)
    eng = m.engine
    shapes = [int(s) for s in args.shapes.split(",")]
    flop = 2 * args.blocks * bench.conv_flop(args.ch)
    lib.azg_pv_set_tuning(19, 1)
    for B in (int(b) for b in args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=B)).cuda()
        lib.azg_pv_set_tuning(5, 0)
        _, _, l0 = eng.forward(x, want_logits=True)
        best = {s: 1e30 for s in shapes}
        lib.azg_pv_set_tuning(5, 1)
        for rnd in range(4):
            for s in shapes:
                lib.azg_pv_set_tuning(6, s)
                eng.forward(x)
                torch.cuda.synchronize()
                eng.profile_enable(True)
                for _ in range(args.reps):
                    eng.forward(x)
                prof = eng.profile_read()
                eng.profile_enable(False)
                ms = sum(v[0] for k, v in prof.items() if k in ("tower", "tower16", "board")) / args.reps
                best[s] = min(best[s], ms)
        for s in shapes:
            lib.azg_pv_set_tuning(6, s)
            _, _, l1 = eng.forward(x, want_logits=True)
            same = bool(torch.equal(l0, l1))
            dmax = float((l0 - l1).abs().max())
            print(f"B={B} shape {s}: tower {best[s]:.3f} ms = {flop * B / best[s] / 1e9:.1f} TFLOP/s "
                  f"({flop * B / best[s] / 1e9 / 838.9 * 100:.1f} % of the split roofline), bitwise {same} "
                  f"max|dlogit| {dmax:.2e}", flush=True)
        lib.azg_pv_set_tuning(5, 2)


if __name__ == "__main__":
    main()
