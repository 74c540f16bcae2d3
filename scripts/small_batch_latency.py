"""Eval-forward latency at small batches for the two split-fp16 arithmetics (key 19 = 1:
the tuner's pick among per-layer / tile towers / 32x32 board tower; 2: the 16x16x32 board
tower, one board per workgroup, or at B <= key 52 three workgroups per board).  Device time per forward (hipEvent profile, best of 3
rounds of 20) and wall time per synchronous predict.

    python scripts/small_batch_latency.py [--batches 1,4,16,64,256,512]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="1,4,16,64,256,512")
    args = ap.parse_args()
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device="cuda", n_res_blocks=6, channels=128)
    eng = m.engine
    for B in (int(b) for b in args.batches.split(",")):
        xs = synth_encoded(B, seed=B)
        x = torch.from_numpy(xs).cuda()
        row = []
        for cls, split in ((1, 85), (2, 0), (2, 85)):
            lib.azg_pv_set_tuning(19, cls)
            lib.azg_pv_set_tuning(52, split)
            eng.forward(x)
            torch.cuda.synchronize()
            best = 1e30
            for _ in range(3):
                eng.profile_enable(True)
                for _ in range(20):
                    eng.forward(x)
                prof = eng.profile_read()
                eng.profile_enable(False)
                best = min(best, sum(v[0] for v in prof.values()) / 20)
            m.predict(xs)
            t0 = time.perf_counter()
            for _ in range(20):
                m.predict(xs)
            wall = (time.perf_counter() - t0) / 20 * 1e3
            row.append(f"key19={cls}{' split' if cls == 2 and split else ''}: device {best:.3f} ms, "
                       f"predict wall {wall:.3f} ms")
        print(f"B={B}: " + " | ".join(row), flush=True)
    lib.azg_pv_set_tuning(19, 2)
    lib.azg_pv_set_tuning(52, 85)


if __name__ == "__main__":
    main()
