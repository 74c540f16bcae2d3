"""End-to-end self-play throughput (BASELINE configs[2] shape, scaled down by
flags): G concurrent games x S simulations/move through the native C++ search
(default) or the reference-semantics Python MCTS (--python) + batched HIP forward.  Reports leaf boards/s (NN-evaluated boards
per second), moves/s and the share of wall time inside the forward.

    python scripts/bench_selfplay.py --games 64 --sims 100 --moves 6 [--blocks 6 --channels 128]
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
    ap.add_argument("--games", type=int, default=64)
    ap.add_argument("--sims", type=int, default=100)
    ap.add_argument("--moves", type=int, default=6, help="moves per game (max_moves)")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--python", action="store_true", help="Python search instead of the native one")
    args = ap.parse_args()
    from games.gomoku import Gomoku
    from network import PyTorchModel
    import selfplay

    torch.manual_seed(0)
    np.random.seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=args.blocks, channels=args.channels)
    m.predict(np.zeros((8, 3, 15, 15), np.float32))
    t0 = time.perf_counter()
    ex, winners, drv = selfplay.selfplay_games(m, Gomoku, args.games, args.sims, 1.0, lambda n: 1.0, 0.05, 0.15, 10,
                                               max_moves=args.moves, native=not args.python)
    dt = time.perf_counter() - t0
    moves = len(ex) // 8
    print(json.dumps({"games": args.games, "sims": args.sims, "net": f"{args.blocks}x{args.channels}",
                      "leaf_boards": drv.boards, "forwards": drv.forwards, "max_batch": drv.max_batch,
                      "seconds": round(dt, 2), "boards_per_s": round(drv.boards / dt, 1),
                      "moves_per_s": round(moves / dt, 2), "nn_share": round(drv.nn_seconds / dt, 3),
                      "mean_batch": round(drv.boards / max(drv.forwards, 1), 1),
                      "search": "python" if args.python else "native",
                      "search_share": round(getattr(drv, "search_seconds", 0.0) / dt, 3)}))


if __name__ == "__main__":
    main()
