"""Study: do two board16 forwards on two HIP streams fill each other's tail round?

A board16 launch runs ceil(B / 256) rounds of one board per CU; its last round leaves
256 - B % 256 CUs idle.  Two engines (two handles, own workspaces) evaluate batches of the
same size back to back, either on one stream or on one stream each; the wall time of the
pairs is compared.

    python scripts/lab/two_stream_ab.py [--batches 512,2039,2100,3000] [--reps 20]
"""
import argparse
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="512,2039,2100,2300,3000")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    from network import PyTorchModel
    torch.manual_seed(0)
    ms = [PyTorchModel(board_size=15, device="cuda", n_res_blocks=6, channels=128) for _ in range(2)]
    g = torch.Generator().manual_seed(1)
    for B in (int(b) for b in args.batches.split(",")):
        bufs = []
        for _ in ms:
            boards = torch.randint(0, 3, (B, 225), generator=g, dtype=torch.int8).cuda()
            players = torch.randint(1, 3, (B,), generator=g, dtype=torch.int8).cuda()
            outs = [torch.empty((B, 225), device="cuda"), torch.empty((B, 1), device="cuda"),
                    torch.empty((B, 225), device="cuda")]
            bufs.append((boards, players, outs))
        streams = [torch.cuda.Stream(), torch.cuda.Stream()]

        def run(two):
            for _ in range(args.reps):
                for i, m in enumerate(ms):
                    s = streams[i] if two else streams[0]
                    with torch.cuda.stream(s):
                        b, p, (pr, v, pri) = bufs[i]
                        m.engine.forward_boards_into(b, p, pr, v, pri)
            torch.cuda.synchronize()

        res = {}
        for two in (False, True, False, True):
            run(two)
            t0 = time.perf_counter()
            run(two)
            dt = time.perf_counter() - t0
            res.setdefault(two, []).append(2 * args.reps * B / dt)
        one, two = max(res[False]), max(res[True])
        print(f"B={B}: one stream {one:,.0f} boards/s, two streams {two:,.0f} boards/s ({two / one:.3f}x)",
              flush=True)


if __name__ == "__main__":
    main()
