"""In-process A/B of train-step tuning variants (6x128, B=128): every variant
trains the SAME model copy from the same state, the results must be bitwise
identical (the keys only change cache policy / scheduling), and the variants are
timed interleaved (rounds x steps) so box drift hits all of them alike.

    python scripts/train_ab.py --variant 18=0 --variant 18=7 [--variant 18=1,12=1] [--rounds 5 --steps 20]
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
    ap.add_argument("--variant", action="append", required=True, help="KEY=VAL[,KEY=VAL...]")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--no-bitwise", action="store_true", help="timing-only variants (study keys): skip the check")
    args = ap.parse_args()
    import _native
    lib = _native.load_library()
    from network import PyTorchModel
    from synth import synth_encoded

    variants = [[tuple(int(t) for t in kv.split("=")) for kv in v.split(",")] for v in args.variant]
    keys = sorted({k for v in variants for k, _ in v})
    defaults = {k: lib.azg_pv_set_tuning(k, -12345) for k in keys}   # read the defaults back
    for k, v in defaults.items():
        lib.azg_pv_set_tuning(k, v)

    def select(v):
        for k in keys:
            lib.azg_pv_set_tuning(k, defaults[k])
        for k, val in v:
            lib.azg_pv_set_tuning(k, val)

    dev = torch.device("cuda", 0)
    B = args.batch
    rng = np.random.default_rng(5)
    x = torch.from_numpy(synth_encoded(B, seed=5)).to(dev)
    pi = rng.random((B, 225)).astype(np.float32)
    pi /= pi.sum(1, keepdims=True)
    pi = torch.from_numpy(pi).to(dev)
    z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).to(dev)
    torch.manual_seed(0)
    model = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=args.blocks, channels=args.channels)
    state = {k: v.clone() for k, v in model.net.state_dict().items()}
    opt = model.optimizer.state_dict()

    # bitwise: two steps from the same state under every variant
    ref = None
    for v in ([] if args.no_bitwise else variants):
        select(v)
        model.net.load_state_dict(state)
        model.optimizer.load_state_dict(opt)
        for _ in range(2):
            model.train_batch_device(x, pi, z, return_tensor=True)
        torch.cuda.synchronize()
        got = torch.cat([t.detach().reshape(-1).float().cpu() for t in model.net.state_dict().values()])
        if ref is None:
            ref = got
        else:
            same = torch.equal(ref, got)
            print(json.dumps({"variant": v, "bitwise_equal_to_first": same}), flush=True)
            if not same:
                sys.exit(3)

    times = {i: [] for i in range(len(variants))}
    for r in range(args.rounds):
        for i, v in enumerate(variants):
            select(v)
            for _ in range(3):
                model.train_batch_device(x, pi, z, return_tensor=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                model.train_batch_device(x, pi, z, return_tensor=True)
            torch.cuda.synchronize()
            times[i].append((time.perf_counter() - t0) / args.steps * 1e3)
    flop = None
    for i, v in enumerate(variants):
        t = np.array(times[i])
        print(json.dumps({"variant": v, "ms_min": round(float(t.min()), 4), "ms_median": round(float(np.median(t)), 4),
                          "ms_all": [round(float(a), 4) for a in t]}), flush=True)


if __name__ == "__main__":
    main()
