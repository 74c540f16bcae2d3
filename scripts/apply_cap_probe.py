"""How many workgroups of the fused dgrad + BN-backward apply launch (key 45) can wait
for each other at once: one 6x128 train step per batch size with key 46 lifted to the
occupancy bound; a launch whose tiles do not all fit defers the tiles whose waits time
out to the finalizer (pv_halo.h ApX): correct, but the step time shows it.

    python scripts/apply_cap_probe.py [--batches 128,132,...]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="128,132,136,138,140,142,144")
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=6)
    args = ap.parse_args()
    import numpy as np
    import torch
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    C = args.channels
    occ = lib.azg_pv_set_tuning(46, -C)
    print(f"C={C}: occupancy bound {occ} workgroups", flush=True)
    lib.azg_pv_set_tuning(46, 100000)
    for B in (int(b) for b in args.batches.split(",")):
        tiles = ((B * 225 + 127) // 128) * (C // 64)
        torch.manual_seed(0)
        m = PyTorchModel(board_size=15, device="cuda", n_res_blocks=args.blocks, channels=C)
        rng = np.random.default_rng(B)
        x = torch.from_numpy(synth_encoded(B, seed=B)).cuda()
        pi = rng.random((B, 225)).astype(np.float32)
        pi /= pi.sum(1, keepdims=True)
        pi = torch.from_numpy(pi).cuda()
        z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).cuda()
        res = []
        import time
        for mode in (1, 0):   # fused (key 45 = 1, bound lifted) vs separate passes
            lib.azg_pv_set_tuning(45, mode)
            m.train_batch_device(x, pi, z, return_tensor=True)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(5):
                m.train_batch_device(x, pi, z, return_tensor=True)
            torch.cuda.synchronize()
            m.engine.check_status()
            res.append(f"{(time.perf_counter() - t0) / 5 * 1e3:.3f}")
        lib.azg_pv_set_tuning(45, 1)
        print(f"B={B}: {tiles} tiles: ms/step fused {res[0]} separate {res[1]}", flush=True)
        del m
        torch.cuda.empty_cache()
    lib.azg_pv_set_tuning(46, 0)


if __name__ == "__main__":
    main()
