"""Bitwise cross-library check of the train step: run the same seeded train steps
with the policy/value library named by AZG_PV_LIB (or the in-tree product library)
and dump every parameter, gradient, Adam moment, BN buffer and loss; `--compare`
diffs two dumps bit for bit.  Used to show that a schedule change (e.g. the
persistent train backward) leaves the results of the previous round's library
unchanged:

    AZG_PV_LIB=scripts/_ref/libazg_pv_r3.so python scripts/train_lib_compare.py --out a.npz
    python scripts/train_lib_compare.py --out b.npz
    python scripts/train_lib_compare.py --compare a.npz b.npz

Cases: (blocks, channels, batch, steps) = (6, 128, 128, 3) -- configs[3]'s shape --,
(3, 64, 37, 2) ragged, (2, 256, 16, 2); --tune KEY=VALUE sets tuning keys first.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import numpy as np

CASES = [(6, 128, 128, 3), (3, 64, 37, 2), (2, 256, 16, 2)]


def run(out, tune):
    import torch
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    for kv in tune:
        k, v = (int(t) for t in kv.split("="))
        lib.azg_pv_set_tuning(k, v)
    res = {}
    for nb, ch, B, steps in CASES:
        tag = f"{nb}x{ch}_b{B}"
        torch.manual_seed(3)
        m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=nb, channels=ch)
        rng = np.random.default_rng(nb * 1000 + ch + B)
        x = torch.from_numpy(synth_encoded(B, seed=nb + ch)).cuda()
        pi = rng.random((B, 225)).astype(np.float32)
        pi /= pi.sum(1, keepdims=True)
        pi = torch.from_numpy(pi).cuda()
        z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).cuda()
        for s in range(steps):
            losses = m.train_batch_device(x, pi, z, return_tensor=True)
            res[f"{tag}/loss{s}"] = losses.detach().cpu().numpy()
        torch.cuda.synchronize()
        eng = m.engine
        res[f"{tag}/params"] = eng.flat_params.detach().cpu().numpy()
        res[f"{tag}/grads"] = eng.flat_grads.detach().cpu().numpy()
        res[f"{tag}/m"] = m.optimizer.flat_exp_avg.detach().cpu().numpy()
        res[f"{tag}/v"] = m.optimizer.flat_exp_avg_sq.detach().cpu().numpy()
        for k, v in m.net.state_dict().items():
            if "running" in k or "num_batches" in k:
                res[f"{tag}/{k}"] = v.detach().cpu().numpy()
        print(f"{tag}: {steps} steps, last losses {res[f'{tag}/loss{steps - 1}']}", flush=True)
        del m
        torch.cuda.empty_cache()
    np.savez(out, **res)


def compare(a, b):
    A, Bz = np.load(a), np.load(b)
    bad = 0
    for k in sorted(set(A.files) | set(Bz.files)):
        if k not in A.files or k not in Bz.files:
            print(f"MISSING {k}")
            bad += 1
            continue
        x, y = A[k], Bz[k]
        same = x.shape == y.shape and np.array_equal(np.atleast_1d(x).view(np.uint8), np.atleast_1d(y).view(np.uint8))
        if not same:
            d = np.abs(x.astype(np.float64) - y.astype(np.float64)).max() if x.shape == y.shape else -1
            print(f"DIFF {k}: max|d| {d:.3e}, {np.count_nonzero(x != y)} of {x.size}")
            bad += 1
    print(f"{len(A.files)} arrays compared, {bad} differ")
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    ap.add_argument("--compare", nargs=2)
    ap.add_argument("--tune", action="append", default=[])
    args = ap.parse_args()
    if args.compare:
        sys.exit(1 if compare(*args.compare) else 0)
    run(args.out, args.tune)


if __name__ == "__main__":
    main()
