"""Per-item timeline of the persistent train backward (pv_bwd_tower.hip).

    python scripts/bwd_trace.py --run out.bin [--blocks 6 --channels 128 --batch 128]
    python scripts/bwd_trace.py out.bin

--run trains a few steps with AZG_BWD_TRACE=out.bin (the library records, for every
work item of the last launch, {claim, workgroup, start, dependencies met, end} in
wall_clock64 ticks of 10 ns) and writes the file when the workspace is freed; the
analysis prints per item kind the count, mean wait and mean run time, per conv the
span of its A / D / W / R items, and the share of workgroup-time spent running items,
waiting on dependencies and between items.
"""
import argparse
import os
import subprocess
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run(path, blocks, ch, batch, steps):
    code = f"""
import sys, numpy as np, torch
sys.path[:0] = [{REPO!r}, {os.path.join(REPO, 'alphazero-gomoku_amd')!r}]
from network import PyTorchModel
from synth import synth_encoded
torch.manual_seed(0)
m = PyTorchModel(device='cuda', n_res_blocks={blocks}, channels={ch})
B = {batch}
rng = np.random.default_rng(0)
x = torch.from_numpy(synth_encoded(B, seed=11)).cuda()
pi = rng.random((B, 225)).astype(np.float32); pi /= pi.sum(1, keepdims=True)
pi = torch.from_numpy(pi).cuda()
z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).cuda()
for _ in range({steps}):
    m.train_batch_device(x, pi, z, return_tensor=True)
torch.cuda.synchronize()
del m
import gc; gc.collect()
"""
    env = dict(os.environ, AZG_BWD_TRACE=path)
    subprocess.run([sys.executable, "-c", code], check=True, env=env)


def analyze(path):
    raw = np.fromfile(path, dtype=np.uint8)
    C, nconv, M, S = np.frombuffer(raw[:16].tobytes(), dtype=np.int32)
    tr = np.frombuffer(raw[16:].tobytes(), dtype=np.uint64).reshape(-1, 5).astype(np.int64)
    ntt = (M + 127) // 128
    nt = 1 if C < 128 else C // 128
    nA, nD, nW, nR = ntt, ntt * (C // 64), 9 * nt * nt * S, (9 * C * C + 4095) // 4096
    G0, G = nA + nD + nW, nA + nD + nW + nR
    w = tr[:, 0]
    p = np.where(w < G0, 0, (w - G0) // G + 1)
    off = np.where(w < G0, w, (w - G0) - (p - 1) * G)
    kind = np.full(len(w), 3)
    main = p < nconv
    kind[main & (off < nA)] = 0
    kind[main & (off >= nA) & (off < nA + nD)] = 1
    kind[main & (off >= nA + nD) & (off < G0)] = 2
    conv = np.where(kind == 3, np.where(main, p - 1, nconv - 1), p)
    t0, t1, t2 = tr[:, 2], tr[:, 3], tr[:, 4]
    base = t0.min()
    us = lambda t: (t - base) / 100.0   # 100 MHz ticks -> us
    span = (t2.max() - base) / 100.0
    nslot = int(tr[:, 1].max()) + 1
    print(f"C={C} nconv={nconv} M={M} S={S}: {len(w)} items on {nslot} workgroups, launch span {span:.1f} us "
          f"({span / nconv:.1f} per conv)")
    names = "A D W R".split()
    for k in range(4):
        s = kind == k
        print(f"  {names[k]}: {s.sum():5d} items, wait {np.mean(t1[s] - t0[s]) / 100:7.2f} us, "
              f"run {np.mean(t2[s] - t1[s]) / 100:7.2f} us (min {np.min(t2[s] - t1[s]) / 100:.2f}, "
              f"max {np.max(t2[s] - t1[s]) / 100:.2f})")
    run_t = np.sum(t2 - t1) / 100.0
    wait_t = np.sum(t1 - t0) / 100.0
    print(f"  workgroup-time: running {run_t / (span * nslot):.3f}, waiting {wait_t / (span * nslot):.3f}, "
          f"other {1 - (run_t + wait_t) / (span * nslot):.3f}")
    print("  conv: [A start-end] [D start-end] [W start-end] [R start-end] (us from launch start)")
    for c in range(nconv):
        row = []
        for k in range(4):
            s = (conv == c) & (kind == k)
            row.append(f"{names[k]} {us(t1[s].min()):7.1f}-{us(t2[s].max()):7.1f}" if s.any() else f"{names[k]} -")
        print(f"  {c:2d} " + "  ".join(row))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--run", action="store_true")
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--steps", type=int, default=4)
    args = ap.parse_args()
    if args.run:
        run(args.path, args.blocks, args.channels, args.batch, args.steps)
    analyze(args.path)


if __name__ == "__main__":
    main()
