"""Train-step throughput: PyTorchModel.train_batch_device on a resident batch
(6x128, B=128 per GPU = the reference's batch_size, train.py:849-889), with a
per-kernel-class breakdown from the engine's hipEvent instrumentation, and the
oracle (reference train_batch on CPU) timed beside it for a few steps.

    python scripts/bench_train.py [--steps 20] [--batch 128] [--blocks 6 --channels 128]
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
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--cpu-steps", type=int, default=3)
    ap.add_argument("--tune", action="append", default=[], help="KEY=VALUE tuning key (include/azg_pv.h)")
    args = ap.parse_args()
    import _native
    lib = _native.load_library()
    for kv in args.tune:
        k, v = (int(t) for t in kv.split("="))
        lib.azg_pv_set_tuning(k, v)
    from network import PyTorchModel
    from synth import synth_encoded

    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=args.blocks, channels=args.channels)
    B = args.batch
    rng = np.random.default_rng(0)
    x = torch.from_numpy(synth_encoded(B, seed=11)).cuda()
    pi = rng.random((B, 225)).astype(np.float32)
    pi /= pi.sum(1, keepdims=True)
    pi = torch.from_numpy(pi).cuda()
    z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).cuda()
    for _ in range(args.warmup):
        m.train_batch_device(x, pi, z)
    torch.cuda.synchronize()
    eng = m.engine
    # reference semantics: losses returned as floats (one host sync per step)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.train_batch_device(x, pi, z)
    torch.cuda.synchronize()
    dt_sync = time.perf_counter() - t0
    # pipelined: losses stay on the device
    # pipelined, no instrumentation: host enqueue time vs device time
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.train_batch_device(x, pi, z, return_tensor=True)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt_pipe = time.perf_counter() - t0
    eng.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        m.train_batch_device(x, pi, z, return_tensor=True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile_enable(False)
    fwd_flop = 2 * 225 * args.channels * 9 * args.channels * (2 * args.blocks)   # tower convs per sample
    out = {"net": f"{args.blocks}x{args.channels}", "batch": B, "steps": args.steps, "tune": args.tune,
           "ms_per_step_profiled": round(dt / args.steps * 1e3, 3), "samples_per_s": round(B * args.steps / dt, 1),
           "ms_per_step_sync": round(dt_sync / args.steps * 1e3, 3),
           "ms_per_step_pipelined": round(dt_pipe / args.steps * 1e3, 3),
           "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 3),
           "tower_tflops_fwd_bwd": round(3 * fwd_flop * B * args.steps / dt / 1e12, 2),
           "kernel_ms_per_step": {k: round(v[0] / args.steps, 3) for k, v in prof.items()},
           "launches_per_step": {k: v[1] // args.steps for k, v in prof.items()}}
    if args.cpu_steps:
        from oracle.ref_net import RefModel
        torch.set_num_threads(max(1, min(16, os.cpu_count() or 1)))
        ref = RefModel(args.blocks, args.channels)
        xs, ps, zs = x.cpu().numpy(), pi.cpu().numpy(), z.cpu().numpy()
        ref.train_batch(xs, ps, zs)
        t0 = time.perf_counter()
        for _ in range(args.cpu_steps):
            ref.train_batch(xs, ps, zs)
        cdt = time.perf_counter() - t0
        out["cpu_oracle_samples_per_s"] = round(B * args.cpu_steps / cdt, 1)
        out["cpu_threads"] = torch.get_num_threads()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
