"""Train-step timing probe (configs[3] shape: 6x128, B = 128), product library:

  * pipelined: K back-to-back steps, one sync at the end (the bench's train leg);
  * host enqueue: the same K steps enqueued behind a long GPU spin (torch.cuda._sleep),
    so the host loop never waits on a full queue -- what the host alone costs per step;
  * graph: backward + clip/Adam captured once in a HIP graph and replayed (fixed step
    count inside, timing only) -- the device-bound floor without launch gaps;
  * key 24 = 0 / 1: BN finalize in separate kernels vs fused into the producing conv's
    last workgroup (acquire hand-off); key 25 = 32 / 0: train convs with buffer-
    resource addressing vs 64-bit pointers; key 26 = 8 / 16: 128x64 tiles with 8 waves
    vs 128x128 tiles with 16 waves (one workgroup per CU).

    python scripts/train_r3_probe.py [--steps 30]
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
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--splits", default="", help="comma list of wgrad split counts to time (key 27; 0 = auto)")
    ap.add_argument("--only-splits", action="store_true")
    ap.add_argument("--ab", default="26=8,25=32,24=1;26=8,25=32,24=0;26=8,25=0,24=1;26=16,25=32,24=1",
                    help="';'-separated sets of comma-separated KEY=VALUE tuning keys to time against each other")
    args = ap.parse_args()
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    dev = torch.device("cuda", 0)
    B, K = args.batch, args.steps
    rng = np.random.default_rng(5)
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=args.blocks, channels=args.channels)
    x = torch.from_numpy(synth_encoded(B, seed=5)).to(dev)
    pi = rng.random((B, 225)).astype(np.float32)
    pi /= pi.sum(1, keepdims=True)
    pi = torch.from_numpy(pi).to(dev)
    z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).to(dev)
    eng, opt = m.engine, m.optimizer
    flop = 3 * 2 * 225 * args.channels * 9 * args.channels * 2 * args.blocks * B
    out = {"net": f"{args.blocks}x{args.channels}", "batch": B, "steps": K}

    def step():
        m.train_batch_device(x, pi, z, return_tensor=True)

    for _ in range(5):
        step()
    torch.cuda.synchronize()
    def timed(tag):
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        torch.cuda.synchronize()
        out.setdefault(tag, []).append(round((time.perf_counter() - t0) / K * 1e3, 4))

    if args.splits:
        for rnd in range(2):
            for S in (int(v) for v in args.splits.split(",")):
                lib.azg_pv_set_tuning(27, S)
                timed(f"pipelined_ms_splits_{S}")
        lib.azg_pv_set_tuning(27, 0)
    # A/B of tuning-key sets, interleaved rounds (default: the round-3 train keys)
    for rnd in range(0 if args.only_splits else 2):
        for cfg in args.ab.split(";"):
            kv = [tuple(int(t) for t in item.split("=")) for item in cfg.split(",") if item]
            if any(k == 26 and v == 16 for k, v in kv) and args.channels != 128:
                continue
            prev = [(k, lib.azg_pv_set_tuning(k, v)) for k, v in kv]
            timed("pipelined_ms_" + (cfg.replace("=", "_").replace(",", "__") or "default"))
            for k, v in reversed(prev):
                lib.azg_pv_set_tuning(k, v)
    if hasattr(torch.cuda, "_sleep") and not args.only_splits:
        torch.cuda.synchronize()
        torch.cuda._sleep(int(2.4e9 * 0.5))        # ~0.5 s spin ahead of the queue
        t0 = time.perf_counter()
        for _ in range(K):
            step()
        host = (time.perf_counter() - t0) / K * 1e3
        torch.cuda.synchronize()
        out["host_enqueue_ms_per_step_gpu_blocked"] = round(host, 4)
    # graph replay of backward + apply (fixed step count: timing only)
    losses = torch.empty(3, device=dev)
    opt._ensure_state()
    g = opt.param_groups[0]

    def raw():
        s = torch.cuda.current_stream().cuda_stream
        eng.lib.azg_pv_train_backward(eng.h, x.data_ptr(), pi.data_ptr(), z.data_ptr(), B, losses.data_ptr(), s)
        eng.lib.azg_pv_train_apply(eng.h, opt.flat_exp_avg.data_ptr(), opt.flat_exp_avg_sq.data_ptr(), 7,
                                   float(g["lr"]), 0.9, 0.999, 1e-8, float(g["weight_decay"]), 3.0, None, s)
    try:
        if args.only_splits:
            raise RuntimeError("skipped")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            raw()
        torch.cuda.current_stream().wait_stream(s)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            raw()
        torch.cuda.synchronize()
        for _ in range(3):
            graph.replay()
        torch.cuda.synchronize()
        for _ in range(2):
            t0 = time.perf_counter()
            for _ in range(K):
                graph.replay()
            torch.cuda.synchronize()
            out.setdefault("graph_ms", []).append(round((time.perf_counter() - t0) / K * 1e3, 4))
    except Exception as e:  # noqa: BLE001 -- a probe: report, do not fail the run
        out["graph_error"] = repr(e)[:300]
    best = min(min(v) for k, v in out.items() if k.startswith("pipelined_ms"))
    out["best_pipelined_mfma_frac"] = round(flop / (best * 1e-3) / 157.3e12, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
