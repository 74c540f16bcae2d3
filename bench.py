"""Benchmark: BASELINE.json configs[1] -- batch-512 policy/value forward of the
6-block/128-filter ResNet on synthetic legal 15x15 positions, one MI355X per rank.

    python bench.py [--gpus N] [--steps K] [--warmup W]

N>1 is launched by the driver as torchrun (one process per GPU, RCCL).  Self-play
leaf evaluation shards by game, so every rank runs its own independent batches
(weak scaling, no collective in the timed region).  A step = one forward of 512
boards already resident in HBM.  Prints ONE JSON line on rank 0 with a live
`roofline` for the dominant kernel (the fused 3x3 conv, timed by hipEvents on its
own stream over the timed region) and a bounded `cpu_baseline` (the CPU oracle,
i.e. the reference's PyTorch-CPU algorithm, timed on this host).

After the timed forward loop, a `selfplay` object reports BASELINE configs[2] end to
end on every rank: 256 concurrent games x 400 simulations/move through the native
C++ search (int8 leaves, on-GPU encoding, search of one half of the games overlapped
with the forward of the other), for --sp-moves moves per game; leaf boards summed over
ranks / max wall time over ranks (weak scaling, no collective inside).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
for _p in (REPO, os.path.join(REPO, "alphazero-gomoku_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np
import torch

METRIC = json.load(open(os.path.join(REPO, "BASELINE.json")))["metric"]
BLOCKS, CHANNELS, BATCH = 6, 128, 512
FLOP_CONV = 2 * 225 * CHANNELS * 9 * CHANNELS            # per board per 3x3 res conv = 66,355,200
FLOP_BOARD = 798_221_828                                 # whole forward, SURVEY §8(d)
PEAK_F32_MFMA = 157.3e12                                 # MI355X_MICROARCH.md: FP32 matrix peak


def dist_setup(n_gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return rank, world, local, dist
    return 0, 1, 0, None


def barrier_sync(dist, local):
    if dist is not None:
        dist.barrier(device_ids=[local])
    torch.cuda.synchronize()


def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float = 12.0) -> dict:
    """Oracle (PyTorch-CPU restatement of reference network.py) timed on this host:
    batches of 64 boards, ~2/3 of `seconds` at up to 16 threads (the reported value)
    and ~1/3 single-threaded (1 thread and all cores)."""
    from oracle.boards import encode_batch, synth_positions
    from oracle.ref_net import RefModel

    def timed(threads, budget):
        torch.set_num_threads(threads)
        n = 0
        ref.predict(x)                   # warm-up at this thread count
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget:
            ref.predict(x)
            n += 64
        return n, time.perf_counter() - t0

    threads = max(1, min(16, os.cpu_count() or 1))
    torch.manual_seed(0)
    ref = RefModel(BLOCKS, CHANNELS)
    b, p = synth_positions(64, seed=99)
    x = encode_batch(b, p)
    n, dt = timed(threads, seconds * 2 / 3)
    n1, dt1 = timed(1, seconds / 3)
    return {"value": round(n / dt, 2), "unit": "boards/s", "cores": threads, "kind": "port",
            "sample": f"{n} boards as {n // 64} predict() batches of 64, 6x128, torch-CPU oracle "
                      f"(oracle/ref_net.py = reference network.py:168-183 restated), {dt:.1f}s, "
                      f"{threads} threads",
            "value_1_thread": round(n1 / dt1, 2), "cpu_model": _cpu_model(),
            "host_cpus_visible": os.cpu_count()}


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` ("tower" or "conv3x3") from the committed PMC
    pass (profiles/conv_traffic.json, scripts/summarize_profile.py), or None."""
    path = os.path.join(REPO, "profiles", "conv_traffic.json")
    if not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        if d.get("config") == f"{BLOCKS}x{CHANNELS}_B{BATCH}" and d.get("kernel", "conv3x3") == kernel:
            return d.get("hbm_bytes_per_launch")
    except Exception:
        pass
    return None


def selfplay_leg(model, args, rank, dist, dev, local):
    """BASELINE configs[2]: G games x S sims/move on this rank (native search +
    pipelined board evaluator); returns aggregate leaf boards/s over ranks."""
    from games.gomoku import Gomoku
    from mcts.native_mcts import NativeSelfPlay
    G, S = args.sp_games, args.sp_sims
    sp = NativeSelfPlay(None, Gomoku, G, S, cpuct=1.0, dirichlet_alpha=0.03, epsilon=0.25,
                        apply_dirichlet_n_first_moves=10, evaluator_factory=model.board_evaluator, groups=2)
    warm = NativeSelfPlay(None, Gomoku, 8, 64, evaluator_factory=model.board_evaluator, groups=2)
    warm.play(lambda n: 1.0, max_moves=1, use_symmetries=False, seeds=list(range(8)))
    # conv tile autotuning is cached per batch bucket: visit the buckets the timed
    # run's leaf batches (up to G/2 x 32 boards per group) fall in
    top = (G + 1) // 2 * 32
    z8 = np.zeros((top, 225), np.int8)
    for b in sorted({max(1, top * k // 16) for k in range(4, 17)}):
        model.predict_boards(z8[:b], np.ones(b, np.int8))
    barrier_sync(dist, local)
    t0 = time.perf_counter()
    sp.play(lambda n: 1.0, max_moves=args.sp_moves, use_symmetries=False,
            seeds=[1000 * rank + i for i in range(G)])
    barrier_sync(dist, local)
    dt = time.perf_counter() - t0
    v = torch.tensor([float(sp.boards), dt], dtype=torch.float64, device=dev)
    if dist is not None:
        b = v[:1].clone()
        dist.all_reduce(b)
        m = v[1:].clone()
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        v = torch.cat([b, m])
    boards, dt = float(v[0]), float(v[1])
    return {"config": f"configs[2]: {G} concurrent games/GPU x {S} sims/move, {args.sp_moves} moves/game, "
                      f"native C++ search + batched HIP forward (6x128)",
            "boards_per_s": round(boards / dt, 1), "leaf_boards": int(boards), "seconds": round(dt, 3),
            "moves_per_s": round(G * args.sp_moves * (dist.get_world_size() if dist else 1) / dt, 1),
            "nn_share_rank0": round(sp.nn_seconds / dt, 3), "search_share_rank0": round(sp.search_seconds / dt, 3),
            "mean_batch": round(sp.boards / max(sp.forwards, 1), 1)}


def big_net_leg(args, rank, dist, dev, local):
    """BASELINE configs[4] network (10-block/256-filter ResNet, 15x15 Pente boards use
    the same 3-plane input) at batch 512 per GPU: forward boards/s and the persistent
    tower's MFMA fraction (device time of its launches, hipEvents)."""
    from network import PyTorchModel
    from synth import synth_encoded
    nb, ch, B = 10, 256, 512
    torch.manual_seed(1)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=nb, channels=ch)
    eng = m.engine
    x = torch.from_numpy(synth_encoded(B, seed=77 + rank)).to(dev)
    probs = torch.empty((B, 225), device=dev)
    values = torch.empty((B, 1), device=dev)
    for _ in range(3):
        eng.forward_into(x, probs, values)
    barrier_sync(dist, local)
    eng.profile_enable(True)
    t0 = time.perf_counter()
    for _ in range(args.big_steps):
        eng.forward_into(x, probs, values)
    barrier_sync(dist, local)
    dt = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile_enable(False)
    v = torch.tensor([dt], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
    dt = float(v.item())
    world = dist.get_world_size() if dist is not None else 1
    flop_conv = 2 * 225 * ch * 9 * ch * B * 2 * nb
    tower_ms, tower_n = prof.get("tower", (0.0, 0))
    if not tower_n:
        tower_ms, tower_n = prof.get("conv3x3", (0.0, 0))
        tower_n = max(tower_n // (2 * nb), 1)
    conv_s = tower_ms / 1e3 / max(tower_n, 1)
    return {"config": f"configs[4] network: {nb}x{ch} ResNet, batch {B}/GPU forward (eval BN)",
            "boards_per_s": round(B * args.big_steps * world / dt, 1),
            "ms_per_step": round(dt / args.big_steps * 1e3, 3),
            "residual_convs_ms": round(conv_s * 1e3, 3),
            "residual_convs_mfma_frac": round(flop_conv / conv_s / PEAK_F32_MFMA, 4) if conv_s > 0 else None}


def train_leg(model, args, rank, world, dist, dev, local):
    """BASELINE configs[3] train half: PyTorchModel.train_batch_device on 128 samples
    per GPU (global 128 x N) with the flat-gradient all-reduce over RCCL between
    backward and clip+Adam (distributed.grad_hook); max step time over ranks."""
    import distributed as D
    from synth import synth_encoded
    B, K = 128, args.train_steps
    rng = np.random.default_rng(77 + rank)
    x = torch.from_numpy(synth_encoded(B, seed=77 + rank)).to(dev)
    pi = rng.random((B, 225)).astype(np.float32)
    pi /= pi.sum(1, keepdims=True)
    pi = torch.from_numpy(pi).to(dev)
    z = torch.from_numpy(rng.integers(-1, 2, (B, 1)).astype(np.float32)).to(dev)
    model.grad_hook = D.grad_hook() if world > 1 else None
    for _ in range(3):
        model.train_batch_device(x, pi, z, return_tensor=True)
    barrier_sync(dist, local)
    t0 = time.perf_counter()
    for _ in range(K):
        losses = model.train_batch_device(x, pi, z, return_tensor=True)
    barrier_sync(dist, local)
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    dt = float(dt.item())
    assert torch.isfinite(losses).all()
    return {"config": f"configs[3] train step: 6x128, {B} samples/GPU (global {B * world}), "
                      f"{'RCCL all-reduce of the flat fp32 gradient (7.57 MB) + ' if world > 1 else ''}clip 3.0 + Adam",
            "samples_per_s": round(B * K * world / dt, 1), "ms_per_step": round(dt / K * 1e3, 3), "steps": K}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=BATCH)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--sp-games", type=int, default=256)
    ap.add_argument("--sp-sims", type=int, default=400)
    ap.add_argument("--sp-moves", type=int, default=2, help="moves per game in the self-play leg (0: skip)")
    ap.add_argument("--train-steps", type=int, default=20, help="steps of the data-parallel train leg (0: skip)")
    ap.add_argument("--big-steps", type=int, default=10, help="forward steps of the 10x256 net leg (0: skip)")
    args = ap.parse_args()

    rank, world, local, dist = dist_setup(args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from network import PyTorchModel
    from synth import synth_encoded

    torch.manual_seed(0)
    model = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=BLOCKS, channels=CHANNELS)
    eng = model.engine
    B = args.batch
    x = torch.from_numpy(synth_encoded(B, seed=1234 + rank)).to(dev)
    probs = torch.empty((B, 225), device=dev)
    values = torch.empty((B, 1), device=dev)

    for _ in range(args.warmup):
        eng.forward_into(x, probs, values)
    barrier_sync(dist, local)

    eng.profile_enable(True)
    barrier_sync(dist, local)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        eng.forward_into(x, probs, values)
    barrier_sync(dist, local)
    elapsed = time.perf_counter() - t0
    prof = eng.profile_read()
    eng.profile_enable(False)

    assert torch.isfinite(probs).all() and torch.isfinite(values).all()

    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    elapsed = float(t.item())

    selfplay = None
    if args.sp_moves > 0:
        selfplay = selfplay_leg(model, args, rank, dist, dev, local)
    train = None
    if args.train_steps > 0:
        train = train_leg(model, args, rank, world, dist, dev, local)

    big = None
    if args.big_steps > 0:
        big = big_net_leg(args, rank, dist, dev, local)

    if rank != 0:
        dist.destroy_process_group()
        return

    boards = B * args.steps * world
    value = boards / elapsed
    tower = bool(prof.get("tower", (0.0, 0))[1])
    if tower:
        # persistent residual tower: one launch runs all 2*BLOCKS convs
        conv_ms, conv_n = prof["tower"]
        flop_launch = FLOP_CONV * B * 2 * BLOCKS
        kname = ("azg::conv_tower<128,*> (persistent residual tower: all 12 fused 3x3 conv + BN + "
                 "residual + ReLU layers in one launch, halo-staged tiles)")
    else:
        conv_ms, conv_n = prof.get("conv3x3", (0.0, 0))
        flop_launch = FLOP_CONV * B
        kname = "azg::conv3x3_halo<128,*> (fused 3x3 conv + BN + residual + ReLU, halo-staged)"
    conv_avg_s = conv_ms / 1e3 / max(conv_n, 1)
    achieved = flop_launch / conv_avg_s
    roof = {"bound": "mfma", "achieved": round(achieved / 1e12, 3), "peak": PEAK_F32_MFMA / 1e12,
            "unit": "TFLOP/s", "frac": round(achieved / PEAK_F32_MFMA, 4),
            "traffic": load_traffic("tower" if tower else "conv3x3"),
            "kernel": kname, "avg_launch_us": round(conv_avg_s * 1e6, 2), "launches": conv_n,
            "flop_per_launch": flop_launch}
    out = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "boards/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic (seeded legal 15x15 positions; seeded Kaiming init weights, no checkpoint)",
        "config": {"workload": "configs[1]: batch-512 policy/value forward (eval BN, softmax + tanh), "
                               "6-block/128-filter ResNet, inputs resident in HBM",
                   "global_batch": B * world, "per_gpu_batch": B, "net": f"{BLOCKS}x{CHANNELS}",
                   "parallelism": f"replicas{world} (games shard by GPU; no collective in timed region)"},
        "roofline": roof,
        "whole_forward_mfma_frac": round(value / world * FLOP_BOARD / PEAK_F32_MFMA, 4),
        "kernel_ms_per_step": {k: round(v[0] / args.steps, 4) for k, v in prof.items()},
        "selfplay": selfplay,
        "train": train,
        "net_10x256": big,
    }
    if not args.no_cpu_baseline and world == 1:
        out["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
    else:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
