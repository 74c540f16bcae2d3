"""Benchmark: BASELINE.json's metric -- self-play boards/s on 15x15 Gomoku with the
6-block/128-filter ResNet at 400 sims/move (configs[2]: 256 concurrent games per
GPU), every game played to its end, one MI355X per rank.

    python bench.py [--gpus N] [--steps K] [--warmup W]

N>1 is launched by the driver as torchrun (one process per GPU, RCCL).  Self-play
shards by game: every rank plays its own 256 games (weak scaling, no collective
inside the timed region); value = leaf boards summed over ranks / max wall time.

Headline (`value`): one self-play generation as train.py plays it
(train.py:360-412 per game, __main__ settings train.py:847-889: cpuct 1.0,
Dirichlet alpha 0.05 / eps 0.15 on the first 10 moves, temperature max(0, 1 - n/10),
8-fold symmetry augmentation, max_moves 225), through the native C++ search and
the batched HIP forward.  Every game runs until is_game_over(); the run ends when
the last game does, so the shrinking batches of the tail are inside the timed
region.  A "step" is one move round (every live game makes one move, 400
simulations); `steps` is the number of rounds the generation took (its longest
game), NOT --steps: the workload is fixed by the config, --steps K / --warmup W
size the configs[1] forward sub-leg.  `roofline` is the persistent residual tower
(`conv_tower`, the dominant kernel) over its launches INSIDE the self-play run:
algorithmic FLOPs of the boards each launch evaluated / hipEvent device time of
those launches on the stream they ran on.

Sub-legs (extra keys): `selfplay_fp32` (the headline self-play again with the eval residual
convs in fp32 MFMA, tuning key 19 = 0), `forward_b512` (configs[1]: K forwards of 512 boards
in HBM, own roofline), `train` (configs[3] train step, 6x128, B=128/GPU, RCCL all-reduce
at N>1), `pente_10x256` (configs[4]: Pente self-play with the 10x256 net at 800
sims, 32 games per GPU played to their end, its 10x256 forward at B=512 and train
step at B=128), and `cpu_baseline` (rank 0 at N=1: the reference CPU path, i.e. the oracle
restatement of network.py + the reference-semantics Python MCTS, on this host).
"""
from __future__ import annotations

import argparse
import json
import os
import platform
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
PEAK_F32_MFMA = 157.3e12                                 # MI355X_MICROARCH.md: FP32 matrix peak
PEAK_F16_MFMA = 16 * PEAK_F32_MFMA                       # dense F16/BF16 MFMA (the guide: 16x the fp32 rate)
# split-fp16 residual convs (key 19 = 1, the default): three fp16 MFMAs per fp32-equivalent
# product, so their roofline is the fp16 peak / 3 in fp32-equivalent FLOP/s
PEAK_H3 = PEAK_F16_MFMA / 3


def conv_peak():
    """(peak FLOP/s of the residual convs' instructions, dtype label) for the eval
    arithmetic the library runs now (tuning key 19)."""
    import _native
    lib = _native.load_library()
    k = lib.azg_pv_set_tuning(19, -1)
    if k in (1, 2):   # 2: the 16x16x32 board tower (C = 128); the same F16 instruction peak
        return PEAK_H3, "f16x3->f32"
    return PEAK_F32_MFMA, "f32"


def train_fwd_peak():
    """(peak FLOP/s of the train step's forward convs, label) for tuning key 49: 2 (default)
    split-fp16 with four products (the F16 MFMA peak / 4), 1 three products, 0 fp32 MFMA."""
    import _native
    k = _native.load_library().azg_pv_set_tuning(49, -1)
    return {2: (PEAK_F16_MFMA / 4, "f16x4"), 1: (PEAK_F16_MFMA / 3, "f16x3")}.get(k, (PEAK_F32_MFMA, "f32"))


def conv_flop(ch: int) -> int:
    """One 3x3 C->C conv on one 15x15 board: 2 * 225 * C * 9C."""
    return 2 * 225 * ch * 9 * ch


def fwd_flop(blocks: int, ch: int) -> int:
    """Whole eval forward per board (6x128 = 798,221,828)."""
    stem = 2 * 225 * ch * 27
    heads = 2 * 225 * ch * 3 + 2 * 450 * 225 + 2 * 225 * 64 + 2 * 64
    return stem + 2 * blocks * conv_flop(ch) + heads


def train_flop(blocks: int, ch: int) -> int:
    """Train step per sample: forward + data grads + weight grads = 3x forward minus
    the stem's data grad (not needed): 6x128 = 2,393 MFLOP."""
    return 3 * fwd_flop(blocks, ch) - 2 * 225 * ch * 27


# selfplay settings of the reference's __main__ (train.py:847-889)
SP_CPUCT, SP_ALPHA, SP_EPS, SP_NOISE_MOVES, SP_TEMP_THRESHOLD = 1.0, 0.05, 0.15, 10, 10


def sp_temp(n: int) -> float:
    return max(0.0, 1.0 - n / SP_TEMP_THRESHOLD)      # train.py:647-648


def dist_setup(n_gpus: int):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        import torch.distributed as dist
        if os.environ.get("AZG_BENCH_SHARE_GPU"):
            # rehearsal of the N>1 path on a 1-GPU box (never a measurement): ranks share
            # the visible GPUs and talk over gloo (RCCL refuses two ranks on one GPU)
            local = local % torch.cuda.device_count()
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        return rank, world, local, dist
    return 0, 1, 0, None


def barrier_sync(dist, local):
    if dist is not None:
        if dist.get_backend() == "nccl":
            dist.barrier(device_ids=[local])
        else:
            dist.barrier()
    torch.cuda.synchronize()


def reduce_(dist, dev, vals, op="sum"):
    """Sum (or max) a list of floats over ranks."""
    v = torch.tensor(vals, dtype=torch.float64, device=dev)
    if dist is not None:
        if dist.get_backend() != "nccl":
            v = v.cpu()
        dist.all_reduce(v, op=dist.ReduceOp.SUM if op == "sum" else dist.ReduceOp.MAX)
    return [float(a) for a in v.tolist()]


def log(msg):
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


# --------------------------------------------------------------------- CPU host
def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def host_cores() -> dict:
    """CPUs this process may run on: affinity mask, cgroup CPU quota, physical cores."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = max(1, int(int(q) // int(period)))
    except (OSError, ValueError):
        pass
    phys = set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" in line:
                k, v = (t.strip() for t in line.split(":", 1))
                cur[k] = v
            elif cur:
                if "physical id" in cur and "core id" in cur:
                    phys.add((cur["physical id"], cur["core id"]))
                cur = {}
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    if phys:
        usable = min(usable, len(phys))      # physical cores, not SMT siblings
    return {"affinity_cpus": aff, "cgroup_quota_cpus": quota, "physical_cores": len(phys) or None,
            "threads_used": usable, "cpu_model": _cpu_model(), "os_cpu_count": os.cpu_count()}


def cpu_baseline(game_seconds: float) -> dict:
    """The reference CPU path on this host (BASELINE.md:50-59), rank 0 at N=1:
      * configs[0]: 1 self-play game, 100 sims/move, 6x128, the oracle's predict
        (oracle/ref_net.py = reference network.py:168-183 restated, PyTorch CPU) driven
        by the reference-semantics Python MCTS (mcts/new_mcts_alpha.py, bit-exact vs
        the reference goldens) at its batch of <= 32 leaves, __main__ settings; played
        to game end or until `game_seconds` of wall time (stated in `sample`);
      * the B=512 forward (configs[1]) and a B=128 train_batch (configs[3] train half);
    each at 1 thread and at all usable physical cores."""
    from games.gomoku import Gomoku
    from mcts.new_mcts_alpha import MCTS
    from oracle.boards import encode_batch, synth_positions, synth_targets
    from oracle.ref_net import RefModel
    from selfplay import sample_action_from_pi

    cores = host_cores()
    nthr = cores["threads_used"]
    torch.manual_seed(0)
    ref = RefModel(BLOCKS, CHANNELS)

    class Counting:
        boards = 0

        def predict(self, x):
            Counting.boards += len(x)
            return ref.predict(x)

    def game(threads):
        torch.set_num_threads(threads)
        np.random.seed(0)
        Counting.boards = 0
        mcts = MCTS(Gomoku, 100, Counting(), cpuct=SP_CPUCT, dirichlet_alpha=SP_ALPHA, epsilon=SP_EPS,
                    apply_dirichlet_n_first_moves=SP_NOISE_MOVES, add_dirichlet_noise=True)
        g = Gomoku(size=15)
        g.current_player = 1
        moves, t0 = 0, time.perf_counter()
        while True:                                 # train.py:369-393
            pi = mcts.run(g, len(g.move_history))
            a = sample_action_from_pi(pi, sp_temp(moves))
            if g.get_valid_moves()[a] != 1.0:
                a = int(np.argmax(pi))
            g.do_move(divmod(a, 15))
            moves += 1
            if g.is_game_over() or moves >= 225:
                ended = True
                break
            if time.perf_counter() - t0 > game_seconds:
                ended = False
                break
        dt = time.perf_counter() - t0
        return {"boards_per_s": round(Counting.boards / dt, 1), "moves_per_s": round(moves / dt, 3),
                "moves": moves, "boards": Counting.boards, "seconds": round(dt, 2), "game_over": ended}

    def forward(threads, reps):
        torch.set_num_threads(threads)
        b, p = synth_positions(BATCH, seed=99)
        x = encode_batch(b, p)
        t0 = time.perf_counter()
        for _ in range(reps):
            ref.predict(x)
        return round(BATCH * reps / (time.perf_counter() - t0), 1)

    def train(threads, reps):
        torch.set_num_threads(threads)
        b, p = synth_positions(128, seed=98)
        x = encode_batch(b, p)
        pi, z = synth_targets(128, seed=97)
        t0 = time.perf_counter()
        for _ in range(reps):
            ref.train_batch(x, pi, z)
        return round(128 * reps / (time.perf_counter() - t0), 1)

    out = {}
    g_all = game(nthr)
    g_one = game(1)
    forward(nthr, 1)                                # warm the allocator / weights in cache
    fwd_all, fwd_one = forward(nthr, 3), forward(1, 1)
    trn_all, trn_one = train(nthr, 3), train(1, 1)
    torch.set_num_threads(nthr)
    out.update({
        "value": g_all["boards_per_s"], "unit": "boards/s", "cores": nthr, "kind": "port",
        "sample": (f"configs[0]: 1 self-play game, 100 sims/move, 6x128, torch-CPU oracle predict (reference "
                   f"network.py:168-183 restated) under the reference-semantics Python MCTS (batch <= 32), "
                   f"{g_all['moves']} moves / {g_all['boards']} leaf boards in {g_all['seconds']} s at {nthr} "
                   f"threads ({'to game end' if g_all['game_over'] else 'stopped at the time bound'})"),
        "configs0_game": {"threads_all": g_all, "threads_1": g_one},
        "forward_b512_boards_per_s": {"threads_all": fwd_all, "threads_1": fwd_one},
        "train_b128_samples_per_s": {"threads_all": trn_all, "threads_1": trn_one},
        "value_1_thread": g_one["boards_per_s"],
        "host": cores,
    })
    return out


# --------------------------------------------------------------------- GPU legs
def traffic_records():
    """HBM-traffic records of the residual-conv kernels from the committed PMC passes
    (profiles/conv_traffic.json: scripts/summarize_pmc_r3.py, summarize_conv_pmc.py)."""
    try:
        d = json.load(open(os.path.join(REPO, "profiles", "conv_traffic.json")))
        return d.get("records", [d])
    except Exception:
        return []


# profile class -> (convs per launch as a multiple of blocks (0: one conv), PMC record shape prefix)
TOWER_CLASSES = {"tower16": (2, "conv_tower<128, 128, 4, 1, 16"), "tower": (2, "conv_tower<"),
                 "board": (2, "board_tower"), "board16": (2, "board16_tower"), "conv3x3": (0, None)}


def roofline_from_profile(prof, boards, blocks, ch, knames, traffic=True):
    """Residual-conv roofline from hipEvent-timed launches.  The kernel is the
    DOMINANT class by device time: the persistent tower with 16-wave tiles
    (`tower16`), with 64x64 / 128x64 tiles (`tower`), or per-layer conv3x3 launches
    (`conv3x3`); the other classes are reported beside it.  traffic: HBM bytes per
    launch from the committed PMC record of that kernel and net at the batch closest
    to this run's average launch, scaled per board to it."""
    cf = conv_flop(ch)
    peak, _ = conv_peak()
    cls = {}
    for k, (mult, _) in TOWER_CLASSES.items():
        ms, n = prof.get(k, (0.0, 0))
        if n:
            convs = mult * blocks if mult else 1
            flop = cf * convs * boards.get(k, 0)
            cls[k] = {"kernel": knames.get(k, k), "launches": n, "device_ms": round(ms, 1),
                      "avg_launch_us": round(ms / n * 1e3, 2), "flop_per_launch": round(flop / n),
                      "boards_per_launch": round(boards.get(k, 0) / n, 1),
                      "frac": round(flop / (ms / 1e3) / peak, 4), "_flop": flop, "_ms": ms}
    if not cls:
        return None
    dom = max(cls, key=lambda k: cls[k]["_ms"])
    d = cls[dom]
    achieved = d["_flop"] / (d["_ms"] / 1e3)
    out = {"bound": "mfma", "achieved": round(achieved / 1e12, 3), "peak": round(peak / 1e12, 1),
           "unit": "TFLOP/s", "frac": round(achieved / peak, 4), "traffic": None}
    if peak == PEAK_H3:
        inst = "v_mfma_f32_16x16x32_f16" if dom == "board16" else "v_mfma_f32_32x32x16_f16"
        out["peak_basis"] = (f"split-fp16 products: 3 {inst} per fp32-equivalent product, "
                             "dense F16 MFMA peak 2516.8 TFLOP/s / 3 (both f16 shapes); achieved counts the "
                             "fp32-equivalent conv FLOPs (2 x 225 x C x 9C per board per conv)")
        # a ratio, not a fraction: the split tower's fp32-equivalent rate over the fp32-MFMA peak
        out["speedup_over_fp32_mfma_peak"] = round(achieved / PEAK_F32_MFMA, 4)
    out.update({k: v for k, v in d.items() if not k.startswith("_") and k != "frac"})
    pref = TOWER_CLASSES[dom][1]
    h3 = peak == PEAK_H3
    if h3 and dom == "tower16":   # split-fp16: class 7 is the h3_tile 128x128 tower (shape 12, VAR 355)
        pref = f"conv_tower<{ch}, 128, 2, 2, 4, 355"
    if dom in ("board", "board16"):   # traffic records of the board-resident towers are keyed by class
        pref = None
        recs = [r for r in traffic_records() if r.get("kernel") == dom and
                r.get("config", "").startswith(f"{blocks}x{ch}_B")]
        if traffic and recs:
            bpl = d["boards_per_launch"]
            r = min(recs, key=lambda r: abs(r["boards_per_launch"] - bpl))
            out["traffic"] = round(r["hbm_bytes_per_launch"] / r["boards_per_launch"] * bpl)
            out["traffic_over_algorithmic"] = r["traffic_over_algorithmic"]
            out["traffic_basis"] = (f"PMC FETCH_SIZE x2 + WRITE_SIZE of {TOWER_CLASSES[dom][1]} at {r['config']} ({r['tag']}): "
                                    f"{r['hbm_bytes_per_launch'] / 1e6:.1f} MB per launch, "
                                    f"{r['traffic_over_algorithmic']}x algorithmic; scaled per board to this run's "
                                    f"average launch ({bpl} boards)")
    if traffic and pref:
        net = f"{blocks}x{ch}_B"
        # the split-fp16 128x64 towers: halo_tile VAR 99 (98 before round 5's end); h3_tile VAR 355
        recs = [r for r in traffic_records() if r.get("kernel") == "tower" and r.get("config", "").startswith(net)
                and r.get("shape", "").startswith(pref) and (dom != "tower" or "16>" not in r["shape"])
                and any(f", {v}, 0>" in r["shape"] for v in ((99, 98, 355) if h3 else (16, 32, 33)))]
        if h3 and dom == "tower" and any(", 99, 0>" in r["shape"] for r in recs):   # the current body's record first
            recs = [r for r in recs if ", 99, 0>" in r["shape"]]
        if recs:
            bpl = d["boards_per_launch"]
            r = min(recs, key=lambda r: abs(r["boards_per_launch"] - bpl))
            out["traffic"] = round(r["hbm_bytes_per_launch"] / r["boards_per_launch"] * bpl)
            out["traffic_over_algorithmic"] = r["traffic_over_algorithmic"]
            out["traffic_basis"] = (f"PMC FETCH_SIZE x2 + WRITE_SIZE of {r['shape']} at {r['config']} ({r['tag']}): "
                                    f"{r['hbm_bytes_per_launch'] / 1e6:.1f} MB per launch, "
                                    f"{r['traffic_over_algorithmic']}x algorithmic; scaled per board to this run's "
                                    f"average launch ({bpl} boards)")
    others = [k for k in cls if k != dom]
    if others:
        tot_f = sum(c["_flop"] for c in cls.values())
        tot_ms = sum(c["_ms"] for c in cls.values())
        out["all_residual_convs_frac"] = round(tot_f / (tot_ms / 1e3) / peak, 4)
        out["other_classes"] = {k: {kk: vv for kk, vv in cls[k].items() if not kk.startswith("_")} for k in others}
    return out


def tower_knames(ch, blocks):
    n = 2 * blocks
    return {"board16": (f"azg::board16_tower (board-resident residual tower on v_mfma_f32_16x16x32_f16: one board "
                        f"per 12-wave workgroup, its activations in LDS as split fp16 through all {n} fused 3x3 conv + "
                        f"BN (+ residual) + ReLU layers, split-fp16 products, LDS-DMA weight stages; then the heads' three 1x1 "
                        f"projections from the fp32 tower output in LDS)"),
            "board": (f"azg::board_tower (board-resident residual tower: one board per 16-wave workgroup, its "
                      f"activations in LDS as split fp16 through all {n} fused 3x3 conv + BN (+ residual) + ReLU "
                      f"layers, split-fp16 products, LDS-DMA weight stages)"),
            "tower16": (f"azg::conv_tower<{ch},128,2,2,4,355> (persistent residual tower, h3_tile 128x128 tiles: 4 "
                        f"waves of 64x64, split-fp16 products, LDS-DMA weight stages: {n} fused 3x3 conv + BN "
                        f"(+ residual) + ReLU layers per launch)" if conv_peak()[0] == PEAK_H3 else
                        f"azg::conv_tower<{ch},128,4,1,16,16> (persistent residual tower, 16-wave 128x128 tiles, one "
                        f"workgroup per CU: {n} fused 3x3 conv + BN (+ residual) + ReLU layers per launch)"),
            "tower": (f"azg::conv_tower<{ch},64,*,99> (persistent residual tower, 128x64 / 64x64 "
                      f"tiles, split-fp16 products, acquire hand-off: {n} fused 3x3 conv + BN (+ residual) + ReLU layers "
                      f"per launch)" if conv_peak()[0] == PEAK_H3 else
                      f"azg::conv_tower<{ch},64,*,{33 if ch >= 256 else 32}> (persistent residual tower, 128x64 / 64x64 "
                      f"tiles, acquire hand-off: {n} fused 3x3 conv + BN (+ residual) + ReLU layers per launch)"),
            "conv3x3": f"azg::conv3x3_halo<{ch},*> (per-layer fused 3x3 conv + BN (+ residual) + ReLU)"}


def batch_buckets(top):
    """Every batch bucket of the engine's autotuning caches up to `top` boards (the
    C++ conv_batch_bucket, pv_conv.hip: multiples of 16 up to 256 boards, then
    1/8-octave steps), each as the largest batch that falls in it."""
    out = set(range(16, min(top, 256) + 1, 16))
    p = 256
    while p < top:
        q = p // 8
        out.update(range(p + q, min(2 * p, top) + 1, q))
        p *= 2
    out.add(top)
    return sorted(b for b in out if b <= top)


def visit_buckets(model, top):
    """Conv/tower variant autotuning is cached per batch bucket: visit EVERY bucket a
    self-play run's leaf batches can fall in, so no tuning happens in the timed region
    (a missed bucket tunes mid-run: ~10 shapes x 4 timed launches + a stream sync)."""
    z8 = np.zeros((top, 225), np.int8)
    for b in sorted(set(batch_buckets(top)) | {1, 2, 4, 8}):
        model.predict_boards(z8[:b], np.ones(b, np.int8))


SP_GROUPS = int(os.environ.get("AZG_SP_GROUPS", "2"))   # pipelined search / evaluate groups


def selfplay_run(model, game_class, G, S, max_moves, seeds, profile=True):
    """One self-play generation of G concurrent games (native search, pipelined
    int8-board evaluator, SP_GROUPS groups: the host searches one while the GPU
    evaluates the others; results are identical for any grouping) -> (driver, seconds,
    profile, boards per class)."""
    from mcts.native_mcts import NativeSelfPlay
    sp = NativeSelfPlay(None, game_class, G, S, cpuct=SP_CPUCT, dirichlet_alpha=SP_ALPHA, epsilon=SP_EPS,
                        apply_dirichlet_n_first_moves=SP_NOISE_MOVES, evaluator_factory=model.board_evaluator,
                        groups=min(SP_GROUPS, G))
    eng = model.engine
    eng.clear_status()
    eng.tower_diag_clear()
    if profile:
        eng.profile_enable(True)
    t0 = time.perf_counter()
    last = [t0]

    def progress(live):
        now = time.perf_counter()
        if now - last[0] > 20.0:
            last[0] = now
            log(f"  {live} games live, {sp.moves} moves, {sp.boards} leaf boards, {now - t0:.0f} s")
    results = sp.play(sp_temp, max_moves=max_moves, use_symmetries=True, seeds=seeds, progress=progress)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    prof = eng.profile_read() if profile else {}
    boards = eng.profile_boards() if profile else {}
    if profile:
        eng.profile_enable(False)
    eng.check_status()   # every timed-out tower launch was recomputed at its evaluator's wait
    sp.tower = tower_waits(eng)
    return sp, dt, prof, boards, results


def tower_waits(eng) -> dict:
    """The persistent tower's dependency waits in the leg just run (azg_pv_tower_diag):
    the histogram, timeouts (each one a launch recomputed per layer) and, if any timed
    out, the first one's record."""
    d = eng.tower_diag()
    if d["timeouts"] or d["waits_suspended"] or d["max_wall_us"] > 1000:
        log(f"pid {os.getpid()} tower waits: {d}")
    out = {k: d[k] for k in ("waits_over_100us", "waits_over_1ms", "waits_over_10ms", "max_wait_us", "max_wall_us",
                             "waits_suspended", "timeouts", "recovered", "breaker_trips", "breaker_launches")}
    if d["timeouts"]:
        out["first_timeout"] = {k: d[k] for k in ("layer", "mtile", "wait_mtile", "observed", "needed", "waited_us",
                                                  "wall_us", "waiter_xcc", "waiter_cu", "producer_claimed",
                                                  "producer_started", "producer_xcc", "producer_cu",
                                                  "producer_start_us")}
    return out


PRETRAIN_STEPS = 20


def pretrain(model, dev, steps=PRETRAIN_STEPS, batch=128):
    """SURVEY.md §8(d) / §7 synthetic setup: the benchmarked weights are the seeded
    init (torch.manual_seed(0)) + 20 train_batch steps (network.py:199-235) on synthetic
    data -- legal boards (synth_encoded, seed = step), pi ~ normalised U[0,1)^225,
    z in {-1, 0, 1} (np.random.default_rng(0)), batch 128 (train.py's batch_size).
    Fresh Kaiming init is not what a self-play generation runs on (its logits
    reach +-48); ~0.06 s of GPU time, outside every timed region."""
    from synth import synth_encoded
    rng = np.random.default_rng(0)
    for s in range(steps):
        x = torch.from_numpy(synth_encoded(batch, seed=s)).to(dev)
        pi = rng.random((batch, 225)).astype(np.float32)
        pi /= pi.sum(1, keepdims=True)
        z = rng.integers(-1, 2, (batch, 1)).astype(np.float32)
        model.train_batch_device(x, torch.from_numpy(pi).to(dev), torch.from_numpy(z).to(dev), return_tensor=True)
    torch.cuda.synchronize()
    model.engine.check_status()
    model.net.eval()


def selfplay_leg(model, args, rank, world, dist, dev, local):
    """configs[2] headline: G games x S sims/move per rank, every game to its end."""
    from games.gomoku import Gomoku
    G, S = args.sp_games, args.sp_sims
    model.net.eval()
    warm_seeds = [10_000 + i for i in range(8)]
    selfplay_run(model, Gomoku, 8, 64, 2, warm_seeds, profile=False)       # code objects, pinned pools
    visit_buckets(model, (G + 1) // 2 * 32)
    barrier_sync(dist, local)
    log(f"self-play: {G} games x {S} sims/move to game end")
    sp, dt, prof, boards, results = selfplay_run(model, Gomoku, G, S, args.sp_max_moves,
                                                 [1000 * rank + i for i in range(G)])
    barrier_sync(dist, local)
    n_boards, n_moves, n_games, n_ex = reduce_(dist, dev, [float(sp.boards), float(sp.moves), float(G),
                                                           float(sum(len(ex) for ex, _ in results))])
    dt_max, rounds_max = reduce_(dist, dev, [dt, float(sp.rounds)], op="max")
    winners = {w: sum(1 for _, x in results if x == w) for w in (0, 1, 2)}
    lengths = np.asarray(sp.game_lengths)
    roof = roofline_from_profile(prof, boards, BLOCKS, CHANNELS, tower_knames(CHANNELS, BLOCKS))
    nn_ms = sum(v[0] for v in prof.values())
    return {
        "boards": n_boards, "seconds": dt_max, "rounds": int(rounds_max),
        "boards_per_s": n_boards / dt_max, "moves_per_s": n_moves / dt_max, "games": int(n_games),
        "examples": int(n_ex),
        "detail": {
            "moves_per_game": "to game end (is_game_over(), max_moves 225)",
            "game_length_rank0": {"mean": round(float(lengths.mean()), 1), "min": int(lengths.min()),
                                  "max": int(lengths.max())},
            "winners_rank0": winners,
            "leaf_boards_rank0": sp.boards, "forwards_rank0": sp.forwards,
            "mean_batch_rank0": round(sp.boards / max(sp.forwards, 1), 1), "max_batch_rank0": sp.max_batch,
            "gpu_busy_share_rank0": round(nn_ms / 1e3 / dt, 3),
            "host_wait_share_rank0": round(sp.nn_seconds / dt, 3),
            "host_search_share_rank0": round(sp.search_seconds / dt, 3),
            "kernel_ms_rank0": {k: round(v[0], 1) for k, v in prof.items()},
            "kernel_launches_rank0": {k: v[1] for k, v in prof.items()},
            "tower_waits_rank0": sp.tower,
            "settings": f"cpuct {SP_CPUCT}, Dirichlet alpha {SP_ALPHA} eps {SP_EPS} on the first {SP_NOISE_MOVES} "
                        f"moves, temperature max(0, 1 - n/{SP_TEMP_THRESHOLD}), 8 symmetries, leaf batch 32 "
                        f"per game (train.py:847-889, mcts/new_mcts_alpha.py:12)",
        },
        "roofline": roof,
    }


def selfplay_fp32_leg(model, args, rank, world, dist, dev, local, sp):
    """The headline self-play (same games, sims, seeds) with the eval residual convs in fp32
    MFMA (tuning key 19 = 0): what the split-fp16 arithmetic buys end to end, and the rate
    a caller gets who keeps the fp32 chain's numerics."""
    import _native
    lib = _native.load_library()
    prev = lib.azg_pv_set_tuning(19, 0)
    try:
        G = args.sp32_games
        a = argparse.Namespace(**{**vars(args), "sp_games": G})
        r = selfplay_leg(model, a, rank, world, dist, dev, local)
    finally:
        lib.azg_pv_set_tuning(19, prev)
    log(f"fp32 self-play done: {r['boards_per_s']:.0f} boards/s over {r['seconds']:.1f} s")
    roof = r["roofline"] or {}
    return {"tuning": "key 19 = 0 (fp32 MFMA residual convs; stem, heads unchanged)", "games": r["games"],
            "boards": r["boards"], "seconds": round(r["seconds"], 2), "rounds": r["rounds"],
            "boards_per_s": round(r["boards_per_s"], 1),
            "headline_over_fp32": round(sp["boards_per_s"] / r["boards_per_s"], 3),
            "mean_batch_rank0": r["detail"]["mean_batch_rank0"],
            "gpu_busy_share_rank0": r["detail"]["gpu_busy_share_rank0"],
            "roofline": {k: roof.get(k) for k in ("kernel", "achieved", "peak", "unit", "frac", "avg_launch_us",
                                                  "boards_per_launch")}}


def forward_leg(model, args, rank, world, dist, dev, local, blocks=BLOCKS, ch=CHANNELS, B=BATCH, steps=None,
                warmup=None):
    """configs[1] (and the configs[4] network): `steps` forwards of B synthetic boards
    resident in HBM; roofline of the residual tower from hipEvents."""
    from synth import synth_encoded
    steps = args.steps if steps is None else steps
    warmup = args.warmup if warmup is None else warmup
    eng = model.engine
    x = torch.from_numpy(synth_encoded(B, seed=1234 + rank)).to(dev)
    probs = torch.empty((B, 225), device=dev)
    values = torch.empty((B, 1), device=dev)
    for _ in range(max(warmup, 1)):
        eng.forward_into(x, probs, values)
    torch.cuda.synchronize()
    eng.tower_diag_clear()
    barrier_sync(dist, local)
    eng.profile_enable(True)
    barrier_sync(dist, local)
    t0 = time.perf_counter()
    for _ in range(steps):
        eng.forward_into(x, probs, values)
    barrier_sync(dist, local)
    elapsed = time.perf_counter() - t0
    prof = eng.profile_read()
    boards = eng.profile_boards()
    eng.profile_enable(False)
    # every launch read x and wrote probs / values: recovering the last one settles the
    # outputs; earlier timed-out launches are counted (tower_waits) and dropped
    eng.recover(eng.last_seq())
    waits = tower_waits(eng)
    eng.clear_status()
    assert torch.isfinite(probs).all() and torch.isfinite(values).all()
    (elapsed,) = reduce_(dist, dev, [elapsed], op="max")
    roof = roofline_from_profile(prof, boards, blocks, ch, tower_knames(ch, blocks))
    return {"config": f"{blocks}x{ch} ResNet, batch {B}/GPU eval forward (BN running stats, softmax + tanh), "
                      f"inputs resident in HBM",
            "boards_per_s": round(B * steps * world / elapsed, 1), "ms_per_step": round(elapsed / steps * 1e3, 4),
            "steps": steps, "warmup": warmup,
            # the whole forward against the peaks of the instructions it issues: its residual
            # convs at the conv roofline (split-fp16: F16 peak / 3), stem and heads at fp32
            "whole_forward_frac_of_instruction_peak": round(
                (2 * blocks * conv_flop(ch) / conv_peak()[0] + (fwd_flop(blocks, ch) - 2 * blocks * conv_flop(ch))
                 / PEAK_F32_MFMA) * B * steps / elapsed, 4),
            "kernel_ms_per_step": {k: round(v[0] / steps, 4) for k, v in prof.items()},
            "tower_waits_rank0": waits, "roofline": roof}


def train_leg(model, args, rank, world, dist, dev, local, blocks=BLOCKS, ch=CHANNELS, steps=None):
    """configs[3] train half: PyTorchModel.train_batch_device on 128 samples per GPU
    (global 128 x N) with the flat-gradient all-reduce over RCCL between backward
    and clip+Adam (distributed.grad_hook); max step time over ranks."""
    import distributed as D
    from synth import synth_encoded
    B = 128
    K = args.train_steps if steps is None else steps
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
    (dt,) = reduce_(dist, dev, [time.perf_counter() - t0], op="max")
    assert torch.isfinite(losses).all()
    model.grad_hook = None
    flop = train_flop(blocks, ch) * B
    fwd_conv = 2 * blocks * conv_flop(ch) * B
    fwd_peak, fwd_label = train_fwd_peak()
    nparam = model.engine.nparam
    coll = "RCCL" if dist is not None and dist.get_backend() == "nccl" else "gloo (shared-GPU rehearsal)"
    return {"config": f"{blocks}x{ch}, {B} samples/GPU (global {B * world}), "
                      f"{f'{coll} all-reduce of the flat fp32 gradient ({nparam * 4 / 1e6:.2f} MB) + ' if world > 1 else ''}"
                      f"clip 3.0 + Adam",
            "samples_per_s": round(B * K * world / dt, 1), "ms_per_step": round(dt / K * 1e3, 3), "steps": K,
            "flop_per_step": flop,
            # against the peaks of the instructions the step issues: the forward convs at the
            # key-49 arithmetic's roofline (default: four split-fp16 products, F16 peak / 4),
            # data and weight gradients, stem and heads at the fp32-MFMA peak
            "frac_of_instruction_peak": round((fwd_conv / fwd_peak + (flop - fwd_conv) / PEAK_F32_MFMA) / (dt / K), 4),
            "peak_basis": f"forward convs {fwd_label} ({fwd_peak / 1e12:.1f} TFLOP/s), everything else fp32 MFMA "
                          f"({PEAK_F32_MFMA / 1e12:.1f} TFLOP/s)"}


def pente_leg(args, rank, world, dist, dev, local):
    """configs[4] on one GPU: the 10x256 net -- Pente self-play at 800 sims/move
    (default: 32 games, every game to its end), the B=512 forward and the B=128 train
    step."""
    from games.pente import Pente
    from network import PyTorchModel
    nb, ch = 10, 256
    torch.manual_seed(1)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=nb, channels=ch)
    # the benchmarked weights are the seeded init + the same synthetic
    # train_batch steps as the 6x128 headline (pretrain), not a raw Kaiming init
    pretrain(m, dev, args.pretrain_steps)
    out = {"net": f"{nb}x{ch}",
           "weights": f"torch.manual_seed(1) init + {args.pretrain_steps} train_batch steps on synthetic data"}
    out["forward_b512"] = forward_leg(m, args, rank, world, dist, dev, local, nb, ch, BATCH, args.big_steps, 2)
    out["train_b128"] = train_leg(m, args, rank, world, dist, dev, local, nb, ch, steps=args.big_train_steps)
    if args.pente_moves > 0:
        G, S = args.pente_games, 800
        m.net.eval()
        selfplay_run(m, Pente, 4, 32, 1, [20_000 + i for i in range(4)], profile=False)
        visit_buckets(m, (G + 1) // 2 * 32)
        barrier_sync(dist, local)
        sp, dt, prof, boards, _ = selfplay_run(m, Pente, G, S, args.pente_moves, [2000 * rank + i for i in range(G)])
        barrier_sync(dist, local)
        (nbd,) = reduce_(dist, dev, [float(sp.boards)])
        (dtm,) = reduce_(dist, dev, [dt], op="max")
        lengths = np.asarray(sp.game_lengths)
        span = ("every game played to its end (is_game_over(), max_moves 225; train.py:369-393)"
                if args.pente_moves >= 225 else f"first {args.pente_moves} moves of every game (max_moves window)")
        out["selfplay"] = {
            "config": f"Pente (capture rules), {G} concurrent games/GPU x {S} sims/move, {span}, __main__ settings, "
                      f"native C++ search + batched HIP forward ({nb}x{ch})",
            "boards_per_s": round(nbd / dtm, 1), "leaf_boards": int(nbd), "seconds": round(dtm, 2),
            "games": G, "rounds": int(sp.rounds), "moves": int(sp.moves),
            "game_length_rank0": {"mean": round(float(lengths.mean()), 1), "min": int(lengths.min()),
                                  "max": int(lengths.max())},
            "mean_batch_rank0": round(sp.boards / max(sp.forwards, 1), 1),
            "roofline": roofline_from_profile(prof, boards, nb, ch, tower_knames(ch, nb))}
    del m
    torch.cuda.empty_cache()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50, help="forwards of the configs[1] sub-leg")
    ap.add_argument("--warmup", type=int, default=10, help="untimed forwards before the configs[1] sub-leg")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-game-seconds", type=float, default=12.0,
                    help="wall-time bound per configs[0] CPU game (1 thread and all cores)")
    ap.add_argument("--sp-games", type=int, default=256)
    ap.add_argument("--sp-sims", type=int, default=400)
    ap.add_argument("--sp-max-moves", type=int, default=225, help="train.py's max_moves (board size squared)")
    ap.add_argument("--sp32-games", type=int, default=256,
                    help="games of the fp32-arithmetic self-play sub-leg (key 19 = 0; 0: skip)")
    ap.add_argument("--train-steps", type=int, default=60,
                    help="steps of the configs[3] train leg (0: skip; 60 steps amortise the first step's enqueue)")
    ap.add_argument("--big-steps", type=int, default=10, help="10x256 forwards (configs[4] net; 0: skip the leg)")
    ap.add_argument("--big-train-steps", type=int, default=10)
    ap.add_argument("--pente-games", type=int, default=32)
    ap.add_argument("--pente-moves", type=int, default=225,
                    help="max_moves of the configs[4] Pente self-play (225 = every game to its end)")
    ap.add_argument("--skip-forward", action="store_true", help="profiling runs: no configs[1] sub-leg")
    ap.add_argument("--pretrain-steps", type=int, default=PRETRAIN_STEPS,
                    help="seeded train_batch steps on synthetic data before the legs (SURVEY §8(d); 0: raw init)")
    ap.add_argument("--tune", action="append", default=[], help="KEY=VALUE tuning key (A/B and profiling runs)")
    args = ap.parse_args()
    if args.tune:
        import _native
        lib = _native.load_library()
        for kv in args.tune:
            k, v = (int(t) for t in kv.split("="))
            lib.azg_pv_set_tuning(k, v)

    rank, world, local, dist = dist_setup(args.gpus)
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from network import PyTorchModel

    torch.manual_seed(0)
    model = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=BLOCKS, channels=CHANNELS)
    if args.pretrain_steps > 0:
        pretrain(model, dev, args.pretrain_steps)

    fwd = sp = None
    if not args.skip_forward:
        log("configs[1] forward leg")
        fwd = forward_leg(model, args, rank, world, dist, dev, local)
    sp32 = None
    if args.sp_games > 0:
        sp = selfplay_leg(model, args, rank, world, dist, dev, local)
        log(f"self-play done: {sp['boards_per_s']:.0f} boards/s over {sp['seconds']:.1f} s")
        if args.sp32_games > 0:
            sp32 = selfplay_fp32_leg(model, args, rank, world, dist, dev, local, sp)
    train = None
    if args.train_steps > 0:
        log("configs[3] train leg")
        train = train_leg(model, args, rank, world, dist, dev, local)
    big = None
    if args.big_steps > 0:
        log("configs[4] 10x256 legs")
        del model
        torch.cuda.empty_cache()
        big = pente_leg(args, rank, world, dist, dev, local)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline (reference CPU path on the host)")
        cpu = cpu_baseline(args.cpu_game_seconds)

    if rank != 0:
        dist.destroy_process_group()
        return
    if sp is None:      # profiling runs only (--sp-games 0): not the headline metric
        print(json.dumps({"profiling_run": True, "forward_b512": fwd, "train": train, "pente_10x256": big}),
              flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    out = {
        "metric": METRIC,
        "value": round(sp["boards_per_s"], 1),
        "unit": "boards/s",
        "n_gpus": world,
        "steps": sp["rounds"],
        "warmup": args.warmup,
        "ms_per_step": round(sp["seconds"] / max(sp["rounds"], 1) * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": conv_peak()[1],
        "data": (f"synthetic (self-play from the empty board; 6x128 weights = seeded init + {args.pretrain_steps} "
                 f"train_batch steps on synthetic boards / pi / z, SURVEY §8(d); no checkpoint)"),
        "config": {"workload": f"configs[2]: {args.sp_games} concurrent self-play games/GPU x {args.sp_sims} "
                               f"sims/move, 15x15 Gomoku, 6-block/128-filter ResNet, every game played to its end "
                               f"(train.py:360-412); value = NN-evaluated leaf boards / wall time of the whole "
                               f"generation incl. its tail",
                   "step": "one move round (every live game makes one move); steps = rounds of the generation",
                   "moves_per_game": "to game end",
                   "games_per_gpu": args.sp_games, "sims_per_move": args.sp_sims, "net": f"{BLOCKS}x{CHANNELS}",
                   "global_batch": "leaf batch varies: up to 32 x games per forward",
                   "parallelism": f"replicas{world} (games shard by GPU; no collective in the timed region)"},
        "roofline": sp["roofline"],
        "selfplay": {k: v for k, v in sp.items() if k != "roofline"},
        "selfplay_fp32": sp32,
        "forward_b512": fwd,
        "train": train,
        "pente_10x256": big,
        "cpu_baseline": cpu,
        "steps_requested": args.steps,
    }
    print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
