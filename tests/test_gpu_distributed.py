"""Data parallelism THROUGH THE PRODUCT: world size 2, gloo, both
ranks on the HIP engine (cuda:0 here -- one GPU box; the collectives stage through
host memory under gloo, RCCL's path differs only in transport).  Each rank builds
PyTorchModel from a DIFFERENT seed, `distributed.broadcast_model` makes rank 1 a
copy of rank 0 (params, BN stats and counters, Adam moments and step), then K
`train_batch` steps on rank-local batches with `distributed.grad_hook()` between
azg_pv_train_backward and azg_pv_train_apply, and `sync_bn_stats` at the end.

Checked: params, Adam moments and step, BN running stats and counters bitwise
identical across ranks, and equal (<= 2e-6) to a single-process run that evaluates
both ranks' batches with azg_pv_train_backward, averages the two flat gradients,
and applies clip + Adam once per step (BN running stats evolved per rank, then
averaged -- what sync_bn_stats does).  Two shapes: 2x64 at B = 32/rank, and
configs[3]'s per-rank shape, 6x128 at B = 128/rank (7.57 MB flat gradient; the
reference step network.py:199-235 at train.py:849-889's batch).

`test_collectives_see_device_tensors_under_rccl`: with the backend reported as
"nccl" (RCCL has no CPU path), every tensor reaching a collective from
broadcast_model / grad_hook / sync_bn_stats / allreduce_* is a HIP tensor."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, REPO, has_gpu

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]

SHAPES = {"2x64_b32": (3, 32, 2, 64), "6x128_b128": (2, 128, 6, 128)}   # K steps, B per rank, blocks, channels


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _batch(rank, step, B):
    from oracle.boards import encode_batch, synth_positions, synth_targets
    b, p = synth_positions(B, seed=1000 + 10 * step + rank)
    pi, z = synth_targets(B, seed=2000 + 10 * step + rank)
    return encode_batch(b, p), pi, z


def _state(m):
    eng, opt = m.engine, m.optimizer
    torch.cuda.synchronize()
    return {"params": eng.flat_params.cpu().numpy().copy(), "bn": eng.flat_bn.cpu().numpy().copy(),
            "nbt": eng.flat_nbt.cpu().numpy().copy(), "m": opt.flat_exp_avg.cpu().numpy().copy(),
            "v": opt.flat_exp_avg_sq.cpu().numpy().copy(),
            "step": np.array([float(opt.state[eng.params[0]]["step"])])}


def _worker(rank, world, port, out_dir, shape):
    K, B, BLOCKS, CH = SHAPES[shape]
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    torch.set_num_threads(1)
    torch.distributed.init_process_group("gloo")
    import distributed as D
    from network import PyTorchModel
    torch.manual_seed(rank)                              # replicas start DIFFERENT
    m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=BLOCKS, channels=CH)
    if rank == 1:                                        # and a different Adam history
        x, pi, z = _batch(7, 7, B)
        m.train_batch(x, pi, z)
    D.broadcast_model(m, 0)
    m.grad_hook = D.grad_hook()
    for s in range(K):
        x, pi, z = _batch(rank, s, B)
        m.train_batch(x, pi, z)
    D.sync_bn_stats(m)
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **_state(m))
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("shape", list(SHAPES))
def test_dp_train_through_hip_engine_world2(tmp_path, shape):
    K, B, BLOCKS, CH = SHAPES[shape]
    port = _free_port()
    mp.spawn(_worker, args=(2, port, str(tmp_path), shape), nprocs=2, join=True)
    r0, r1 = (dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(2))
    for k in r0:
        assert np.array_equal(r0[k], r1[k]), k          # replicas bitwise identical

    # single process: both ranks' batches through azg_pv_train_backward, averaged
    # flat gradient, one clip + Adam per step; per-rank BN running stats, averaged
    from network import PyTorchModel
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=BLOCKS, channels=CH)
    eng = m.engine
    bn = [eng.flat_bn.clone(), eng.flat_bn.clone()]
    nbt0 = eng.flat_nbt.clone()
    losses = torch.empty(3, device=eng.device)
    m.net.train()
    for s in range(K):
        gs = []
        for r in range(2):
            x, pi, z = (torch.from_numpy(np.asarray(a, np.float32)).to(eng.device) for a in _batch(r, s, B))
            with torch.no_grad():
                eng.flat_bn.copy_(bn[r])
            eng.flat_nbt.copy_(nbt0)
            eng.train_backward(x, pi, z.reshape(-1, 1), losses)
            gs.append(eng.flat_grads.clone())
            bn[r] = eng.flat_bn.clone()
        with torch.no_grad():
            eng.flat_grads.copy_((gs[0] + gs[1]) / 2)
        m.optimizer.hip_step(m.max_grad_norm)
        nbt0 += 1
    with torch.no_grad():
        eng.flat_bn.copy_((bn[0] + bn[1]) / 2)
        eng.flat_nbt.copy_(nbt0)
    want = _state(m)
    for k in ("params", "m", "v", "bn"):
        d = float(np.abs(r0[k] - want[k]).max())
        print(f"{shape} {k}: max |dp - single| = {d:.2e}")
        assert d <= 2e-6, (k, d)
    assert np.array_equal(r0["nbt"], want["nbt"]) and r0["step"][0] == want["step"][0] == K


def test_collectives_see_device_tensors_under_rccl(monkeypatch):
    """under RCCL every collective operand must be a HIP tensor --
    broadcast_model's Adam step counter used to be a CPU float64 tensor.  The backend
    is reported as "nccl" and world size 2; the collectives record their operands."""
    import distributed as D
    import torch.distributed as dist
    from network import PyTorchModel
    seen = []

    def rec(name):
        def f(t, *a, **k):
            seen.append((name, t.device.type, tuple(t.shape), t.dtype))
        return f
    monkeypatch.setattr(D, "world", lambda: 2)
    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "nccl")
    monkeypatch.setattr(dist, "broadcast", rec("broadcast"))
    monkeypatch.setattr(dist, "all_reduce", rec("all_reduce"))
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=1, channels=64)
    D.broadcast_model(m, 0)
    D.grad_hook()(m.engine.flat_grads)
    D.sync_bn_stats(m)
    D.allreduce_sum_(torch.zeros(3, dtype=torch.int64))            # a host tensor: staged through the GPU
    assert D.allreduce_min_int(5, "cpu") == 5
    assert len(seen) >= 8
    assert all(dev == "cuda" for _, dev, _, _ in seen), seen


def test_bench_collectives_see_device_tensors_under_rccl(monkeypatch):
    """bench.py's own collectives: under a backend reported as "nccl"
    (RCCL), reduce_ hands a HIP tensor to all_reduce (sum and max) and barrier_sync
    passes the rank's device to dist.barrier; both return the right values."""
    import importlib
    import torch.distributed as dist
    bench = importlib.import_module("bench")
    seen = []

    def all_reduce(t, op=None, **k):
        seen.append(("all_reduce", t.device.type, t.dtype, op))
        t.mul_(2)                      # a 2-rank sum of equal contributions

    def barrier(*a, **k):
        seen.append(("barrier", k.get("device_ids")))

    monkeypatch.setattr(dist, "get_backend", lambda *a, **k: "nccl")
    monkeypatch.setattr(dist, "all_reduce", all_reduce)
    monkeypatch.setattr(dist, "barrier", barrier)
    dev = torch.device("cuda", 0)
    assert bench.reduce_(dist, dev, [1.5, 2.0]) == [3.0, 4.0]
    assert bench.reduce_(dist, dev, [7.0], op="max") == [14.0]
    bench.barrier_sync(dist, 0)
    assert [s[:3] for s in seen[:2]] == [("all_reduce", "cuda", torch.float64)] * 2
    assert seen[0][3] == dist.ReduceOp.SUM and seen[1][3] == dist.ReduceOp.MAX
    assert seen[2] == ("barrier", [0])


def _loop_worker(rank, world, port, out_dir):
    """One train_alphazero iteration (reference train.py:575-845) on this rank: sharded
    self-play, DP training with the flat-gradient all-reduce, BN-stat sync, sharded
    gating with the summed win count, and the accept/reject decision -- every collective
    of the loop on HIP models, under gloo (two ranks share the box's GPU)."""
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    torch.set_num_threads(1)
    torch.distributed.init_process_group("gloo")   # train_alphazero keeps an initialised group
    import random
    import train
    random.seed(100 + rank)                        # rank-local opening moves of the gating games
    np.random.seed(200 + rank)
    torch.manual_seed(rank)                        # broadcast_model must make the replicas equal
    seen = {}
    play = train._play_eval_games
    evaluate = train.evaluate_models

    def play_wrap(model_new, model_best, games, starts, *a, **k):
        winners = play(model_new, model_best, games, starts, *a, **k)
        seen["local_wins"] = sum(1 for w, s in zip(winners, starts) if (w == 1 and s) or (w == 2 and not s))
        seen["local_games"] = len(games)
        return winners

    def evaluate_wrap(*a, **k):
        out = evaluate(*a, **k)
        seen["global_wins"] = out[0]
        return out

    train._play_eval_games = play_wrap
    train.evaluate_models = evaluate_wrap
    best = train.train_alphazero(num_iterations=1, games_per_iteration=4, n_simulations=16, batch_size=64,
                                 epochs_per_iter=2, eval_games=4, eval_mcts_simulations=12,
                                 win_rate_threshold=0.0,
                                 model_dir=os.path.join(out_dir, "models"), n_res_blocks=2, channels=128,
                                 max_moves=24)
    st = _state(best)
    st.update({k: np.array([v]) for k, v in seen.items()})
    np.savez(os.path.join(out_dir, f"loop_rank{rank}.npz"), **st)
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(600)
def test_train_alphazero_world2_through_hip_engine(tmp_path):
    """train_alphazero at world size 2 end to end on HIP models
    (gloo; both ranks on this box's GPU).  After one iteration both ranks hold bitwise-
    identical params, BN buffers and counters, Adam moments and step (the accepted
    candidate: win_rate_threshold 0 accepts), and the gating win count every rank saw
    is the sum of the ranks' local wins over their shard of the games."""
    port = _free_port()
    mp.spawn(_loop_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (dict(np.load(tmp_path / f"loop_rank{r}.npz")) for r in range(2))
    for k in ("params", "bn", "nbt", "m", "v", "step"):
        assert np.array_equal(r0[k], r1[k]), k
    assert r0["global_wins"][0] == r1["global_wins"][0] == r0["local_wins"][0] + r1["local_wins"][0]
    assert r0["local_games"][0] + r1["local_games"][0] == 4
    assert r0["step"][0] > 0                                         # trained: Adam stepped


def _ovf_batches(B=32):
    """Rank 0: random legal positions with ONE input element set to 1000 (a pixel
    neighbourhood the batch statistics see once in 7,200: its normalised stem outputs
    reach ~60 sigma); rank 1: random legal positions (~5 sigma at most)."""
    from oracle.boards import encode_batch, synth_positions, synth_targets
    b0, p0 = synth_positions(B, seed=4241)
    x0 = encode_batch(b0, p0).copy()
    x0[0, 0, 7, 7] = 1000.0
    b1, p1 = synth_positions(B, seed=4242)
    pi, z = synth_targets(B, seed=4243)
    return [(x0, pi, z), (encode_batch(b1, p1), pi, z)]


def _stem_gamma(m, batches):
    """Per-channel stem BN gamma that drives rank 0's largest activation beyond fp16's
    range (65504) and keeps rank 1's below it: the geometric mean of 65520 / (the two
    batches' largest normalised stem outputs), where rank 0's is at least 8x rank 1's;
    other channels keep gamma 1 (train-mode BN statistics, float64)."""
    import torch.nn.functional as F
    w = m.net.conv.weight.detach().double().cpu()
    mx = []
    for x, _, _ in batches:
        zz = F.conv2d(torch.from_numpy(np.asarray(x, np.float64)), w, padding=1)
        mean = zz.mean(dim=(0, 2, 3), keepdim=True)
        var = zz.var(dim=(0, 2, 3), unbiased=False, keepdim=True)
        mx.append(((zz - mean) / torch.sqrt(var + 1e-5)).amax(dim=(0, 2, 3)))
    sel = mx[0] > 8 * mx[1].clamp_min(1e-3)
    gamma = torch.where(sel, 65520.0 / torch.sqrt(mx[0] * mx[1].clamp_min(1e-3)), torch.ones_like(mx[0]))
    return gamma.float(), int(sel.sum())


def _ovf_worker(rank, world, port, out_dir):
    import sys
    sys.path[:0] = [REPO, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK="0")
    torch.set_num_threads(1)
    torch.distributed.init_process_group("gloo")
    import _native
    import distributed as D
    from network import PyTorchModel
    lib = _native.load_library()
    batches = _ovf_batches()
    x, pi, z = batches[rank]
    out = {}
    for tag, key49 in (("split", 2), ("fp32", 0)):
        torch.manual_seed(11)
        m = PyTorchModel(board_size=15, device="cuda:0", n_res_blocks=2, channels=64)
        gamma, nsel = _stem_gamma(m, batches)
        with torch.no_grad():
            m.net.bn.weight.copy_(gamma.to(m.engine.device))
        m.engine.mark_dirty()
        m.grad_hook = D.grad_hook()
        prev = lib.azg_pv_set_tuning(49, key49)
        try:
            losses = m.train_batch(x, pi, z)
        finally:
            lib.azg_pv_set_tuning(49, prev)
        D.sync_bn_stats(m)   # running stats are rank-local until averaged (train.py does it per iteration)
        out.update({f"{tag}_{k}": v for k, v in _state(m).items()})
        out[f"{tag}_losses"] = np.array([losses[k] for k in ("policy_loss", "value_loss", "total_loss")])
        out[f"{tag}_recoveries"] = np.array([m.engine.train_recoveries])
        out[f"{tag}_skips"] = np.array([m.engine.train_skips()])
        out["channels"] = np.array([nsel])
    np.savez(os.path.join(out_dir, f"ovf_rank{rank}.npz"), **out)
    torch.distributed.destroy_process_group()


@pytest.mark.timeout(300)
def test_dp_train_overflow_on_one_rank_skips_everywhere(tmp_path):
    """a split-fp16 train-forward range overflow on ONE rank must not
    hang or split the replicas.  Its skip word rides the gradient all-reduce, so every rank
    skips the step on the device and redoes it in fp32 -- rank 0 overflows (its stem BN
    drives one channel past 65504 on its batch only), rank 1 does not.  Checked: both
    ranks redid the step (one recovery, one skipped step each), the replicas are bitwise
    identical, and bitwise equal to a world-2 run with key 49 = 0."""
    port = _free_port()
    mp.spawn(_ovf_worker, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    r0, r1 = (dict(np.load(tmp_path / f"ovf_rank{r}.npz")) for r in range(2))
    assert r0["channels"][0] >= 1, "no stem channel separates the two batches"
    for r in (r0, r1):
        assert r["split_recoveries"][0] == 1 and r["split_skips"][0] == 1, r
        assert r["fp32_recoveries"][0] == 0 and r["fp32_skips"][0] == 0, r
        assert np.isfinite(r["split_losses"]).all()
        for k in ("params", "bn", "nbt", "m", "v", "step", "losses"):
            assert np.array_equal(r[f"split_{k}"], r[f"fp32_{k}"]), k
    for k in ("params", "bn", "nbt", "m", "v", "step"):
        assert np.array_equal(r0[f"split_{k}"], r1[f"split_{k}"]), k
    print(f"one-rank overflow: {int(r0['channels'][0])} stem channels, both ranks redid the step in fp32")
