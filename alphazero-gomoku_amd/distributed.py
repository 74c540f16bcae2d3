"""One process per GPU, torch.distributed over RCCL ("nccl" backend on ROCm) or
gloo on CPU.  Used in exactly two places:

  * self-play: games are sharded across ranks (independent replicas, no
    per-move communication);
  * training: data-parallel step with ONE all-reduce (average) of the flat fp32
    gradient buffer between backward and clip+Adam, so the clip sees the global
    gradient; BN running stats are averaged once per iteration; weights and Adam
    moments are broadcast from rank 0 when replicas must agree.
"""
from __future__ import annotations

import os
from typing import Optional

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


def init_from_env(backend: Optional[str] = None) -> tuple:
    """Initialise from torchrun env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).
    Returns (rank, world, local_rank, device)."""
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    r = int(os.environ.get("RANK", "0"))
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    use_gpu = torch.cuda.is_available() and backend != "gloo"
    device = torch.device("cuda", lr) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(device)
    if ws > 1 and not dist.is_initialized():
        backend = backend or ("nccl" if use_gpu else "gloo")
        if backend == "nccl":
            dist.init_process_group(backend, device_id=device)
        else:
            dist.init_process_group(backend)
    return r, ws, lr, device


def _on_host(t: torch.Tensor, fn) -> torch.Tensor:
    """Run collective `fn` on `t` where the backend can reach it: a device tensor
    under gloo is staged through host memory (gloo is the CPU test backend:
    world-size-2 DP tests of the HIP engine); a host tensor under RCCL ("nccl",
    which has no CPU path) is staged through the current HIP device."""
    nccl = dist.get_backend() == "nccl"
    if t.is_cuda and not nccl:
        h = t.detach().to("cpu")
        fn(h)
        t.copy_(h)
    elif not t.is_cuda and nccl:
        d = t.detach().to(torch.device("cuda", torch.cuda.current_device()))
        fn(d)
        t.copy_(d.cpu())
    else:
        fn(t)
    return t


def allreduce_mean_(t: torch.Tensor) -> torch.Tensor:
    """In-place average across ranks: RCCL's AVG (one pass over xGMI, no extra
    kernel) on GPU tensors, SUM then scale on gloo (no AVG there)."""
    n = world()
    if n > 1:
        if t.is_cuda and dist.get_backend() == "nccl":
            dist.all_reduce(t, op=dist.ReduceOp.AVG)
        else:
            def f(x):
                dist.all_reduce(x, op=dist.ReduceOp.SUM)
                x.div_(n)
            _on_host(t, f)
    return t


def allreduce_sum_(t: torch.Tensor) -> torch.Tensor:
    if world() > 1:
        _on_host(t, lambda x: dist.all_reduce(x, op=dist.ReduceOp.SUM))
    return t


def broadcast_(t: torch.Tensor, src: int = 0) -> torch.Tensor:
    if world() > 1:
        _on_host(t, lambda x: dist.broadcast(x, src))
    return t


def allreduce_min_int(v: int, device) -> int:
    if world() == 1:
        return int(v)
    t = torch.tensor([int(v)], dtype=torch.int64, device=device)
    _on_host(t, lambda x: dist.all_reduce(x, op=dist.ReduceOp.MIN))
    return int(t.item())


def grad_hook():
    """Hook for PyTorchModel.grad_hook: average the flat gradient buffer."""
    return allreduce_mean_


def broadcast_model(model, src: int = 0) -> None:
    """Make every replica identical to `src`: params, BN stats and counters, Adam
    moments and the Adam step counter (bias correction)."""
    if world() == 1:
        return
    eng = model.engine
    for t in (eng.flat_params, eng.flat_bn, eng.flat_nbt):
        broadcast_(t, src)
    opt = model.optimizer
    broadcast_(opt.flat_exp_avg, src)
    broadcast_(opt.flat_exp_avg_sq, src)
    opt._ensure_state()
    # on the engine's device: RCCL has no CPU tensors (gloo stages it through the host)
    step = torch.tensor([float(opt.state[eng.params[0]]["step"])], dtype=torch.float64, device=eng.device)
    broadcast_(step, src)
    for p in eng.params:
        opt.state[p]["step"].fill_(float(step.item()))
    eng.mark_dirty()


def sync_bn_stats(model) -> None:
    """Average BN running statistics (each rank saw its own local batches)."""
    if world() > 1:
        allreduce_mean_(model.engine.flat_bn)
        model.engine.mark_dirty()


def shard(n: int, r: Optional[int] = None, w: Optional[int] = None) -> range:
    """Contiguous share of n items for rank r (sizes differ by at most one)."""
    r = rank() if r is None else r
    w = world() if w is None else w
    base, extra = divmod(n, w)
    start = r * base + min(r, extra)
    return range(start, start + base + (1 if r < extra else 0))
