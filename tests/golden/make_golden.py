"""Generate golden vectors by importing the REFERENCE (read-only, /root/reference)
in this container.  The reference never travels to the GPU box; only the small
.npz fixtures written here do.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

For each net size (3x64 = reference default, network.py:145-146; 6x128 = BASELINE
configs 2-4):
  * weights: torch.manual_seed(0) + reference PyTorchModel ctor, then 20 seeded
    reference ``train_batch`` steps (fresh Kaiming init explodes activations),
    then every float tensor rounded to fp16-representable values and stored as fp16
    (exact when widened back to fp32), so fixtures stay small;
  * forward: reference ``PyTorchModel.predict`` (network.py:168-183) on 64 seeded
    synthetic positions, plus logits and an fp64 re-run (the tolerance floor);
  * train: a fresh reference PyTorchModel loaded with those weights runs two
    ``train_batch`` calls (network.py:199-235); we keep the losses and a seeded
    subset of the updated params, BN buffers and Adam moments;
  * init checksums of the raw seed-0 construction (pins the oracle's RNG order,
    which the box uses to regenerate 10x256 weights).
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
sys.path.insert(0, REPO)

import network as ref_network  # noqa: E402  (the reference module)
from oracle.boards import encode_batch, synth_positions, synth_targets  # noqa: E402

SUBSET = 2048


def _subset_idx(n: int, seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    k = min(n, SUBSET)
    return np.sort(rng.choice(n, size=k, replace=False))


def make(blocks: int, channels: int) -> None:
    torch.set_num_threads(8)
    tag = f"{blocks}x{channels}"
    out = {}

    torch.manual_seed(0)
    m = ref_network.PyTorchModel(board_size=15, device="cpu", n_res_blocks=blocks, channels=channels)
    for k, v in m.net.state_dict().items():
        if v.dtype.is_floating_point:
            out[f"init_sum/{k}"] = np.float64(v.double().sum().item())
            out[f"init_abs/{k}"] = np.float64(v.double().abs().sum().item())

    # 20 seeded warm-up steps (reference train_batch)
    for step in range(20):
        b, p = synth_positions(128, seed=1000 + step)
        pi, z = synth_targets(128, seed=2000 + step)
        m.train_batch(encode_batch(b, p), pi, z, epochs=1)

    sd = m.net.state_dict()
    rounded = {}
    for k, v in sd.items():
        if v.dtype.is_floating_point:
            h = v.detach().half()
            rounded[k] = h.float()
            out[f"w/{k}"] = h.numpy()
        else:
            rounded[k] = v.clone()
            out[f"w/{k}"] = v.numpy()
    m.net.load_state_dict(rounded)

    # forward goldens
    b, p = synth_positions(64, seed=123)
    x = encode_batch(b, p)
    probs, values = m.predict(x)
    m.net.eval()
    with torch.no_grad():
        logits, _ = m.net(torch.from_numpy(x))
        net64 = ref_network.AlphaZeroNet(n_res_blocks=blocks, channels=channels).double()
        net64.load_state_dict({k: (v.double() if v.dtype.is_floating_point else v) for k, v in rounded.items()})
        net64.eval()
        l64, v64 = net64(torch.from_numpy(x).double())
        p64 = torch.softmax(l64, dim=1)
    out["fwd/boards"] = b
    out["fwd/players"] = p
    out["fwd/probs"] = probs
    out["fwd/values"] = values
    out["fwd/logits"] = logits.numpy()
    out["fwd/probs64"] = p64.numpy()
    out["fwd/values64"] = v64.numpy()
    out["fwd/logits64"] = l64.numpy()

    # train goldens: fresh model (fresh Adam), two steps
    torch.manual_seed(0)
    t = ref_network.PyTorchModel(board_size=15, device="cpu", n_res_blocks=blocks, channels=channels)
    t.net.load_state_dict(rounded)
    losses = []
    for step in range(2):
        bb, pp = synth_positions(128, seed=3000 + step)
        pi, z = synth_targets(128, seed=4000 + step)
        out[f"train/boards{step}"] = bb
        out[f"train/players{step}"] = pp
        out[f"train/pi{step}"] = pi
        out[f"train/z{step}"] = z
        li = t.train_batch(encode_batch(bb, pp), pi, z, epochs=1)
        losses.append([li["policy_loss"], li["value_loss"], li["total_loss"]])
    out["train/losses"] = np.array(losses, dtype=np.float64)
    names = [n for n, _ in t.net.named_parameters()]
    params = dict(t.net.named_parameters())
    for i, n in enumerate(names):
        pt = params[n].detach().reshape(-1)
        idx = _subset_idx(pt.numel(), seed=i)
        st = t.optimizer.state[params[n]]
        out[f"train/idx/{n}"] = idx
        out[f"train/param/{n}"] = pt.numpy()[idx]
        out[f"train/exp_avg/{n}"] = st["exp_avg"].reshape(-1).numpy()[idx]
        out[f"train/exp_avg_sq/{n}"] = st["exp_avg_sq"].reshape(-1).numpy()[idx]
    for k, v in t.net.state_dict().items():
        if "running" in k or "num_batches" in k:
            out[f"train/buf/{k}"] = v.numpy().copy()

    path = os.path.join(HERE, f"net_{tag}.npz")
    np.savez_compressed(path, **out)
    print(f"wrote {path} ({os.path.getsize(path) / 1e6:.2f} MB)")


if __name__ == "__main__":
    make(3, 64)
    make(6, 128)
