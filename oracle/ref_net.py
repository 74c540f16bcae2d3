"""Oracle: PyTorch-CPU restatement of the reference policy/value network and its
train step.  TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Restates, operation for operation (same ATen ops, same order, same state_dict
keys, same RNG consumption at init):

* ``ResidualBlock``          -- reference ``network.py:9-26``
* ``AlphaZeroNet``           -- reference ``network.py:29-117`` (init ``:75-83``)
* ``predict``                -- reference ``network.py:168-183``
* ``train_batch``            -- reference ``network.py:199-235`` with the optimiser
  and loss objects built in ``PyTorchModel.__init__`` (``network.py:141-163``):
  Adam(lr=1e-3, weight_decay=1e-4), MSELoss(), KLDivLoss('batchmean'),
  clip_grad_norm_(3.0).

Pinned against goldens generated from the reference itself
(``tests/golden/make_golden.py`` -> ``tests/golden/*.npz``), see
``tests/test_oracle_golden.py``.  It is also the ``cpu_baseline`` ("port") that
``bench.py`` times on the GPU box's host cores, since the reference source never
travels there.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F


def _conv3(cin: int, cout: int) -> nn.Conv2d:
    return nn.Conv2d(cin, cout, kernel_size=3, padding=1, bias=False)


class RefBlock(nn.Module):
    """network.py:9-26: relu(bn2(conv2(relu(bn1(conv1(x))))) + x)."""

    def __init__(self, c: int):
        super().__init__()
        self.conv1 = _conv3(c, c)
        self.bn1 = nn.BatchNorm2d(c)
        self.conv2 = _conv3(c, c)
        self.bn2 = nn.BatchNorm2d(c)

    def forward(self, x):
        h = F.relu(self.bn1(self.conv1(x)))
        h = self.bn2(self.conv2(h))
        h += x                       # in-place add, as network.py:24
        return F.relu(h)


class RefNet(nn.Module):
    """network.py:29-117.  Module registration order == reference order, so the
    state_dict keys and the RNG stream consumed by construction + re-init match."""

    def __init__(self, blocks: int = 6, channels: int = 128, board: int = 15,
                 in_ch: int = 3, actions: int | None = None):
        super().__init__()
        actions = board * board if actions is None else actions
        self.board_size, self.action_size, self.channels = board, actions, channels
        self.conv = _conv3(in_ch, channels)
        self.bn = nn.BatchNorm2d(channels)
        self.res_blocks = nn.ModuleList(RefBlock(channels) for _ in range(blocks))
        self.policy_conv = nn.Conv2d(channels, 2, kernel_size=1, bias=False)
        self.policy_bn = nn.BatchNorm2d(2)
        self.policy_fc = nn.Linear(2 * board * board, actions)
        self.value_conv = nn.Conv2d(channels, 1, kernel_size=1, bias=False)
        self.value_bn = nn.BatchNorm2d(1)
        self.value_fc1 = nn.Linear(board * board, 64)
        self.value_fc2 = nn.Linear(64, 1)
        # network.py:75-83 -- re-init in self.modules() order
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, nonlinearity="relu")
            elif isinstance(m, nn.Linear):
                nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
                nn.init.constant_(m.bias, 0)

    def forward(self, x):
        h = F.relu(self.bn(self.conv(x)))
        for blk in self.res_blocks:
            h = blk(h)
        p = F.relu(self.policy_bn(self.policy_conv(h)))
        logits = self.policy_fc(p.view(p.shape[0], -1))
        v = F.relu(self.value_bn(self.value_conv(h)))
        v = F.relu(self.value_fc1(v.view(v.shape[0], -1)))
        value = torch.tanh(self.value_fc2(v))
        return logits, value


class RefModel:
    """network.py:132-235 restated (CPU only)."""

    def __init__(self, blocks=6, channels=128, board=15, lr=1e-3, weight_decay=1e-4,
                 dtype=torch.float32):
        self.board_size = board
        self.action_size = board * board
        self.net = RefNet(blocks, channels, board).to(dtype)
        self.dtype = dtype
        self.optimizer = torch.optim.Adam(self.net.parameters(), lr=lr,
                                          weight_decay=weight_decay)
        self.value_loss_fn = nn.MSELoss()
        self.policy_loss_fn = nn.KLDivLoss(reduction="batchmean")

    def predict(self, x: np.ndarray, with_logits: bool = False):
        """network.py:168-183: eval mode + no_grad, softmax(dim=1), restore mode."""
        was_training = self.net.training
        self.net.eval()
        with torch.no_grad():
            xt = torch.from_numpy(np.asarray(x).astype(np.float32)).to(self.dtype)
            logits, value = self.net(xt)
            probs = F.softmax(logits, dim=1).numpy()
            values = value.numpy()
        self.net.train(was_training)
        if with_logits:
            return probs, values, logits.numpy()
        return probs, values

    def train_batch(self, states, target_pis, target_vs, epochs: int = 1) -> dict:
        """network.py:199-235."""
        self.net.train()
        s = torch.from_numpy(np.asarray(states).astype(np.float32)).to(self.dtype)
        t = torch.from_numpy(np.asarray(target_pis).astype(np.float32)).to(self.dtype)
        z = torch.from_numpy(np.asarray(target_vs).astype(np.float32)).to(self.dtype)
        acc = np.zeros(3)
        for _ in range(epochs):
            self.optimizer.zero_grad()
            logits, values = self.net(s)
            pl = self.policy_loss_fn(F.log_softmax(logits, dim=1), t)
            vl = self.value_loss_fn(values, z)
            loss = pl + vl
            loss.backward()
            torch.nn.utils.clip_grad_norm_(self.net.parameters(), 3.0)
            self.optimizer.step()
            acc += [float(pl.item()), float(vl.item()), float(loss.item())]
        acc /= float(epochs)
        return {"policy_loss": acc[0], "value_loss": acc[1], "total_loss": acc[2]}


def state_to_numpy(net: nn.Module) -> dict:
    return {k: v.detach().cpu().numpy().copy() for k, v in net.state_dict().items()}


def load_numpy_state(net: nn.Module, state: dict) -> None:
    sd = net.state_dict()
    new = {}
    for k, v in sd.items():
        new[k] = torch.from_numpy(np.asarray(state[k])).to(v.dtype)
    net.load_state_dict(new)


def param_count(blocks: int, channels: int, board: int = 15) -> int:
    """Trainable parameter count of network.py:41-73 (BN affine included)."""
    c, a = channels, board * board
    stem = c * 27 + 2 * c
    tower = blocks * 2 * (c * c * 9 + 2 * c)
    pol = 2 * c + 4 + (2 * a) * a + a
    val = c + 2 + a * 64 + 64 + 64 + 1
    return stem + tower + pol + val


def masked_forward_fp64(net: nn.Module, x, masks: dict):
    """Train-mode forward in float64 where every ReLU is replaced by the caller's
    0/1 mask (e.g. the GPU's own forward).  Returns (logits, value, pre) where
    pre[name] is the fp64 PRE-activation of the masked ReLU `name` (a0, h{i}, xo{i},
    fp, fv, hv) given the masks upstream of it -- what a flipped mask is judged by."""
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)
    mk = {k: t(v) for k, v in masks.items()}
    pre = {}
    z = net.bn(net.conv(t(x)))
    pre["a0"] = z
    h = z * mk["a0"]
    for i, blk in enumerate(net.res_blocks):
        z = blk.bn1(blk.conv1(h))
        pre[f"h{i}"] = z
        hh = z * mk[f"h{i}"]
        z = blk.bn2(blk.conv2(hh)) + h
        pre[f"xo{i}"] = z
        h = z * mk[f"xo{i}"]
    B = h.shape[0]
    z = net.policy_bn(net.policy_conv(h)).reshape(B, -1)
    pre["fp"] = z
    logits = net.policy_fc(z * mk["fp"])
    z = net.value_bn(net.value_conv(h)).reshape(B, -1)
    pre["fv"] = z
    z = net.value_fc1(z * mk["fv"])
    pre["hv"] = z
    value = torch.tanh(net.value_fc2(z * mk["hv"]))
    return logits, value, pre


def masked_grads_fp64(state: dict, blocks: int, channels: int, x, pi, z, masks: dict, return_pre: bool = False):
    """Autograd gradients of the train-step loss (network.py:213-222) in float64,
    with every ReLU's 0/1 derivative mask SUPPLIED by the caller (e.g. the GPU's
    own forward) instead of recomputed.  A pre-activation within fp32 rounding of
    zero flips a mask between two correct fp32 implementations and the gradient
    jumps there; fixing the masks makes the comparison well-conditioned.
    masks: a0 [B,C,15,15], h{i}, xo{i} (NCHW), fp [B,450], fv [B,225], hv [B,64];
    1.0 where the GPU's ReLU output was > 0.  Returns (grads dict, (pl, vl)), and
    the fp64 pre-activations (numpy) as a third element when return_pre."""
    net = RefNet(blocks, channels).double()
    load_numpy_state(net, {k: (np.asarray(v, dtype=np.float64) if np.asarray(v).dtype.kind == "f" else v)
                           for k, v in state.items()})
    net.train()
    t = lambda a: torch.as_tensor(np.asarray(a), dtype=torch.float64)
    logits, value, pre = masked_forward_fp64(net, x, masks)
    pl = F.kl_div(F.log_softmax(logits, dim=1), t(pi), reduction="batchmean")
    vl = F.mse_loss(value, t(z))
    (pl + vl).backward()
    grads = {n: q.grad.numpy() for n, q in net.named_parameters()}
    losses = (float(pl.detach()), float(vl.detach()))
    if return_pre:
        return grads, losses, {k: v.detach().numpy() for k, v in pre.items()}
    return grads, losses
