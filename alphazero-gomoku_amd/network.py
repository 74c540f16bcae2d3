"""Drop-in replacement for the reference ``network.py`` whose compute runs on
hand-written gfx950 HIP kernels (libazg_pv.so, include/azg_pv.h).

Same public surface as the reference (network.py:9-265):
  * ``ResidualBlock``, ``AlphaZeroNet`` -- same sub-module names, parameter order,
    state_dict keys and initialisation (so ``torch.manual_seed(s)`` + ctor gives the
    reference's weights bit for bit); ``forward`` runs the HIP eval path.
  * ``PyTorchModel(board_size, action_size, device, n_res_blocks=3, channels=64, lr,
    weight_decay)`` with ``predict``, ``predict_batch``, ``train_batch``, ``save``,
    ``load``, ``make_batch_from_states`` and the attributes ``.net``, ``.optimizer``,
    ``.board_size``, ``.action_size``, ``.device``; plus ``policy_value`` /
    ``train_step`` aliases named by the north star, and device-resident variants
    (``predict_device``) for the batched self-play driver.

Differences, by design: the device must be a HIP GPU (there is no CPU path: the
reference's CPU fallback, network.py:152, raises here) and the board must be 15x15.
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch
import torch.nn as nn

from engine import PolicyValueEngine


class ResidualBlock(nn.Module):
    """Parameter container of reference network.py:9-26 (compute: pv_conv.hip)."""

    def __init__(self, channels: int):
        super().__init__()
        self.conv1 = nn.Conv2d(channels, channels, kernel_size=3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(channels)
        self.conv2 = nn.Conv2d(channels, channels, kernel_size=3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(channels)


class AlphaZeroNet(nn.Module):
    """Reference network.py:29-117.  Parameters live in the engine's flat buffers
    once attached to a device (``attach``); forward() is the HIP eval path."""

    def __init__(self, in_channels: int = 3, board_size: int = 15, action_size: int = 15 * 15,
                 n_res_blocks: int = 6, channels: int = 128):
        super().__init__()
        self.board_size = board_size
        self.action_size = action_size
        self.channels = channels
        self.n_res_blocks = n_res_blocks
        self.conv = nn.Conv2d(in_channels, channels, kernel_size=3, padding=1, bias=False)
        self.bn = nn.BatchNorm2d(channels)
        self.res_blocks = nn.ModuleList([ResidualBlock(channels) for _ in range(n_res_blocks)])
        self.policy_conv = nn.Conv2d(channels, 2, kernel_size=1, bias=False)
        self.policy_bn = nn.BatchNorm2d(2)
        self.policy_fc = nn.Linear(2 * board_size * board_size, action_size)
        self.value_conv = nn.Conv2d(channels, 1, kernel_size=1, bias=False)
        self.value_bn = nn.BatchNorm2d(1)
        self.value_fc1 = nn.Linear(board_size * board_size, 64)
        self.value_fc2 = nn.Linear(64, 1)
        self._init_weights()
        self.engine: Optional[PolicyValueEngine] = None

    def _init_weights(self):
        # network.py:75-83 (same RNG consumption order)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, nonlinearity="relu")
            elif isinstance(m, nn.Linear):
                nn.init.kaiming_uniform_(m.weight, nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def attach(self, device) -> "AlphaZeroNet":
        """Move parameters into the engine's device buffers (once)."""
        if self.engine is None:
            self.engine = PolicyValueEngine(self, self.n_res_blocks, self.channels, self.board_size, device)
        return self

    def to(self, *args, **kwargs):  # keep `.to("cuda")` working like the reference
        dev = None
        if args and isinstance(args[0], (str, torch.device)):
            dev = torch.device(args[0])
        elif "device" in kwargs:
            dev = torch.device(kwargs["device"])
        if dev is not None and dev.type == "cuda":
            return self.attach(dev)
        if self.engine is not None:
            raise RuntimeError("AlphaZeroNet is bound to a HIP device; moving it is not supported")
        return super().to(*args, **kwargs)

    def mark_dirty(self):
        """Call after mutating parameters through ``.data`` (not tracked by autograd versions)."""
        if self.engine is not None:
            self.engine.mark_dirty()

    def forward(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """(logits [B,225], value [B,1]) with BN running statistics (eval semantics).
        Train-mode BN runs only inside PyTorchModel.train_batch (fused with backward)."""
        if self.engine is None:
            raise RuntimeError("AlphaZeroNet.forward needs a HIP device: call .to('cuda') first")
        if self.training:
            raise RuntimeError("train-mode forward is fused into PyTorchModel.train_batch; "
                               "call .eval() for inference")
        eng = self.engine
        x = x.to(eng.device, torch.float32).contiguous()
        _, value, logits = eng.forward(x, want_logits=True)
        # a host-visible result, like the reference's: settle the launch now (x is alive)
        seq = eng.last_seq()
        if seq:
            torch.cuda.current_stream(eng.device).synchronize()
            eng.recover(seq)
            eng.check_orphans()
        return logits, value

    def predict(self, state):
        """network.py:119-129: single unbatched state -> (logits, value)."""
        st = torch.as_tensor(np.asarray(state), dtype=torch.float32).unsqueeze(0)
        return self(st)


class HipAdam(torch.optim.Adam):
    """torch.optim.Adam bookkeeping (param_groups, state_dict format: step /
    exp_avg / exp_avg_sq per parameter) whose moments live in flat device buffers
    updated by the fused clip+Adam kernel (azg_pv_train_apply)."""

    def __init__(self, net: AlphaZeroNet, lr: float = 1e-3, weight_decay: float = 1e-4):
        super().__init__(net.parameters(), lr=lr, weight_decay=weight_decay)
        self._net = net
        eng = net.engine
        self.flat_exp_avg = torch.zeros_like(eng.flat_params)
        self.flat_exp_avg_sq = torch.zeros_like(eng.flat_params)

    def get_step(self) -> int:
        self._ensure_state()
        return int(self.state[self._net.engine.params[0]]["step"].item())

    def set_step(self, step: int) -> None:
        self._ensure_state()
        for p in self._net.engine.params:
            self.state[p]["step"].fill_(float(step))

    def _views(self, p, i):
        eng = self._net.engine
        o = int(eng.param_views[i].storage_offset())
        return (self.flat_exp_avg[o:o + p.numel()].view_as(p), self.flat_exp_avg_sq[o:o + p.numel()].view_as(p))

    def _ensure_state(self):
        """Lazily create torch-format state (as torch does on the first step)."""
        for i, p in enumerate(self._net.engine.params):
            st = self.state[p]
            if "exp_avg" not in st:
                ea, es = self._views(p, i)
                ea.zero_()
                es.zero_()
                st["step"] = torch.tensor(0.0, dtype=torch.float32)
                st["exp_avg"] = ea
                st["exp_avg_sq"] = es

    def load_state_dict(self, state_dict):
        super().load_state_dict(state_dict)
        with torch.no_grad():
            for i, p in enumerate(self._net.engine.params):
                st = self.state.get(p)
                if not st or "exp_avg" not in st:
                    continue
                ea, es = self._views(p, i)
                ea.copy_(st["exp_avg"])
                es.copy_(st["exp_avg_sq"])
                st["exp_avg"], st["exp_avg_sq"] = ea, es
                # a private step counter: torch's load_state_dict hands back the SOURCE
                # step tensor, and hip_step's fill_ would otherwise advance the other
                # optimizer's step too (the moments above are private copies as well --
                # clean copy semantics; the reference aliases both, train.py:817,827)
                st["step"] = torch.tensor(float(st["step"]), dtype=torch.float32)

    def hip_step(self, max_norm: float = float("inf"), total_norm: Optional[torch.Tensor] = None):
        """One optimiser step on the bound flat grads: clip to max_norm, then Adam."""
        self._ensure_state()
        g = self.param_groups[0]
        if g.get("amsgrad") or g.get("maximize"):
            raise NotImplementedError("amsgrad/maximize are not used by the reference")
        first = self.state[self._net.engine.params[0]]
        step = int(first["step"].item()) + 1
        b1, b2 = g["betas"]
        self._net.engine.train_apply(self.flat_exp_avg, self.flat_exp_avg_sq, step, g["lr"], b1, b2,
                                     g["eps"], g["weight_decay"], max_norm, total_norm)
        for p in self._net.engine.params:
            self.state[p]["step"].fill_(float(step))

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        self.hip_step()
        return loss


class BoardEvaluator:
    """Asynchronous leaf evaluation for the native search: pinned host staging
    (the search writes int8 boards straight into it), non-blocking H2D, the
    board-input forward, non-blocking D2H of the masked priors and values, and an
    event to wait on.  Two evaluators let the host search one half of the games
    while the GPU evaluates the other."""

    def __init__(self, model: "PyTorchModel", capacity: int):
        self.model = model
        dev = model.engine.device
        self.capacity = int(capacity)
        self.h_boards = torch.empty((capacity, 225), dtype=torch.int8).pin_memory()
        self.h_players = torch.empty((capacity,), dtype=torch.int8).pin_memory()
        self.h_priors = torch.empty((capacity, 225), dtype=torch.float32).pin_memory()
        self.h_values = torch.empty((capacity, 1), dtype=torch.float32).pin_memory()
        self.d_boards = torch.empty((capacity, 225), dtype=torch.int8, device=dev)
        self.d_players = torch.empty((capacity,), dtype=torch.int8, device=dev)
        self.d_probs = torch.empty((capacity, 225), dtype=torch.float32, device=dev)
        self.d_priors = torch.empty((capacity, 225), dtype=torch.float32, device=dev)
        self.d_values = torch.empty((capacity, 1), dtype=torch.float32, device=dev)
        self.boards = self.h_boards.numpy()      # views the search writes into
        self.players = self.h_players.numpy()
        self.event = torch.cuda.Event()
        self.n = 0
        self.seq = 0                             # tower launch number of the batch in flight

    def submit(self, n: int) -> None:
        self.n = n
        if n == 0:
            return
        self.d_boards[:n].copy_(self.h_boards[:n], non_blocking=True)
        self.d_players[:n].copy_(self.h_players[:n], non_blocking=True)
        eng = self.model.engine
        eng.forward_boards_into(self.d_boards[:n], self.d_players[:n], self.d_probs[:n],
                                self.d_values[:n], self.d_priors[:n])
        self.seq = eng.last_seq()
        self.h_priors[:n].copy_(self.d_priors[:n], non_blocking=True)
        self.h_values[:n].copy_(self.d_values[:n], non_blocking=True)
        self.event.record()

    def wait(self):
        """-> (priors [n,225], values [n,1]) numpy views of the pinned buffers.  A batch
        whose persistent-tower forward timed out is recomputed per layer here (the device
        inputs and outputs of this evaluator are intact until its next submit)."""
        if self.n:
            self.event.synchronize()
            eng = self.model.engine
            if eng.recover(self.seq):
                n = self.n
                self.h_priors[:n].copy_(self.d_priors[:n], non_blocking=True)
                self.h_values[:n].copy_(self.d_values[:n], non_blocking=True)
                self.event.record()
                self.event.synchronize()
            eng.check_orphans(self.seq)
        return self.h_priors.numpy()[:self.n], self.h_values.numpy()[:self.n]


class PyTorchModel:
    """Reference network.py:132-265 surface over the HIP engine."""

    def __init__(self,
                 board_size: int = 15,
                 action_size: Optional[int] = None,
                 device: Optional[str] = None,
                 n_res_blocks: int = 3,
                 channels: int = 64,
                 lr: float = 1e-3,
                 weight_decay: float = 1e-4):
        self.board_size = board_size
        self.action_size = action_size if action_size is not None else board_size * board_size
        self.device = device or ("cuda" if torch.cuda.is_available() else "cpu")
        if not str(self.device).startswith("cuda"):
            raise RuntimeError(
                f"PyTorchModel(device={self.device!r}): this build computes only on HIP devices "
                "(MI355X, gfx950); there is no CPU fallback")
        self.net = AlphaZeroNet(in_channels=3, board_size=board_size, action_size=self.action_size,
                                n_res_blocks=n_res_blocks, channels=channels).attach(self.device)
        self.optimizer = HipAdam(self.net, lr=lr, weight_decay=weight_decay)
        self.value_loss_fn = nn.MSELoss()
        self.policy_loss_fn = nn.KLDivLoss(reduction="batchmean")
        self.max_grad_norm = 3.0                        # network.py:223
        self.grad_hook = None                           # DP: all-reduce of the flat grads (+ skip word)
        self._losses = None
        self._skips_seen = 0                            # device-skipped steps already accounted for

    @property
    def engine(self) -> PolicyValueEngine:
        return self.net.engine

    # ---------------- inference ----------------
    def predict(self, encoded_states: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
        """network.py:168-183: (probs [B,225] float32, values [B,1] float32) with BN
        running stats; the module's train/eval flag is left as it was."""
        eng = self.engine
        x = torch.from_numpy(np.ascontiguousarray(encoded_states, dtype=np.float32)).to(eng.device)
        probs, values = self.predict_device(x)
        seq = eng.last_seq()
        out = probs.cpu().numpy(), values.cpu().numpy()
        if eng.recover(seq):   # a timed-out tower wait: recomputed per layer in place
            out = probs.cpu().numpy(), values.cpu().numpy()
        eng.check_orphans()
        return out

    def predict_device(self, x: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Device-resident predict: x [B,3,15,15] -> (probs, values) on the GPU.
        Asynchronous: a caller that synchronises should settle the forward with
        engine.recover(engine.last_seq()) (x must still be intact), as predict does;
        a forward nobody settles is checked at the engine's next settle point
        (check_orphans: a posted one raises TowerFault there)."""
        eng = self.engine
        probs, values, _ = eng.forward(x)
        eng.track(eng.last_seq())
        return probs, values

    policy_value = predict

    def predict_boards(self, boards: np.ndarray, players: np.ndarray, masked: bool = True):
        """Leaf evaluation from int8 boards [B,15,15] or [B,225] and the side to move
        [B]: the encoding (games/gomoku.py:130-150) runs inside the stem kernel.
        Returns (priors = probs * valid if masked else probs, values [B,1]) as numpy."""
        eng = self.engine
        b = torch.from_numpy(np.ascontiguousarray(boards, dtype=np.int8).reshape(len(boards), 225)).to(eng.device)
        pl = torch.from_numpy(np.ascontiguousarray(players, dtype=np.int8).reshape(-1)).to(eng.device)
        B = int(b.shape[0])
        probs = torch.empty((B, 225), dtype=torch.float32, device=eng.device)
        values = torch.empty((B, 1), dtype=torch.float32, device=eng.device)
        priors = torch.empty_like(probs) if masked else None
        eng.forward_boards_into(b, pl, probs, values, priors)
        seq = eng.last_seq()
        out = (priors if masked else probs).cpu().numpy(), values.cpu().numpy()
        if eng.recover(seq):
            out = (priors if masked else probs).cpu().numpy(), values.cpu().numpy()
        eng.check_orphans()
        return out

    def board_evaluator(self, capacity: int) -> "BoardEvaluator":
        return BoardEvaluator(self, capacity)

    def predict_batch(self, states_list: list) -> Tuple[np.ndarray, np.ndarray]:
        return self.predict(self.make_batch_from_states(states_list))

    # ---------------- training ----------------
    def train_batch(self, states: np.ndarray, target_pis: np.ndarray, target_vs: np.ndarray,
                    epochs: int = 1) -> dict:
        """network.py:199-235: per epoch zero_grad, train-mode forward, KLDiv(batchmean)
        + MSE, backward, clip_grad_norm_(3.0), Adam step.  Leaves the net in train mode."""
        self.net.train()
        dev = self.engine.device
        s = torch.from_numpy(np.ascontiguousarray(states, dtype=np.float32)).to(dev)
        t = torch.from_numpy(np.ascontiguousarray(target_pis, dtype=np.float32)).to(dev)
        z = torch.from_numpy(np.ascontiguousarray(target_vs, dtype=np.float32).reshape(-1, 1)).to(dev)
        return self.train_batch_device(s, t, z, epochs)

    def train_batch_device(self, s: torch.Tensor, t: torch.Tensor, z: torch.Tensor, epochs: int = 1,
                           return_tensor: bool = False):
        """train_batch on device-resident tensors.  return_tensor=True returns the
        mean losses as a float32 [3] device tensor (policy, value, total) without a
        host sync, so consecutive steps pipeline on the stream.

        A step whose split-fp16 forward (tuning key 49) met an activation beyond fp16's
        range on any rank does not commit on the device (include/azg_pv.h
        azg_pv_train_apply: params, moments and BN buffers keep the values it started
        from).  Synchronous callers (return_tensor=False) see it with the losses and redo
        the step with fp32 forward convs on every rank -- the result is the key-49 = 0
        step, bitwise.  Pipelined callers (return_tensor=True) do not wait for it: the
        skipped step's batch is dropped, its Adam step number is given back at the next
        call (steps already queued behind it used numbers one higher), and
        engine.train_skips() counts it."""
        self.net.train()
        eng = self.engine
        self._settle_skips()
        losses = torch.empty(3, dtype=torch.float32, device=eng.device)
        acc = None
        vals = None
        for _ in range(epochs):
            step0 = self.optimizer.get_step()
            self._one_step(s, t, z, losses)
            if not return_tensor:
                # one host sync per step (the reference reads its losses per step too)
                v = torch.cat((losses, eng.flat_grads_ext[-1:])).double().tolist()
                if v[3] != 0.0:
                    # skipped on the device on every rank (the all-reduced skip word): redo in fp32
                    self.optimizer.set_step(step0)
                    eng.train_recoveries += 1
                    self._skips_seen += 1
                    eng.train_fp32_once()
                    self._one_step(s, t, z, losses)
                    v = losses.double().tolist()
                vals = v[:3] if vals is None else [a + b for a, b in zip(vals, v[:3])]
            elif epochs > 1:
                acc = losses.double() if acc is None else acc + losses
        if return_tensor:
            return losses if epochs == 1 else (acc / float(epochs)).float()
        vals = [a / float(epochs) for a in vals]
        return {"policy_loss": vals[0], "value_loss": vals[1], "total_loss": vals[2]}

    def _one_step(self, s, t, z, losses):
        eng = self.engine
        eng.train_backward(s, t, z, losses)
        if self.grad_hook is not None:
            self.grad_hook(eng.flat_grads_ext)   # the gradients AND the step's skip word
        self.optimizer.hip_step(self.max_grad_norm)

    def _settle_skips(self):
        """Give back the Adam step numbers of pipelined steps the device skipped."""
        n = self.engine.train_skips()
        if n < self._skips_seen:       # clear_status reset the count
            self._skips_seen = n
        elif n > self._skips_seen:
            self.optimizer.set_step(self.optimizer.get_step() - (n - self._skips_seen))
            self._skips_seen = n

    train_step = train_batch

    # ---------------- checkpoints ----------------
    def save(self, path: str) -> None:
        """network.py:240-248 format: {"net", "opt", "board_size", "action_size"}."""
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        torch.cuda.current_stream(self.engine.device).synchronize()
        self._settle_skips()
        net_sd = {k: v.detach().clone() for k, v in self.net.state_dict().items()}
        opt_sd = self.optimizer.state_dict()
        opt_sd = {"state": {i: {k: (v.detach().clone() if torch.is_tensor(v) else v) for k, v in st.items()}
                            for i, st in opt_sd["state"].items()},
                  "param_groups": opt_sd["param_groups"]}
        torch.save({"net": net_sd, "opt": opt_sd, "board_size": self.board_size,
                    "action_size": self.action_size}, path)

    def load(self, path: str, map_location: Optional[str] = None) -> None:
        """network.py:250-258; optimizer-state errors are ignored as in the reference."""
        map_location = map_location or self.device
        state = torch.load(path, map_location=map_location, weights_only=True)
        self.net.load_state_dict(state["net"])
        if "opt" in state and state["opt"] is not None:
            try:
                self.optimizer.load_state_dict(state["opt"])
            except Exception:
                pass

    @staticmethod
    def make_batch_from_states(list_of_encoded_states: list) -> np.ndarray:
        return np.stack(list_of_encoded_states, axis=0).astype(np.float32)
