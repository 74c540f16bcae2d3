"""PolicyValueEngine: owns one libazg_pv handle and the torch-owned flat buffers
it computes on (parameters, gradients, Adam moments, BN running stats).

Layout contract (include/azg_pv.h): parameters / gradients / moments are flat
fp32 buffers in nn.Module.parameters() order with torch's per-tensor layout;
BN running stats are [mean(c) | var(c)] per BatchNorm layer in module order.
Each nn.Parameter / BN buffer of the module becomes a view into these buffers,
so state_dict(), load_state_dict() and torch.save() keep working unchanged.
"""
from __future__ import annotations

import ctypes

import torch
import torch.nn as nn

from _native import AzgConfig, check, load_library, ptr


def _stream(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


class TowerFault(RuntimeError):
    """A persistent-tower forward computed on stale inputs and could not be recomputed."""


class PolicyValueEngine:
    def __init__(self, net: nn.Module, blocks: int, channels: int, board: int, device):
        if board != 15:
            raise ValueError("the gfx950 kernels are built for 15x15 boards only")
        self.lib = load_library()
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError("PolicyValueEngine needs a HIP (MI355X) device; there is no CPU path")
        cfg = AzgConfig(blocks, channels, board, 3)
        h = ctypes.c_void_p()
        check(self.lib.azg_pv_create(ctypes.byref(cfg), ctypes.byref(h)), self.lib)
        self.h = h
        self.net = net
        self.blocks, self.channels = blocks, channels
        n = self.lib.azg_pv_num_param_tensors(h)
        offs = (ctypes.c_int64 * n)()
        nums = (ctypes.c_int64 * n)()
        check(self.lib.azg_pv_param_layout(h, offs, nums), self.lib)
        params = list(net.parameters())
        if len(params) != n or any(p.numel() != nums[i] for i, p in enumerate(params)):
            raise RuntimeError("module parameters do not match the engine layout")
        self.nparam = int(self.lib.azg_pv_param_count(h))
        dev = self.device
        with torch.no_grad():
            self.flat_params = torch.empty(self.nparam, dtype=torch.float32, device=dev)
            # the gradients + ONE skip word (include/azg_pv.h azg_pv_bind, ABI 3): a DP
            # all-reduce of flat_grads_ext carries a rank's split-fp16 range overflow to
            # every rank, and train_apply commits the step only where the word is 0
            ng = int(self.lib.azg_pv_grad_count(h))
            if ng != self.nparam + 1:
                raise RuntimeError("libazg_pv: unexpected gradient buffer layout")
            self.flat_grads_ext = torch.zeros(ng, dtype=torch.float32, device=dev)
            self.flat_grads = self.flat_grads_ext[:self.nparam]
            self.param_views = []
            self.grad_views = []
            for i, p in enumerate(params):
                o, k = int(offs[i]), int(nums[i])
                v = self.flat_params[o:o + k].view_as(p)
                v.copy_(p.data.to(dev, torch.float32))
                p.data = v
                gv = self.flat_grads[o:o + k].view_as(p)
                p.grad = gv
                self.param_views.append(v)
                self.grad_views.append(gv)
            bns = [m for m in net.modules() if isinstance(m, nn.BatchNorm2d)]
            self.nbn = int(self.lib.azg_pv_bn_count(h))
            if sum(2 * b.num_features for b in bns) != self.nbn:
                raise RuntimeError("BatchNorm layers do not match the engine layout")
            self.flat_bn = torch.empty(self.nbn, dtype=torch.float32, device=dev)
            self.flat_nbt = torch.zeros(len(bns), dtype=torch.int64, device=dev)
            o = 0
            for i, b in enumerate(bns):
                c = b.num_features
                self.flat_bn[o:o + c].copy_(b.running_mean)
                self.flat_bn[o + c:o + 2 * c].copy_(b.running_var)
                self.flat_nbt[i].copy_(b.num_batches_tracked)
                b.running_mean = self.flat_bn[o:o + c]
                b.running_var = self.flat_bn[o + c:o + 2 * c]
                b.num_batches_tracked = self.flat_nbt[i]
                o += 2 * c
        self.params = params
        check(self.lib.azg_pv_bind(h, ptr(self.flat_params), ptr(self.flat_grads_ext), ptr(self.flat_bn)), self.lib)
        if self.lib.azg_pv_num_bn_layers(h) != len(bns):
            raise RuntimeError("BatchNorm layer count does not match the engine layout")
        # num_batches_tracked advances inside the train kernels (no extra launch)
        check(self.lib.azg_pv_bind_counters(h, ptr(self.flat_nbt)), self.lib)
        self._seen = self._versions()
        self._out_cache = {}
        self.recoveries = 0         # tower launches recomputed per layer (recover)
        self.train_recoveries = 0   # train steps skipped on the device and redone in fp32 (network.train_batch)
        self._unsettled = []        # launch numbers of forwards no host sync has settled yet (predict_device)

    # -- housekeeping -------------------------------------------------------
    def _versions(self):
        # nn.Parameter keeps its own version counter after `p.data = view`, so sum them;
        # BN buffers ARE views of flat_bn and share its counter.
        return (self.flat_params._version, self.flat_bn._version, sum(p._version for p in self.params))

    def sync_dirty(self):
        """Parameters or BN stats were modified in place through torch (load_state_dict,
        copy_, optimizer from outside): re-derive packed weights before the next call."""
        v = self._versions()
        if v != self._seen:
            check(self.lib.azg_pv_mark_dirty(self.h), self.lib)
            self._seen = v

    def mark_dirty(self):
        check(self.lib.azg_pv_mark_dirty(self.h), self.lib)

    def last_seq(self) -> int:
        """Launch number of the last forward if it ran the persistent tower, else 0
        (include/azg_pv.h azg_pv_last_seq)."""
        return int(self.lib.azg_pv_last_seq(self.h))

    def recover(self, seq: int) -> bool:
        """Call after synchronising with forward `seq`: if one of its tower waits timed
        out, recompute it with per-layer convs (bitwise what an undisturbed tower gives)
        into the same device outputs, stream-ordered, and return True.  The forward's
        input and output buffers must still be intact."""
        if not seq:
            return False
        if seq in self._unsettled:
            self._unsettled.remove(seq)
        done = ctypes.c_int32(0)
        check(self.lib.azg_pv_recover(self.h, int(seq), ctypes.byref(done), _stream(self.device)), self.lib)
        if done.value:
            self.recoveries += 1
        return bool(done.value)

    def track(self, seq: int) -> None:
        """Register a forward whose caller synchronises later without settling it
        (PyTorchModel.predict_device): the next settle point checks it."""
        if seq:
            self._unsettled.append(int(seq))
            del self._unsettled[:-1024]

    def check_orphans(self, upto: int = 0) -> None:
        """Settle point (the caller has synchronised this engine's stream): raise
        TowerFault if a tracked forward older than `upto` (0: every tracked one) timed out
        or met a split-fp16 range overflow -- its buffers may be gone, so it cannot be
        recomputed, and its outputs are invalid."""
        keep, bad = [], []
        for s in self._unsettled:
            if upto and s >= upto:
                keep.append(s)
            elif int(self.lib.azg_pv_posted(self.h, s)):
                bad.append(s)
        self._unsettled = keep
        if bad:
            raise TowerFault(f"libazg_pv: forward launch(es) {bad} timed out or left fp16's range and were never "
                             f"settled (predict_device outputs consumed without recover); their outputs are invalid "
                             f"({self.tower_diag()})")

    def check_status(self):
        """Raise TowerFault if an eval launch this handle ran timed out or met a split-fp16
        range overflow and was not recovered (azg_pv_status: a plain host load, complete
        for every forward the caller has synchronised with).  The product recovers every
        such launch at its host sync (recover), so this fires only for forwards nobody
        settled.  The posted launches stay until clear_status()."""
        s = int(self.lib.azg_pv_status(self.h))
        if s:
            d = self.tower_diag()
            raise TowerFault(f"libazg_pv: {s} eval launch(es) timed out or left fp16's range and were not "
                             f"recomputed; their outputs are invalid ({d})")

    def train_skips(self) -> int:
        """Train steps the Adam kernel skipped since clear_status (azg_pv_train_status: a
        plain host load, complete for every step the caller has synchronised with)."""
        return int(self.lib.azg_pv_train_status(self.h))

    def train_fp32_once(self):
        """The next train_backward runs its forward convs with fp32 MFMA (the redo of a
        skipped step)."""
        check(self.lib.azg_pv_train_fp32_once(self.h), self.lib)

    def clear_status(self):
        check(self.lib.azg_pv_clear_status(self.h), self.lib)

    def tower_diag(self) -> dict:
        """The tower's wait record since the last tower_diag_clear (include/azg_pv.h
        azg_pv_tower_diag): wait histogram, timeouts, and the first timed-out wait."""
        from _native import TowerDiag
        d = TowerDiag()
        check(self.lib.azg_pv_tower_diag_read(self.h, ctypes.byref(d), _stream(self.device)), self.lib)
        return d.as_dict()

    def tower_diag_clear(self):
        check(self.lib.azg_pv_tower_diag_clear(self.h, _stream(self.device)), self.lib)

    def reattach_grads(self):
        for p, g in zip(self.params, self.grad_views):
            if p.grad is None or p.grad.data_ptr() != g.data_ptr():
                p.grad = g

    def close(self):
        if getattr(self, "h", None) is not None and self.h.value:
            self.lib.azg_pv_destroy(self.h)
            self.h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- compute ------------------------------------------------------------
    def forward(self, x: torch.Tensor, want_logits: bool = False):
        """Eval-mode forward on device.  x: [B,3,15,15] fp32 (any device/dtype)."""
        x = x.to(self.device, torch.float32).contiguous()
        B = int(x.shape[0])
        probs = torch.empty((B, 225), dtype=torch.float32, device=self.device)
        values = torch.empty((B, 1), dtype=torch.float32, device=self.device)
        logits = torch.empty((B, 225), dtype=torch.float32, device=self.device) if want_logits else None
        self.forward_into(x, probs, values, logits)
        return probs, values, logits

    def forward_into(self, x, probs, values, logits=None):
        self.sync_dirty()
        check(self.lib.azg_pv_forward(self.h, ptr(x), int(x.shape[0]), ptr(probs), ptr(values), ptr(logits),
                                      _stream(self.device)), self.lib)

    def forward_boards_into(self, boards, players, probs, values, priors=None):
        """Eval forward from device int8 boards [B,225] + players [B] (on-GPU encode);
        priors (optional) = probs * (board == 0)."""
        self.sync_dirty()
        check(self.lib.azg_pv_forward_boards(self.h, ptr(boards), ptr(players), int(boards.shape[0]), ptr(probs),
                                             ptr(values), ptr(priors), _stream(self.device)), self.lib)

    def train_backward(self, x, pis, zs, losses):
        self.sync_dirty()
        check(self.lib.azg_pv_train_backward(self.h, ptr(x), ptr(pis), ptr(zs), int(x.shape[0]), ptr(losses),
                                             _stream(self.device)), self.lib)
        self._seen = self._versions()
        self.reattach_grads()

    def train_apply(self, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps, wd, max_norm, total_norm=None):
        check(self.lib.azg_pv_train_apply(self.h, ptr(exp_avg), ptr(exp_avg_sq), int(step), float(lr),
                                          float(beta1), float(beta2), float(eps), float(wd), float(max_norm),
                                          ptr(total_norm), _stream(self.device)), self.lib)

    # -- instrumentation ----------------------------------------------------
    DEBUG_BUFFERS = {"z0": 0, "a0": 1, "z1": 2, "h": 3, "z2": 4, "xo": 5, "gX": 6, "DZ": 7, "DH": 8, "GR": 9, "snap": 10}

    HEAD_BUFFERS = {"fp": (11, 450), "fv": (12, 225), "hv": (13, 64)}

    def debug_tensor(self, name: str, batch: int, index: int = 0) -> torch.Tensor:
        """Interior [batch,15,15,C] of a train-workspace buffer from the last train step
        (head features fp/fv/hv: [batch, n])."""
        if name in self.HEAD_BUFFERS:
            which, n = self.HEAD_BUFFERS[name]
            out = torch.empty((batch, n), dtype=torch.float32, device=self.device)
            check(self.lib.azg_pv_debug_copy(self.h, which, 0, ptr(out), batch, _stream(self.device)), self.lib)
            return out
        out = torch.empty((batch, 15, 15, self.channels), dtype=torch.float32, device=self.device)
        check(self.lib.azg_pv_debug_copy(self.h, self.DEBUG_BUFFERS[name], index, ptr(out), batch,
                                         _stream(self.device)), self.lib)
        return out

    def profile_enable(self, on: bool = True):
        check(self.lib.azg_pv_profile_enable(self.h, 1 if on else 0), self.lib)

    def profile_read(self) -> dict:
        """{class: (ms_total, launches)} since the last profile_enable (synchronises)."""
        from _native import PROF_CLASSES
        k = len(PROF_CLASSES)
        ms = (ctypes.c_double * k)()
        n = (ctypes.c_int64 * k)()
        check(self.lib.azg_pv_profile_read(self.h, ms, n), self.lib)
        return {PROF_CLASSES[i]: (ms[i], int(n[i])) for i in range(k) if n[i]}

    def profile_boards(self) -> dict:
        """{class: boards processed} since the last profile_enable."""
        from _native import PROF_CLASSES
        k = len(PROF_CLASSES)
        b = (ctypes.c_int64 * k)()
        check(self.lib.azg_pv_profile_boards(self.h, b), self.lib)
        return {PROF_CLASSES[i]: int(b[i]) for i in range(k) if b[i]}
