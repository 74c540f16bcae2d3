"""ctypes binding of libazg_pv.so (C-ABI declared in include/azg_pv.h).

The library is the only compute path: there is no CPU or eager-PyTorch
fallback.  If it is missing or cannot load, importing the product raises.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  -- load torch's HIP runtime first so the library binds to it

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AZG_PV_LIB", os.path.join(_HERE, "libazg_pv.so"))


class AzgConfig(ctypes.Structure):
    _fields_ = [("blocks", ctypes.c_int32), ("channels", ctypes.c_int32),
                ("board", ctypes.c_int32), ("in_ch", ctypes.c_int32)]


class TowerDiag(ctypes.Structure):
    """include/azg_pv.h azg_pv_tower_diag."""
    _fields_ = [(n, ctypes.c_uint32) for n in (
        "timeouts", "waits_over_100us", "waits_over_1ms", "waits_over_10ms", "waits_over_100ms", "max_wait_us",
        "recovered", "seq", "layer", "mtile", "wait_mtile", "observed", "needed", "waited_us", "wall_us",
        "waiter_hwid", "waiter_xcc", "claims", "producer_claimed", "producer_started", "producer_hwid",
        "producer_xcc")] + [("producer_start_us", ctypes.c_int32), ("max_wall_us", ctypes.c_uint32),
                             ("waits_suspended", ctypes.c_uint32), ("breaker_trips", ctypes.c_uint32),
                             ("breaker_launches", ctypes.c_uint32), ("h3_overflows", ctypes.c_uint32),
                             ("train_h3_overflows", ctypes.c_uint32), ("reserved", ctypes.c_uint32 * 3)]

    def as_dict(self) -> dict:
        d = {n: getattr(self, n) for n, _ in self._fields_ if n != "reserved"}
        for k in ("waiter_hwid", "producer_hwid"):   # gfx9 HW_ID fields
            v = d[k]
            d[k.replace("hwid", "cu")] = {"wave": v & 15, "simd": (v >> 4) & 3, "cu": (v >> 8) & 15,
                                          "sh": (v >> 12) & 1, "se": (v >> 13) & 7, "vmid": (v >> 20) & 15,
                                          "queue": (v >> 24) & 7}
        return d


_P = ctypes.c_void_p
_SIGS = {
    "azg_pv_abi_version": (ctypes.c_int32, []),
    "azg_pv_last_error": (ctypes.c_char_p, []),
    "azg_pv_create": (ctypes.c_int32, [ctypes.POINTER(AzgConfig), ctypes.POINTER(_P)]),
    "azg_pv_destroy": (ctypes.c_int32, [_P]),
    "azg_pv_param_count": (ctypes.c_int64, [_P]),
    "azg_pv_bn_count": (ctypes.c_int64, [_P]),
    "azg_pv_num_param_tensors": (ctypes.c_int32, [_P]),
    "azg_pv_param_layout": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]),
    "azg_pv_bind": (ctypes.c_int32, [_P, _P, _P, _P]),
    "azg_pv_mark_dirty": (ctypes.c_int32, [_P]),
    "azg_pv_bind_counters": (ctypes.c_int32, [_P, _P]),
    "azg_pv_num_bn_layers": (ctypes.c_int32, [_P]),
    "azg_pv_forward": (ctypes.c_int32, [_P, _P, ctypes.c_int32, _P, _P, _P, _P]),
    "azg_pv_forward_boards": (ctypes.c_int32, [_P, _P, _P, ctypes.c_int32, _P, _P, _P, _P]),
    "azg_pv_train_backward": (ctypes.c_int32, [_P, _P, _P, _P, ctypes.c_int32, _P, _P]),
    "azg_pv_train_apply": (ctypes.c_int32, [_P, _P, _P, ctypes.c_int64, ctypes.c_float, ctypes.c_float,
                                            ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                            _P, _P]),
    "azg_pv_profile_enable": (ctypes.c_int32, [_P, ctypes.c_int32]),
    "azg_pv_profile_read": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]),
    "azg_pv_profile_boards": (ctypes.c_int32, [_P, ctypes.POINTER(ctypes.c_int64)]),
    "azg_pv_set_tuning": (ctypes.c_int32, [ctypes.c_int32, ctypes.c_int32]),
    "azg_pv_tower_status": (ctypes.c_int32, [ctypes.c_void_p, ctypes.c_void_p]),
    "azg_pv_last_seq": (ctypes.c_uint32, [_P]),
    "azg_pv_recover": (ctypes.c_int32, [_P, ctypes.c_uint32, ctypes.POINTER(ctypes.c_int32), _P]),
    "azg_pv_status": (ctypes.c_int32, [_P]),
    "azg_pv_clear_status": (ctypes.c_int32, [_P]),
    "azg_pv_train_status": (ctypes.c_int32, [_P]),
    "azg_pv_tower_diag_read": (ctypes.c_int32, [_P, ctypes.POINTER(TowerDiag), _P]),
    "azg_pv_tower_diag_clear": (ctypes.c_int32, [_P, _P]),
    "azg_pv_debug_copy": (ctypes.c_int32, [_P, ctypes.c_int32, ctypes.c_int32, _P, ctypes.c_int32, _P]),
    "azg_pv_grad_count": (ctypes.c_int64, [_P]),
    "azg_pv_train_fp32_once": (ctypes.c_int32, [_P]),
    "azg_pv_posted": (ctypes.c_int32, [_P, ctypes.c_uint32]),
}
EXPORTS = tuple(_SIGS)
PROF_CLASSES = ("conv3x3", "stem", "heads", "train_conv", "train_wgrad", "train_other", "tower", "tower16", "board",
                "board16")
ABI_VERSION = 3   # 2: tower launch numbers, azg_pv_recover, the wait record (round 5); 3: the gradient
                  # buffer's skip word, azg_pv_train_fp32_once, azg_pv_posted (round 6)

_lib = None


def load_library(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type the C-ABI.  Raises with build instructions if absent."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(
            f"HIP policy/value library not found at {p}. Build it with "
            "`python -c 'import __graft_entry__ as g; g.build()'` (or `make -C alphazero-gomoku_amd/csrc`). "
            "There is no CPU fallback.")
    lib = ctypes.CDLL(p)
    for name, (res, args) in _SIGS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.azg_pv_abi_version() != ABI_VERSION:
        raise RuntimeError(f"libazg_pv ABI {lib.azg_pv_abi_version()} != expected {ABI_VERSION}")
    if path is None:
        _lib = lib
    return lib


def check(rc: int, lib: ctypes.CDLL | None = None) -> None:
    if rc != 0:
        lib = lib or load_library()
        raise RuntimeError("libazg_pv: " + (lib.azg_pv_last_error() or b"?").decode())


def ptr(t) -> int | None:
    return None if t is None else t.data_ptr()
