"""Stem kernel timing ablation (timing-only switches compiled into stem_mfma, C=128
float-plane path): device time of the stem per forward for each mask.
    python scripts/stem_ablate.py [--batch 512]"""
import os as _os

# A/B study variants live only in the study build (make -C alphazero-gomoku_amd/csrc study)
_os.environ.setdefault("AZG_PV_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                   "alphazero-gomoku_amd", "libazg_pv_study.so"))
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--masks", default="0,1,2,4,8,6,14,15")
    args = ap.parse_args()
    from network import PyTorchModel
    from synth import synth_encoded
    import _native
    lib = _native.load_library()
    m = PyTorchModel(device="cuda", n_res_blocks=6, channels=128)
    eng = m.engine
    B = args.batch
    x = torch.from_numpy(synth_encoded(B, seed=5)).cuda()
    probs = torch.empty((B, 225), device="cuda")
    values = torch.empty((B, 1), device="cuda")
    res = {}
    for rnd in range(3):
        for v in ["valu"] + args.masks.split(","):
            lib.azg_pv_set_tuning(9, 0 if v == "valu" else 1)
            lib.azg_pv_set_tuning(11, 0 if v == "valu" else int(v))
            eng.forward_into(x, probs, values)
            eng.profile_enable(True)
            for _ in range(10):
                eng.forward_into(x, probs, values)
            torch.cuda.synchronize()
            prof = eng.profile_read()
            eng.profile_enable(False)
            us = prof["stem"][0] / 10 * 1e3
            res[v] = min(res.get(v, 1e9), us)
    lib.azg_pv_set_tuning(11, 0)
    lib.azg_pv_set_tuning(9, 1)
    print(json.dumps({"batch": B, "stem_us": {k: round(v, 2) for k, v in res.items()}}))


if __name__ == "__main__":
    main()
