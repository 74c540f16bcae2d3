"""In-process A/B of the eval residual tower's hand-off forms (round 3), study build
(AZG_PV_LIB=.../libazg_pv_study.so): 6x128 forward at several batches, tower device
time per forward from the engine's hipEvents on the tower's stream, interleaved
rounds, plus a bitwise check of every variant's outputs against per-layer launches.

  layer      per-layer launches (no in-launch hand-off)
  t5         64x64 / 4 waves, acquire, buffer addressing (VAR 32)
  t8         128x64 / 8 waves, acquire, buffer addressing (VAR 32)       [product]
  t8_flat    128x64 / 8 waves, acquire, 64-bit pointer loads (VAR 0)     [round-2 acquire form]
  t8_sc1     128x64 / 8 waves, sc1 loads, no acquire, 2 WG/CU (VAR 16)   [round-2 default; outside envelope]
  t10        128x128 / 16 waves, sc1 loads, 1 WG/CU (VAR 16)              [product]
  t10_acq    128x128 / 16 waves, acquire, buffer addressing (VAR 32)

    AZG_PV_LIB=alphazero-gomoku_amd/libazg_pv_study.so python scripts/tower_r3_ab.py [--batches 512,2048]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch

VARIANTS = {   # name: (key 5 mode, key 6 shape, key 10 var, key 31)
    "layer": (0, 8, 0, 0),
    "t5": (1, 5, 0, 0),
    "t8": (1, 8, 0, 0),
    "t8_flat": (1, 8, 13, 0),
    "t8_sc1": (1, 8, 0, 1),
    "t10": (1, 10, 0, 0),
    "t10_acq": (1, 10, 1, 0),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="512,1024,2048,3456,4096")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    args = ap.parse_args()
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    study = lib.azg_pv_set_tuning(15, 0) == 1
    names = [v for v in args.variants.split(",") if study or VARIANTS[v][2] == 0 and VARIANTS[v][3] == 0]
    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=6, channels=128)
    eng = m.engine

    def setv(name):
        mode, shape, var, coh = VARIANTS[name]
        lib.azg_pv_set_tuning(5, mode)
        lib.azg_pv_set_tuning(6, shape)
        lib.azg_pv_set_tuning(10, var)
        lib.azg_pv_set_tuning(31, coh)

    for B in (int(b) for b in args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=B)).cuda()
        ref = None
        same = {}
        for name in names:
            setv(name)
            p, v, _ = eng.forward(x)
            torch.cuda.synchronize()
            eng.check_status()
            if ref is None:
                ref = (p.clone(), v.clone())
            same[name] = bool(torch.equal(p, ref[0]) and torch.equal(v, ref[1]))
        res = {n: [] for n in names}
        for r in range(args.rounds):
            for name in names:
                setv(name)
                for _ in range(2):
                    eng.forward(x)
                eng.profile_enable(True)
                for _ in range(args.steps):
                    eng.forward(x)
                prof = eng.profile_read()
                eng.profile_enable(False)
                ms = sum(prof.get(c, (0.0, 0))[0] for c in ("tower", "tower16", "conv3x3"))
                res[name].append(ms / args.steps)
        eng.check_status()
        flop = 12 * 2 * 225 * 128 * 9 * 128 * B
        for name, t in res.items():
            t = sorted(t)
            print(json.dumps({"batch": B, "variant": name, "tower_ms_min": round(t[0], 4),
                              "tower_ms_median": round(t[len(t) // 2], 4),
                              "frac_best": round(flop / (t[0] * 1e-3) / 157.3e12, 4),
                              "bitwise_equal_to_first": same[name]}), flush=True)
    setv("t10")
    lib.azg_pv_set_tuning(5, 2)


if __name__ == "__main__":
    main()
