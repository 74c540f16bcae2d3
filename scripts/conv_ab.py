"""Interleaved A/B of 3x3-conv tile shapes in ONE process (6x128, B=512 forward).
Each round runs every shape for K forwards and reads the conv launches' average
device time from the engine's hipEvent instrumentation.  Also checks that every
shape produces bitwise-identical outputs (the K order does not depend on tiling).

    python scripts/conv_ab.py [--shapes 0,6,3] [--variants 1,0] [--rounds 5] [--steps 10] [--batch 512]

--variants: conv kernel variants (1 halo-staged product kernel, 0 per-chunk A staging);
outputs are compared bitwise within a variant (the K order differs between variants).
"""
import os as _os

# A/B study variants live only in the study build (make -C alphazero-gomoku_amd/csrc study)
_os.environ.setdefault("AZG_PV_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                   "alphazero-gomoku_amd", "libazg_pv_study.so"))
import argparse
import json
import os
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shapes", default="0,6,3,1")
    ap.add_argument("--variants", default="1")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--blocks", type=int, default=6)
    ap.add_argument("--channels", type=int, default=128)
    args = ap.parse_args()
    from network import PyTorchModel
    from synth import synth_encoded
    import _native

    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=args.blocks, channels=args.channels)
    eng = m.engine
    x = torch.from_numpy(synth_encoded(args.batch, seed=5)).cuda()
    probs = torch.empty((args.batch, 225), device="cuda")
    values = torch.empty((args.batch, 1), device="cuda")
    shapes = [(v, int(s)) for v in map(int, args.variants.split(",")) for s in args.shapes.split(",")]
    ref = {}
    times = {s: [] for s in shapes}
    for r in range(args.rounds):
        for s in shapes:
            lib.azg_pv_set_tuning(4, s[0])
            lib.azg_pv_set_tuning(0, s[1])
            eng.forward_into(x, probs, values)      # warm
            eng.profile_enable(True)
            for _ in range(args.steps):
                eng.forward_into(x, probs, values)
            prof = eng.profile_read()
            eng.profile_enable(False)
            ms, n = prof["conv3x3"]
            times[s].append(ms / n * 1e3)
            if s[0] not in ref:
                ref[s[0]] = probs.clone()
            elif not torch.equal(ref[s[0]], probs):
                print(f"variant/shape {s}: outputs differ within the variant "
                      f"(max {float((ref[s[0]] - probs).abs().max()):.3e})")
    if len(ref) > 1:
        a, b = list(ref.values())[:2]
        print(f"variants {list(ref)}: max |dprobs| between variants {float((a - b).abs().max()):.3e}")
    lib.azg_pv_set_tuning(0, -1)
    lib.azg_pv_set_tuning(4, 1)
    flop = 2 * 225 * args.channels * 9 * args.channels * args.batch
    out = {f"v{s[0]}s{s[1]}": {"median_us": round(statistics.median(t), 2), "min_us": round(min(t), 2),
               "tflops": round(flop / (statistics.median(t) * 1e-6) / 1e12, 2)} for s, t in times.items()}
    print(json.dumps({"batch": args.batch, "net": f"{args.blocks}x{args.channels}", "conv": out}))


if __name__ == "__main__":
    main()
