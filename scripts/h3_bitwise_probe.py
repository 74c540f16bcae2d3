"""Bitwise agreement of the eval forward's forms (per-layer 64x64 / 128x64, tower
64x64 / 128x64) under split-fp16 (key 19 = 1) and fp32 (0), seeded vs pretrained
weights, several batches: max |d probs| against per-layer 64x64 and whether equal.

    python scripts/h3_bitwise_probe.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import torch


def main():
    import _native
    import bench
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    dev = torch.device("cuda", 0)
    for pre in (0, 1):
        torch.manual_seed(0)
        m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=6, channels=128)
        if pre:
            bench.pretrain(m, dev)
        m.net.eval()
        eng = m.engine
        for h3 in (1, 0):
            lib.azg_pv_set_tuning(19, h3)
            for B in (128, 512, 2048):
                x = torch.from_numpy(synth_encoded(B, seed=B)).to(dev)
                res = {}
                ref = None
                for name, mode, shape, ov in (("layer5", 0, 8, 5), ("layer8", 0, 8, 8), ("tower5", 1, 5, -1),
                                             ("tower8", 1, 8, -1)):
                    lib.azg_pv_set_tuning(5, mode)
                    lib.azg_pv_set_tuning(6, shape)
                    lib.azg_pv_set_tuning(0, ov)
                    for rep in range(3):
                        p, v, lg = eng.forward(x, want_logits=True)
                        torch.cuda.synchronize()
                        if ref is None:
                            ref = lg.clone()
                        d = float((lg - ref).abs().max())
                        res[f"{name}.{rep}"] = 0.0 if torch.equal(lg, ref) else d
                lib.azg_pv_set_tuning(0, -1)
                lib.azg_pv_set_tuning(5, 2)
                print(json.dumps({"pretrained": pre, "h3": h3, "batch": B, "max_dlogit_vs_layer5": res}), flush=True)
    lib.azg_pv_set_tuning(19, 1)


if __name__ == "__main__":
    main()
