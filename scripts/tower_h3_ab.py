"""Split-fp16 (H3) eval tower vs the fp32-MFMA tower, in one process.

The 6x128 (and 10x256) net after bench.py's synthetic pretraining: per batch, the
tower's device time (hipEvents, profile class 'tower') of the fp32 tower (key 19 = 0)
and the H3 tower (key 19 = 1), interleaved rounds, and the H3 outputs against the fp32
outputs and against the float64 oracle forward (oracle/ref_net.py).

    python scripts/tower_h3_ab.py [--batches 512,3456] [--rounds 4] [--reps 5]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]

import numpy as np
import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", default="512,3456")
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--net", default="6x128")
    ap.add_argument("--oracle", type=int, default=64, help="boards checked against the fp64 oracle (0: skip)")
    args = ap.parse_args()
    import _native
    import bench
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    nb, ch = (int(v) for v in args.net.split("x"))
    dev = torch.device("cuda", 0)
    torch.manual_seed(0 if ch == 128 else 1)
    m = PyTorchModel(board_size=15, device=str(dev), n_res_blocks=nb, channels=ch)
    bench.pretrain(m, dev)
    eng = m.engine
    lib.azg_pv_set_tuning(5, 1)
    lib.azg_pv_set_tuning(6, 8)
    res = {"net": args.net}
    for B in (int(b) for b in args.batches.split(",")):
        x = torch.from_numpy(synth_encoded(B, seed=B)).to(dev)
        outs, times = {}, {0: [], 1: []}
        for r in range(args.rounds):
            for v in (0, 1):
                lib.azg_pv_set_tuning(19, v)
                p, val, lg = eng.forward(x, want_logits=True)    # warm / pack
                torch.cuda.synchronize()
                eng.profile_enable(True)
                for _ in range(args.reps):
                    p, val, lg = eng.forward(x, want_logits=True)
                prof = eng.profile_read()
                eng.profile_enable(False)
                times[v].append(prof["tower"][0] / prof["tower"][1])
                outs[v] = (p.clone(), val.clone(), lg.clone())
        lib.azg_pv_set_tuning(19, 0)
        flop = 2 * 225 * ch * 9 * ch * 2 * nb * B
        d = {"batch": B}
        for v in (0, 1):
            t = min(times[v])
            d[("fp32" if v == 0 else "h3") + "_tower_ms"] = round(t, 4)
            d[("fp32" if v == 0 else "h3") + "_tflops"] = round(flop / (t * 1e-3) / 1e12, 1)
        d["speedup"] = round(min(times[0]) / min(times[1]), 3)
        p0, v0, l0 = outs[0]
        p1, v1, l1 = outs[1]
        d["h3_vs_fp32"] = {"max_dprob": float((p0 - p1).abs().max()), "max_dvalue": float((v0 - v1).abs().max()),
                           "max_dlogit": float((l0 - l1).abs().max())}
        if args.oracle:
            from oracle.ref_net import RefModel
            n = min(args.oracle, B)
            r64 = RefModel(nb, ch, dtype=torch.float64)
            r64.net.load_state_dict({k: (v.detach().cpu().double() if v.dtype.is_floating_point else v.cpu())
                                     for k, v in m.net.state_dict().items()})
            pr, vr = r64.predict(x[:n].cpu().numpy())
            for tag, (pp, vv, _) in (("fp32", outs[0]), ("h3", outs[1])):
                d[tag + "_vs_fp64_oracle"] = {"max_dprob": float(np.abs(pp[:n].cpu().numpy() - pr).max()),
                                              "max_dvalue": float(np.abs(vv[:n].cpu().numpy() - vr).max())}
        print(json.dumps(d), flush=True)
        res[B] = d
    return res


if __name__ == "__main__":
    main()
