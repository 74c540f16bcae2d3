"""Ablation timing of the halo-staged 3x3 conv tile (C=128; argv: batch [default 512],
tile shape 5 = 64x64 / 8 = 128x64 [default 5]), per-layer launches:
mask bit 1 = no weight loads, 2 = no halo loads, 4 = no per-chunk barrier,
8 = no LDS fragment reads, 16 = no epilogue stores.
Only conv1 launches (EPI_BN_RELU) are ablated; we time those."""
import os as _os

# A/B study variants live only in the study build (make -C alphazero-gomoku_amd/csrc study)
_os.environ.setdefault("AZG_PV_LIB", _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                                                   "alphazero-gomoku_amd", "libazg_pv_study.so"))
import os, sys, json, statistics
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]
import torch


def main():
    from network import PyTorchModel
    from synth import synth_encoded
    import _native
    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(device="cuda", n_res_blocks=6, channels=128)
    eng = m.engine
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    shape = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    lib.azg_pv_set_tuning(5, 0)        # per-layer launches (ablations apply there)
    lib.azg_pv_set_tuning(0, shape)    # un-ablated conv2 launches use the same shape
    lib.azg_pv_set_tuning(7, shape)
    x = torch.from_numpy(synth_encoded(B, seed=5)).cuda()
    probs = torch.empty((B, 225), device="cuda"); values = torch.empty((B, 1), device="cuda")
    res = {}
    for rnd in range(3):
        for mask in (0, 1, 2, 3, 4, 8, 16, 7, 31):
            lib.azg_pv_set_tuning(3, mask)
            eng.forward_into(x, probs, values)
            eng.profile_enable(True)
            for _ in range(5):
                eng.forward_into(x, probs, values)
            ms, n = eng.profile_read()["conv3x3"]
            eng.profile_enable(False)
            res.setdefault(mask, []).append(ms / n * 1e3)
    lib.azg_pv_set_tuning(3, 0)
    med = {k: statistics.median(v) for k, v in res.items()}
    normal = med[0]
    print(json.dumps({"batch": B, "shape": shape, "avg_us": {str(k): round(v, 1) for k, v in med.items()},
                      "ablated_conv1_us": {str(k): round(2 * v - normal, 1) for k, v in med.items()}}))
    print("note: mixes ablated conv1 (6/step) with normal conv2 (6/step); ablated time = 2*avg - normal")


main()
