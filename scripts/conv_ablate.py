"""Ablation timing of the 3x3 conv main loop (shape 64x64, C=128, B from argv, default 512):
mask bit 1 = no global loads, 2 = no LDS fragment reads, 4 = no barrier, 8 = no epilogue stores.
Only conv1 launches (EPI_BN_RELU) are ablated; we time those."""
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
    x = torch.from_numpy(synth_encoded(B, seed=5)).cuda()
    probs = torch.empty((B, 225), device="cuda"); values = torch.empty((B, 1), device="cuda")
    res = {}
    for rnd in range(3):
        for mask in (0, 1, 2, 3, 4, 7, 8, 15):
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
    print(json.dumps({"batch": B, "avg_us": {str(k): round(v, 1) for k, v in med.items()},
                      "ablated_conv1_us": {str(k): round(2 * v - normal, 1) for k, v in med.items()}}))
    print("note: mixes ablated conv1 (6/step) with normal conv2 (6/step); ablated time = 2*avg - normal")


main()
