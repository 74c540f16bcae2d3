"""Ablation timing of the 3x3 conv main loop (shape 160x128, C=128, B=512):
mask bit 1 = no global loads, 2 = no LDS fragment reads, 4 = no barrier.
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
    x = torch.from_numpy(synth_encoded(512, seed=5)).cuda()
    probs = torch.empty((512, 225), device="cuda"); values = torch.empty((512, 1), device="cuda")
    res = {}
    for rnd in range(3):
        for mask in (0, 1, 2, 3, 4, 7):
            lib.azg_pv_set_tuning(3, mask)
            eng.forward_into(x, probs, values)
            eng.profile_enable(True)
            for _ in range(5):
                eng.forward_into(x, probs, values)
            ms, n = eng.profile_read()["conv3x3"]
            eng.profile_enable(False)
            res.setdefault(mask, []).append(ms / n * 1e3)
    lib.azg_pv_set_tuning(3, 0)
    print(json.dumps({str(k): round(statistics.median(v), 1) for k, v in res.items()}))
    print("note: mixes ablated conv1 (6/step) with normal conv2 (6/step); ablated time = 2*avg - normal")


main()
