"""Train step A/B: conv weight grads overlapped on a side stream (default) vs on
the caller's stream (tuning key 12), 6x128, B=128; then the per-class device time
of the serial schedule (each class alone on the GPU).
    WGRAD_BK=32,16 python scripts/train_ab.py   (wgrad K chunks to compare, key 13)"""
import os, sys, time, json
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd")]
import numpy as np, torch
from network import PyTorchModel
import _native
from oracle.boards import encode_batch, synth_positions, synth_targets
lib = _native.load_library()
torch.manual_seed(0)
m = PyTorchModel(device="cuda", n_res_blocks=6, channels=128)
B = 128
b, p = synth_positions(B, seed=3); x = torch.from_numpy(encode_batch(b, p)).cuda()
pi, z = synth_targets(B, seed=4); pi = torch.from_numpy(pi).cuda(); z = torch.from_numpy(z).cuda()
res = {}
BKS = [int(v) for v in os.environ.get("WGRAD_BK", "32").split(",")]
for rnd in range(4):
    for mode in [(o, bk) for o in (0, 1) for bk in BKS]:
        lib.azg_pv_set_tuning(12, mode[0])
        lib.azg_pv_set_tuning(13, mode[1])
        for _ in range(3): m.train_batch_device(x, pi, z)
        torch.cuda.synchronize(); t0 = time.perf_counter()
        for _ in range(20): m.train_batch_device(x, pi, z)
        torch.cuda.synchronize(); dt = (time.perf_counter() - t0) / 20 * 1e3
        res[mode] = min(res.get(mode, 1e9), dt)
lib.azg_pv_set_tuning(12, 0)
lib.azg_pv_set_tuning(13, 32)
print(json.dumps({("serial" if o else "overlapped") + f"_bk{bk}_ms": round(v, 3) for (o, bk), v in res.items()}))
lib.azg_pv_set_tuning(12, 1)
lib.azg_pv_set_tuning(13, BKS[-1])
eng = m.engine
eng.profile_enable(True)
for _ in range(10): m.train_batch_device(x, pi, z)
torch.cuda.synchronize()
prof = eng.profile_read(); eng.profile_enable(False)
lib.azg_pv_set_tuning(12, 0)
lib.azg_pv_set_tuning(13, 32)
print(json.dumps({k: (round(v[0] / 10, 3), v[1] // 10) for k, v in prof.items()}))
