"""GPU debug: one train step on the golden fixture -- per-tensor gradient error
(GPU vs the fp32 oracle autograd and vs fp64), BN batch statistics / running stats,
and the fraction of params whose post-Adam value differs by > 2e-5.

    python scripts/debug_train2.py [blocks ch]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd"), os.path.join(REPO, "tests")]

import numpy as np
import torch
import torch.nn.functional as F

from conftest import golden_state, load_golden
from oracle.boards import encode_batch
from oracle.ref_net import RefModel, load_numpy_state


def main():
    blocks, ch = (int(a) for a in sys.argv[1:3]) if len(sys.argv) > 2 else (6, 128)
    torch.set_num_threads(8)
    g = load_golden(f"{blocks}x{ch}")
    st = golden_state(g)
    from network import PyTorchModel
    m = PyTorchModel(device="cuda", n_res_blocks=blocks, channels=ch)
    m.net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    ref = RefModel(blocks, ch)
    load_numpy_state(ref.net, st)
    r64 = RefModel(blocks, ch, dtype=torch.float64)
    r64.net.load_state_dict({k: (torch.from_numpy(np.asarray(v)).double() if np.asarray(v).dtype.kind == "f"
                                 else torch.from_numpy(np.asarray(v))) for k, v in st.items()})
    x = encode_batch(g["train/boards0"], g["train/players0"])
    pi, z = g["train/pi0"], g["train/z0"]
    B = len(x)
    print("B =", B)

    def grads_of(r, dt):
        r.net.train()
        r.optimizer.zero_grad()
        lg, v = r.net(torch.from_numpy(x).to(dt))
        pl = r.policy_loss_fn(F.log_softmax(lg, 1), torch.from_numpy(pi).to(dt))
        vl = r.value_loss_fn(v, torch.from_numpy(z).to(dt).reshape(-1, 1))
        (pl + vl).backward()
        return {n: p.grad.detach().double().numpy().copy() for n, p in r.net.named_parameters()}

    g32 = grads_of(ref, torch.float32)
    g64 = grads_of(r64, torch.float64)
    eng = m.engine
    dev = eng.device
    losses = torch.empty(3, device=dev)
    m.net.train()
    eng.train_backward(torch.from_numpy(x).to(dev), torch.from_numpy(pi).to(dev),
                       torch.from_numpy(z).reshape(-1, 1).to(dev), losses)
    torch.cuda.synchronize()
    print("losses", losses.cpu().numpy())
    for (n, p), gv in zip(m.net.named_parameters(), eng.grad_views):
        got = gv.detach().double().cpu().numpy()
        a, b = g32[n], g64[n]
        sc = np.abs(b).max() + 1e-30
        print(f"{n:32s} max|g|={sc:.3e} |gpu-64|/max={np.abs(got - b).max() / sc:.2e} "
              f"|cpu32-64|/max={np.abs(a - b).max() / sc:.2e} |gpu-cpu32|/max={np.abs(got - a).max() / sc:.2e}")
    # ReLU-mask agreement of the train-mode forward: GPU vs the fp32 and fp64 oracles
    def fwd_acts(r, dt):
        net = r.net
        out = {}
        with torch.no_grad():
            X = F.relu(net.bn(net.conv(torch.from_numpy(x).to(dt))))
            out["a0"] = X
            for i, blk in enumerate(net.res_blocks):
                z1 = blk.conv1(X)
                h = F.relu(blk.bn1(z1))
                X = F.relu(blk.bn2(blk.conv2(h)) + X)
                out[f"z1_{i}"], out[f"h_{i}"], out[f"xo_{i}"] = z1, h, X
        return {k: v.permute(0, 2, 3, 1).double().numpy() for k, v in out.items()}
    ref2 = RefModel(blocks, ch)
    load_numpy_state(ref2.net, st)
    ref2.net.train()
    c32 = fwd_acts(ref2, torch.float32)
    r642 = RefModel(blocks, ch, dtype=torch.float64)
    r642.net.load_state_dict(r64.net.state_dict())
    c64 = fwd_acts(r642, torch.float64)
    for i in range(blocks):
        for nm, key in (("h", "h"), ("xo", "xo")):
            gv = eng.debug_tensor(nm, B, i).double().cpu().numpy()
            a, b = c32[f"{key}_{i}"], c64[f"{key}_{i}"]
            print(f"block {i} {nm}: flips gpu-vs-64 {int(((gv > 0) != (b > 0)).sum())} cpu32-vs-64 "
                  f"{int(((a > 0) != (b > 0)).sum())}  max|gpu-64| {np.abs(gv - b).max():.2e} max|cpu32-64| "
                  f"{np.abs(a - b).max():.2e}")
    # BN running stats after the train-mode forward (ref: reference buffers after one step)
    sd = m.net.state_dict()
    rsd = ref.net.state_dict()   # ref has not updated: do a forward pass to update its running stats
    for k in sd:
        if "running" in k:
            d = np.abs(sd[k].cpu().numpy() - r64.net.state_dict()[k].numpy()).max()
            print(f"{k:32s} |gpu-fp64| {d:.2e}")


if __name__ == "__main__":
    main()
