"""GPU debug: compare train-step intermediates (engine workspace) with the oracle
autograd.  Run on the GPU box:  python scripts/debug_train.py [blocks ch B]"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "alphazero-gomoku_amd"), os.path.join(REPO, "tests")]

import numpy as np
import torch
import torch.nn.functional as F

from conftest import golden_state, load_golden
from oracle.boards import encode_batch, synth_positions, synth_targets
from oracle.ref_net import RefModel, load_numpy_state


def main():
    blocks, ch, B = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (3, 64, 128)
    torch.set_num_threads(8)
    tag = f"{blocks}x{ch}"
    g = load_golden(tag)
    st = golden_state(g)
    from network import PyTorchModel
    m = PyTorchModel(device="cuda", n_res_blocks=blocks, channels=ch)
    m.net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    ref = RefModel(blocks, ch)
    load_numpy_state(ref.net, st)
    b, p = synth_positions(B, seed=77 + B)
    x = encode_batch(b, p)
    pi, z = synth_targets(B, seed=78 + B)

    net = ref.net
    net.train()
    xt = torch.from_numpy(x)
    acts = {}
    z0 = net.conv(xt); z0.retain_grad(); acts["z0"] = z0
    a0 = F.relu(net.bn(z0)); a0.retain_grad(); acts["a0"] = a0
    X = a0
    for i, blk in enumerate(net.res_blocks):
        z1 = blk.conv1(X); z1.retain_grad(); acts[f"z1{i}"] = z1
        h = F.relu(blk.bn1(z1)); h.retain_grad(); acts[f"h{i}"] = h
        z2 = blk.conv2(h); z2.retain_grad(); acts[f"z2{i}"] = z2
        xo = F.relu(blk.bn2(z2) + X); xo.retain_grad(); acts[f"xo{i}"] = xo
        X = xo
    pp = F.relu(net.policy_bn(net.policy_conv(X)))
    logits = net.policy_fc(pp.view(B, -1))
    v = F.relu(net.value_bn(net.value_conv(X)))
    v = torch.tanh(net.value_fc2(F.relu(net.value_fc1(v.view(B, -1)))))
    loss = ref.policy_loss_fn(F.log_softmax(logits, 1), torch.from_numpy(pi)) + ref.value_loss_fn(v, torch.from_numpy(z))
    loss.backward()

    eng = m.engine
    dev = eng.device
    losses = torch.empty(3, device=dev)
    eng.train_backward(torch.from_numpy(x).to(dev), torch.from_numpy(pi).to(dev), torch.from_numpy(z).to(dev), losses)

    def cmp(name, got, want):
        want = want.detach().permute(0, 2, 3, 1).numpy()
        got = got.cpu().numpy()
        err = np.abs(got - want)
        scale = np.abs(want).max()
        idx = np.unravel_index(err.argmax(), err.shape)
        print(f"{name:10s} max|d|={err.max():.3e} scale={scale:.3e} rel={err.max() / (scale + 1e-30):.2e} at {idx}")
        return err

    cmp("z0", eng.debug_tensor("z0", B), acts["z0"])
    cmp("a0", eng.debug_tensor("a0", B), acts["a0"])
    for i in range(blocks):
        cmp(f"z1[{i}]", eng.debug_tensor("z1", B, i), acts[f"z1{i}"])
        cmp(f"h[{i}]", eng.debug_tensor("h", B, i), acts[f"h{i}"])
        cmp(f"z2[{i}]", eng.debug_tensor("z2", B, i), acts[f"z2{i}"])
        cmp(f"xo[{i}]", eng.debug_tensor("xo", B, i), acts[f"xo{i}"])
    if os.environ.get("AZG_DEBUG_SNAP"):
        names = [f"xo{blocks - 1}"] + [f"xo{blocks - 2 - k}" if blocks - 2 - k >= 0 else "a0" for k in range(blocks)]
        for k, nm in enumerate(names):
            err = cmp(f"snap{k}=d{nm}", eng.debug_tensor("snap", B, k), acts[nm].grad)
            bb = np.unravel_index(err.argmax(), err.shape)[0]
            e = err[bb].max(axis=2)
            print(f"  board {bb} err by (y,x) / max:\n", np.array2string(e / (e.max() + 1e-30), precision=1, max_line_width=200))
    # final backward state: gX = d/d a0, DH = d/d h[0], GR = block-0 residual dy
    cmp("gX=da0", eng.debug_tensor("gX", B), acts["a0"].grad)
    cmp("DH=dh0", eng.debug_tensor("DH", B), acts["h0"].grad)
    dy0 = acts["xo0"].grad * (acts["xo0"] > 0)
    cmp("GR=dy0", eng.debug_tensor("GR", B), dy0)
    err = cmp("DZ=dz0", eng.debug_tensor("DZ", B), acts["z0"].grad)
    e = err.max(axis=(0, 3))
    print("DZ err by (y,x):\n", np.array2string(e / (e.max() + 1e-30), precision=2, max_line_width=200))


if __name__ == "__main__":
    main()
