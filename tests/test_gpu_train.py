"""GPU parity of the train step (azg_pv_train_backward + azg_pv_train_apply via
PyTorchModel.train_batch) against the CPU oracle (autograd) and the reference
goldens.

Tolerances (fp32; stated per check):
  * gradients: |g_gpu - g_64| <= 2e-5 * max|g_64| (per tensor) + 1e-8 against fp64
    autograd that uses the GPU's own ReLU masks; every mask flip (GPU vs the exact
    fp64 pre-activation) must sit at |pre-activation| <= max(1e-6 x the layer's max,
    2 x the GPU's own max error on that layer), and flips vs the fp32 oracle's own
    masks are counted and printed;
  * losses: 1e-5 relative;
  * params after 2 steps (clip + Adam): <= 1 % of elements beyond 2e-5 -- against
    the fp64 trajectory with the GPU's masks (all params), and against the
    reference goldens for every param not below a mask flip (a flip at block k
    perturbs the gradients of blocks <= k and the stem at ~1e-3 relative, and Adam
    turns that into +-lr; those blocks are reported, and covered by the fp64
    trajectory test).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import golden_state, has_gpu, load_golden
from oracle.boards import encode_batch, synth_positions, synth_targets
from oracle.ref_net import RefModel, load_numpy_state, state_to_numpy

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not has_gpu(), reason="needs a HIP device")]


def make_model(blocks, ch, state=None, seed=0):
    from network import PyTorchModel
    torch.manual_seed(seed)
    m = PyTorchModel(board_size=15, device="cuda", n_res_blocks=blocks, channels=ch)
    if state is not None:
        m.net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in state.items()})
    return m


def oracle_grads(ref, x, pi, z):
    """network.py:213-222 up to loss.backward() (no clip, no step)."""
    ref.net.train()
    ref.optimizer.zero_grad()
    logits, values = ref.net(torch.from_numpy(x))
    pl = ref.policy_loss_fn(F.log_softmax(logits, dim=1), torch.from_numpy(pi))
    vl = ref.value_loss_fn(values, torch.from_numpy(z))
    (pl + vl).backward()
    return ({n: p.grad.detach().numpy().copy() for n, p in ref.net.named_parameters()},
            (float(pl), float(vl), float(pl + vl)))


def mask_flips(mk: dict, pre: dict, gpu_err: dict = None):
    """Per masked ReLU: positions where the GPU's mask disagrees with the exact
    (fp64) pre-activation's sign, and the largest |pre| there relative to the
    layer's max|pre|."""
    out = {}
    for k, m in mk.items():
        p = pre[k]
        flip = (m > 0) != (p > 0)
        n = int(flip.sum())
        mx = float(np.abs(p).max()) + 1e-30
        worst = float(np.abs(p[flip]).max()) if n else 0.0
        out[k] = (n, worst, mx)
    return out


def flipped_block(flips: dict, blocks: int) -> int:
    """Highest residual block whose gradients a flip perturbs (-1: none, blocks:
    a head mask flipped, so every block is below it)."""
    hi = -1
    for k, (n, _, _) in flips.items():
        if not n:
            continue
        if k == "a0":
            hi = max(hi, 0)
        elif k[0] in "hx":
            hi = max(hi, int(k.lstrip("hxo")))
        else:
            hi = blocks
    return hi


def block_of(name: str, blocks: int) -> int:
    """Residual block index of a parameter (stem: 0, heads: blocks)."""
    if name.startswith("res_blocks."):
        return int(name.split(".")[1])
    if name.startswith("conv.") or name.startswith("bn."):
        return 0
    return blocks


def gpu_masks(eng, blocks, B):
    """0/1 ReLU masks of the GPU's own train-mode forward (NCHW / [B, n])."""
    nchw = lambda t: (t > 0).double().permute(0, 3, 1, 2).cpu().numpy()
    mk = {"a0": nchw(eng.debug_tensor("a0", B))}
    for i in range(blocks):
        mk[f"h{i}"] = nchw(eng.debug_tensor("h", B, i))
        mk[f"xo{i}"] = nchw(eng.debug_tensor("xo", B, i))
    for n in ("fp", "fv", "hv"):
        mk[n] = (eng.debug_tensor(n, B) > 0).double().cpu().numpy()
    return mk


@pytest.mark.parametrize("tag,blocks,ch,B", [("3x64", 3, 64, 128), ("6x128", 6, 128, 128), ("3x64", 3, 64, 37),
                                             (None, 2, 128, 16), (None, 10, 256, 12),
                                             # configs[4]'s net at the bench's train shape (B = 128)
                                             pytest.param(None, 10, 256, 128, marks=pytest.mark.timeout(900)),
                                             # fused BN apply / finalize at 160 and 48 samples (C = 64 / 256)
                                             (None, 2, 64, 160), (None, 2, 256, 48),
                                             # B > kHeadFoldMaxB (512): the unfolded head-BN backward
                                             # (head_bn_bwd_fin_kernel -> heads_bwd_fused with dg_nwg = 0)
                                             pytest.param(None, 1, 64, 520, marks=pytest.mark.timeout(600))])
def test_gradients_match_oracle(tag, blocks, ch, B):
    """Gradients vs fp64 autograd with the GPU's ReLU masks (oracle.masked_grads_fp64):
    |g_gpu - g_64| <= 2e-5 * max|g_64| + 1e-8 per tensor.  The fp32 CPU oracle (own
    masks) is reported beside it: mask flips at near-zero pre-activations make two
    correct fp32 implementations differ by up to ~1e-2 relative there."""
    import os
    from oracle.ref_net import masked_grads_fp64
    torch.set_num_threads(max(8, min(16, len(os.sched_getaffinity(0)))))
    if tag is None:      # no golden at this size (Pente config 10x256): seeded init state
        torch.manual_seed(blocks * 1000 + ch)
        st = state_to_numpy(RefModel(blocks, ch).net)
    else:
        st = golden_state(load_golden(tag))
    m = make_model(blocks, ch, st)
    b, p = synth_positions(B, seed=77 + B)
    x = encode_batch(b, p)
    pi, z = synth_targets(B, seed=78 + B)
    eng = m.engine
    dev = eng.device
    losses = torch.empty(3, device=dev)
    eng.train_backward(torch.from_numpy(x).to(dev), torch.from_numpy(pi).to(dev), torch.from_numpy(z).to(dev),
                       losses)
    torch.cuda.synchronize()
    eng.check_status()   # no in-kernel wait of the step timed out
    mk = gpu_masks(eng, blocks, B)
    want, (pl, vl), pre = masked_grads_fp64(st, blocks, ch, x, pi, z, mk, return_pre=True)
    np.testing.assert_allclose(losses.cpu().numpy(), [pl, vl, pl + vl], rtol=1e-5, atol=1e-7)
    # mask flips: GPU vs exact, and GPU vs the fp32 oracle's own masks
    flips = mask_flips(mk, pre)
    ref_masks = fp32_masks(st, blocks, ch, x)
    nchw = lambda t: t.permute(0, 3, 1, 2).double().cpu().numpy()
    gpu_pre = {"a0": nchw(eng.debug_tensor("a0", B))}
    for i in range(blocks):
        gpu_pre[f"h{i}"] = nchw(eng.debug_tensor("h", B, i))
        gpu_pre[f"xo{i}"] = nchw(eng.debug_tensor("xo", B, i))
    for n_ in ("fp", "fv", "hv"):
        gpu_pre[n_] = eng.debug_tensor(n_, B).double().cpu().numpy()
    for k, (n, worst, mx) in flips.items():
        n32 = int(((mk[k] > 0) != (ref_masks[k] > 0)).sum())
        # GPU's own error on this layer (post-ReLU values, where both are positive)
        err = float(np.abs(gpu_pre[k] - np.maximum(pre[k], 0)).max()) if k in gpu_pre else 0.0
        if n or n32:
            print(f"mask flips {k}: gpu-vs-fp64 {n} (worst |pre| {worst:.2e} = {worst / mx:.1e} x max), "
                  f"gpu-vs-fp32-oracle {n32}, gpu max err {err:.2e}")
        assert worst <= max(1e-6 * mx, 2 * err), (k, n, worst, mx, err)
    ref = RefModel(blocks, ch)
    load_numpy_state(ref.net, st)
    want32, _ = oracle_grads(ref, x, pi, z)
    bad = []
    for n, prm in m.net.named_parameters():
        gg = prm.grad.detach().cpu().numpy().astype(np.float64)
        w = want[n]
        err, scale = np.abs(gg - w).max(), np.abs(w).max()
        e32 = np.abs(want32[n] - w).max()
        print(f"{tag} B={B} {n:28s} |gpu-64|={err:.2e} |cpu32-64|={e32:.2e} max|g|={scale:.2e} "
              f"rel={err / (scale + 1e-30):.1e}")
        if err > 2e-5 * scale + 1e-8:
            bad.append(n)
    assert not bad, bad


def fp32_masks(st, blocks, ch, x):
    """The fp32 CPU oracle's own ReLU masks (train-mode forward), NCHW / [B, n]."""
    net = RefModel(blocks, ch).net
    load_numpy_state(net, st)
    net.train()
    out = {}
    with torch.no_grad():
        h = F.relu(net.bn(net.conv(torch.from_numpy(x))))
        out["a0"] = h
        for i, blk in enumerate(net.res_blocks):
            hh = F.relu(blk.bn1(blk.conv1(h)))
            out[f"h{i}"] = hh
            h = F.relu(blk.bn2(blk.conv2(hh)) + h)
            out[f"xo{i}"] = h
        B = h.shape[0]
        p = F.relu(net.policy_bn(net.policy_conv(h))).reshape(B, -1)
        v = F.relu(net.value_bn(net.value_conv(h))).reshape(B, -1)
        out["fp"], out["fv"], out["hv"] = p, v, F.relu(net.value_fc1(v))
    return {k: (t > 0).double().numpy() for k, t in out.items()}


def _golden_steps(g):
    for s in range(2):
        yield encode_batch(g[f"train/boards{s}"], g[f"train/players{s}"]), g[f"train/pi{s}"], g[f"train/z{s}"]


@pytest.mark.parametrize("tag,blocks,ch", [("3x64", 3, 64), ("6x128", 6, 128)])
def test_train_batch_matches_reference_goldens(tag, blocks, ch):
    """Two train_batch steps vs the reference's own two steps.  Losses to 1e-5; the
    optimizer state in torch format; params <= 1 % beyond 2e-5 for every block above
    the highest GPU mask flip (flips: GPU masks vs the exact fp64 pre-activations of
    the GPU's own params, see the module docstring); the flipped-below blocks are
    reported here and gated by test_two_steps_match_fp64_trajectory."""
    from oracle.ref_net import masked_grads_fp64
    g = load_golden(tag)
    m = make_model(blocks, ch, golden_state(g))
    losses, hi = [], -1
    for x, pi, z in _golden_steps(g):
        st = state_to_numpy(m.net)
        li = m.train_batch(x, pi, z)
        losses.append([li["policy_loss"], li["value_loss"], li["total_loss"]])
        mk = gpu_masks(m.engine, blocks, len(x))
        _, _, pre = masked_grads_fp64(st, blocks, ch, x, pi, z, mk, return_pre=True)
        fl = mask_flips(mk, pre)
        print({k: v[0] for k, v in fl.items() if v[0]})
        hi = max(hi, flipped_block(fl, blocks))
    np.testing.assert_allclose(np.array(losses), g["train/losses"], rtol=1e-5, atol=1e-6)
    bad = tot = 0
    for n, p in m.net.named_parameters():
        idx = g[f"train/idx/{n}"]
        d = np.abs(p.detach().reshape(-1).cpu().numpy()[idx] - g[f"train/param/{n}"])
        assert d.max() <= 2 * 2 * 1e-3 * 1.01, (n, d.max())      # two Adam steps, any sign
        nb = int((d > 2e-5).sum())
        if block_of(n, blocks) > hi:
            bad += nb
            tot += d.size
        elif nb:
            print(f"{n}: {nb}/{d.size} beyond 2e-5 (below a mask flip at block {hi})")
    print(f"highest flipped block {hi}: {bad}/{tot} compared elements beyond 2e-5")
    assert bad <= 0.01 * tot, (bad, tot)
    sd = m.net.state_dict()
    for k in sd:
        if ("running" in k or "num_batches" in k) and block_of(k, blocks) > hi:
            # step-2 stats come from step-1 params that already differ (see above)
            np.testing.assert_allclose(sd[k].cpu().numpy(), g[f"train/buf/{k}"], atol=5e-4, rtol=1e-3, err_msg=k)
    assert int(sd["bn.num_batches_tracked"]) == int(g["train/buf/bn.num_batches_tracked"])
    # optimizer state in torch format
    osd = m.optimizer.state_dict()
    assert len(osd["state"]) == len(list(m.net.parameters()))
    assert float(osd["state"][0]["step"]) == 2.0


@pytest.mark.parametrize("tag,blocks,ch", [("3x64", 3, 64), ("6x128", 6, 128)])
def test_two_steps_match_fp64_trajectory(tag, blocks, ch):
    """Two GPU train_batch steps vs the exact trajectory: fp64 autograd with the
    GPU's ReLU masks of each step + torch clip_grad_norm_(3.0) + Adam(1e-3, wd 1e-4)
    in fp64.  Every param: <= 1 % of elements beyond 2e-5 (Adam's first steps move
    every element by ~lr * sign(g), so only gradients within fp32 rounding of zero
    may disagree)."""
    from oracle.ref_net import RefNet, masked_grads_fp64
    g = load_golden(tag)
    st0 = golden_state(g)
    m = make_model(blocks, ch, st0)
    net64 = RefNet(blocks, ch).double()
    load_numpy_state(net64, {k: (np.asarray(v, np.float64) if np.asarray(v).dtype.kind == "f" else v)
                             for k, v in st0.items()})
    opt = torch.optim.Adam(net64.parameters(), lr=1e-3, weight_decay=1e-4)
    for x, pi, z in _golden_steps(g):
        m.train_batch(x, pi, z)
        mk = gpu_masks(m.engine, blocks, len(x))
        st = {k: v.detach().numpy() for k, v in net64.state_dict().items()}
        grads, _ = masked_grads_fp64(st, blocks, ch, x, pi, z, mk)
        for n, p in net64.named_parameters():
            p.grad = torch.from_numpy(grads[n])
        torch.nn.utils.clip_grad_norm_(net64.parameters(), 3.0)
        opt.step()
    bad = tot = 0
    want = dict(net64.named_parameters())
    for n, p in m.net.named_parameters():
        d = np.abs(p.detach().double().cpu().numpy() - want[n].detach().numpy())
        nb = int((d > 2e-5).sum())
        if nb:
            print(f"{n}: {nb}/{d.size} beyond 2e-5, max {d.max():.2e}")
        assert d.max() <= 2 * 2 * 1e-3 * 1.01, (n, d.max())
        bad += nb
        tot += d.size
    print(f"{tag}: {bad}/{tot} params beyond 2e-5 of the fp64 trajectory")
    assert bad <= 0.01 * tot, (bad, tot)


def test_clip_and_adam_match_torch():
    """azg_pv_train_apply == clip_grad_norm_(3.0) + torch Adam on identical grads,
    including a clipping case (grads scaled up) and weight decay."""
    m = make_model(1, 64)
    eng = m.engine
    torch.manual_seed(3)
    params0 = eng.flat_params.detach().cpu().clone()
    for scale in (1e-3, 10.0):
        grads = torch.randn(eng.nparam) * scale
        eng.flat_grads.copy_(grads.to(eng.device))
        m.optimizer.hip_step(3.0)
        torch.cuda.synchronize()
    # torch reference on CPU
    p = torch.nn.Parameter(params0.clone())
    opt = torch.optim.Adam([p], lr=1e-3, weight_decay=1e-4)
    torch.manual_seed(3)
    for scale in (1e-3, 10.0):
        p.grad = torch.randn(eng.nparam) * scale
        torch.nn.utils.clip_grad_norm_([p], 3.0)
        opt.step()
    got = eng.flat_params.detach().cpu()
    np.testing.assert_allclose(got.numpy(), p.detach().numpy(), atol=2e-6, rtol=0)
    st = opt.state[p]
    np.testing.assert_allclose(m.optimizer.flat_exp_avg.cpu().numpy(), st["exp_avg"].numpy(), rtol=1e-5, atol=1e-9)
    # v ~ g^2 doubles the relative error of the clip coefficient, which the kernel
    # takes from an fp64 global norm and torch from an fp32 vector norm (7e-6 apart)
    np.testing.assert_allclose(m.optimizer.flat_exp_avg_sq.cpu().numpy(), st["exp_avg_sq"].numpy(), rtol=1e-4,
                               atol=1e-12)


def test_train_then_predict_uses_new_weights():
    m = make_model(2, 64)
    b, p = synth_positions(64, seed=5)
    x = encode_batch(b, p)
    pi, z = synth_targets(64, seed=6)
    p0, _ = m.predict(x)
    m.train_batch(x, pi, z, epochs=3)
    p1, v1 = m.predict(x)
    ref = RefModel(2, 64)
    load_numpy_state(ref.net, state_to_numpy(m.net))
    rp, rv = ref.predict(x)
    assert not np.allclose(p0, p1)
    np.testing.assert_allclose(p1, rp, atol=1e-5)
    np.testing.assert_allclose(v1, rv, atol=1e-5)


def train_state_after(x, pi, z, blocks, ch, steps=2, seed=3):
    """params, BN buffers, grads and Adam moments after `steps` train steps."""
    m = make_model(blocks, ch, seed=seed)
    for _ in range(steps):
        m.train_batch(x, pi, z)
    got = [t.detach().cpu().clone() for t in m.net.state_dict().values()]
    got += [m.engine.flat_grads.cpu().clone(), m.optimizer.flat_exp_avg.cpu().clone(),
            m.optimizer.flat_exp_avg_sq.cpu().clone()]
    return got


@pytest.mark.parametrize("key,values", [(23, (1, 0)), (24, (1, 0)), (44, (0, 512, 97)), (48, (1, 0))])
def test_train_schedule_keys_bitwise(key, values):
    """The train step's product tuning keys change only the schedule: where the forward
    BN applies run (23: folded into the next conv's halo staging, or separate passes),
    where the BN finalizes run (24: by the producing conv's last workgroup, or separate
    kernels) and how many workgroups the BN apply passes use (44, grid-stride): two
    steps from one state must give bitwise-identical params, grads, BN buffers and Adam
    moments under every value.  Key 48 selects the weight-grad tile (1: round 5's row-table /
    buffer-DMA / MFMA-layout-slab form, 0: round 4's): the same MFMA chain per output and
    the same slab sum order."""
    import _native
    lib = _native.load_library()
    b, p = synth_positions(128, seed=91)
    x = encode_batch(b, p)
    pi, z = synth_targets(128, seed=92)
    prev = lib.azg_pv_set_tuning(key, values[0])
    ref = None
    try:
        for v in values:
            lib.azg_pv_set_tuning(key, v)
            got = train_state_after(x, pi, z, 2, 128)
            if ref is None:
                ref = got
            else:
                assert all(torch.equal(a, c) for a, c in zip(ref, got)), (key, v)
    finally:
        lib.azg_pv_set_tuning(key, prev)


@pytest.mark.parametrize("key,value", [(27, 16), (27, 64), (49, 0), (49, 1)])
@pytest.mark.parametrize("tag,blocks,ch,B", [("6x128", 6, 128, 128), ("3x64", 3, 64, 37)])
def test_train_sum_order_variants_match_oracle(key, value, tag, blocks, ch, B):
    """The weight-grad split count (key 27) changes an fp32 summation order, and key 49 = 0 / 1
    runs the forward convs in fp32 MFMA / three split-fp16 products instead of the default
    four: each holds the
    oracle tolerance of test_gradients_match_oracle (no bitwise test); 64 splits are the
    largest slab the workspace holds."""
    import _native
    lib = _native.load_library()
    prev = lib.azg_pv_set_tuning(key, value)
    try:
        test_gradients_match_oracle(tag, blocks, ch, B)
    finally:
        lib.azg_pv_set_tuning(key, prev)


def _overflow_model(lib=None):
    """2x64 net whose stem BN (gamma x 1e6, beta + 1e5) drives every staged activation of
    the first split-fp16 train conv beyond fp16's range (65504)."""
    m = make_model(2, 64, seed=5)
    with torch.no_grad():
        m.net.bn.weight.mul_(1e6)
        m.net.bn.bias.add_(1e5)
    m.engine.mark_dirty()
    return m


def _full_state(m):
    torch.cuda.synchronize()
    st = [t.detach().cpu().clone() for t in m.net.state_dict().values()]   # params, BN stats, counters
    st += [m.optimizer.flat_exp_avg.cpu().clone(), m.optimizer.flat_exp_avg_sq.cpu().clone(),
           torch.tensor([float(m.optimizer.get_step())])]
    return st


def test_train_h3_range_overflow_is_redone_in_fp32():
    """VERDICT r5 next 2 / ADVICE r5: a split-fp16 train forward (key 49 = 2, the default)
    that meets an activation beyond fp16's range must not corrupt the model.  The step's
    skip word (the gradient buffer's last float) makes azg_pv_train_apply leave params,
    moments and gradients alone and restore the BN running stats and counters; train_batch
    sees it with the losses and redoes the step with fp32 forward convs.  Checked: the
    device-skipped step leaves params, moments and BN buffers bitwise as they were; the
    redone step returns finite losses, and its params, moments, BN buffers, counters and
    Adam step are bitwise those of a key-49 = 0 step."""
    import _native
    lib = _native.load_library()
    b, p = synth_positions(32, seed=91)
    x = encode_batch(b, p)
    pi, z = synth_targets(32, seed=92)
    prev = lib.azg_pv_set_tuning(49, 2)
    try:
        # 1. the device skip alone (pipelined call: no redo)
        m = _overflow_model()
        before = _full_state(m)
        dev = m.engine.device
        xd, pd, zd = (torch.from_numpy(np.asarray(a, np.float32)).to(dev) for a in (x, pi, z.reshape(-1, 1)))
        m.train_batch_device(xd, pd, zd, return_tensor=True)
        torch.cuda.synchronize()
        assert m.engine.train_skips() == 1
        m._settle_skips()                      # gives the skipped step's Adam number back
        after = _full_state(m)
        assert all(torch.equal(a, c) for a, c in zip(before, after)), "a skipped step changed the model"
        # 2. train_batch: skipped on the device, redone in fp32
        got = m.train_batch(x, pi, z)
        assert all(np.isfinite(v) for v in got.values()), got
        assert m.engine.train_recoveries == 1 and m.engine.train_skips() == 2
        lib.azg_pv_set_tuning(49, 0)
        r = _overflow_model()
        want = r.train_batch(x, pi, z)
        lib.azg_pv_set_tuning(49, 2)
        assert got == want, (got, want)
        assert all(torch.equal(a, c) for a, c in zip(_full_state(m), _full_state(r))), "redo != key-49 = 0 step"
        print(f"overflow step redone in fp32: losses {got}")
        m.engine.clear_status()
        assert lib.azg_pv_status(m.engine.h) == 0 and m.engine.train_skips() == 0
    finally:
        lib.azg_pv_set_tuning(49, prev)
