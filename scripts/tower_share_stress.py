"""Persistent-tower dependency waits with the GPU to itself vs shared by several
processes (what let a waiter poll for seconds in the round-4
shared-GPU rehearsal).

Each worker process builds the 6x128 net, forces the persistent 128x64 tower
(key 5 = 1, key 6 = 8), sets the awake-time wait bound (key 14, microseconds) and
runs back-to-back forwards at alternating batches for --seconds.  Every launch is
synchronised and settled with engine.recover (a timed-out launch is recomputed per
layer) and compared bitwise with a per-layer reference computed first.  The worker
prints one JSON line: launches, timeouts, recoveries, mismatches after recovery, and
the tower's wait record (azg_pv_tower_diag: wait histogram, the first timed-out wait
with waiter / producer placement).

The parent never touches the GPU: it starts the workers as child processes (they run
concurrently on the same GPU) and writes their lines to --out.

    python scripts/tower_share_stress.py --procs 2 --seconds 30 --wait-us 20000 \
        --out gpurun_out/share2.json
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def worker(args):
    sys.path[:0] = [os.path.join(REPO, "alphazero-gomoku_amd"), REPO]
    import numpy as np
    import torch
    import _native
    from network import PyTorchModel
    from synth import synth_encoded
    lib = _native.load_library()
    torch.manual_seed(0)
    m = PyTorchModel(board_size=15, device="cuda", n_res_blocks=6, channels=128)
    m.net.eval()
    eng = m.engine
    batches = [int(b) for b in args.batches.split(",")]
    xs = {B: torch.from_numpy(synth_encoded(B, seed=B)).cuda() for B in batches}
    outs = {B: (torch.empty((B, 225), device="cuda"), torch.empty((B, 1), device="cuda")) for B in batches}
    lib.azg_pv_set_tuning(5, 0)
    ref = {}
    for B in batches:
        eng.forward_into(xs[B], *outs[B])
        ref[B] = (outs[B][0].clone(), outs[B][1].clone())
    lib.azg_pv_set_tuning(5, 1)
    lib.azg_pv_set_tuning(6, 8)
    for B in batches:   # warm (code objects)
        eng.forward_into(xs[B], *outs[B])
    torch.cuda.synchronize()
    lib.azg_pv_set_tuning(14, args.wait_us)
    lib.azg_pv_set_tuning(18, 0)   # no per-layer breaker: every launch runs the tower
    eng.clear_status()
    eng.tower_diag_clear()
    launches = timeouts = mism = 0
    per_batch = {B: 0 for B in batches}
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < args.seconds:
        B = batches[i % len(batches)]
        i += 1
        eng.forward_into(xs[B], *outs[B])
        seq = eng.last_seq()
        torch.cuda.synchronize()
        launches += 1
        per_batch[B] += 1
        if eng.recover(seq):
            timeouts += 1
            torch.cuda.synchronize()
        if not (torch.equal(outs[B][0], ref[B][0]) and torch.equal(outs[B][1], ref[B][1])):
            mism += 1
    dt = time.perf_counter() - t0
    d = eng.tower_diag()
    lib.azg_pv_set_tuning(14, -1)
    print(json.dumps({"pid": os.getpid(), "seconds": round(dt, 2), "launches": launches, "per_batch": per_batch,
                      "timed_out_launches": timeouts, "recoveries": eng.recoveries,
                      "mismatches_after_recovery": mism, "status_after": int(lib.azg_pv_status(eng.h)),
                      "diag": d}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=30.0)
    ap.add_argument("--wait-us", type=int, default=20000, help="key 14: awake-time bound per wait")
    ap.add_argument("--batches", default="512,3456")
    ap.add_argument("--out", default=None)
    ap.add_argument("--worker", action="store_true")
    args = ap.parse_args()
    if args.worker:
        worker(args)
        return
    cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--seconds", str(args.seconds), "--wait-us",
           str(args.wait_us), "--batches", args.batches]
    procs = [subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True) for _ in range(args.procs)]
    lines, rc = [], 0
    for p in procs:
        out, _ = p.communicate(timeout=args.seconds + 600)
        rc |= p.returncode
        lines += [json.loads(l) for l in out.splitlines() if l.startswith("{")]
    res = {"procs": args.procs, "seconds": args.seconds, "wait_us": args.wait_us, "batches": args.batches,
           "workers": lines}
    txt = json.dumps(res, indent=1)
    print(txt)
    if args.out:
        os.makedirs(os.path.dirname(args.out) or ".", exist_ok=True)
        with open(args.out, "w") as f:
            f.write(txt)
    sys.exit(rc)


if __name__ == "__main__":
    main()
