"""Timeline of the persistent fixed-mode launch (pqp_persist.hip) at
n_dual = 1024: workgroup 0's per-wave events (s_memtime clocks) for updates
10..29 of a 1000-iteration solve: how long each wave waits for its y slice
(the cross-workgroup exchange), when its turn in the add chain comes, and how
long its adds take.  Run on the GPU box: python scripts/persist_trace.py"""
from __future__ import annotations

import ctypes as C
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main(N: int = 1024, iters: int = 1000, n_trace: int = 40):
    import numpy as np
    import torch

    import pqp_amd

    M = N // 2
    b = pqp_amd.Batch(1, N).generate(seed=1, inst0=0, M=M)
    P = dict(Qd=b.qd_rowmajor(0), Fd=b.Fd[0, :N].cpu().numpy(), Md=b.Md[:1].cpu().numpy(),
             Qp=np.zeros(M * M, np.float32), Qp_inv=np.zeros(M * M, np.float32), Fp=np.zeros(M, np.float32),
             Mp=np.zeros(1, np.float32), Gp=np.zeros(N * M, np.float32), Kp=np.zeros(N, np.float32), N=N, M=M)
    L = pqp_amd.lib()
    KB = (N + 3) // 4
    # pqp_persist.hip: slices of 24, 36, then 49 packets (persist_slice0)
    first = lambda w: 0 if w == 0 else (24 if w == 1 else 60 + (w - 2) * 49)  # noqa: E731
    W = 1
    while first(W) < KB:
        W += 1
    tr = torch.zeros(n_trace * W * 12, dtype=torch.int64, device="cuda")
    with pqp_amd.Problem(P) as prob:
        prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
        t0 = time.perf_counter()
        prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
        untraced = time.perf_counter() - t0
        assert L.pqp_tune_persist_trace(C.c_void_p(tr.data_ptr()), n_trace) == 0
        t0 = time.perf_counter()
        prob.solve(pqp_amd.MODE_FIXED, num_iter=iters)
        traced = time.perf_counter() - t0
        L.pqp_tune_persist_trace(None, 0)
    full = tr.cpu().numpy().astype(np.int64)
    t = full[: n_trace * W * 4].reshape(n_trace, W, 4)
    fine = full[n_trace * W * 4:].reshape(n_trace, W, 8)
    lo, hi = 10, 30
    period = float(np.median(np.diff(t[lo:hi, 0, 2])))  # wave 0's turn, update to update
    us_per_update = untraced / (iters - 1) * 1e6
    out = {"n_dual": N, "waves": W, "us_per_update_untraced": us_per_update,
           "us_per_update_traced": traced / (iters - 1) * 1e6, "clocks_per_update": period,
           "clock_GHz_implied": period / us_per_update / 1e3, "per_wave_median_clocks": {}}
    for w in range(W):
        ev = t[lo:hi, w, :]
        out["per_wave_median_clocks"][f"wave{w}"] = {
            "y_wait (sweep start -> staged)": float(np.median(ev[:, 1] - ev[:, 0])),
            "staged -> turn": float(np.median(ev[:, 2] - ev[:, 1])),
            "adds (turn -> chain done)": float(np.median(ev[:, 3] - ev[:, 2])),
        }
    # critical path split: last wave's chain done -> wave 0 staged (exchange),
    # wave 0 staged -> turn (products), turn(w) -> turn(w+1) (adds + hand-off)
    ex = [t[u + 1, 0, 1] - t[u, W - 1, 3] for u in range(lo, hi)]
    out["exchange_clocks (last wave done u -> wave 0 staged u+1)"] = float(np.median(ex))
    out["handoff_clocks (wave w done -> wave w+1 turn)"] = float(np.median(
        [t[u, w + 1, 2] - t[u, w, 3] for u in range(lo, hi) for w in range(W - 1)]))
    out["handoff_clocks_per_pair"] = {f"{w}->{w + 1}": float(np.median([t[u, w + 1, 2] - t[u, w, 3] for u in range(lo, hi)]))
                                      for w in range(W - 1)}
    out["raw_update_10"] = (t[10] - t[10, 0, 0]).tolist()
    # each later wave's chain in sevenths: clocks per seventh (median over updates)
    out["chain_sevenths_clocks"] = {
        f"wave{w}": np.median(np.diff(fine[lo:hi, w, :], axis=1), axis=0).tolist() for w in range(1, W)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
