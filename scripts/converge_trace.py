"""Timeline of the persistent converge launch (pqp_converge.hip) on one
synthetic problem: s_memrealtime marks (100 MHz, chip-wide) of workgroup 0 of
every role, per iterate and wave: start, inputs staged, turn (running sums in;
DEC: its dot summed), done.  Prints medians over steady-state iterates in us:
each wave's period and phases, and the hand-over latencies between roles."""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))

ROLES = ("UPD", "T1", "T2", "T3")
KW = 7  # wave slots per role (pqp_converge.hip kMaxW)
NIDS = 5 * KW  # 4 chain roles x KW wave slots, then DEC's kDecW = KW waves (pqp_converge.hip kTraceIds)
# DEC's waves: 0 decides; 1, 2 dot 1 (Fd.Y) of even / odd iterates; 3, 4 dot 4
# ((Y'Qd).Y) of even / odd iterates; 5 dots 2 and 3 of every iterate


def waves_of(K):
    # pqp_converge.hip: slices of 24, 36, then 49 packets (slice0_of)
    KB = (K + 3) // 4
    first = lambda w: 0 if w == 0 else (24 if w == 1 else 60 + (w - 2) * 49)  # noqa: E731
    W = 1
    while first(W) < KB:
        W += 1
    return W


def main(N: int = 1024, cap: int = 200, n_trace: int = 120):
    import numpy as np
    import torch

    import pqp_amd

    M = N // 2
    pb = pqp_amd.ProblemBatch.synthetic(1, 0, 1, N, M)
    P = pb.problem(0)
    del pb
    L = pqp_amd.lib()
    tr = torch.zeros(2 * n_trace * NIDS * 4, dtype=torch.int64, device="cuda")
    with pqp_amd.Problem(P) as prob:
        prob.solve(max_updates=cap)
        L.pqp_tune_converge_trace(pqp_amd.C.c_void_p(tr.data_ptr()), n_trace)
        r = prob.solve(max_updates=cap)
        L.pqp_tune_converge_trace(None, 0)
    torch.cuda.synchronize()
    both = tr.cpu().numpy().reshape(2, n_trace, NIDS, 4).astype(np.float64)
    t = both[0] / 100.0  # us
    clk = both[1]  # shader clocks
    lo, hi = n_trace // 3, n_trace - 10
    W = {"UPD": waves_of(N), "T1": waves_of(N), "T2": waves_of(M), "T3": waves_of(M)}
    med = lambda x: float(np.median(x))
    out = {"n_dual": N, "m": M, "h": r["h"], "iterates": [lo, hi], "roles": {}}
    # the shader clock the launch ran at: clocks over chip time, per role's wave 0
    out["clock_GHz"] = {role: float((clk[hi, ri * KW, 0] - clk[lo, ri * KW, 0]) / ((t[hi, ri * KW, 0] - t[lo, ri * KW, 0]) * 1e3))
                        for ri, role in enumerate(ROLES)}
    for ri, role in enumerate(ROLES):
        for w in range(W[role]):
            i = ri * KW + w
            x = t[lo:hi, i]
            out["roles"][f"{role}.w{w}"] = {
                "period": med(np.diff(t[lo:hi + 1, i, 0])), "stage": med(x[:, 1] - x[:, 0]),
                "turn_wait": med(x[:, 2] - x[:, 1]) if w else 0.0, "adds": med(x[:, 3] - x[:, 2]) if w else
                med(x[:, 3] - x[:, 1])}
    x = t[lo:hi, 4 * KW]
    out["roles"]["DEC.w0 (decision)"] = {"period": med(np.diff(t[lo:hi + 1, 4 * KW, 0])),
                                         "feasibility": med(x[:, 1] - x[:, 0]), "dots_wait": med(x[:, 2] - x[:, 1]),
                                         "decide": med(x[:, 3] - x[:, 2])}
    for d in range(1, KW):
        i = 4 * KW + d
        x = t[lo:hi, i]
        on = x[:, 0] > 0  # parity waves mark every other iterate
        xs = x[on]
        out["roles"][f"DEC.w{d}"] = {"period": med(np.diff(xs[:, 0])) if len(xs) > 1 else 0.0,
                                     "gather": med(xs[:, 1] - xs[:, 0]), "sum": med(xs[:, 2] - xs[:, 1])}
    lastw = lambda role: ROLES.index(role) * KW + W[role] - 1
    u = np.arange(lo, hi)
    out["handover"] = {
        "UPD done u -> UPD.w0 staged u+1": med(t[u + 1, 0, 1] - t[u, lastw("UPD"), 3]),
        "UPD done u -> T1.w0 staged u+1": med(t[u + 1, 6, 1] - t[u, lastw("UPD"), 3]),
        "T1 done u -> T2.w0 staged u": med(t[u, 12, 1] - t[u, lastw("T1"), 3]),
        "T2 done u -> T3.w0 staged u": med(t[u, 18, 1] - t[u, lastw("T2"), 3]),
        "T3 done u -> DEC.w5 gathered u": med(t[u, 29, 1] - t[u, lastw("T3"), 3]),
        "T1 done u -> DEC dot-4 wave gathered u": med(np.maximum(t[u, 27, 1], t[u, 28, 1]) - t[u, lastw("T1"), 3]),
        "DEC decided u": med(t[u, 4 * KW, 3] - t[u, lastw("UPD"), 3]),
        "y_u published -> DEC decided u (latency)": med(t[u, 4 * KW, 3] - t[u - 1, lastw("UPD"), 3]),
        "DEC decided u-8 -> y_u published": med(t[u - 1, lastw("UPD"), 3] - t[u - 8, 4 * KW, 3]),
        "UPD ahead of DEC (iterates)": med(np.searchsorted(t[:, lastw("UPD"), 3], t[u, 4 * KW, 3]) - u),
    }
    # absolute timeline of a few iterates, relative to DEC's decision of u - 8
    # (the decision that lets y_u be published)
    sample = {}
    for uu in range(lo, lo + 4):
        base = t[uu - 8, 4 * KW, 3]
        ev = {"y_u published (UPD last wave)": t[uu - 1, lastw("UPD"), 3],
              "T1.w0 staged": t[uu, 6, 1], "T1 last done": t[uu, lastw("T1"), 3],
              "T2.w0 staged": t[uu, 12, 1], "T2 last done": t[uu, lastw("T2"), 3],
              "T3.w0 staged": t[uu, 18, 1], "T3 last done": t[uu, lastw("T3"), 3],
              "DEC dot-4 gathered": max(t[uu, 27, 1], t[uu, 28, 1]), "DEC dot-4 summed": max(t[uu, 27, 2], t[uu, 28, 2]),
              "DEC.w5 summed": t[uu, 29, 2],
              "DEC.w0 feasibility": t[uu, 4 * KW, 1], "DEC.w0 dots in": t[uu, 4 * KW, 2],
              "DEC decided": t[uu, 4 * KW, 3]}
        sample[f"u={uu}"] = {k: round(float(v - base), 2) for k, v in ev.items()}
    out["timeline_from_decision_u-8"] = sample
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:]))
