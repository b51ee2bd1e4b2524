"""Problem data for the timing scripts, from the committed fixtures only --
scripts never import oracle/ (test infrastructure): the bundled example's
dual (tests/golden/bundled.npz, generated from the reference build by
tests/golden/make_golden.py) and k copies of a dual problem on the diagonal
(the horizon-size class of the bench's horizon leg)."""
from __future__ import annotations

from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
KEYS = ("Qd", "Fd", "Md", "Qp", "Qp_inv", "Fp", "Mp", "Gp", "Kp")


def bundled_problem() -> dict:
    g = np.load(ROOT / "tests" / "golden" / "bundled.npz")
    P = {k: np.ascontiguousarray(g[k], dtype=np.float32) for k in KEYS}
    P.update(N=int(g["N"]), M=int(g["M"]))
    return P


def block_diag_problem(P: dict, k: int) -> dict:
    """k copies of P on the diagonal: Qd, Gp, Qp, Qp_inv block-diagonal, the
    vectors tiled, Md and Mp times k (every block's iterate is P's own)."""
    N, M = int(P["N"]), int(P["M"])

    def bd(a, r, c):
        out = np.zeros((k * r, k * c), np.float32)
        a = np.asarray(a, np.float32).reshape(r, c)
        for b in range(k):
            out[b * r:(b + 1) * r, b * c:(b + 1) * c] = a
        return out.reshape(-1)

    def tile(a):
        return np.tile(np.asarray(a, np.float32).reshape(-1), k)

    return dict(Qd=bd(P["Qd"], N, N), Gp=bd(P["Gp"], N, M), Qp=bd(P["Qp"], M, M), Qp_inv=bd(P["Qp_inv"], M, M),
                Fd=tile(P["Fd"]), Kp=tile(P["Kp"]), Fp=tile(P["Fp"]),
                Md=(np.asarray(P["Md"], np.float32) * np.float32(k)).reshape(1),
                Mp=(np.asarray(P["Mp"], np.float32) * np.float32(k)).reshape(1), N=k * N, M=k * M)
