"""Debug: updates of a small problem through the streaming and the relay
split kernels, in one or several row blocks; reports the first divergence."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (ROOT / "pqp-for-mpc_amd", ROOT / "oracle"):
    sys.path.insert(0, str(p))
import numpy as np
import torch

import pqp_amd
from oracle import Oracle

orc = Oracle()
N = 28
P = orc.synth_problem(17, 1, N, N // 2, with_qp=False)
Qd = torch.from_numpy(P["Qd"]).cuda()
Fd = torch.from_numpy(P["Fd"]).cuda()
L = pqp_amd.lib()
for var in (1 << 14, 5 << 14, (5 << 14) | (4 << 17)):
    for cuts in ([], [9, 10]):
        L.pqp_tune_set_variant(var)
        edges = [0] + cuts + [N]
        blocks = [pqp_amd.RowBlock(Qd[a * N:], Fd, N, a, b - a) for a, b in zip(edges[:-1], edges[1:])]
        Y = torch.full((N,), 1000.0, device="cuda")
        for it in range(1, 6):
            Yn = torch.full((N,), -7.0, device="cuda")
            for blk in blocks:
                blk.update(Y, Yn[blk.row0:blk.row0 + blk.rows])
            torch.cuda.synchronize()
            got = Yn.cpu().numpy()
            want = orc.iterate(P["Qd"], P["Fd"], N, it)
            ok = np.array_equal(got.view(np.uint32), want.view(np.uint32))
            if not ok:
                bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
                print(hex(var), cuts, "iter", it, "DIFF rows", bad[:10], got[bad[:4]], want[bad[:4]], flush=True)
                break
            Y = Yn
        else:
            print(hex(var), cuts, "exact through 5 updates", flush=True)
L.pqp_tune_set_variant(0)
