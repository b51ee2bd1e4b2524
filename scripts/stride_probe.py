"""Does the problem stride / column stride of QdT change the hot kernel's HBM
rate?  Every problem is 4 MiB = a power of two, so 768 concurrent workgroup
streams start at addresses that differ only above bit 22.  This probe lays the
same 4096 generated problems out with padded strides (extra floats between
problems, or a padded column stride ldq), checks that the iterates are
bit-identical to the unpadded layout, and times pqp_batch_iterate and the
k_stream_read ceiling of each layout, interleaved in one process.

    python scripts/stride_probe.py [--batch 4096] [--rounds 5] [--launches 10]
"""
from __future__ import annotations

import argparse
import ctypes as C
import statistics
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=1024)
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--launches", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch

    import pqp_amd

    L = pqp_amd.lib()
    N, B = a.n, a.batch
    M = N // 2
    alg = (4 * N * N + 16 * N) * B
    s = torch.cuda.current_stream()
    sp = C.c_void_p(s.cuda_stream)
    p = lambda t: C.c_void_p(t.data_ptr())  # noqa: E731
    # (name, ldq, extra floats between problems)
    layouts = [("base", N, 0), ("pad 256 B", N, 64), ("pad 1 KiB", N, 256), ("pad 4 KiB", N, 1024),
               ("pad 64 KiB+1 KiB", N, 16384 + 256), ("ldq+32", N + 32, 0)]
    ldv = N
    Fd = torch.empty(B * ldv, device="cuda")
    Md = torch.empty(B, device="cuda")
    th = torch.empty(B * ldv, device="cuda")
    Y = torch.empty(B * ldv, device="cuda")
    out = torch.empty(B * 256, device="cuda")
    bufs = []
    for name, ldq, pad in layouts:
        qs = N * ldq + pad
        Q = torch.zeros(B * qs, device="cuda")
        rc = L.pqp_batch_generate(1, 0, B, N, M, p(Q), ldq, C.c_longlong(qs), p(Fd), p(Md), p(th), ldv, sp)
        assert rc == 0, rc
        bufs.append((name, ldq, qs, Q))
    torch.cuda.synchronize()

    def it(ldq, qs, Q, n):
        rc = L.pqp_batch_iterate(B, N, p(Q), ldq, C.c_longlong(qs), p(th), p(Fd), ldv, None, p(Y), n, sp)
        assert rc == 0, rc

    ref = None
    for name, ldq, qs, Q in bufs:
        it(ldq, qs, Q, 3)
        y = Y.view(B, ldv)[:64, :N].cpu().numpy().copy()
        if ref is None:
            ref = y
        assert np.array_equal(y.view(np.uint32), ref.view(np.uint32)), f"{name} differs"
    print("iterates bit-identical across layouts", flush=True)

    def t_iter(ldq, qs, Q):
        it(ldq, qs, Q, 1)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.launches):
            it(ldq, qs, Q, 1)
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / a.launches

    def t_read(ldq, qs, Q):
        L.pqp_tune_stream_read(B, N, p(Q), ldq, C.c_longlong(qs), p(out), 1, sp)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(a.launches):
            L.pqp_tune_stream_read(B, N, p(Q), ldq, C.c_longlong(qs), p(out), 1, sp)
        e1.record(s)
        e1.synchronize()
        return e0.elapsed_time(e1) / a.launches

    res = {}
    for r in range(a.rounds):
        for name, ldq, qs, Q in bufs:
            res.setdefault(("iterate", name), []).append(t_iter(ldq, qs, Q))
            res.setdefault(("stream_read nt", name), []).append(t_read(ldq, qs, Q))
        print(f"round {r} done", flush=True)
    for (kind, name), v in res.items():
        med = statistics.median(v)
        print(f"{kind:15s} {name:18s} median {med:.4f} ms  {alg / med / 1e9:.0f} GB/s  "
              f"min {min(v):.4f} max {max(v):.4f}", flush=True)


if __name__ == "__main__":
    main()
