"""profiles/pmc_traffic.json records for the batched converge solvers
(k_solve_pipe, or k_solve_single with PIPE_OFF=1) from
separate rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE) of scripts/batch_converge_one.py 8: the dispatch of
the 8-update call (9 terminate() + 8 updates per problem, n_dual 1024, M 512,
4096 problems).  Bytes as MI355X_MICROARCH.md prescribes for the hot kernel,
(2*FETCH_SIZE + WRITE_SIZE) * 1024; the ratio to the bytes the kernel is
designed to move says whether anything is re-read.
Usage: python scripts/pmc_single.py FETCH.csv WRITE.csv infeasible|feasible [pipe|single]"""
from __future__ import annotations

import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
KERNELS = {"single": "k_solve_single<256, true", "pipe": "k_solve_pipe<256"}
N, M, B, K = 1024, 512, 4096, 8


def dispatches(path: str, counter: str, kernel: str) -> list[float]:
    vals = []
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"] and row["Counter_Name"] == counter:
                vals.append(float(row["Counter_Value"]))
    return vals


def design_bytes(case: str, which: str) -> float:
    """Bytes per problem the 8-update dispatch moves by design."""
    q, g, qi, qp = 4.0 * N * N, 4.0 * N * M, 4.0 * M * M, 4.0 * M * M
    if which == "pipe":
        # Gp'Y of the first iterate, then per iterate Qp_inv and one pass over
        # Gp, and an update before every iterate but the capped one
        if case == "infeasible":
            return g + K * q + (K + 1) * (qi + g)
        # feasible: iterates 1..K fused (a launch's first iterate fuses too),
        # the capped iterate K+1 no update but Y'Qd's pass; Qp for U'Qp every
        # iterate
        return g + (K + 1) * q + (K + 1) * (qi + g + qp)
    if case == "infeasible":  # 8 updates; 9 terminates stopping at checkFeas (Gp'Y, Qp_inv, and Gp U
        # over its first 256 rows, where a row over its bound decides the iterate)
        return K * q + (K + 1) * (g + 4.0 * min(N, 256) * M + qi)
    # feasible: terminate 1 reads Qd for Y'Qd, then update 1 (unfused), then
    # 8 fused passes (update + Y'Qd, the last one speculative); Qp for U'Qp each time
    return (K + 2) * q + (K + 1) * (2 * g + qi + qp)


def main():
    fetch_csv, write_csv, case = sys.argv[1], sys.argv[2], sys.argv[3]
    which = sys.argv[4] if len(sys.argv) > 4 else "pipe"
    kernel = KERNELS[which]
    f, w = dispatches(fetch_csv, "FETCH_SIZE", kernel), dispatches(write_csv, "WRITE_SIZE", kernel)
    if len(f) < 2 or len(w) < 2:
        raise SystemExit(f"expected >= 2 {kernel} dispatches, got {len(f)} / {len(w)}")
    fetch, write = f[1], w[1]  # [0] is the warm-up call (1 update)
    sys.path.insert(0, str(ROOT))
    from bench import kernel_src_hash

    hbm = (2 * fetch + write) * 1024
    design = design_bytes(case, which) * B
    name = "k_solve_pipe" if which == "pipe" else "k_solve_single"
    khash = kernel_src_hash("solve-single", "solve-pipe") if which == "pipe" else kernel_src_hash("solve-single")
    rec = {"kernel": "k_solve_pipe<256>" if which == "pipe" else "k_solve_single<256,true>", "kernel_src_sha256": khash,
           "case": case, "dispatch": f"the {K}-update call: {K + 1} terminate() + {K} updates per problem, "
                                     f"{B} problems, n_dual {N}, M {M}",
           "fetch_size_kb": fetch, "write_size_kb": write, "hbm_bytes": hbm, "design_bytes": design,
           "traffic_ratio": hbm / design,
           "correction": "bytes = (2*FETCH_SIZE + WRITE_SIZE) * 1024 (MI355X_MICROARCH.md, HBM)",
           "source": f"{fetch_csv}, {write_csv} (separate rocprofv3 --pmc passes of scripts/batch_converge_one.py)"}
    out = ROOT / "profiles" / "pmc_traffic.json"
    db = json.loads(out.read_text()) if out.exists() else {}
    db[f"{name}_{case}"] = rec
    out.write_text(json.dumps(db, indent=1) + "\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
