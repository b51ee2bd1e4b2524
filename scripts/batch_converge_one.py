"""One batched converge-mode call at n_dual 1024 x 4096 problems (the bench's
batch_converge leg), for kernel traces: python scripts/batch_converge_one.py [K]
FEASIBLE=1: every iterate feasible (Kp = 1e30 seen by checkFeas only), so
terminate() runs all of computeCost; PQP_BATCH_OPTS: pqp_tune_batch_converge;
PIPE_OFF=1: k_solve_single (Gp read twice per iteration) instead of k_solve_pipe."""
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "pqp-for-mpc_amd"))


def main():
    import torch

    import pqp_amd

    K = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    pb = pqp_amd.ProblemBatch.synthetic(3, 0, 4096, 1024, 512)
    if os.environ.get("FEASIBLE"):
        pb.Kp.fill_(1e30)
    if os.environ.get("PQP_BATCH_OPTS"):
        pqp_amd.lib().pqp_tune_batch_converge(int(os.environ["PQP_BATCH_OPTS"]))
    if os.environ.get("PIPE_OFF"):
        pqp_amd.tune("pipe_off", 1)
    pb.solve(max_updates=1)
    torch.cuda.synchronize()
    print("kernel", "k_solve_pipe" if pqp_amd.tune_get("last_batch_kernel") else "k_solve_single", flush=True)
    for k in (K, 3 * K):
        t0 = time.perf_counter()
        pb.solve(max_updates=k)
        torch.cuda.synchronize()
        print(f"updates {k}: {(time.perf_counter() - t0) * 1e3:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
