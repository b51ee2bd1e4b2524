"""bench.py at N > 1: the headline line survives a failing or hanging
optional leg.  The row-sharded leg runs on CPU over gloo
with a test-only block standing in for the GPU kernel, one rank made to fail
inside its timed updates (PQP_BENCH_FAULT, as in a GPU rehearsal); a leg that
never returns is ended by the Emitter's watchdog, which prints the line and
exits 0."""
from __future__ import annotations

import json
import os
import socket
import subprocess
import sys
import time

import pytest
import torch.multiprocessing as mp

from conftest import ROOT


def _bench():
    if str(ROOT) not in sys.path:
        sys.path.insert(0, str(ROOT))
    import bench

    return bench


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _HalfBlock:
    """Test-only row block: Y_next[i] = Y[i] / 2 + 1 for its rows."""

    def __init__(self, N, row0, rows):
        self.N, self.row0, self.rows = N, row0, rows

    def update(self, Y, Y_rows):
        Y_rows[: self.rows] = Y[self.row0:self.row0 + self.rows] * 0.5 + 1.0


def _worker(rank, world, port, fault, out_dir):
    sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    bench = _bench()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    if fault:
        os.environ["PQP_BENCH_FAULT"] = fault
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=30))
    result = {"value": 123.0, "n_gpus": world} if rank == 0 else None
    em = bench.Emitter(rank, result, leg_timeout_s=60)
    out = em.leg("rowshard", lambda: bench.rowshard_bench(None, dist, rank, world, torch.device("cpu"), 16, 20,
                                                           graph=False, make_block=_HalfBlock))
    with open(os.path.join(out_dir, f"r{rank}.json"), "w") as f:
        json.dump({"leg": out, "result": result, "failed": em.failed}, f)
    if em.failed:  # as bench.main: do not wait on a peer stuck in the failed collective
        os._exit(0)
    dist.destroy_process_group()


@pytest.mark.parametrize("fault", ["", "rowshard:1", "rowshard:0"])
def test_rowshard_leg_failure_keeps_headline(tmp_path, fault):
    t0 = time.monotonic()
    mp.spawn(_worker, args=(2, _free_port(), fault, str(tmp_path)), nprocs=2, join=True)
    assert time.monotonic() - t0 < 120
    r0 = json.loads((tmp_path / "r0.json").read_text())
    assert r0["result"]["value"] == 123.0  # the headline is untouched
    leg = r0["result"]["rowshard"]
    if not fault:
        assert "error" not in leg and leg["ranks"] == 2 and leg["finite_nonneg"] and leg["us_per_update"] > 0
        # the block update timed alone beside update + all-gather
        assert leg["us_per_update_block_only"] > 0
        assert leg["allgather_us_per_update"] == pytest.approx(leg["us_per_update_eager"] - leg["us_per_update_block_only"])
    else:
        assert "error" in leg, leg
        r1 = json.loads((tmp_path / "r1.json").read_text())
        assert "error" in r1["leg"]


def test_setup_failure_on_one_rank_is_agreed(tmp_path):
    """A rank whose block cannot be built: every rank sees the error before
    any all-gather of the leg (no peer left waiting)."""
    code = f"""
import json, os, sys
sys.path.insert(0, {str(ROOT)!r}); sys.path.insert(0, {str(ROOT / 'tests')!r})
sys.path.insert(0, {str(ROOT / 'pqp-for-mpc_amd')!r})
from datetime import timedelta
import torch, torch.distributed as dist
import bench
rank = int(os.environ['RANK'])
dist.init_process_group('gloo', timeout=timedelta(seconds=30))
def make(N, row0, rows):
    if rank == 1:
        raise MemoryError('no room for the block')
    from test_bench_legs import _HalfBlock
    return _HalfBlock(N, row0, rows)
em = bench.Emitter(rank, {{'value': 1.0}} if rank == 0 else None, 60)
out = em.leg('rowshard', lambda: bench.rowshard_bench(None, dist, rank, 2, torch.device('cpu'), 8, 4,
                                                     graph=False, make_block=make))
open(os.path.join({str(tmp_path)!r}, 'r%d' % rank), 'w').write(json.dumps(out))
dist.destroy_process_group()
"""
    bench = _bench()
    t0 = time.monotonic()
    assert bench.launch_ranks(2, [sys.executable, "-c", code], grace_s=30) == 0
    assert time.monotonic() - t0 < 90
    e0 = json.loads((tmp_path / "r0").read_text())["error"]
    e1 = json.loads((tmp_path / "r1").read_text())["error"]
    assert "another rank" in e0 and "no room" in e1


def test_hung_leg_prints_line_and_exits_zero():
    code = f"""
import sys, time
sys.path.insert(0, {str(ROOT)!r})
import bench
em = bench.Emitter(0, {{"value": 7.0, "n_gpus": 2}}, leg_timeout_s=1.0)
em.leg("gather", lambda: {{"ms": 1.0, "ok": True}})
em.leg("rowshard", lambda: time.sleep(600))
print("not reached")
"""
    t0 = time.monotonic()
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    assert time.monotonic() - t0 < 60
    lines = [ln for ln in out.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, lines
    rec = json.loads(lines[0])
    assert rec["value"] == 7.0 and rec["gather"]["ok"] is True
    assert "timed out" in rec["rowshard"]["error"]


def test_emitter_prints_once_and_records_errors(capsys):
    bench = _bench()
    res = {"value": 1.0}
    em = bench.Emitter(0, res, leg_timeout_s=30)

    def boom():
        raise ValueError("leg broke")

    assert em.leg("bad", boom)["error"].startswith("ValueError")
    assert em.leg("good", lambda: {"x": 1}) == {"x": 1}
    em.emit()
    em.emit()
    lines = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()]
    assert len(lines) == 1 and em.failed
    rec = json.loads(lines[0])
    assert rec["bad"]["error"] == "ValueError: leg broke" and rec["good"] == {"x": 1}
    # other ranks print nothing
    em1 = bench.Emitter(1, None, 30)
    em1.leg("x", lambda: {})
    em1.emit()
    assert capsys.readouterr().out == ""


def test_failed_leg_ends_every_rank_before_the_next_leg(tmp_path):
    """Two collective legs, rank 1 failing inside the first (abort_on_failure,
    as bench.main runs N > 1): rank 0 prints the line with the first leg's
    error, nobody meets a peer inside the wrong leg's collectives, and the job
    ends quickly with status 0."""
    code = f"""
import os, sys
sys.path.insert(0, {str(ROOT)!r}); sys.path.insert(0, {str(ROOT / 'tests')!r})
sys.path.insert(0, {str(ROOT / 'pqp-for-mpc_amd')!r})
from datetime import timedelta
import torch, torch.distributed as dist
import bench
from test_bench_legs import _HalfBlock
rank = int(os.environ['RANK'])
os.environ['PQP_BENCH_FAULT'] = 'rowshard:1'
dist.init_process_group('gloo', timeout=timedelta(seconds=60))
em = bench.Emitter(rank, {{'value': 5.0}} if rank == 0 else None, 60, abort_on_failure=True)
for name, n in (('rowshard', 16), ('rowshard_8', 8)):
    em.leg(name, lambda n=n: bench.rowshard_bench(None, dist, rank, 2, torch.device('cpu'), n, 20, graph=False,
                                                  make_block=_HalfBlock))
em.emit()
dist.destroy_process_group()
"""
    out_file = tmp_path / "out.txt"
    bench = _bench()
    t0 = time.monotonic()
    with open(out_file, "w") as f:
        old = os.dup(1)
        os.dup2(f.fileno(), 1)
        try:
            rc = bench.launch_ranks(2, [sys.executable, "-c", code], grace_s=30)
        finally:
            os.dup2(old, 1)
            os.close(old)
    assert rc == 0 and time.monotonic() - t0 < 90
    lines = [ln for ln in out_file.read_text().splitlines() if ln.startswith("{")]
    assert len(lines) == 1, lines
    rec = json.loads(lines[0])
    assert rec["value"] == 5.0 and "error" in rec["rowshard"] and "rowshard_8" not in rec


def _spread_worker(rank, world, port, out_dir):
    from datetime import timedelta

    import torch
    import torch.distributed as dist

    bench = _bench()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world, timeout=timedelta(seconds=30))
    dev = torch.device("cpu")
    spread = bench.rank_spread(dist, dev, timed_s=1.0 + rank, kern_ms=10.0 * (rank + 1))
    g = bench.rank_spread(dist, dev, gather_ms=3.0 - rank)["gather_ms"]
    if rank == 0:
        res = bench.headline(None, rank, world, 1024, 4096, 20, 5, 10, spread["timed_s"]["max"],
                             spread["kern_ms"]["max"], 2, True, False, spread=spread)
        res.setdefault("per_rank", {})["gather_ms"] = g
        with open(os.path.join(out_dir, "r0.json"), "w") as f:
            json.dump({"result": res, "summary": bench.summary(res)}, f)
    dist.destroy_process_group()


def test_per_rank_spread_at_world_size_2(tmp_path):
    """at N > 1 the line carries each rank's timed region
    and gather time as min / max over ranks (a slow or stuck rank is visible
    in the first 8-GPU record); value uses the max."""
    mp.spawn(_spread_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    rec = json.loads((tmp_path / "r0.json").read_text())
    res, S = rec["result"], rec["summary"]
    assert res["per_rank"]["timed_s"] == {"min": 1.0, "max": 2.0}
    assert res["per_rank"]["kern_ms"] == {"min": 10.0, "max": 20.0}
    assert res["per_rank"]["gather_ms"] == {"min": 2.0, "max": 3.0}
    assert res["value"] == pytest.approx(4096 * 2 * 20 / 2.0)  # whole job over the slowest rank
    assert S["per_rank_timed_s"] == {"min": 1.0, "max": 2.0} and S["gather_ms"] == {"min": 2.0, "max": 3.0}


def test_summary_is_the_last_key(capsys):
    """every leg's key numbers in a compact object at the
    END of the line (the driver's record keeps the line's tail)."""
    bench = _bench()
    res = {"value": 1.5e6, "n_gpus": 1, "roofline": {"frac": 0.95, "avg_launch_ms": 22.5, "traffic": 1.5e11,
                                                     "alg_bytes_per_launch": 1.72e11},
           "batch_converge": {"infeasible": {"ms_per_iteration": 4.4, "frac_of_hbm_peak": 0.85}},
           "horizon": {"H4": {"converge_ms": 28.0, "roofline": {"frac": 0.32, "alg_frac": 0.21}}},
           "bundled": {"error": "RuntimeError: x"}}
    em = bench.Emitter(0, res, leg_timeout_s=30)
    em.leg("single_n1024", lambda: {"ms_per_solve": 3.6})
    em.emit()
    line = [ln for ln in capsys.readouterr().out.splitlines() if ln.strip()][0]
    rec = json.loads(line)
    assert list(rec)[-1] == "summary"
    S = rec["summary"]
    assert S["hbm_frac"] == 0.95 and S["traffic_ratio"] == pytest.approx(1.5e11 / 1.72e11, abs=1e-4)
    assert S["batch_converge_infeasible"] == {"ms_per_iter": 4.4, "hbm_frac": 0.85}
    assert S["batch_converge_feasible"] == {"ms_per_iter": None, "hbm_frac": None}
    assert S["horizon_H4"] == {"ms": 28.0, "valu_frac": 0.32, "alg_frac": 0.21}
    assert S["single_n1024_ms_per_1000"] == 3.6 and S["bundled_fixed1000_ms"] is None
    assert S["legs_with_errors"] == ["bundled"]
    assert len(line.split('"summary"')[1]) < 2500  # compact


def test_kernel_hash_covers_included_headers(tmp_path, monkeypatch):
    """a change to a header the kernels include (here
    pqp_device.h, where gap_stop lives) changes the source hash, so the PMC
    record measured before it is reported as stale, not as `traffic`."""
    import shutil

    bench = _bench()
    src = ROOT / "pqp-for-mpc_amd"
    (tmp_path / "pqp-for-mpc_amd").mkdir()
    shutil.copytree(src / "csrc", tmp_path / "pqp-for-mpc_amd" / "csrc")
    shutil.copy(src / "Makefile", tmp_path / "pqp-for-mpc_amd" / "Makefile")
    monkeypatch.setattr(bench, "ROOT", tmp_path)
    h0 = bench.hot_kernel_hash()
    assert h0 == bench.kernel_src_hash("hot-kernel", root=ROOT)
    (tmp_path / "profiles").mkdir()
    (tmp_path / "profiles" / "pmc_traffic.json").write_text(json.dumps(
        {"n1024_b4096_c10": {"kernel_src_sha256": h0, "hbm_bytes_per_launch": 1.6e11, "source": "test"}}))
    fresh = bench.headline(None, 0, 1, 1024, 4096, 20, 5, 10, 0.05, 47.0, 2, True, False)
    assert fresh["roofline"]["traffic"] == 1.6e11
    for h in bench.KERNEL_HEADERS:
        f = tmp_path / "pqp-for-mpc_amd" / "csrc" / h
        f.write_text(f.read_text() + "\n// edited\n")
        assert bench.hot_kernel_hash() != h0
        assert bench.kernel_src_hash("solve-mid2") != bench.kernel_src_hash("solve-mid2", root=ROOT)
        stale = bench.headline(None, 0, 1, 1024, 4096, 20, 5, 10, 0.05, 47.0, 2, True, False)
        assert stale["roofline"]["traffic"] is None and stale["roofline"]["traffic_source"].startswith("stale")
        f.write_text(f.read_text().replace("\n// edited\n", ""))
    assert bench.hot_kernel_hash() == h0


def test_horizon_roofline_peak_and_alg_flops():
    """VALU issue peak = one wave64 instruction per SIMD
    every 2 clocks (1228.8 G/s), algorithmic flops 6N^2 + 4NM + 4M^2 per
    feasible iterate against 78.6 T op/s."""
    bench = _bench()
    assert bench.VALU_PEAK_GWI == pytest.approx(1228.8)
    assert bench.VALU_LANE_OPS == pytest.approx(78.6432e12)
    N, M = 112, 28
    assert bench.converge_alg_flops(1, N, M) == 6 * N * N + 4 * N * M + 4 * M * M
    assert bench.converge_alg_flops(1, N, M, feasible=False) == 4 * N * N + 4 * N * M + 2 * M * M
    r = bench.valu_roofline("no_such_record", "solve-mid2", 5128195, 0.028, N, M)
    assert r["achieved"] is None and r["peak"] == pytest.approx(1228.8)
    assert r["alg_TFLOPs"] == pytest.approx(5128195 * 90944 / 0.028 / 1e12)
