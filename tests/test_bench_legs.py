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
