"""bench.py's batch_converge leg alone (one JSON line)."""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "pqp-for-mpc_amd"))

import bench  # noqa: E402
import pqp_amd  # noqa: E402

print(json.dumps(bench.batch_converge_bench(pqp_amd)), flush=True)
