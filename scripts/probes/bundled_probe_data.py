"""Write the bundled example's N, Qd, Fd and the reference's Y after 999
fixed-mode updates (tests/golden/bundled.npz) as one binary file for
bundled_probe.hip."""
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[2]
d = np.load(ROOT / "tests" / "golden" / "bundled.npz")
out = Path(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/bundled.bin")
out.parent.mkdir(parents=True, exist_ok=True)
with open(out, "wb") as f:
    f.write(np.int32(int(d["N"])).tobytes())
    for k in ("Qd", "Fd", "Y_fixed999"):
        f.write(np.ascontiguousarray(d[k], dtype=np.float32).tobytes())
print(out)
