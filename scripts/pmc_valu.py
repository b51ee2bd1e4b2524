"""Build profiles/pmc_valu.json from the rocprofv3 passes of
`scripts/gpu_r05.sh hpmc` (scripts/horizon_pmc.py H under --pmc SQ_INSTS_VALU
SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE): k_solve_mid2's VALU
wave-instructions for the bench's horizon solve (the second dispatch of each
pass: the timed one after the warm-up), keyed by the hash of the kernel's
source region (<solve-mid2>) and the headers it includes.  bench.py divides
the count by its own timed solve to report the horizon rows' VALU-issue
roofline (peak 1228.8 G wave-instr/s: one wave64 instruction per SIMD every
2 clocks, MI355X_MICROARCH.md).  Passes h2, h4, h5 are the stacked plant
(records mid2_H2/4/5); d112, d140 the dense companion (mid2_dense_N112/140).
Usage: python scripts/pmc_valu.py gpurun_out/TAG"""
import collections
import csv
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def main(d: str):
    sys.path.insert(0, str(ROOT))
    from bench import kernel_src_hash

    out = ROOT / "profiles" / "pmc_valu.json"
    db = json.loads(out.read_text()) if out.exists() else {}
    for H in ("2", "4", "5", "d112", "d140"):
        sub = Path(d) / (f"h{H}" if not H.startswith("d") else H)
        if not sub.exists():
            continue
        by = collections.defaultdict(dict)
        meta = {}
        for r in csv.DictReader(open(sub / "pmc_counter_collection.csv")):
            if "k_solve_mid2" not in r["Kernel_Name"]:
                continue
            c = by[int(r["Dispatch_Id"])]
            c[r["Counter_Name"]] = c.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
            meta[int(r["Dispatch_Id"])] = (r["Kernel_Name"], r["Start_Timestamp"], r["End_Timestamp"])
        disp = sorted(by)[-1]  # the timed solve (after the warm-up)
        c = by[disp]
        name, t0, t1 = meta[disp]
        ms = (int(t1) - int(t0)) / 1e6
        info = json.loads([ln for ln in (sub.parent / f"{sub.name}.json").read_text().splitlines()
                           if ln.startswith("{")][-1])
        key = f"mid2_H{H}" if not H.startswith("d") else f"mid2_dense_N{H[1:]}"
        db[key] = {
            "kernel": name, "kernel_src_sha256": kernel_src_hash("solve-mid2"), "n_dual": info["n_dual"],
            "problems": info["problems"], "h_sum": info["h_sum"], "sq_insts_valu": c["SQ_INSTS_VALU"],
            "sq_active_inst_valu": c["SQ_ACTIVE_INST_VALU"], "sq_busy_cycles": c["SQ_BUSY_CYCLES"],
            "grbm_gui_active": c["GRBM_GUI_ACTIVE"], "dispatch_ms_under_counters": ms,
            "clock_ghz": c["GRBM_GUI_ACTIVE"] / 8 / (ms * 1e-3) / 1e9,
            "valu_issue_frac_under_counters": c["SQ_INSTS_VALU"] / (ms * 1e-3) / (256 * 4 * 2.4e9 / 2),
            "source": f"{sub} (rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE "
                      f"-- python3 scripts/horizon_pmc.py {H})"}
        print(H, json.dumps(db[key]))
    out.write_text(json.dumps(db, indent=1) + "\n")


if __name__ == "__main__":
    main(sys.argv[1])
