"""Summarise one rocprofv3 SQ/GRBM `--pmc` pass over tools/pmc_probe.py into per-kernel issue
figures: effective clock under load (GRBM_GUI_ACTIVE / 8 XCDs / dispatch time, the DVFS
read-out of MI355X_MICROARCH.md), VALU issue occupancy per SIMD, wave-state split
(active / issue-stalled / parked) and VALU instructions per launch.

    rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU \
        SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY -d gpurun_out/pmc_issue -o issue \
        --output-format csv -- python3 tools/pmc_probe.py
    python tools/pmc_issue.py gpurun_out/pmc_issue > profiles/pmc_issue.json

SQ_* cycle counters count quad-cycles (x4), summed over waves; 256 CUs x 4 SIMDs.
"""
import collections
import csv
import glob
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import short  # noqa: E402

SIMDS = 256 * 4


def main():
    d = sys.argv[1]
    disp = collections.defaultdict(dict)   # dispatch id -> counters (+ name, ns)
    for f in glob.glob(os.path.join(d, "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            s = short(r["Kernel_Name"])
            if s is None:
                continue
            e = disp[(f, r["Dispatch_Id"])]
            e["name"] = s
            e["ns"] = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
            e[r["Counter_Name"]] = e.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    per = collections.defaultdict(list)
    for e in disp.values():
        per[e["name"]].append(e)
    out = {}
    for k, es in per.items():
        def avg(c):
            v = [e[c] for e in es if c in e]
            return sum(v) / len(v) if v else None
        ns = avg("ns")
        gui = avg("GRBM_GUI_ACTIVE")
        clk = gui / 8.0 / ns if gui else None          # GHz (cycles per ns)
        cyc = gui / 8.0 if gui else None                # shader cycles of the dispatch
        wave = avg("SQ_WAVE_CYCLES")
        o = {"launches": len(es), "avg_ms": ns / 1e6, "eff_clock_GHz": clk,
             "valu_insts_per_launch": avg("SQ_INSTS_VALU")}
        if cyc and avg("SQ_ACTIVE_INST_VALU") is not None:
            o["valu_issue_busy_per_simd"] = 4 * avg("SQ_ACTIVE_INST_VALU") / (cyc * SIMDS)
        if wave:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY"):
                if avg(c) is not None:
                    o[c.lower() + "_frac_of_wave_cycles"] = avg(c) / wave
            o["avg_waves_per_simd"] = 4 * wave / (cyc * SIMDS) if cyc else None
        out[k] = o
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
