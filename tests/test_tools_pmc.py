"""The PMC summarisers behind bench.py's roofline.traffic and the DESIGN §3 issue table
(tools/pmc_traffic.py, tools/pmc_issue.py), on a synthetic rocprofv3 counter CSV."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIELDS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id",
          "Grid_Size", "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size",
          "Scratch_Size", "VGPR_Count", "Accum_VGPR_Count", "SGPR_Count", "Counter_Name",
          "Counter_Value", "Start_Timestamp", "End_Timestamp"]
BWD = "void dicp::sym_bwd_pk_kernel<3>(dicp::Args, dicp::Scal, long, int, int, float*, long, int, int)"


def _write(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        for disp, name, counter, value, t0, t1 in rows:
            w.writerow({k: 0 for k in FIELDS} | {"Dispatch_Id": disp, "Kernel_Name": name,
                                                 "Counter_Name": counter, "Counter_Value": value,
                                                 "Start_Timestamp": t0, "End_Timestamp": t1})


def _run(tool, d):
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", tool), str(d)],
                         check=True, capture_output=True, text=True).stdout
    return json.loads(out)


def test_pmc_traffic_gfx950_correction(tmp_path):
    _write(tmp_path / "f_counter_collection.csv",
           [(1, BWD, "FETCH_SIZE", 100.0, 0, 10), (2, BWD, "FETCH_SIZE", 300.0, 0, 10),
            (3, "void at::native::other_kernel()", "FETCH_SIZE", 5.0, 0, 10)])
    _write(tmp_path / "w_counter_collection.csv",
           [(1, BWD, "WRITE_SIZE", 50.0, 0, 10), (2, BWD, "WRITE_SIZE", 50.0, 0, 10)])
    d = _run("pmc_traffic.py", tmp_path)
    assert set(d) == {"ode_self_bwd"}           # torch kernels are not attributed
    b = d["ode_self_bwd"]
    assert b["fetch_kb_per_launch"] == 200.0 and b["write_kb_per_launch"] == 50.0
    assert b["hbm_bytes_per_launch"] == (2 * 200.0 + 50.0) * 1024      # 2 x FETCH + WRITE
    assert b["hbm_bytes_per_launch_raw"] == (200.0 + 50.0) * 1024


def test_pmc_issue_clock_and_valu_occupancy(tmp_path):
    ns = 1_000_000                               # 1 ms dispatch
    gui = 8 * 2.0 * ns                           # 8 XCDs at 2.0 GHz
    cyc = gui / 8
    rows = [(7, BWD, "GRBM_GUI_ACTIVE", gui, 0, ns),
            (7, BWD, "SQ_WAVE_CYCLES", 4 * cyc * 1024 / 4, 0, ns),      # 4 waves per SIMD
            (7, BWD, "SQ_ACTIVE_INST_VALU", 0.9 * cyc * 1024 / 4, 0, ns),
            (7, BWD, "SQ_INSTS_VALU", 1e9, 0, ns)]
    _write(tmp_path / "issue_counter_collection.csv", rows)
    d = _run("pmc_issue.py", tmp_path)["ode_self_bwd"]
    assert abs(d["eff_clock_GHz"] - 2.0) < 1e-12
    assert abs(d["valu_issue_busy_per_simd"] - 0.9) < 1e-12
    assert abs(d["avg_waves_per_simd"] - 4.0) < 1e-12
    assert d["valu_insts_per_launch"] == 1e9 and d["launches"] == 1
