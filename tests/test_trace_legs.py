"""CPU tests of tools/trace_legs.py, which pairs a rocprofv3 kernel trace of a
bench.py run with the legs bench.py recorded (--legs-out): library-internal
dispatches (the routine-table probe, a JIT prefetch's one-workgroup warm
launch) are skipped, the bsr name forms map to their traced kernels, and any
other name mismatch makes the tool exit non-zero."""
import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "trace_legs.py")
NS = "zfec_hip::(anonymous namespace)::"
FIELDS = ["Dispatch_Id", "Kernel_Name", "Grid_Size_X", "Workgroup_Size_X", "Start_Timestamp", "End_Timestamp"]


def write_trace(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=FIELDS)
        w.writeheader()
        t = 1000
        for i, (name, grid, us) in enumerate(rows):
            w.writerow({"Dispatch_Id": i + 1, "Kernel_Name": name, "Grid_Size_X": grid, "Workgroup_Size_X": 256,
                        "Start_Timestamp": t, "End_Timestamp": t + int(us * 1000)})
            t += int(us * 1000) + 500


def run(tmp_path, legs, rows):
    lp, tp, op = tmp_path / "legs.json", tmp_path / "kt.csv", tmp_path / "out.json"
    lp.write_text(json.dumps({"workload": "cfg4", "legs": legs}))
    write_trace(tp, rows)
    p = subprocess.run([sys.executable, TOOL, str(lp), str(tp), str(op)], capture_output=True, text=True)
    return p, (json.loads(op.read_text()) if op.exists() else None)


def test_internal_dispatches_skipped_and_forms_mapped(tmp_path):
    rows = [
        ("void %smatapply_reg<3, 7, 3, true, true>(%sRegJob<3, 7>)" % (NS, NS), 5462, 40.0),
        ("void %sbsr_table_probe(unsigned long*)" % NS, 1, 3.0),
        ("zfec_hip_bitslice_k20_r40_676996c653b3266d", 256, 0.5),  # prefetch warm launch: one workgroup
        ("void %smatapply_bsr<10, true, false, %sBsrTblJob>(%sBsrTblJob)" % (NS, NS, NS), 262144, 660.0),
        ("void %smatapply_bsr<10, false, false, %sBsrJob>(%sBsrJob)" % (NS, NS, NS), 262144, 400.0),
        ("void %smatapply_bsr_solo<6>(%sBsrJob)" % (NS, NS), 5000, 60.0),
        ("zfec_hip_bitslice_k20_r40_676996c653b3266d", 262144, 600.0),
        ("zfec_hip_bitslice_k20_r40_676996c653b3266d", 262144, 602.0),
    ]
    legs = [["encode cold", "matapply_reg<3,7>", 1], ["first launch", "matapply_bsr<10,lds,tbl>", 1],
            ["first seen", "matapply_bsr<10,lds>", 1], ["decode fresh", "matapply_bsr<6>", 1],
            ["timed loop", "zfec_hip_bitslice_k20_r40_676996c653b3266d", 2]]
    p, res = run(tmp_path, legs, rows)
    assert p.returncode == 0, p.stderr
    assert res["name_mismatches"] == 0 and res["internal_skipped"] == 2 and res["paired"] == len(rows)
    tl = res["legs"]["timed loop | zfec_hip_bitslice_k20_r40_676996c653b3266d"]
    assert tl["launches"] == 2 and abs(tl["mean_us"] - 601.0) < 0.01
    assert abs(res["legs"]["first launch | matapply_bsr<10,lds,tbl>"]["mean_us"] - 660.0) < 0.01


def test_mismatch_fails(tmp_path):
    rows = [("void %smatapply_reg<3, 3, 3, false, false>(%sRegJob<3, 3>)" % (NS, NS), 5462, 24.0),
            ("void %smatapply_reg<3, 7, 3, true, true>(%sRegJob<3, 7>)" % (NS, NS), 5462, 40.0)]
    legs = [["encode cold", "matapply_reg<3,7>", 1], ["decode cold", "matapply_reg<3,3>", 1]]
    p, res = run(tmp_path, legs, rows)
    assert p.returncode != 0 and "do not match" in p.stderr
    assert res["name_mismatches"] == 2 and res["first_mismatch"]["leg"] == "encode cold"


def test_bsr_form_must_match_its_job_type(tmp_path):
    """A table-form launch recorded as the argument form is a mismatch."""
    rows = [("void %smatapply_bsr<10, true, false, %sBsrTblJob>(%sBsrTblJob)" % (NS, NS, NS), 262144, 660.0)]
    p, res = run(tmp_path, [["first seen", "matapply_bsr<10,lds>", 1]], rows)
    assert p.returncode != 0 and res["name_mismatches"] == 1
