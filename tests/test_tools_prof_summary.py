"""CPU: tools/prof_summary.py -- the steady-state window and the per-(kernel, grid) table it
prints from a rocprofv3 ``--kernel-trace`` CSV (synthetic trace of the same columns)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, steps=6):
    # a warm-up (autotune) burst that must fall outside the window, then `steps` identical steps
    rows, t = [], 0
    for _ in range(5):
        rows.append(("void grace::gemm_f32_kernel<64, 64, 0, 1>(Args)", 9, 50_000))
        t += 1
    step = [("void grace::bn_reduce_kernel<float, true>(Red)", 25088, 12_000),
            ("void grace::bn_reduce_kernel<float, true>(Red)", 133888, 98_000),
            ("Cijk_Ailk_Bjlk_S_B", 64, 30_000),
            ("void grace::topk2_split_kernel(float const*)", 426752, 36_000)]
    for _ in range(steps):
        rows.extend(step)
    out, t = [], 0
    for name, grid, dur in rows:
        out.append({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + dur,
                    "Grid_Size_X": grid, "Grid_Size_Y": 1})
        t += dur + 1000
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=list(out[0]))
        w.writeheader()
        w.writerows(out)


def test_window_and_grid_table(tmp_path):
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof_summary.py"), str(p), "--steps", "3",
                        "--marker", "topk2_split", "--per-step-markers", "1", "--grid-match", "grace::"],
                       capture_output=True, text=True, check=True)
    out = r.stdout
    assert "kernels 4/step" in out  # the warm-up GEMMs are outside the window
    assert "gemm_f32" not in out
    lines = [ln.split() for ln in out.splitlines()]
    big = next(ln for ln in lines if len(ln) > 4 and ln[3] == "133888x1")
    small = next(ln for ln in lines if len(ln) > 4 and ln[3] == "25088x1")
    assert float(big[0]) == 98.0 and float(big[1]) == 1.0  # us/step, calls/step
    assert float(small[2]) == 12.0  # mean us
    table = out.split("per (kernel, grid)")[1].split("\n\n")[0]
    assert "Cijk" not in table  # only the kernels matching --grid-match
