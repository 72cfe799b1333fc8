"""scripts/trace_summary.py: per-workload kernel averages from a rocprofv3
kernel trace (host-only; no GPU)."""
import csv
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_splits_k1_by_duration_and_others_by_grid(tmp_path):
    rows = [  # (kernel name, grid x, duration ms)
        ("void sdgpu::k_leaves3<5>(unsigned char const*)", 327680, 13.5),
        ("void sdgpu::k_leaves3<5>(unsigned char const*)", 327680, 14.5),
        ("void sdgpu::k_leaves3<5>(unsigned char const*)", 327680, 0.3),
        ("sdgpu::k_bucket_group(HIP_vector_type<unsigned int, 4u> const*)", 4194304, 0.13),
        ("sdgpu::k_bucket_group(HIP_vector_type<unsigned int, 4u> const*)", 131072, 0.01),
        ("void at::native::elementwise_kernel<128>()", 1024, 1.0),
    ]
    path = tmp_path / "run_kernel_trace.csv"
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp", "Grid_Size_X"])
        t = 1_000_000
        for name, grid, ms in rows:
            w.writerow([name, t, t + int(ms * 1e6), grid])
            t += int(ms * 1e6) + 1000
    out = tmp_path / "summary.txt"
    subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_summary.py"), str(path),
                    str(out)], check=True, capture_output=True)
    lines = {tuple(l.split()[:2]): l.split()[2:] for l in out.read_text().splitlines()[1:]}
    assert lines[("k_leaves3", "1M-file")][0:2] == ["step", "2"]
    assert abs(float(lines[("k_leaves3", "1M-file")][2]) - 14.0) < 1e-6
    assert lines[("k_leaves3", "other")][0] == "1"
    assert lines[("k_bucket_group", "4194304")][0] == "1"
    assert lines[("k_bucket_group", "131072")][0] == "1"
    assert not any(k[0].startswith("void") or "elementwise" in k[0] for k in lines)
