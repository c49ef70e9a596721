"""tools/c3_trace.py's trace analysis (CPU): blocks split at host gaps, the
modal kernel count picks the timed blocks, span / busy / gap medians."""
import csv
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _trace(path, blocks):
    with open(path, "w", newline="") as fh:
        w = csv.DictWriter(fh, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 0
        for kernels in blocks:
            for name, dur_us, gap_us in kernels:
                t += int(gap_us * 1000)
                w.writerow({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + int(dur_us * 1000)})
                t += int(dur_us * 1000)
            t += 2_000_000                     # 2 ms host gap between blocks


def test_analyse_splits_blocks(tmp_path):
    warm = [[("plan_build(int)", 50.0, 1.0)] * 7]            # a block of another size
    block = [("a(int)", 5.0, 0.0), ("b(int)", 10.0, 1.0), ("c(int)", 4.0, 2.0)]
    p = tmp_path / "run_kernel_trace.csv"
    _trace(p, warm + [block] * 5)
    out = subprocess.run([sys.executable, os.path.join(REPO, "tools", "c3_trace.py"), "analyse", str(p),
                          "--gap-us", "500", "--blocks", "4"], capture_output=True, text=True, check=True).stdout
    d = json.loads(out)
    assert d["blocks"] == 4 and d["kernels_per_block"] == 3
    assert abs(d["busy_us_median"] - 19.0) < 1e-6
    assert abs(d["span_us_median"] - 22.0) < 1e-6        # 5 + 1 + 10 + 2 + 4
    assert abs(d["gaps_us_median"] - 3.0) < 1e-6
    assert [k["name"] for k in d["kernels"]] == ["a", "b", "c"]
