"""bench.py's CPU-only line (BASELINE.json configs[0]): problem-16 on the
CPU ProgramEvaluator restatement at num_threads = 1, no GPU -- the
reference's plumbing configuration.  The oracle is the measured thing here
only because configs[0] is a CPU configuration; bench.py's GPU lines never
call it except for cpu_baseline."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpu_only_line_is_configs0():
    out = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--cpu-only",
                          "--steps", "2"], capture_output=True, text=True, timeout=600,
                         cwd=REPO)
    assert out.returncode == 0, out.stderr[-2000:]
    line = json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])
    assert "problem-16" in line["metric"] and "configs[0]" in line["metric"]
    assert line["n_gpus"] == 0 and line["value"] > 0
    assert line["config"]["blocks"] == 83718
    assert line["residual_only"]["value"] > line["value"]  # no Jets, no Jacobian stores
