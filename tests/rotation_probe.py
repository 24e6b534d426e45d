#!/usr/bin/env python3
"""Test helper (not collected): parity errors of
tests/test_rotation_paths_gpu.py's problems for one
library build (default lib/libcse.so; --lib another build of the same ABI),
without asserting: norm-wise and per-element figures for every output."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
sys.path.insert(0, os.path.join(REPO, "oracle"))
from ceres_amd import _cse  # noqa: E402

if "--lib" in sys.argv:
    _cse.use_library(os.path.abspath(sys.argv[sys.argv.index("--lib") + 1]))

import numpy as np  # noqa: E402
import ceres_amd as ca  # noqa: E402
import oracle_py as O  # noqa: E402
from parity_util import elementwise_report  # noqa: E402
import test_rotation_paths_gpu as T  # noqa: E402

for kind in ("small", "large", "mixed", "beyond_pi"):
    for fmt in (ca.BLOCK_SPARSE,):
        prog = T._problem(T._angles(kind, 3), 3, ca.Loss.huber(1.0), fmt)
        op = O.OracleProgram.from_program(prog, apply_loss_function=True)
        ok_r, cost_r, r_r, g_r, j_r = op.evaluate(prog.state, None, num_threads=8)
        ev = ca.Evaluator(prog)
        ok_g, cost_g, r_g, g_g, j_g = ev.evaluate()
        ev.close()
        out = [kind, f"ok {ok_g}/{ok_r}", f"cost {abs(cost_g - cost_r) / abs(cost_r):.2e}"]
        for name, a, b in (("r", r_g, r_r), ("g", g_g, g_r), ("J", j_g, j_r)):
            nrm = np.linalg.norm(a - b) / np.linalg.norm(b)
            rep = elementwise_report(a, b)
            out.append(f"{name}: norm {nrm:.2e} bound_ratio {rep['bound_ratio']:.3f}")
        out.append(f"|g|/(|J||r|) {np.linalg.norm(g_r) / (np.linalg.norm(j_r) * np.linalg.norm(r_r)):.2e}")
        print("  ".join(out), flush=True)
