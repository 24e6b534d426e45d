"""Compare one affine variant ($CSE_AFFINE_VARIANT) with the oracle on a small
BAL problem and print where they differ (GPU box, from the repo root)."""
import os
import sys

import numpy as np

sys.path[:0] = ["ceres-solver-cuda_amd", "oracle", "tests"]
import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402
import oracle_py as O  # noqa: E402

C, P, N = (int(x) for x in (sys.argv[1:4] if len(sys.argv) > 3 else (16, 600, 2300)))
prog = bal.synthetic_program((C, P, N), loss=None, format=ca.BLOCK_SPARSE, seed=7)
ev = ca.Evaluator(prog, check_finite=False)
ok, cost, r, g, j = ev.evaluate(gradient=False)
ev.close()
ref = O.OracleProgram.from_program(prog).evaluate(prog.state, num_threads=4)
print("variant", os.environ.get("CSE_AFFINE_VARIANT"), "ok", ok, "cost", cost, "ref", ref[1])
rr = ref[2].reshape(-1, 2)
rg = r.reshape(-1, 2)
bad = np.nonzero(np.abs(rg - rr).max(axis=1) > 1e-9 * (1 + np.abs(rr).max(axis=1)))[0]
print("residual blocks bad:", len(bad), "of", len(rr))
for b in bad[:12]:
    print(f"  block {b} (chunk {b // 64}, lane {b % 64}): got {rg[b]} ref {rr[b]}")
nO = len(rr)
E = j[: 6 * nO].reshape(-1, 6)
Er = ref[4][: 6 * nO].reshape(-1, 6)
F = j[6 * nO:].reshape(-1, 18)
Fr = ref[4][6 * nO:].reshape(-1, 18)
print("E bad:", int((np.abs(E - Er).max(axis=1) > 1e-9 * (1 + np.abs(Er).max(axis=1))).sum()),
      "F bad:", int((np.abs(F - Fr).max(axis=1) > 1e-9 * (1 + np.abs(Fr).max(axis=1))).sum()))
