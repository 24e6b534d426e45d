#!/usr/bin/env python3
"""Write the bench's problem-13682 inputs as raw binaries for
tools/membench2 (MB_INPUTS=<dir>): ids int32[O][2] (camera, point),
obs double[O][2], points double[P][3], cameras repacked at 10 doubles."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))
from ceres_amd import bal  # noqa: E402

out = sys.argv[1]
os.makedirs(out, exist_ok=True)
C, P, O = bal.CONFIGS["problem-13682-4456117"]
cams, pts, ci, pi, obs = bal.synthetic(C, P, O)
np.stack([ci, pi], 1).astype(np.int32).tofile(os.path.join(out, "ids.bin"))
np.ascontiguousarray(obs, np.float64).tofile(os.path.join(out, "obs.bin"))
np.ascontiguousarray(pts, np.float64).tofile(os.path.join(out, "pts.bin"))
c80 = np.zeros((C, 10))
c80[:, :9] = cams
c80.tofile(os.path.join(out, "cam80.bin"))
print("wrote", out)
