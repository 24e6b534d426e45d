"""Product hygiene on the GPU: environment variables cannot change results,
and evaluators release every device buffer."""
import os

import numpy as np
import pytest

import ceres_amd as ca
from ceres_amd import bal

pytestmark = pytest.mark.gpu

# Names of the variables older builds (and the round-5 tuning build) honoured.
STRAY = {"CSE_AFFINE_VARIANT": "21", "CSE_VALUES_VARIANT": "3", "CSE_WG_PER_CU": "1",
         "CSE_NO_DMA_GATHER": "1", "CSE_ATOMIC_GRADIENT": "1", "CSE_TUNE_VARIANT": "5",
         "CSE_PIPE_WAVES": "2", "CSE_STREAM_WAVES": "1", "CSE_TIMELINE": "/dev/null"}


def _evaluate_all(prog):
    ev = ca.Evaluator(prog)
    try:
        out = [ev.evaluate(), ev.evaluate(jacobian=False, gradient=False),
               ev.evaluate(residuals=False, jacobian=False, gradient=False)]
    finally:
        ev.close()
    return out


def test_stray_cse_environment_has_no_effect(gpu):
    prog = bal.synthetic_program((20, 900, 3500), loss=ca.Loss.huber(1.0), seed=17)
    clean = _evaluate_all(prog)
    saved = {k: os.environ.get(k) for k in STRAY}
    try:
        os.environ.update(STRAY)
        dirty = _evaluate_all(prog)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    for a, b in zip(clean, dirty):
        assert a[0] == b[0] and a[1] == b[1]
        for x, y in zip(a[2:], b[2:]):
            assert (x is None and y is None) or np.array_equal(x, y)


def test_create_evaluate_destroy_does_not_leak(gpu):
    # Every evaluator buffer -- group tables, gradient plans, fused-gradient
    # scratch, CGNR scratch, host-path staging -- is released by cse_destroy.
    import torch
    prog = bal.synthetic_program((30, 4000, 16000), loss=ca.Loss.huber(1.0), seed=4)
    dev = torch.device("cuda", 0)
    x = torch.ones(prog.num_effective_parameters, dtype=torch.float64, device=dev)
    y = torch.zeros_like(x)
    jac = torch.empty(prog.num_jacobian_values, dtype=torch.float64, device=dev)
    st = torch.from_numpy(prog.state).to(dev)
    cost = torch.zeros(1, dtype=torch.float64, device=dev)

    def cycle():
        ev = ca.Evaluator(prog, device=0)
        ev.evaluate()  # host path: staging buffers, fused gradient
        ev.evaluate_device(st.data_ptr(), cost.data_ptr(), None, None, jac.data_ptr())
        ev.cgnr_multiply_device(jac.data_ptr(), None, x.data_ptr(), y.data_ptr())
        ev.plus(prog.state, np.zeros(prog.num_effective_parameters))
        assert ev.wait() == 0
        ev.close()

    cycle()
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info(dev)
    for _ in range(12):
        cycle()
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info(dev)
    # A leak of even the smallest per-evaluator buffer that matters (the
    # 1.3 MB camera-contribution scratch) would exceed this after 12 cycles.
    assert free0 - free1 < 2 << 20, (free0, free1)
