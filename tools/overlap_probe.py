#!/usr/bin/env python3
"""Probe: do two evaluations on two HIP streams overlap usefully?

Times (a) the fused-gradient evaluation of problem-13682 alone, (b) a
residual+Jacobian evaluation alone, (c) both queued on two streams at once,
and (d) both on one stream, to size what splitting the gradient's camera
gather from the evaluation (running it beside the next half) could gain.
"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ceres-solver-cuda_amd"))

import ceres_amd as ca  # noqa: E402
from ceres_amd import bal  # noqa: E402


def main():
    import torch
    dev = torch.device("cuda", 0)
    f64 = torch.float64
    prog = bal.synthetic_program("problem-13682-4456117", loss=ca.Loss.huber(1.0))
    sa = torch.cuda.Stream(dev)
    sb = torch.cuda.Stream(dev)
    ea = ca.Evaluator(prog, device=0, stream=sa.cuda_stream)
    eb = ca.Evaluator(prog, device=0, stream=sb.cuda_stream)
    state = torch.from_numpy(prog.state).to(dev)
    bufs = []
    for _ in range(2):
        bufs.append(dict(cost=torch.zeros(1, dtype=f64, device=dev),
                         r=torch.empty(prog.num_residuals, dtype=f64, device=dev),
                         j=torch.empty(prog.num_jacobian_values, dtype=f64, device=dev),
                         g=torch.empty(prog.num_effective_parameters, dtype=f64, device=dev)))

    def grad_eval(ev, b):
        ev.evaluate_device(state.data_ptr(), b["cost"].data_ptr(), b["r"].data_ptr(),
                           b["g"].data_ptr(), b["j"].data_ptr())

    def jac_eval(ev, b):
        ev.evaluate_device(state.data_ptr(), b["cost"].data_ptr(), b["r"].data_ptr(), None,
                           b["j"].data_ptr())

    def timed(fn, reps=10):
        fn()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize(dev)
        return (time.perf_counter() - t0) / reps * 1e3

    for rnd in range(2):
        ta = timed(lambda: grad_eval(ea, bufs[0]))
        tb = timed(lambda: jac_eval(eb, bufs[1]))
        tc = timed(lambda: (grad_eval(ea, bufs[0]), jac_eval(eb, bufs[1])))
        td = timed(lambda: (grad_eval(ea, bufs[0]), jac_eval(ea, bufs[1])))
        print(f"round {rnd}: gradient eval {ta:.3f} ms, Jacobian eval {tb:.3f} ms, "
              f"both on two streams {tc:.3f} ms, both on one stream {td:.3f} ms", flush=True)
    assert ea.wait() == 0 and eb.wait() == 0
    ea.close()
    eb.close()


if __name__ == "__main__":
    main()
