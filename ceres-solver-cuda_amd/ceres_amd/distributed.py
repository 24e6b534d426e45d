"""Block-sharded evaluation across GPUs (BASELINE configs[4]).

One process per GPU.  Each rank owns a point-bucket shard of the one
Schur-ordered Program (ceres_amd.shard): its points, every camera, and the
residual blocks of its points.  A rank evaluates its shard through libcse.so
on its own device; the exchange step is an all-reduce of the scalar cost and,
when the gradient is requested, of the camera rows of the gradient (RCCL over
xGMI on the real node; gloo in the CPU tests and in a 1-GPU rehearsal where
several ranks share one device).

The reference has no multi-GPU path: ProgramEvaluatorCUDA evaluates the
whole program on one device and copies residuals and Jacobian back to the
host (program_evaluator_cuda.h:98-138; the D2H seam is README.md:198-200).
Here each rank's outputs are contiguous strips of the global arrays
(Shard.residual_strip, Shard.jacobian_strips), so handing them back to the
host solve is one D2H copy per strip into pinned memory
(ShardedEvaluator.copy_strips_to_host).
"""
import numpy as np

from . import shard as _shard
from .problem import BLOCK_SPARSE, Evaluator


class ShardedEvaluator:
    """ProgramEvaluatorCUDA::Evaluate over one rank's shard.

    cameras/points/cam_idx/pt_idx/obs: the whole (point-major) BAL problem,
    identical on every rank.  `device`: this rank's HIP device index.
    Outputs live in HBM as torch tensors: `residuals`, `jacobian` (the
    rank-local strips, in the rank-local layout) and, with the gradient,
    `gradient` (local points, then every camera, summed over ranks).
    """

    def __init__(self, cameras, points, cam_idx, pt_idx, obs, rank, world, device, loss=None,
                 format=BLOCK_SPARSE, gradient=False, gradient_mode=0, stream=None, group=None,
                 quaternion_manifold=False, constant_cameras=(), jacobian_form="closed",
                 exchange=None):
        import torch
        import torch.distributed as dist
        self.torch, self.dist, self.group = torch, dist, group
        self.rank, self.world = rank, world
        self.num_points, self.num_cameras = points.shape[0], cameras.shape[0]
        # gradient rows: the active cameras only
        self.num_cameras -= len(set(int(c) for c in constant_cameras))
        # camera gradient rows: the tangent size (9 for the quaternion camera
        # on its manifold)
        self.cam_size = cameras.shape[1] - (1 if quaternion_manifold else 0)
        self.program, self.shard = _shard.shard_program(cameras, points, cam_idx, pt_idx, obs,
                                                        rank, world, loss=loss, format=format,
                                                        quaternion_manifold=quaternion_manifold,
                                                        constant_cameras=constant_cameras)
        self.device = torch.device("cuda", device)
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        self.stream = stream
        self.evaluator = Evaluator(self.program, device=device, profile=True,
                                   stream=stream.cuda_stream, gradient_mode=gradient_mode,
                                   jacobian_form=jacobian_form)
        p = self.program
        f64 = torch.float64
        dev = self.device
        self.state = torch.from_numpy(p.state).to(dev)
        self.cost = torch.zeros(1, dtype=f64, device=dev)
        self.residuals = torch.empty(p.num_residuals, dtype=f64, device=dev)
        self.jacobian = torch.empty(p.num_jacobian_values, dtype=f64, device=dev)
        self.gradient = (torch.empty(p.num_effective_parameters, dtype=f64, device=dev)
                         if gradient else None)
        # Camera rows of the local gradient: after the shard's points
        # (Schur order: points are the eliminated group, first).
        npts = self.shard.points[1] - self.shard.points[0]
        self._cam_rows = (3 * npts, 3 * npts + self.cam_size * self.num_cameras)
        # The exchange runs whenever the process group has several ranks
        # (also for replica shards, world == 1 here).  gloo reduces host
        # tensors; RCCL reduces in place in HBM.  exchange=True forces it on a
        # one-rank group (the RCCL path on a one-GPU box), False switches it off.
        grouped = dist.is_available() and dist.is_initialized()
        if exchange is None:
            self.exchange = grouped and dist.get_world_size(group) > 1
        else:
            if exchange and not grouped:
                raise ValueError("exchange=True needs an initialised process group")
            self.exchange = bool(exchange)
        self._host_reduce = self.exchange and dist.get_backend(group) == "gloo"
        self._pending = []

    # ---- evaluation -------------------------------------------------------
    def evaluate(self, residuals=True, jacobian=True, gradient=None, cost=None, overlap=False,
                 new_evaluation_point=True):
        """One Evaluate of this rank's shard, then the exchange step.

        The evaluation is asynchronous on the rank's stream.  The cost goes to
        `cost` (a one-element device tensor, default self.cost).  With
        overlap=False the all-reduce is ordered before anything queued after
        it on the stream (torch.distributed's default).  With overlap=True
        (RCCL only) the cost all-reduce runs on the collective stream while
        the next evaluation proceeds; its handle is kept until
        wait_exchange(), so each call must pass its own `cost` buffer.  The
        gradient's camera rows are always reduced in order (the gradient
        buffer is shared).  new_evaluation_point=False: the state
        equals the previous evaluation's (CSE_EVAL_SAME_POINT)."""
        gradient = self.gradient is not None if gradient is None else gradient
        if gradient and self.gradient is None:
            raise ValueError("ShardedEvaluator built without a gradient buffer")
        cost = self.cost if cost is None else cost
        ptr = lambda t, want: t.data_ptr() if (t is not None and want) else None
        self.evaluator.evaluate_device(self.state.data_ptr(), cost.data_ptr(),
                                       ptr(self.residuals, residuals),
                                       ptr(self.gradient, gradient),
                                       ptr(self.jacobian, jacobian),
                                       new_evaluation_point=new_evaluation_point)
        if self.exchange:
            # The collectives are ordered against the evaluation's stream: a
            # collective (and gloo's host copy) follows torch's current
            # stream, so it is issued with self.stream current.
            with self.torch.cuda.stream(self.stream):
                if overlap and not self._host_reduce:
                    self._pending.append(self.dist.all_reduce(cost, group=self.group,
                                                              async_op=True))
                else:
                    self._all_reduce(cost)
                if gradient:
                    lo, hi = self._cam_rows
                    self._all_reduce(self.gradient[lo:hi])

    def wait_exchange(self):
        """Order every overlapped all-reduce before later work on the stream."""
        with self.torch.cuda.stream(self.stream):
            for w in self._pending:
                w.wait()
        self._pending = []

    def _all_reduce(self, t):
        """All-reduce t (sum) after the work queued on self.stream."""
        if self._host_reduce:
            h = t.cpu()
            self.dist.all_reduce(h, group=self.group)
            t.copy_(h)
        else:
            self.dist.all_reduce(t, group=self.group)

    def wait(self):
        """cse_wait: the status of the evaluations queued so far (0 = ok)."""
        return self.evaluator.wait()

    # ---- the D2H seam: strips back to the host ------------------------------
    def host_buffers(self, pin=True):
        """Pinned host buffers for this rank's residual and Jacobian strips."""
        torch = self.torch
        p = self.program
        return (torch.empty(p.num_residuals, dtype=torch.float64, pin_memory=pin),
                torch.empty(p.num_jacobian_values, dtype=torch.float64, pin_memory=pin))

    def copy_strips_to_host(self, host_res, host_jac):
        """Queue the D2H copies of the rank's strips on its stream.  The
        rank-local arrays are the global strips (Shard.residual_strip,
        Shard.jacobian_strips) in global order, so a host solve addresses
        them at those offsets without any reshuffle."""
        with self.torch.cuda.stream(self.stream):
            host_res.copy_(self.residuals, non_blocking=True)
            host_jac.copy_(self.jacobian, non_blocking=True)

    def d2h_bytes(self):
        p = self.program
        return 8 * (p.num_residuals + p.num_jacobian_values)

    def strips(self):
        """(residual strip, [(local_begin, global_begin, length), ...])."""
        return self.shard.residual_strip, self.shard.jacobian_strips(cam_size=self.cam_size)

    def point_gradient_rows(self):
        """(local begin, global begin, length) of this rank's point rows."""
        return _shard.gradient_maps(self.shard, self.num_points, self.num_cameras,
                                    cam_size=self.cam_size)[0]

    def close(self):
        self.evaluator.close()


def assemble_gradient(shards, point_rows, camera_rows, num_points, num_cameras, cam_size=9):
    """The global gradient from each rank's point rows and the (already
    summed) camera rows."""
    g = np.full(3 * num_points + cam_size * num_cameras, np.nan)
    for sh, rows in zip(shards, point_rows):
        _, gb, n = _shard.gradient_maps(sh, num_points, num_cameras, cam_size=cam_size)[0]
        g[gb:gb + n] = rows
    g[3 * num_points:] = camera_rows
    return g
