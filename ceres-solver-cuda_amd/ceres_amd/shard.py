"""Multi-GPU sharding of a Schur-ordered BAL Program.

One process per GPU.  Residual blocks are independent, so the Program is
cut into contiguous, equal-count block ranges whose cut points are moved to
point-bucket boundaries: every point (E block) belongs to exactly one rank,
so its Jacobian cells, residuals and gradient rows are written by one rank
only.  Each rank holds every camera (13,682 x 72 B ~ 1 MB for
problem-13682) and only its points, observations and ids.

The rank-local BlockSparseMatrix ([E cells | F cells] of its blocks) maps
onto two contiguous strips of the global one:
    E strip  [6*b0, 6*b1)                 (points' cells, 2x3 each)
    F strip  [6*O + 18*b0, 6*O + 18*b1)   (cameras' cells, 2x9 each)
and a rank-local CompressedRowSparseMatrix onto one strip
    rows     [24*b0, 24*b1)
Residuals: [2*b0, 2*b1).  The only exchange step is the scalar cost
(and, with the gradient, the camera rows), all-reduced over RCCL.
"""
from dataclasses import dataclass

import numpy as np

from . import bal
from .problem import BLOCK_SPARSE, COMPRESSED_ROW


def point_bucket_cuts(pt_idx, num_points, world, align=4, search=64):
    """Block ranges per rank, cut at point-bucket boundaries.  pt_idx must be
    point-major (nondecreasing).  Returns (point_cuts, block_cuts), each of
    length world + 1.

    Each cut goes to the first point boundary at or after its target.  It
    is then moved on to the next boundary whose block index is a multiple of
    `align` (looking at most `search` boundaries ahead), but only while that
    stays below the next rank's target, so that alignment never empties or
    overruns a rank; otherwise the plain boundary stays.  With align = 4 every
    rank's block count is then a multiple of 4, so its rank-local
    BlockSparseMatrix F cells (at 6 * blocks doubles) start on a 64-byte
    sector and the evaluator's store windows need no partial sectors
    (DESIGN.md §4.3).  Ranks can be empty only when there are fewer points
    than ranks."""
    pt_idx = np.asarray(pt_idx)
    if pt_idx.size and np.any(np.diff(pt_idx) < 0):
        raise ValueError("observations must be point-major (Schur order)")
    counts = np.bincount(pt_idx, minlength=num_points)
    csum = np.concatenate([[0], np.cumsum(counts)])
    O = int(csum[-1])
    pc = [0]
    for r in range(1, world):
        target = O * r // world
        next_target = O * (r + 1) // world
        p = int(np.searchsorted(csum, target))  # first point whose start >= target
        p = max(p, pc[-1])
        if align > 1:
            window = csum[p:p + search]
            hit = np.nonzero((window % align == 0) & (window < next_target))[0]
            if hit.size:
                p += int(hit[0])
        pc.append(min(p, int(num_points)))
    pc.append(int(num_points))
    bc = [int(csum[p]) for p in pc]
    return pc, bc


@dataclass
class Shard:
    rank: int
    world: int
    points: tuple     # [p0, p1)
    blocks: tuple     # [b0, b1)
    num_observations: int
    format: str
    # Held (constant) cameras, BlockSparseMatrix: F cells exist only for the
    # blocks of active cameras -- (cells before b0, cells in the shard).
    f_cells: tuple = None

    @property
    def residual_strip(self):
        b0, b1 = self.blocks
        return (2 * b0, 2 * b1)

    def jacobian_strips(self, cam_size=9, pt_size=3, nres=2):
        """[(local_begin, global_begin, length), ...] mapping the rank-local
        Jacobian values onto the global array."""
        b0, b1 = self.blocks
        n = b1 - b0
        O = self.num_observations
        if self.format == BLOCK_SPARSE:
            e, f = nres * pt_size, nres * cam_size
            f0, fn = self.f_cells if self.f_cells is not None else (b0, n)
            return [(0, e * b0, e * n), (e * n, e * O + f * f0, f * fn)]
        if self.f_cells is not None:
            raise NotImplementedError("held cameras: BlockSparseMatrix strips only")
        w = nres * (cam_size + pt_size)
        return [(0, w * b0, w * n)]


def gradient_maps(shard, num_points, num_cameras, cam_size=9, pt_size=3):
    """(point map, camera map): local -> global gradient ranges.  Point rows
    are disjoint across ranks; camera rows are summed (all-reduce)."""
    p0, p1 = shard.points
    n = p1 - p0
    return ((0, pt_size * p0, pt_size * n),
            (pt_size * n, pt_size * num_points, cam_size * num_cameras))


def shard_program(cameras, points, cam_idx, pt_idx, obs, rank, world, loss=None,
                  format=BLOCK_SPARSE, compile=True, quaternion_manifold=False,
                  constant_cameras=()):
    """The rank's Program: its points (renumbered from 0), every camera, its
    observations; same functor, loss and camera manifold as the full problem."""
    pc, bc = point_bucket_cuts(pt_idx, points.shape[0], world)
    p0, p1, b0, b1 = pc[rank], pc[rank + 1], bc[rank], bc[rank + 1]
    prog = bal.program(cameras, points[p0:p1], cam_idx[b0:b1],
                       np.asarray(pt_idx[b0:b1]) - p0, obs[b0:b1], loss=loss, format=format,
                       compile=compile, quaternion_manifold=quaternion_manifold,
                       constant_cameras=constant_cameras)
    f_cells = None
    if len(constant_cameras):
        active = ~np.isin(np.asarray(cam_idx), np.asarray(constant_cameras))
        f_cells = (int(active[:b0].sum()), int(active[b0:b1].sum()))
    return prog, Shard(rank, world, (p0, p1), (b0, b1), len(cam_idx), format, f_cells)


def assemble(shards, locals_, total):
    """Scatter rank-local Jacobian value arrays into the global array
    (what the per-rank strip D2H copies do on the host)."""
    out = np.full(total, np.nan)
    for sh, vals in zip(shards, locals_):
        for lb, gb, n in sh.jacobian_strips():
            out[gb:gb + n] = vals[lb:lb + n]
    return out
