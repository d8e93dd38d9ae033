"""Work partitioning for multi-GPU runs (pure Python, no device code).

* Volume: 8³ bricks are split into contiguous x-slabs (shard_bricks); rank r owns bricks
  [x0, x1) along x, i.e. voxels [8·x0, min(8·x1, Dx)). Warp + integrate need no halo: every voxel
  is independent (tsdf.py:442-494), node transforms and the frame are replicated.
* GN solve: matches are split into contiguous ranges (match_range); each rank assembles JᵀJ/Jᵀr of
  its range, rank 0 adds the ARAP and motion rows, and one all-reduce (sum) per GN iteration gives
  every rank the identical system (model.py:641-662 is a plain sum over residual rows).
"""


def shard_bricks(n_bricks_x, rank, world):
    """Contiguous x-slab of bricks for `rank` of `world`: returns (x0, x1)."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    base, rem = divmod(int(n_bricks_x), world)
    x0 = rank * base + min(rank, rem)
    return x0, x0 + base + (1 if rank < rem else 0)


def match_range(n_matches, rank, world):
    """Contiguous match range [m0, m1) assembled by `rank`."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"bad rank/world {rank}/{world}")
    return (n_matches * rank) // world, (n_matches * (rank + 1)) // world
