"""Data parallelism for the regressor training step.

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).  Every rank holds the same
epoch permutation (same seed) and takes a contiguous slice of each global batch; the fused
train-step kernel normalises its loss gradient by the GLOBAL element count, so the sum of the
ranks' flat gradients (one all-reduce per step, gradient + [sse, sae] in one buffer) is exactly
the single-device gradient; the L2 term is added once, inside the optimizer kernel, after the
all-reduce.  Inference and evaluation are replicas (each rank owns whole images).
"""


def batch_slice(b0, b1, rank, world):
    """Contiguous [r0, r1) share of global batch rows [b0, b1) for `rank` (sizes differ by <= 1)."""
    nb = b1 - b0
    return b0 + (nb * rank) // world, b0 + (nb * (rank + 1)) // world


def world_info(dist_group=None):
    try:
        import torch.distributed as dist
    except ImportError:
        return 1, 0, None
    if not (dist.is_available() and dist.is_initialized()):
        return 1, 0, None
    return dist.get_world_size(dist_group), dist.get_rank(dist_group), dist


def all_reduce_grad(grad, dist_group=None):
    """Sum the flat gradient buffer (params + loss sums) over ranks: one collective per step."""
    world, _, dist = world_info(dist_group)
    if world > 1:
        dist.all_reduce(grad, group=dist_group)
    return grad
