"""Data parallelism for the training step.

Utterances are independent (timit/timit.lua:240-295 accumulates per-utterance gradients), so
each rank runs its own B utterances and the flat gradient is summed across ranks once per step.
With every rank scaling its local sum by 1/(B * world), the all-reduced buffer equals the
reference's `gradients:div(opt.batchSize)` over the global batch (timit.lua:292-295).
Backend-agnostic: RCCL ("nccl") on GPUs, gloo on CPU tensors (tests).
"""
import torch
import torch.distributed as dist


def world():
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def step_scale(local_batch: int) -> float:
    """scale passed to the local step so that the all-reduced gradient is the global-batch mean."""
    n = local_batch * world()
    return 1.0 / n if n > 1 else 1.0


def allreduce_gradients(flat_grads: torch.Tensor, bucket_elems: int = 0):
    """Sum the flat gradient over ranks in place (one collective, or buckets of bucket_elems)."""
    if world() == 1:
        return flat_grads
    if bucket_elems <= 0 or bucket_elems >= flat_grads.numel():
        dist.all_reduce(flat_grads)
    else:
        for off in range(0, flat_grads.numel(), bucket_elems):
            dist.all_reduce(flat_grads[off:off + bucket_elems])
    return flat_grads


def allreduce_mean_scalar(x: float, device=None) -> float:
    if world() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item()) / world()
