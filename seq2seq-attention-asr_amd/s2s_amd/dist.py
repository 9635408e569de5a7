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


def allreduce_buckets(grads: torch.Tensor, buckets, wait=None, comm_stream=None):
    """Bucketed gradient sum over ranks, overlapped with the rest of the step.

    buckets: [(offset, count)] in the order the step finalises them (ChorowskiBaseline.grad_buckets:
    the decoder, then the encoder layers top-down).  On GPUs, wait(i, comm_stream) makes comm_stream
    wait for bucket i's "final" event (ChorowskiBaseline.wait_bucket, recorded inside the step, also
    under hipGraph replay), and bucket i's all-reduce is issued from comm_stream -- so it runs on
    RCCL while the BPTT of the encoder layers below is still in flight.  The caller's current stream
    then waits for every bucket (the optimizer reads the summed gradient).  Sums are elementwise,
    so the result equals one all-reduce of the flat buffer.  On CPU tensors (gloo) wait(i, None) is called
    before bucket i's all-reduce is issued (tests drive the bucket order with it)."""
    if world() == 1:
        return grads
    works = []
    cur = torch.cuda.current_stream() if grads.is_cuda else None
    for i, (off, n) in enumerate(buckets):
        view = grads[off:off + n]
        if grads.is_cuda:
            if wait is not None:
                wait(i, comm_stream)
            else:
                comm_stream.wait_stream(cur)
            with torch.cuda.stream(comm_stream):
                works.append(dist.all_reduce(view, async_op=True))
        else:  # CPU tensors (gloo): wait(i, None) is the host-side "bucket i is final" hook
            if wait is not None:
                wait(i, None)
            works.append(dist.all_reduce(view, async_op=True))
    for w in works:
        w.wait()
    return grads


def allreduce_mean_scalar(x: float, device=None) -> float:
    if world() == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t)
    return float(t.item()) / world()


def reduce_failure_flag(flag: torch.Tensor) -> torch.Tensor:
    """MAX of every rank's failure flag (Adadelta.failure_flag: 1.0 where a persistent launch of the step failed),
    in place.  A failing rank's invalid gradients are already in every replica's all-reduced sum, so the update
    must be skipped on EVERY rank (Adadelta.step(skip_flag=flag)), or the replicas diverge.  Issued on the
    current stream (RCCL) or as a gloo collective on CPU tensors."""
    if world() > 1:
        dist.all_reduce(flag, op=dist.ReduceOp.MAX)
    return flag
