"""world_size-2 gloo test of the data-parallel step semantics on CPU:
per-rank local gradients (oracle, reference per-utterance semantics) scaled by 1/(B*world) and
all-reduced equal the single-process gradient over the global batch (timit/timit.lua:292-295)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(abi=False):
    """abi: dims the C ABI accepts (hidden / state sizes multiples of 16), for the real bucket layout"""
    from oracle import s2s_oracle as orc
    if abi:
        return orc.ModelConfig(inputFrameSize=6, hiddenFrameSize=16, outputFrameSize=16, scoreDepth=16,
                               stateDepth=16, outputDepth=7, mlpDepth=3, maxoutWindow=2, numLayers=2)
    return orc.ModelConfig(inputFrameSize=6, hiddenFrameSize=4, outputFrameSize=4, scoreDepth=5, stateDepth=4,
                           outputDepth=7, mlpDepth=3, maxoutWindow=2, numLayers=2)


def _worker(rank, world, port, B, out_path, buckets):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import s2s_oracle as orc
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "s2s_dist", os.path.join(ROOT, "seq2seq-attention-asr_amd", "s2s_amd", "dist.py"))
    sd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sd)
    cfg = _cfg(buckets == "events")
    P = orc.init_params(cfg, seed=5)
    x, labels = orc.synthetic_batch(cfg, B * world, 6, 4, seed=9, pad=1, eos=2)
    xs, ls = x[rank * B:(rank + 1) * B], labels[rank * B:(rank + 1) * B]
    # local per-utterance gradient sum (reference semantics), scaled for the global mean
    G = orc.zeros_like_params(P)
    for b in range(B):
        _, g1, _, _ = orc.training_step(xs[b:b + 1], ls[b:b + 1], P, cfg)
        for k in G:
            G[k] += g1[k]
    flat = torch.tensor(orc.flatten(G, cfg)) * (sd.step_scale(B) * 1.0)
    if buckets == "model":
        # the step's bucket order (decoder, then encoder layers top-down) over the flat layout
        import s2s_amd
        mcfg = s2s_amd.ModelConfig(**{f: getattr(cfg, f) for f in (
            "inputFrameSize", "hiddenFrameSize", "outputFrameSize", "scoreDepth", "stateDepth", "outputDepth",
            "mlpDepth", "maxoutWindow", "numLayers")})
        mb = s2s_amd.model.buckets_of_shapes(s2s_amd.param_shapes(mcfg), cfg.numLayers)
        cover = sorted(mb)
        assert cover[0][0] == 0 and sum(n for _, n in mb) == flat.numel()
        assert all(o + n == o2 for (o, n), (o2, _) in zip(cover, cover[1:]))
        sd.allreduce_buckets(flat, mb)
    elif buckets == "events":
        # the real bucket layout from the C ABI (s2s_model_bucket) and the step's "bucket i final" hook: the
        # buffer holds garbage until wait(i) finalises bucket i (as the step's event does on the GPU), so a
        # bucket reduced before its wait -- or a wrong layout -- corrupts the sum
        import s2s_amd
        mcfg = s2s_amd.ModelConfig(**{f: getattr(cfg, f) for f in (
            "inputFrameSize", "hiddenFrameSize", "outputFrameSize", "scoreDepth", "stateDepth", "outputDepth",
            "mlpDepth", "maxoutWindow", "numLayers")})
        mb = s2s_amd.model.grad_buckets(mcfg)
        final = flat.clone()
        flat.fill_(float("nan"))
        order = []

        def wait(i, stream):
            assert stream is None
            off, n = mb[i]
            flat[off:off + n] = final[off:off + n]
            order.append(i)
        sd.allreduce_buckets(flat, mb, wait=wait)
        assert order == list(range(cfg.numLayers + 1)), order
        # decoder first, then encoder layers top-down: bucket 0 starts where the encoder ends
        assert mb[0][0] + mb[0][1] == flat.numel() and mb[-1][0] == 0
    else:
        sd.allreduce_gradients(flat, bucket_elems=buckets)
    if rank == 0:
        np.save(out_path, flat.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("buckets", [0, 37, "model", "events"])
def test_dp_allreduce_equals_global_batch(tmp_path, buckets):
    from oracle import s2s_oracle as orc
    world, B = 2, 2
    out = str(tmp_path / "g.npy")
    mp.start_processes(_worker, args=(world, _free_port(), B, out, buckets), nprocs=world, start_method="spawn")
    got = np.load(out)
    cfg = _cfg(buckets == "events")
    P = orc.init_params(cfg, seed=5)
    x, labels = orc.synthetic_batch(cfg, B * world, 6, 4, seed=9, pad=1, eos=2)
    _, G, _, _ = orc.training_step(x, labels, P, cfg)
    np.testing.assert_allclose(got, orc.flatten(G, cfg), rtol=1e-10, atol=1e-13)


def _flag_worker(rank, world, port, out_path, failing):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "s2s_dist", os.path.join(ROOT, "seq2seq-attention-asr_amd", "s2s_amd", "dist.py"))
    sd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sd)
    # Adadelta.failure_flag's value on this rank: 1.0 where the step's persistent launch failed
    flag = torch.tensor([1.0 if rank == failing else 0.0], dtype=torch.float32)
    sd.reduce_failure_flag(flag)
    np.save(f"{out_path}.{rank}.npy", flag.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("failing", [-1, 0, 1])
def test_failure_flag_reduced_across_ranks(tmp_path, failing):
    """a rank whose persistent launch failed has already sent invalid gradients into the all-reduce,
    so every rank must skip that update.  dist.reduce_failure_flag (the MAX all-reduce of Adadelta.failure_flag)
    gives every rank the same flag: 1 if any rank failed, else 0 (world size 2, gloo)."""
    world = 2
    out = str(tmp_path / "f")
    mp.start_processes(_flag_worker, args=(world, _free_port(), out, failing), nprocs=world, start_method="spawn")
    got = [float(np.load(f"{out}.{r}.npy")[0]) for r in range(world)]
    assert got == [0.0 if failing < 0 else 1.0] * world


def _flag_worker_rccl(rank, world, port, out_path, failing):
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(rank)
    dist.init_process_group("nccl", rank=rank, world_size=world)
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "s2s_dist", os.path.join(ROOT, "seq2seq-attention-asr_amd", "s2s_amd", "dist.py"))
    sd = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(sd)
    flag = torch.tensor([1.0 if rank == failing else 0.0], dtype=torch.float32, device="cuda")
    sd.reduce_failure_flag(flag)  # on the current stream (RCCL), the flag stays on the device
    np.save(f"{out_path}.{rank}.npy", flag.cpu().numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("failing", [-1, 1])
def test_failure_flag_reduced_across_ranks_rccl(tmp_path, failing):
    """the same MAX all-reduce of the failure flag on device tensors over RCCL (world size 2, one GPU per
    rank) -- the form bench.py's data-parallel optimizer leg uses.  Needs two GPUs (skipped on one)."""
    if torch.cuda.device_count() < 2:
        pytest.skip("needs two GPUs")
    world = 2
    out = str(tmp_path / "g")
    mp.start_processes(_flag_worker_rccl, args=(world, _free_port(), out, failing), nprocs=world, start_method="spawn")
    got = [float(np.load(f"{out}.{r}.npy")[0]) for r in range(world)]
    assert got == [0.0 if failing < 0 else 1.0] * world
