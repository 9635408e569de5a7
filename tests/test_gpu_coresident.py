"""GPU: the persistent launches beside a long-running kernel on another stream.

Data parallel runs RCCL's all-reduce kernels on a communication stream while the encoder BPTT's persistent launches
run (s2s_amd.dist.allreduce_buckets; bench.py --gpus N).  Those launches need every member of a chain resident at
once (chain members hand data to each other every step), and the dispatcher does not keep other kernels off the
chains' CUs.  The stand-in here (s2s_debug_lds_hog) is a bounded kernel whose workgroups each hold a block of LDS and
stay resident for a few milliseconds -- launched on a second stream right in front of a config-2 step (B = 32,
L = 128, T = 40; overlap context: exclusive-CU persistent workgroups, side-stream weight gradients), or delayed so
that it lands during the encoder BPTT.  Whatever the dispatcher does with the persistent grids beside it (members
delayed until the hog's CUs free up, members sharing a CU with it), the step must complete with status 0 and with
gradients bitwise equal to the same step run alone: the hand-off waits are bounded by polls, not by time, so a
member that is held back only delays its chain.
"""
import ctypes
import time

import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s2s():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_lds_hog
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_double, ctypes.c_void_p]
    fn.restype = ctypes.c_int
    return s2s_amd


def _batch(cfg, B, L, T, seed):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, L, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, T), generator=g).to(torch.int32).cuda()
    return x, lab


# (hog workgroups, LDS per workgroup in KB, hog duration in us, delay of the hog behind the step's start in us):
# RCCL-like (a few dozen channels) and whole-chip occupancy, from the step's start and during the encoder BPTT
CASES = [(64, 48, 6000, 0), (256, 64, 6000, 0), (64, 32, 4000, 2200), (512, 40, 3000, 2500)]


@pytest.mark.parametrize("nwg,lds_kb,usec,delay", CASES)
def test_config2_step_beside_resident_lds_kernel(s2s, nwg, lds_kb, usec, delay):
    from s2s_amd import _lib
    cfg = s2s.ModelConfig()
    B, L, T = 32, 128, 40
    m = s2s.ChorowskiBaseline(cfg, overlap=True)
    x, lab = _batch(cfg, B, L, T, 11)
    main, comm = torch.cuda.Stream(), torch.cuda.Stream()
    out = torch.zeros(max(nwg, 1), device="cuda")
    # the step alone (twice: the first sizes every buffer)
    for _ in range(2):
        nll0, logp0 = m.step(x, lab, stream=main)
    main.synchronize()
    ref = (m.grads.clone(), logp0.clone(), nll0.clone())
    t_alone = []
    for _ in range(2):
        main.synchronize()
        t0 = time.perf_counter()
        m.step(x, lab, stream=main)
        main.synchronize()
        t_alone.append(time.perf_counter() - t0)
    # the step beside the hog on another stream
    t_beside = []
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        with torch.cuda.stream(comm):
            if delay:  # ~delay us of device time on the comm stream in front of the hog (~2.1 GHz clock)
                torch.cuda._sleep(int(delay * 2100))
            _lib.check(_lib.lib.s2s_debug_lds_hog(ctypes.c_void_p(comm.cuda_stream), nwg, lds_kb * 1024, float(usec),
                                                  ctypes.c_void_p(out.data_ptr())))
        nll, logp = m.step(x, lab, stream=main)
        torch.cuda.synchronize()
        t_beside.append(time.perf_counter() - t0)
        assert m.ctx.status(main, clear=False) == 0, rep
        assert torch.equal(m.grads, ref[0]), rep
        assert torch.equal(logp, ref[1]) and torch.equal(nll, ref[2]), rep
    print(f"hog {nwg} x {lds_kb} KB for {usec} us (+{delay} us): step alone {min(t_alone) * 1e3:.2f} ms, "
          f"beside the hog {min(t_beside) * 1e3:.2f} ms (host wall, hog included)")
