import ctypes, sys, os, torch
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "seq2seq-attention-asr_amd"))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import s2s_amd
from s2s_amd import _lib
from oracle import s2s_oracle as orc
fn = _lib.lib.s2s_debug_dec_pf
fn.argtypes = [ctypes.c_int]
cfg = s2s_amd.ModelConfig(); ocfg = orc.ModelConfig()
for vscale in (1.0, 300.0):
    model = s2s_amd.ChorowskiBaseline(cfg, graph=False)
    if vscale != 1.0:
        P = orc.unflatten(model.params.cpu().double().numpy(), ocfg)
        P["V"] = P["V"] * vscale
        model.params.copy_(torch.tensor(orc.flatten(P, ocfg), dtype=torch.float32))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(32, 96, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (32, 24), generator=g).to(torch.int32).cuda()
    res = []
    for on in (1, 1, 0, 0):
        fn(on)
        _, logp = model.step(x, lab)
        torch.cuda.synchronize()
        res.append((logp.clone(), model.grads.clone()))
    fn(1)
    vh = model.decoder_Vh()
    print(vscale, "pf-pf", torch.equal(res[0][0], res[1][0]), torch.equal(res[0][1], res[1][1]),
          "pt-pt", torch.equal(res[2][0], res[3][0]), torch.equal(res[2][1], res[3][1]),
          "pf-pt", torch.equal(res[0][0], res[2][0]), (res[0][0]-res[2][0]).abs().max().item(),
          (res[0][1]-res[2][1]).abs().max().item(), "vh max", None if vh is None else vh.abs().max().item(), flush=True)
