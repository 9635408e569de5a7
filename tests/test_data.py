"""Data formats, variable-length minibatches and checkpoints.

CPU: the reference's LibriSpeech / TIMIT container layouts (utils_librispeech.lua, timit/timit.lua:40-70,
preprocess_timit.py:341-363) read from .npz archives of the same dataset paths, shape bucketing, and the
checkpoint round trip.  GPU: a ragged minibatch through ChorowskiBaseline.step_ragged equals the
reference's per-utterance loop (timit/timit.lua:240-295) computed by the oracle, 1e-4 relative.
"""
import os

import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc


def test_bucket_by_shape_groups_equal_shapes_in_order():
    from s2s_amd.data import bucket_by_shape
    shapes = [(10, 3), (12, 3), (10, 3), (10, 4), (12, 3), (10, 3)]
    assert bucket_by_shape(shapes) == [[0, 2, 5], [1, 4], [3]]
    assert bucket_by_shape(shapes, max_batch=2) == [[0, 2], [5], [1, 4], [3]]
    assert bucket_by_shape([]) == []


def test_librispeech_layout_roundtrip(tmp_path):
    from s2s_amd import data
    tree = data.synthetic_corpus(5, F=80, O=29, seed=3)
    data.write_npz(str(tmp_path / "train0.npz"), tree)
    (tmp_path / "train.db").write_text(str(tmp_path / "train0.npz") + "\n")
    (tmp_path / "meta.txt").write_text("numSamples 5\nmaxLength 120\nmean 0.5\n")
    fp = data.loadfilepaths(str(tmp_path))
    assert fp["train"] == [str(tmp_path / "train0.npz")] and fp["valid"].endswith("valid.h5")
    meta = data.loadmeta(str(tmp_path))
    assert meta == {"numSamples": 5, "maxLength": 120, "mean": 0.5}
    ds = data.loaddata(fp["train"][0])
    assert ds["numSamples"] == 5
    for i in range(5):
        np.testing.assert_array_equal(ds["x"][i], tree[f"{i}/x"])
        np.testing.assert_array_equal(ds["y"][i], tree[f"{i}/chars"])
        assert ds["y"][i][-1] == 29 and ds["y"][i].min() >= 1  # 1-based, EOS last
        assert (ds["x"][i][0] == 0).all() and (ds["x"][i][-1] == 0).all()  # pad frames
    # batches: every index once
    mb = data.minibatches(ds, 2, seed=1)
    assert sorted(i for b in mb for i in b) == list(range(5)) and [len(b) for b in mb] == [2, 2, 1]


def test_timit_layouts(tmp_path):
    from s2s_amd import data
    rng = np.random.default_rng(0)
    same = {"train/x": rng.standard_normal((3, 8, 4)).astype(np.float32), "train/y": rng.integers(1, 62, (3, 5)),
            "train/ymask": np.ones((3, 5))}
    data.write_npz(str(tmp_path / "same.npz"), same)
    ds = data.load_timit(str(tmp_path / "same.npz"))
    assert ds["numSamples"] == 3 and ds["x"][1].shape == (8, 4) and (ds["y"][2] == same["train/y"][2]).all()
    var = {}
    for k in range(11):  # numeric group order, not lexicographic
        var[f"valid/{k}/x"] = np.full((k + 2, 4), k, np.float32)
        var[f"valid/{k}/y"] = np.arange(1, k + 3)
        var[f"valid/{k}/y39"] = np.arange(1, k + 3) % 39 + 1
    data.write_npz(str(tmp_path / "var.npz"), var)
    ds = data.load_timit(str(tmp_path / "var.npz"), "valid")
    assert [x.shape[0] for x in ds["x"]] == [k + 2 for k in range(11)]
    ds39 = data.load_timit(str(tmp_path / "var.npz"), "valid", predict39=True)
    assert (ds39["y"][10] == var["valid/10/y39"]).all()


PYTABLES_TESTS = "/opt/conda/lib/python3.9/site-packages/tables/tests"


def test_hdf5_reader_known_answers():
    """s2s_amd.hdf5 on real HDF5 files written by the HDF5 C library (PyTables' own test files, shipped in
    this image's conda tree): float.h5 holds (5, 6) arrays arange(6) + arange(5)[:, None] in float16/32/64
    (tables/tests/test_types.py ReadFloatTestCase); python3.h5 has datasets inside a subgroup."""
    import os
    from s2s_amd import data, hdf5
    fp = os.path.join(PYTABLES_TESTS, "float.h5")
    if not os.path.exists(fp):
        pytest.skip("no HDF5 sample files in this image")
    t = hdf5.read_tree(fp)
    ref = np.arange(6) + np.arange(5)[:, None]
    for dt in ("float16", "float32", "float64"):
        assert t[dt].dtype == np.dtype(dt) and t[dt].shape == (5, 6)
        np.testing.assert_array_equal(t[dt], ref.astype(dt))
    t = data._read_tree(os.path.join(PYTABLES_TESTS, "python3.h5"))
    assert t["agroup/anarray1"].shape == (7,) and t["agroup/anarray2"].shape == (1,)


def test_hdf5_reader_refuses_non_hdf5(tmp_path):
    from s2s_amd import hdf5
    p = tmp_path / "x.h5"
    p.write_bytes(b"not an hdf5 file at all")
    with pytest.raises(ValueError, match="not an HDF5 file"):
        hdf5.read_tree(str(p))


def test_checkpoint_roundtrip(tmp_path):
    from s2s_amd import checkpoint, model
    cfg = model.ModelConfig(inputFrameSize=40, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=64,
                            stateDepth=32, outputDepth=29, mlpDepth=8)
    n = sum(int(np.prod(s)) for _, s in model.param_shapes(cfg))
    params = torch.randn(n)
    state = torch.randint(0, 255, (8 * n,), dtype=torch.uint8)
    p = str(tmp_path / "model.safetensors")
    checkpoint.save_flat(p, cfg, params, state, {"epoch": 3, "bestPER": 0.25})
    cfg2, params2, state2, meta = checkpoint.load_flat(p)
    assert cfg2 == cfg and meta == {"epoch": 3, "bestPER": 0.25}
    assert torch.equal(params2, params) and torch.equal(state2, state)
    with pytest.raises(ValueError):
        checkpoint.save_flat(p, cfg, params[:-1])


@pytest.mark.gpu
def test_step_ragged_equals_per_utterance_loop():
    """timit/timit.lua:240-295 with variable-length utterances: sum over utterances of the per-utterance
    gradient, / B -- via equal-shape groups accumulating with scale 1/B."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    kw = dict(inputFrameSize=40, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=64, stateDepth=32,
              outputDepth=29, mlpDepth=8, maxoutWindow=7, numLayers=3)
    m = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(**kw))
    cfg = orc.ModelConfig(**kw)
    rng = np.random.default_rng(5)
    shapes = [(24, 5), (31, 7), (24, 5), (17, 4), (31, 7)]
    xs = [rng.standard_normal((L, 40)).astype(np.float32) for L, _ in shapes]
    ys = [np.append(rng.integers(0, 28, T - 1), 28).astype(np.int32) for _, T in shapes]
    m.grads.fill_(7.0)  # overwritten: the first group zeroes the gradient
    nll, logps = m.step_ragged([torch.tensor(x, device="cuda") for x in xs],
                               [torch.tensor(y, device="cuda") for y in ys])
    torch.cuda.synchronize()
    P = orc.unflatten(m.params.cpu().double().numpy(), cfg)
    gsum = None
    for i, (x, y) in enumerate(zip(xs, ys)):
        nll_i, G, lp, _ = orc.training_step(x[None].astype(np.float64), y[None], P, cfg)
        g = orc.flatten(G, cfg)
        gsum = g if gsum is None else gsum + g
        err = np.abs(logps[i].cpu().numpy() - lp[0]).max() / np.abs(lp).max()
        assert err < 1e-4, (i, err)
    gref = gsum / len(xs)
    g = m.grads.cpu().double().numpy()
    assert np.abs(g - gref).max() / np.abs(gref).max() < 1e-4


def test_checkpoint_seed_base_is_per_rank():
    """Every data-parallel rank loads the same checkpoint: each must re-derive its own dropout seed base from
    the saved user seed and its rank (the ranks' masks stay independent after a resume), and the same rank
    must get back the base it had before saving."""
    from s2s_amd import checkpoint
    from s2s_amd.model import _mix64
    meta = {"steps": 5, "seed": "1234"}
    b0 = checkpoint.seed_base_for(meta, 0, default=-1)
    b1 = checkpoint.seed_base_for(meta, 1, default=-1)
    assert b0 != b1
    assert b0 == _mix64(1234, 0) and b1 == _mix64(1234, 1)
    with pytest.warns(UserWarning, match="no dropout seed"):
        assert checkpoint.seed_base_for({"steps": 5}, 1, default=42) == 42  # nothing saved: keep the model's own
    # an older writer saved its (rank 0) base, not the user seed: rank 0 continues that sequence, every other rank
    # mixes its rank in, so the replicas' masks stay independent
    old = {"steps": 5, "dropout_seed_base": "987"}
    with pytest.warns(UserWarning, match="older format"):
        assert checkpoint.seed_base_for(old, 0, default=42) == 987
    with pytest.warns(UserWarning, match="older format"):
        bases = [checkpoint.seed_base_for(old, r, default=42) for r in range(4)]
    assert bases[0] == 987 and bases[1:] == [_mix64(987, r) for r in range(1, 4)]
    assert len(set(bases)) == 4


@pytest.mark.gpu
def test_checkpoint_restores_model_and_optimizer(tmp_path):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    from s2s_amd import checkpoint, optim
    kw = dict(inputFrameSize=40, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=64, stateDepth=32,
              outputDepth=29, mlpDepth=8)
    m = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(**kw), seed=1)
    opt = optim.Adadelta(m, colnormconstr=True)
    x = torch.randn(2, 20, 40, device="cuda")
    y = torch.randint(0, 28, (2, 5), device="cuda", dtype=torch.int32)
    m.step(x, y)
    opt.step()
    p = os.path.join(str(tmp_path), "model.safetensors")
    checkpoint.save(p, m, opt, {"epoch": 1})
    m2 = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(**kw), seed=2)
    opt2 = optim.Adadelta(m2, colnormconstr=True)
    _, meta = checkpoint.load(p, m2, opt2)
    assert meta["epoch"] == 1
    # the step counter and user seed travel too (a resumed run continues the mask sequence); the same
    # rank re-derives the same seed base
    assert m2._steps == m._steps == 1 and m2.dropout_seed_base == m.dropout_seed_base and m2.seed == 1
    assert torch.equal(m2.params, m.params) and torch.equal(opt2.state, opt.state)
    # the restored pair continues identically
    for mm, oo in ((m, opt), (m2, opt2)):
        mm.step(x, y)
        oo.step()
    torch.cuda.synchronize()
    assert torch.equal(m2.params, m.params)
