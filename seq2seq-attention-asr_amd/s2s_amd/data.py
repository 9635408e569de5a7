"""Data formats and batching.

The reference's corpora are HDF5 files written by its Python-2 preprocessing:
  * TIMIT (timit/preprocess_timit.py:341-363, read whole by timit/timit.lua:40-70): groups
    train / valid / test, each either stacked equal-length arrays x (N, L, F), y (N, T), ymask, or one
    subgroup per utterance "<k>" with x (L, F), y (T), y39, start, finish;
  * LibriSpeech (librispeech/preprocess.py:230-253, read by librispeech/utils_librispeech.lua): a
    directory with train.db (one chunk file per line), valid.h5, test.h5 and meta.txt ("key value"
    lines); every chunk holds one group per utterance "<i>" with x (L, F), chars (T), words.
Labels are 1-based class ids (Torch), EOS included (timit/timit.lua:258-262); this module hands the
C ABI 0-based int32 labels.

.h5 files are read through h5py when it is importable; h5py is not part of this image, so otherwise
through `s2s_amd.hdf5`, a pure-Python reader of the HDF5 subset h5py writes by default (superblock v0,
symbol-table groups, contiguous numeric datasets).  The same layouts are also read from .npz archives
whose keys are the HDF5 paths ("<i>/x", "<i>/chars", "train/x", ...) -- what `write_npz` produces
(synthetic corpora in the reference's layout).

Batching: the trainer runs one utterance per forward (timit/timit.lua:240-265: variable-length
utterances, gradients summed over the minibatch, then divided by B, :292-295).  The batched C ABI takes
padded (B, L_max) batches with per-utterance frame / label lengths (s2s_model_dims.frame_lengths /
label_lengths): masked recurrences, masked attention and loss seed give the per-utterance results
(`ChorowskiBaseline.step_ragged` sorts by length, pads and steps, accumulating with scale 1/B).
`bucket_by_shape` groups exactly equal shapes (no padding at all) for callers that want that.
"""
import os
from collections import OrderedDict

import numpy as np


# ---------------------------------------------------------------- container readers

def _read_tree(path):
    """{hdf5 path: ndarray} of every dataset in an .h5 (via h5py) or .npz archive."""
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            return {k: z[k] for k in z.files}
    try:
        import h5py
    except ImportError:  # not in this image: the built-in reader of the subset h5py writes by default
        from .hdf5 import read_tree
        return read_tree(path)
    out = {}
    with h5py.File(path, "r") as h:
        def visit(name, obj):
            if isinstance(obj, h5py.Dataset):
                out[name] = obj[()]
        h.visititems(visit)
    return out


def write_npz(path, tree):
    """Write {hdf5 path: array} as an .npz archive of the same layout."""
    np.savez(path, **{k: np.asarray(v) for k, v in tree.items()})


def _groups(tree, prefix=""):
    """{group name: {member: array}} of the direct subgroups under prefix."""
    out = OrderedDict()
    for k, v in tree.items():
        if not k.startswith(prefix):
            continue
        parts = k[len(prefix):].split("/")
        if len(parts) == 2:
            out.setdefault(parts[0], {})[parts[1]] = v
    return out


def _numeric_order(keys):
    return sorted(keys, key=lambda s: (0, int(s)) if s.isdigit() else (1, s))


# ---------------------------------------------------------------- LibriSpeech layout

def loadfilepaths(datadir):
    """utils_librispeech.lua:3-17: train chunk paths (train.db lines), valid.h5, test.h5."""
    with open(os.path.join(datadir, "train.db")) as f:
        chunks = [ln.strip() for ln in f if ln.strip()]
    return {"train": chunks, "valid": os.path.join(datadir, "valid.h5"), "test": os.path.join(datadir, "test.h5")}


def loadmeta(datadir):
    """utils_librispeech.lua:38-46: meta.txt "key value" lines -> {key: number}."""
    meta = {}
    with open(os.path.join(datadir, "meta.txt")) as f:
        for ln in f:
            parts = ln.split()
            if len(parts) >= 2:
                v = float(parts[1])
                meta[parts[0]] = int(v) if v.is_integer() else v
    return meta


def loaddata(filepath, labelset="chars"):
    """utils_librispeech.lua:50-66: every utterance group "<i>" -> x (L, F) float32, y (T,) int (1-based)."""
    groups = _groups(_read_tree(filepath))
    xs, ys = [], []
    for k in _numeric_order(groups):
        g = groups[k]
        xs.append(np.asarray(g["x"], dtype=np.float32))
        ys.append(np.asarray(g[labelset]).astype(np.int64).reshape(-1))
    return {"x": xs, "y": ys, "numSamples": len(xs)}


# ---------------------------------------------------------------- TIMIT layout

def load_timit(filepath, split="train", predict39=False):
    """timit/timit.lua:40-70 processData on one split of the preprocess_timit.py:341-363 file: stacked
    equal-length arrays (x, y) or per-utterance subgroups (x, y / y39)."""
    tree = _read_tree(filepath)
    if f"{split}/x" in tree:  # featuresSameLength and phonemesSameLength
        x = np.asarray(tree[f"{split}/x"], dtype=np.float32)
        y = np.asarray(tree[f"{split}/y"]).astype(np.int64)
        return {"x": list(x), "y": list(y), "numSamples": x.shape[0]}
    groups = _groups(tree, f"{split}/")
    key = "y39" if predict39 else "y"
    xs = [np.asarray(groups[k]["x"], dtype=np.float32) for k in _numeric_order(groups)]
    ys = [np.asarray(groups[k][key]).astype(np.int64).reshape(-1) for k in _numeric_order(groups)]
    return {"x": xs, "y": ys, "numSamples": len(xs)}


# ---------------------------------------------------------------- batching

def bucket_by_shape(shapes, max_batch=None):
    """Indices grouped by equal (L, T), in order of first appearance; groups larger than max_batch are
    cut into consecutive pieces.  Deterministic."""
    groups = OrderedDict()
    for i, s in enumerate(shapes):
        groups.setdefault(tuple(s), []).append(i)
    out = []
    for idx in groups.values():
        step = max_batch or len(idx)
        out += [idx[j:j + step] for j in range(0, len(idx), step)]
    return out


def minibatches(dataset, batchSize, seed=None):
    """timit/timit.lua:240-250: minibatches of batchSize utterance indices in shuffled order
    (torch.randperm in the reference; a seeded numpy permutation here), the last one possibly short."""
    n = dataset["numSamples"]
    order = np.random.default_rng(seed).permutation(n) if seed is not None else np.arange(n)
    return [order[t:t + batchSize].tolist() for t in range(0, n, batchSize)]


def to_device_batch(dataset, idx, device):
    """One minibatch as lists of device tensors: x (L_i, F) float32 and 0-based int32 labels (T_i)."""
    import torch
    xs = [torch.from_numpy(np.ascontiguousarray(dataset["x"][i])).to(device) for i in idx]
    ys = [torch.from_numpy((np.asarray(dataset["y"][i]) - 1).astype(np.int32)).to(device) for i in idx]
    return xs, ys


def synthetic_corpus(n, F=80, O=29, L_range=(60, 120), T_range=(10, 30), eos=None, seed=1234, pad=1):
    """A corpus in the LibriSpeech chunk layout ({"<i>/x", "<i>/chars"}): z-normalised features with
    `pad` zero frames each side (librispeech/preprocess.py:192-194) and 1-based labels ending in EOS."""
    rng = np.random.default_rng(seed)
    eos = O if eos is None else eos
    tree = {}
    for i in range(n):
        L = int(rng.integers(L_range[0], L_range[1] + 1))
        T = int(rng.integers(T_range[0], T_range[1] + 1))
        x = rng.standard_normal((L, F)).astype(np.float32)
        x[:pad] = 0
        x[L - pad:] = 0
        y = rng.integers(1, O + 1, size=T)
        y[y == eos] = 1 if eos != 1 else 2
        y[-1] = eos
        tree[f"{i}/x"] = x
        tree[f"{i}/chars"] = y.astype(np.int64)
    return tree
