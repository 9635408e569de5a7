"""ctypes binding of libs2s_hip.so (include/s2s_hip.h).

The product path: every compute call goes through this library.  If the shared object
is missing or fails to load, importing the host layer raises -- there is no CPU
fallback (the CPU oracle under oracle/ is test infrastructure only).
"""
import ctypes
import os

# torch first: it loads the HIP runtime it was built with, and libs2s_hip.so then binds to that same
# (already loaded) libamdhip64.  Loading the library first pulls /opt/rocm/lib's runtime in ahead of
# torch's, and the second runtime of the process then finds no device (seen when build() and smoke()
# ran in one process).
import torch  # noqa: F401

_HERE = os.path.dirname(os.path.abspath(__file__))
# S2S_HIP_LIB overrides the in-tree library (same-box A/B comparisons of two builds)
LIB_PATH = os.environ.get("S2S_HIP_LIB") or os.path.join(_HERE, "libs2s_hip.so")

c_int, c_long, c_float, c_size_t, c_void_p = ctypes.c_int, ctypes.c_long, ctypes.c_float, ctypes.c_size_t, ctypes.c_void_p
P = ctypes.POINTER


class s2s_attn_dims(ctypes.Structure):
    _fields_ = [("B", c_int), ("L", c_int), ("T", c_int), ("annotationDepth", c_int), ("scoreDepth", c_int),
                ("stateDepth", c_int), ("outputDepth", c_int), ("mlpDepth", c_int), ("maxoutWindow", c_int),
                ("penalty", c_float), ("dropout", c_float), ("dropout_seed", ctypes.c_ulonglong),
                ("dropout_mask", c_void_p), ("hybridAttendFilterSize", c_int), ("hybridAttendFeatureMaps", c_int),
                ("external_mlp", c_int), ("decoder_lstm", c_int), ("frame_lengths", c_void_p),
                ("label_lengths", c_void_p)]


class s2s_optim_config(ctypes.Structure):
    _fields_ = [("rho", c_float), ("eps", c_float), ("maxnorm", c_float), ("weightDecay", c_float),
                ("colnorm_max", c_float), ("gradnoise_eta", c_float), ("gradnoise_gamma", c_float),
                ("gradnoise_seed", ctypes.c_ulonglong)]


class s2s_model_dims(ctypes.Structure):
    _fields_ = [("B", c_int), ("L", c_int), ("T", c_int), ("inputFrameSize", c_int), ("hiddenFrameSize", c_int),
                ("outputFrameSize", c_int), ("numLayers", c_int), ("scoreDepth", c_int), ("stateDepth", c_int),
                ("outputDepth", c_int), ("mlpDepth", c_int), ("maxoutWindow", c_int), ("penalty", c_float),
                ("dropout", c_float), ("dropout_seed", ctypes.c_ulonglong), ("dropout_mask", c_void_p),
                ("frame_lengths", c_void_p), ("label_lengths", c_void_p)]


# every symbol include/s2s_hip.h declares: (name, restype, argtypes)
SIGNATURES = [
    ("s2s_version", c_int, []),
    ("s2s_last_error", ctypes.c_char_p, []),
    ("s2s_ctx_create", c_int, [c_int, P(c_void_p)]),
    ("s2s_ctx_destroy", None, [c_void_p]),
    ("s2s_ctx_set_flags", c_int, [c_void_p, c_int]),
    ("s2s_ctx_set_graph_cache", c_int, [c_void_p, c_int]),
    ("s2s_ctx_set_precision", c_int, [c_void_p, c_int]),
    ("s2s_ctx_set_wgrad_overlap", c_int, [c_void_p, c_int]),
    ("s2s_ctx_join_wgrad", c_int, [c_void_p, c_void_p]),
    ("s2s_ctx_side_stream", c_void_p, [c_void_p]),
    ("s2s_ctx_graph_stats", c_int, [c_void_p, P(c_long), P(c_long), P(c_int)]),
    ("s2s_ctx_status", c_int, [c_void_p, c_void_p, P(c_int), c_int]),
    ("s2s_gru_saved_bytes", c_size_t, [c_int, c_int, c_int]),
    ("s2s_gru_scratch_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    ("s2s_gru_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, P(c_int), c_void_p, c_long,
                            P(c_void_p), P(c_void_p), c_long, P(c_void_p), c_void_p, c_void_p, c_size_t]),
    ("s2s_gru_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, P(c_int), c_void_p, c_long,
                            P(c_void_p), P(c_void_p), P(c_void_p), c_long, c_void_p, c_long, c_int, P(c_void_p),
                            c_float, c_void_p, c_void_p, c_size_t]),
    ("s2s_lstm_saved_bytes", c_size_t, [c_int, c_int, c_int]),
    ("s2s_lstm_scratch_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int]),
    ("s2s_lstm_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, P(c_int), c_void_p,
                             c_long, P(c_void_p), P(c_void_p), c_long, P(c_void_p), c_void_p, c_void_p, c_size_t]),
    ("s2s_lstm_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, P(c_int), c_void_p,
                             c_long, P(c_void_p), P(c_void_p), P(c_void_p), c_long, c_void_p, c_long, c_int,
                             P(c_void_p), c_float, c_void_p, c_void_p, c_size_t]),
    ("s2s_attn_saved_bytes", c_size_t, [P(s2s_attn_dims)]),
    ("s2s_attn_scratch_bytes", c_size_t, [P(s2s_attn_dims)]),
    ("s2s_attn_fwd", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_void_p, c_void_p, P(c_void_p), c_void_p,
                             c_void_p, c_void_p, c_size_t]),
    ("s2s_attn_bwd", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_void_p, c_void_p, P(c_void_p), c_void_p,
                             c_void_p, c_void_p, c_int, P(c_void_p), c_float, c_void_p, c_size_t]),
    ("s2s_attn_alpha", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_attn_mlp_input", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_attn_mono_ind", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_attn_maxout_argmax", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_attn_ws", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_attn_vh", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_model_attn_dims", c_int, [P(s2s_model_dims), P(s2s_attn_dims)]),
    ("s2s_model_attn_saved", c_void_p, [P(s2s_model_dims), c_void_p]),
    ("s2s_attn_dropout_mask", c_void_p, [P(s2s_attn_dims), c_void_p]),
    ("s2s_nll_seed", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_void_p, c_void_p, c_void_p, c_int,
                             c_void_p, c_void_p]),
    ("s2s_model_param_count", c_size_t, [P(s2s_model_dims)]),
    ("s2s_model_param_offset", c_long, [P(s2s_model_dims), c_int, P(c_long)]),
    ("s2s_model_workspace_bytes", c_size_t, [P(s2s_model_dims)]),
    ("s2s_model_step", c_int, [c_void_p, c_void_p, P(s2s_model_dims), c_void_p, c_void_p, c_void_p, c_void_p,
                               c_float, c_int, c_void_p, c_void_p, c_void_p, c_size_t]),
    ("s2s_model_encoder_output", c_void_p, [P(s2s_model_dims), c_void_p]),
    ("s2s_prof_enable", c_int, [c_int]),
    ("s2s_prof_collect", c_int, [ctypes.c_char_p, c_size_t]),
    ("s2s_attn_beam_workspace_bytes", c_size_t, [P(s2s_attn_dims), c_int, c_int]),
    ("s2s_attn_beam_search", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_void_p, c_void_p, c_int, c_int, c_int,
                                     c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_size_t]),
    ("s2s_attn_beam_init", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_void_p, c_void_p, c_int, c_int, c_int,
                                   c_void_p, c_size_t]),
    ("s2s_attn_beam_step", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_void_p, c_int, c_int, c_int, c_void_p,
                                   c_size_t]),
    ("s2s_attn_beam_mlp_input", c_void_p, [P(s2s_attn_dims), c_int, c_int, c_void_p]),
    ("s2s_attn_beam_advance", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_int, c_int, c_int, c_int, c_void_p,
                                      c_void_p, c_size_t]),
    ("s2s_attn_beam_done", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_int, c_int, c_void_p, P(c_int)]),
    ("s2s_attn_beam_finish", c_int, [c_void_p, c_void_p, P(s2s_attn_dims), c_int, c_int, c_void_p, c_int, c_void_p,
                                     c_void_p, c_void_p]),
    ("s2s_edit_distance", c_int, [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_int,
                                  c_void_p]),
    ("s2s_optim_state_bytes", c_size_t, [c_size_t]),
    ("s2s_optim_reset", c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
    ("s2s_optim_set_noise_step", c_int, [c_void_p, c_void_p, c_void_p, c_size_t, ctypes.c_uint]),
    ("s2s_optim_adadelta_step", c_int, [c_void_p, c_void_p, P(s2s_optim_config), c_void_p, c_void_p, c_size_t,
                                        c_void_p, c_void_p, c_int, c_void_p]),
    ("s2s_ctx_status_flag", c_int, [c_void_p, c_void_p, c_void_p]),
    ("s2s_optim_adadelta_step_flag", c_int, [c_void_p, c_void_p, P(s2s_optim_config), c_void_p, c_void_p, c_size_t,
                                             c_void_p, c_void_p, c_int, c_void_p, c_void_p]),
    ("s2s_model_weight_matrices", c_int, [P(s2s_model_dims), c_void_p]),
    ("s2s_model_bucket_count", c_int, [P(s2s_model_dims)]),
    ("s2s_model_bucket", c_int, [P(s2s_model_dims), c_int, P(c_size_t), P(c_size_t)]),
    ("s2s_stream_wait_bucket", c_int, [c_void_p, c_void_p, c_int]),
    ("s2s_tconv_scratch_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int]),
    ("s2s_tconv_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p]),
    ("s2s_tconv_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_float, c_void_p, c_size_t]),
    ("s2s_tmaxpool_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p]),
    ("s2s_tmaxpool_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_void_p, c_void_p,
                                 c_void_p]),
    ("s2s_sconv_scratch_bytes", c_size_t, [c_int, c_int, c_int, c_int, c_int, c_int, c_int]),
    ("s2s_sconv_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_size_t]),
    ("s2s_sconv_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_float, c_void_p,
                              c_size_t, c_int]),
    ("s2s_smaxpool_fwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_void_p, c_void_p, c_void_p]),
    ("s2s_smaxpool_bwd", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_int, c_int, c_int, c_int,
                                 c_void_p, c_void_p, c_void_p]),
    ("s2s_swap12", c_int, [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p, c_void_p]),
    ("s2s_relu_fwd", c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p]),
    ("s2s_relu_bwd", c_int, [c_void_p, c_void_p, c_long, c_void_p, c_void_p, c_void_p]),
    ("s2s_logsoftmax_fwd", c_int, [c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p]),
    ("s2s_logsoftmax_bwd", c_int, [c_void_p, c_void_p, c_long, c_int, c_void_p, c_void_p, c_void_p]),
    ("s2s_comm_unique_id", c_int, [c_void_p]),
    ("s2s_comm_init", c_int, [c_void_p, c_void_p, c_int, c_int]),
    ("s2s_allreduce_sum", c_int, [c_void_p, c_void_p, c_void_p, c_size_t]),
]

S2S_CTX_GRAPH = 1
S2S_CTX_OVERLAP = 2
S2S_ZERO_GRADS = 1
S2S_NORMALIZE_NLL = 2
S2S_BUCKET_EVENTS = 4
S2S_ATTN_NPARAMS = 17
S2S_ATTN_NPARAMS_HYBRID = 20
S2S_ATTN_NPARAMS_LSTM = 36
S2S_UNIQUE_ID_BYTES = 128
S2S_PREC_FP32 = 0
S2S_PREC_BF16_GEMM = 1
S2S_PREC_BF16_ALL = 2
S2S_STATUS_HANDOFF_TIMEOUT = 1
S2S_STATUS_ABORTED_REGION = 2


class S2SError(RuntimeError):
    pass


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(the HIP extension is required; there is no CPU fallback)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        try:
            fn = getattr(lib, name)
        except AttributeError:
            # an older build loaded for a same-box A/B (S2S_HIP_LIB): it lacks this round's newer entry points
            if os.environ.get("S2S_HIP_LIB"):
                continue
            raise
        fn.restype = res
        fn.argtypes = args
    return lib


lib = _load()


def check(rc: int):
    if rc != 0:
        raise S2SError(lib.s2s_last_error().decode(errors="replace"))


def ptr_array(ptrs, ctype=c_void_p):
    arr = (ctype * len(ptrs))()
    for i, p in enumerate(ptrs):
        arr[i] = p
    return arr
