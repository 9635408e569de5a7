-- LuaJIT FFI binding of libs2s_hip.so for the reference's Torch7 host (see INTEGRATION.md).
-- The cdef block is generated from include/s2s_hip.h (tools/gen_lua_cdef.py; tests/test_abi.py checks it
-- is current and declares every header symbol).  No LuaJIT/Torch7 exists in the build image or on the GPU
-- box, so the wrappers below are not executed here; the same ABI is exercised through Python ctypes by
-- tests/ and bench.py.
--
-- Conventions of the wrappers: tensors are contiguous torch.CudaTensor (labels / lengths:
-- torch.CudaIntTensor, 0-based class ids), `stream` is a hipStream_t cdata or nil (the default stream),
-- byte buffers (saved / scratch / workspace) are torch.CudaByteTensor resized here.  Errors raise
-- error(s2s_last_error()) as the reference's modules raise error()/assert().
local ffi = require 'ffi'

-- BEGIN GENERATED CDEF (tools/gen_lua_cdef.py)
ffi.cdef[[
typedef struct s2s_ctx s2s_ctx;
typedef void* s2s_stream_t;
int s2s_version(void);
const char* s2s_last_error(void);
int s2s_ctx_create(int device, s2s_ctx** out);
void s2s_ctx_destroy(s2s_ctx* ctx);
int s2s_ctx_set_flags(s2s_ctx* ctx, int flags);
int s2s_ctx_set_graph_cache(s2s_ctx* ctx, int capacity);
int s2s_ctx_set_precision(s2s_ctx* ctx, int precision);
int s2s_ctx_set_wgrad_overlap(s2s_ctx* ctx, int on);
int s2s_ctx_join_wgrad(s2s_ctx* ctx, s2s_stream_t stream);
s2s_stream_t s2s_ctx_side_stream(s2s_ctx* ctx);
int s2s_ctx_graph_stats(s2s_ctx* ctx, long* captures, long* replays, int* cached);
int s2s_ctx_status(s2s_ctx* ctx, s2s_stream_t stream, int* status, int clear);
size_t s2s_gru_saved_bytes(int B, int L, int H);
size_t s2s_gru_scratch_bytes(int ndir, int B, int L, int D, int H);
int s2s_gru_fwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, const int* reverse, const float* x, long ldx, const float* const* W, float* const* y, long ldy, void* const* saved, const int* lengths, void* scratch, size_t scratch_bytes);
int s2s_gru_bwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, const int* reverse, const float* x, long ldx, const float* const* W, void* const* saved, const float* const* dy, long lddy, float* dx, long lddx, int dx_accumulate, float* const* dW, float scale, const int* lengths, void* scratch, size_t scratch_bytes);
size_t s2s_lstm_saved_bytes(int B, int L, int H);
size_t s2s_lstm_scratch_bytes(int ndir, int B, int L, int D, int H, int peepholes);
int s2s_lstm_fwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, int peepholes, const int* reverse, const float* x, long ldx, const float* const* W, float* const* y, long ldy, void* const* saved, const int* lengths, void* scratch, size_t scratch_bytes);
int s2s_lstm_bwd(s2s_ctx* ctx, s2s_stream_t stream, int ndir, int B, int L, int D, int H, int peepholes, const int* reverse, const float* x, long ldx, const float* const* W, void* const* saved, const float* const* dy, long lddy, float* dx, long lddx, int dx_accumulate, float* const* dW, float scale, const int* lengths, void* scratch, size_t scratch_bytes);
typedef struct { int B, L, T; int annotationDepth, scoreDepth, stateDepth, outputDepth, mlpDepth, maxoutWindow; float penalty; float dropout; unsigned long long dropout_seed; const float* dropout_mask; int hybridAttendFilterSize, hybridAttendFeatureMaps; int external_mlp; int decoder_lstm; const int* frame_lengths; const int* label_lengths; } s2s_attn_dims;
size_t s2s_attn_saved_bytes(const s2s_attn_dims* d);
size_t s2s_attn_scratch_bytes(const s2s_attn_dims* d);
int s2s_attn_fwd(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const int* labels, const float* const* params, float* logp, void* saved, void* scratch, size_t scratch_bytes);
int s2s_attn_bwd(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const int* labels, const float* const* params, const void* saved, const float* dlogp, float* dh, int dh_accumulate, float* const* grads, float scale, void* scratch, size_t scratch_bytes);
const float* s2s_attn_mlp_input(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_alpha(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_ws(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_vh(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_mono_ind(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_dropout_mask(const s2s_attn_dims* d, const void* saved);
const int* s2s_attn_maxout_argmax(const s2s_attn_dims* d, const void* saved);
size_t s2s_attn_beam_workspace_bytes(const s2s_attn_dims* d, int K, int maxseqlength);
int s2s_attn_beam_search(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const float* const* params, int eos, int K, int maxseqlength, int* out, int ldo, int* out_len, float* out_score, void* workspace, size_t workspace_bytes);
int s2s_attn_beam_init(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* h, const float* const* params, int eos, int K, int maxseqlength, void* workspace, size_t workspace_bytes);
int s2s_attn_beam_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, const float* const* params, int K, int maxseqlength, int count, void* workspace, size_t workspace_bytes);
const float* s2s_attn_beam_mlp_input(const s2s_attn_dims* d, int K, int maxseqlength, void* workspace);
int s2s_attn_beam_advance(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int eos, int K, int maxseqlength, int count, const float* logp, void* workspace, size_t workspace_bytes);
int s2s_attn_beam_done(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int K, int maxseqlength, void* workspace, int* all_done);
int s2s_attn_beam_finish(s2s_ctx* ctx, s2s_stream_t stream, const s2s_attn_dims* d, int K, int maxseqlength, int* out, int ldo, int* out_len, float* out_score, void* workspace);
int s2s_edit_distance(s2s_ctx* ctx, s2s_stream_t stream, int n, const int* a, const int* alen, int lda, const int* b, const int* blen, int ldb, int* out);
size_t s2s_tconv_scratch_bytes(int B, int L, int Din, int Dout, int kW);
int s2s_tconv_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x, const float* W, const float* b, float* y);
int s2s_tconv_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x, const float* W, const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db, float scale, void* scratch, size_t scratch_bytes);
int s2s_tmaxpool_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int D, int kW, int dW, const float* x, float* y, int* idx);
int s2s_tmaxpool_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int L, int D, int kW, int dW, const int* idx, const float* dy, float* dx);
size_t s2s_sconv_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW);
int s2s_sconv_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x, const float* weight, const float* bias, float* y, void* scratch, size_t scratch_bytes);
int s2s_sconv_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu, const float* x, const float* weight, const float* y, const float* dy, float* dx, int dx_accumulate, float* dweight, float* dbias, float scale, void* scratch, size_t scratch_bytes, int col_from_fwd);
int s2s_smaxpool_fwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH, const float* x, float* y, int* idx);
int s2s_smaxpool_bwd(s2s_ctx* ctx, s2s_stream_t stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH, const int* idx, const float* dy, float* dx);
int s2s_swap12(s2s_ctx* ctx, s2s_stream_t stream, int B, int D1, int D2, int D3, const float* x, float* y);
int s2s_relu_fwd(s2s_ctx* ctx, s2s_stream_t stream, long n, const float* x, float* y);
int s2s_relu_bwd(s2s_ctx* ctx, s2s_stream_t stream, long n, const float* x, const float* dy, float* dx);
int s2s_logsoftmax_fwd(s2s_ctx* ctx, s2s_stream_t stream, long rows, int n, const float* x, float* y);
int s2s_logsoftmax_bwd(s2s_ctx* ctx, s2s_stream_t stream, long rows, int n, const float* y, const float* dy, float* dx);
int s2s_nll_seed(s2s_ctx* ctx, s2s_stream_t stream, int B, int T, int O, const float* logp, const int* labels, const int* label_lengths, int normalize, float* nll, float* dlogp);
typedef struct { int B, L, T; int inputFrameSize, hiddenFrameSize, outputFrameSize, numLayers; int scoreDepth, stateDepth, outputDepth, mlpDepth, maxoutWindow; float penalty; float dropout; unsigned long long dropout_seed; const float* dropout_mask; const int* frame_lengths; const int* label_lengths; } s2s_model_dims;
int s2s_model_bucket_count(const s2s_model_dims* d);
int s2s_model_bucket(const s2s_model_dims* d, int i, size_t* offset, size_t* count);
int s2s_stream_wait_bucket(s2s_ctx* ctx, s2s_stream_t stream, int i);
size_t s2s_model_param_count(const s2s_model_dims* d);
long s2s_model_param_offset(const s2s_model_dims* d, int i, long* numel);
size_t s2s_model_workspace_bytes(const s2s_model_dims* d);
int s2s_model_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_model_dims* d, const float* params, float* grads, const float* x, const int* labels, float scale, int flags, float* logp, float* nll, void* workspace, size_t workspace_bytes);
const float* s2s_model_encoder_output(const s2s_model_dims* d, const void* workspace);
int s2s_model_attn_dims(const s2s_model_dims* d, s2s_attn_dims* out);
const void* s2s_model_attn_saved(const s2s_model_dims* d, const void* workspace);
typedef struct { float rho, eps, maxnorm, weightDecay, colnorm_max; float gradnoise_eta, gradnoise_gamma; unsigned long long gradnoise_seed; } s2s_optim_config;
size_t s2s_optim_state_bytes(size_t n);
int s2s_optim_reset(s2s_ctx* ctx, s2s_stream_t stream, void* state, size_t n);
int s2s_optim_set_noise_step(s2s_ctx* ctx, s2s_stream_t stream, void* state, size_t n, unsigned t);
int s2s_optim_adadelta_step(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params, float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm);
int s2s_ctx_status_flag(s2s_ctx* ctx, s2s_stream_t stream, float* flag);
int s2s_optim_adadelta_step_flag(s2s_ctx* ctx, s2s_stream_t stream, const s2s_optim_config* cfg, float* params, float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm, const float* skip_flag);
int s2s_model_weight_matrices(const s2s_model_dims* d, long* mats);
int s2s_prof_enable(int on);
int s2s_prof_collect(char* buf, size_t cap);
int s2s_comm_unique_id(void* out_bytes);
int s2s_comm_init(s2s_ctx* ctx, const void* id_bytes, int nranks, int rank);
int s2s_allreduce_sum(s2s_ctx* ctx, s2s_stream_t stream, float* buf, size_t count);
]]
-- END GENERATED CDEF

local C = ffi.load('s2s_hip')
local M = {C = C}

-- BEGIN GENERATED CONSTANTS (tools/gen_lua_cdef.py)
M.S2S_CTX_GRAPH = 1
M.S2S_CTX_OVERLAP = 2
M.S2S_PREC_FP32 = 0
M.S2S_PREC_BF16_GEMM = 1
M.S2S_PREC_BF16_ALL = 2
M.S2S_STATUS_HANDOFF_TIMEOUT = 1
M.S2S_STATUS_ABORTED_REGION = 2
M.S2S_ATTN_NPARAMS = 17
M.S2S_ATTN_NPARAMS_HYBRID = 20
M.S2S_ATTN_NPARAMS_LSTM = 36
M.S2S_ZERO_GRADS = 1
M.S2S_NORMALIZE_NLL = 2
M.S2S_BUCKET_EVENTS = 4
M.S2S_UNIQUE_ID_BYTES = 128
-- END GENERATED CONSTANTS

function M.check(rc)
   if rc ~= 0 then error(ffi.string(C.s2s_last_error())) end
end

function M.context(device, flags)
   local out = ffi.new('s2s_ctx*[1]')
   M.check(C.s2s_ctx_create(device or 0, out))
   if flags then M.check(C.s2s_ctx_set_flags(out[0], flags)) end
   return ffi.gc(out[0], C.s2s_ctx_destroy)
end

-- failure status of the context's persistent launches (after syncing `stream`); clear defaults to true.
-- Call it at the trainer's sync points (gradients:norm(), timit/timit.lua:298): a nonzero status means the
-- step's results are invalid, raised as the reference's error() would (RNN.lua:8-9).
function M.ctx_status(ctx, stream, clear)
   local st = ffi.new('int[1]')
   M.check(C.s2s_ctx_status(ctx, stream, st, (clear == false) and 0 or 1))
   return st[0]
end
function M.check_status(ctx, stream)
   local st = M.ctx_status(ctx, stream, true)
   if st ~= 0 then error('s2s: persistent launch failed (status ' .. st .. '): results since the last check are invalid') end
end

-- device pointer of a contiguous CudaTensor (nil -> NULL)
local function dptr(t, ctype)
   if t == nil then return nil end
   return ffi.cast(ctype or 'float*', torch.data(t))
end
M.dptr = dptr
local function iptr(t) return dptr(t, 'int*') end
local function vptr(t) return dptr(t, 'void*') end
local function ptrs(ctype, list)
   local n = #list
   local a = ffi.new(ctype .. '[?]', math.max(n, 1))
   for i = 1, n do a[i - 1] = dptr(list[i]) end
   return a
end

local function as3d(x)
   assert(x:nDimension() == 2 or x:nDimension() == 3, 'input dimension must be 2D or 3D')  -- RNN.lua:128
   if x:nDimension() == 2 then return x:view(1, x:size(1), x:size(2)) end
   return x
end

-- nn.RNN(nn.GRU(D,H), reverse):updateOutput for a (L x D) or (B x L x D) input.
-- W = {Wz, Wr, Wh}: the three LinearZeroBias weights of the cell (GRU.lua:23-26), each (H, H+D).
-- lengths (optional CudaIntTensor of B): frames per utterance of a padded variable-length batch.
function M.gru_forward(ctx, stream, x, W, H, reverse, output, saved, scratch, lengths)
   local x3 = as3d(x)
   local B, L, D = x3:size(1), x3:size(2), x3:size(3)
   output:resize(B, L, H)
   saved:resize(tonumber(C.s2s_gru_saved_bytes(B, L, H)))
   scratch:resize(tonumber(C.s2s_gru_scratch_bytes(1, B, L, D, H)))
   local sv = ffi.new('void*[1]', {vptr(saved)})
   M.check(C.s2s_gru_fwd(ctx, stream, 1, B, L, D, H, ffi.new('int[1]', {reverse and 1 or 0}), dptr(x3), D,
                         ptrs('const float*', W), ptrs('float*', {output}), H, sv, iptr(lengths), vptr(scratch),
                         scratch:nElement()))
   return x:nDimension() == 2 and output[1] or output
end

-- nn.RNN:updateGradInput + accGradParameters(scale) (RNN.lua:169-201, LinearZeroBias.lua:50-74):
-- gradInput (overwritten) and dW = {dWz, dWr, dWh} += scale * ..., after M.gru_forward on the same input.
function M.gru_backward(ctx, stream, x, W, dW, H, reverse, saved, gradOutput, gradInput, scale, scratch, lengths)
   local x3 = as3d(x)
   local B, L, D = x3:size(1), x3:size(2), x3:size(3)
   gradInput:resize(B, L, D)
   scratch:resize(tonumber(C.s2s_gru_scratch_bytes(1, B, L, D, H)))
   local sv = ffi.new('void*[1]', {vptr(saved)})
   local go = gradOutput:contiguous()
   M.check(C.s2s_gru_bwd(ctx, stream, 1, B, L, D, H, ffi.new('int[1]', {reverse and 1 or 0}), dptr(x3), D,
                         ptrs('const float*', W), sv, ptrs('const float*', {go}), H, dptr(gradInput), D, 0,
                         ptrs('float*', dW), scale or 1, iptr(lengths), vptr(scratch), scratch:nElement()))
   return x:nDimension() == 2 and gradInput[1] or gradInput
end

-- s2s_attn_dims for nn.Attention(decoder_recurrent = GRU(S,S), decoder_mlp = Maxout -> Linear -> LogSoftMax, ...)
-- from loadmodel's opt fields (timit/model_chorowski_baseline.lua:37-70)
function M.attention_dims(opt, B, L, T)
   local d = ffi.new('s2s_attn_dims')
   d.B, d.L, d.T = B, L, T
   d.annotationDepth = 2 * opt.outputFrameSize
   d.scoreDepth, d.stateDepth = opt.scoreDepth, opt.stateDepth
   d.outputDepth = opt.numPhonemes or opt.outputDepth
   d.mlpDepth, d.maxoutWindow = opt.mlpDepth, opt.maxoutWindow or 7
   d.penalty, d.dropout = opt.penalty or 0, opt.dropout or 0
   d.hybridAttendFilterSize = opt.hybridAttendFilterSize or 0
   d.hybridAttendFeatureMaps = opt.hybridAttendFeatureMaps or 0
   return d
end

-- Attention:updateOutput({h, labels}) (Attention.lua:305-322): h (B, L, A), labels (B, T) CudaIntTensor,
-- params = the 17 (20 with hybrid features) decoder tensors in the include/s2s_hip.h order; output (B, T, O).
function M.attention_forward(ctx, stream, d, h, labels, params, output, saved, scratch)
   output:resize(d.B, d.T, d.outputDepth)
   saved:resize(tonumber(C.s2s_attn_saved_bytes(d)))
   scratch:resize(tonumber(C.s2s_attn_scratch_bytes(d)))
   M.check(C.s2s_attn_fwd(ctx, stream, d, dptr(h), iptr(labels), ptrs('const float*', params), dptr(output),
                          vptr(saved), vptr(scratch), scratch:nElement()))
   return output
end

-- Attention:updateGradInput + accGradParameters(scale) (Attention.lua:324-327, RNNAttention.lua:203-253):
-- gradOutput = dlogp (B, T, O); gradInput (B, L, A) overwritten; grads (same order as params) += scale * ...
function M.attention_backward(ctx, stream, d, h, labels, params, saved, gradOutput, gradInput, grads, scale, scratch)
   gradInput:resize(d.B, d.L, d.annotationDepth)
   scratch:resize(tonumber(C.s2s_attn_scratch_bytes(d)))
   M.check(C.s2s_attn_bwd(ctx, stream, d, dptr(h), iptr(labels), ptrs('const float*', params), vptr(saved),
                          dptr(gradOutput:contiguous()), dptr(gradInput), 0, ptrs('float*', grads), scale or 1,
                          vptr(scratch), scratch:nElement()))
   return gradInput
end

-- decoder:alpha() / penalty() (B, T, L), decoder:Ws() rows (B, T, Sc) (ExpandAs over L in the reference),
-- decoder.Vh.output (B, L, Sc): device pointers inside `saved` (Attention.lua:241-249, timit/timit.lua:519-521)
function M.attention_views(d, saved)
   local sv = vptr(saved)
   return {alpha = C.s2s_attn_alpha(d, sv), penalty = C.s2s_attn_alpha(d, sv), Ws = C.s2s_attn_ws(d, sv),
           Vh = C.s2s_attn_vh(d, sv)}
end

-- decoder:BeamSearch(annotations, eos, K, maxseqlength) (Attention.lua:332-438) for B utterances; eos and the
-- tokens 0-based.  workspace: a CudaTensor (float; its storage also backs the decoder_mlp input view).
-- mlp (optional): an external decoder_mlp module (d.external_mlp = 1), run between the search's step and
-- advance calls on the (B*K, S+A) hypothesis rows.  Returns out (B, maxlen+1) -1 padded, lengths, scores.
function M.beam_search(ctx, stream, d, h, params, eos, K, maxlen, workspace, mlp)
   local B = d.B
   local bytes = tonumber(C.s2s_attn_beam_workspace_bytes(d, K, maxlen))
   workspace:resize(math.ceil(bytes / 4))
   local out = torch.CudaIntTensor(B, maxlen + 1)
   local len, score = torch.CudaIntTensor(B), torch.CudaTensor(B)
   local P, ws, n = ptrs('const float*', params), vptr(workspace), 4 * workspace:nElement()
   if mlp == nil then
      M.check(C.s2s_attn_beam_search(ctx, stream, d, dptr(h), P, eos, K, maxlen, iptr(out), maxlen + 1, iptr(len),
                                     dptr(score), ws, n))
      return out, len, score
   end
   local R, W = B * K, d.stateDepth + d.annotationDepth
   local off = tonumber(ffi.cast('const float*', C.s2s_attn_beam_mlp_input(d, K, maxlen, ws)) - dptr(workspace))
   local rows = torch.CudaTensor(workspace:storage(), workspace:storageOffset() + off, torch.LongStorage{R, W})
   local done = ffi.new('int[1]')
   M.check(C.s2s_attn_beam_init(ctx, stream, d, dptr(h), P, eos, K, maxlen, ws, n))
   for count = 0, maxlen do
      M.check(C.s2s_attn_beam_step(ctx, stream, d, P, K, maxlen, count, ws, n))
      local logp = mlp:forward(rows):contiguous()
      M.check(C.s2s_attn_beam_advance(ctx, stream, d, eos, K, maxlen, count, dptr(logp), ws, n))
      if count % 4 == 3 or count == maxlen then
         M.check(C.s2s_attn_beam_done(ctx, stream, d, K, maxlen, ws, done))
         if done[0] ~= 0 then break end
      end
   end
   M.check(C.s2s_attn_beam_finish(ctx, stream, d, K, maxlen, iptr(out), maxlen + 1, iptr(len), dptr(score), ws))
   return out, len, score
end

-- the whole autoencoder:forward({X, labelmask}) + NLL + backward(-labelmask) on flat buffers
-- (timit/timit.lua:240-295, getParameters :172): flags = M.S2S_ZERO_GRADS + M.S2S_NORMALIZE_NLL etc.
function M.model_dims(opt, B, L, T, frame_lengths, label_lengths)
   local d = ffi.new('s2s_model_dims')
   d.B, d.L, d.T = B, L, T
   d.inputFrameSize, d.hiddenFrameSize, d.outputFrameSize = opt.inputFrameSize, opt.hiddenFrameSize, opt.outputFrameSize
   d.numLayers = opt.numLayers or 3
   d.scoreDepth, d.stateDepth = opt.scoreDepth, opt.stateDepth
   d.outputDepth = opt.numPhonemes or opt.outputDepth
   d.mlpDepth, d.maxoutWindow = opt.mlpDepth, opt.maxoutWindow or 7
   d.penalty, d.dropout = opt.penalty or 0, opt.dropout or 0
   d.frame_lengths, d.label_lengths = iptr(frame_lengths), iptr(label_lengths)
   return d
end

function M.model_step(ctx, stream, d, params, grads, x, labels, scale, flags, logp, nll, workspace)
   workspace:resize(tonumber(C.s2s_model_workspace_bytes(d)))
   M.check(C.s2s_model_step(ctx, stream, d, dptr(params), dptr(grads), dptr(x), iptr(labels), scale, flags,
                            dptr(logp), dptr(nll), vptr(workspace), workspace:nElement()))
end

-- the trainer's post-backward block (timit/timit.lua:292-347): clip, L2, optim.adadelta, column-norm
-- constraint, on the flat parameters / gradients; state is a CudaByteTensor kept across steps
-- (zeroed on first use, as optim.adadelta's paramVariance / accDelta start at 0).
-- gradnoise: the trainer's table {eta, gamma, t} (timit.lua:185-189; restored from model.gradnoise on a
-- resume, timit.lua:92), passed explicitly.  nil means the exp configs' {eta = 0} (no noise) -- NOT the
-- trainer's own fallback eta = 1e-3 (timit.lua:185-189), which a caller must pass in to get it.  With eta ~= 0
-- the device counter is set to gradnoise.t before the step and the table's t is advanced as the reference
-- does (timit.lua:312), so a resumed run continues the noise schedule; gradnoise.seed (default 0x5EED) keys
-- the counter-based normals and must be equal on every data-parallel rank.
function M.adadelta_step(ctx, stream, d, opt, params, grads, state, gradnorm, gradnoise)
   local n = params:nElement()
   if not M._mats or M._mats_d ~= d then
      local nm = C.s2s_model_weight_matrices(d, nil)
      M._mats = ffi.new('long[?]', 3 * nm)
      C.s2s_model_weight_matrices(d, M._mats)
      M._nmats, M._mats_d = nm, d
   end
   local bytes = tonumber(C.s2s_optim_state_bytes(n))
   if state:nElement() ~= bytes then
      state:resize(bytes)
      M.check(C.s2s_optim_reset(ctx, stream, vptr(state), n))
   end
   local cfg = ffi.new('s2s_optim_config')
   cfg.rho, cfg.eps = opt.rho or 0.95, opt.eps or 1e-8
   cfg.maxnorm, cfg.weightDecay = opt.maxnorm or 1e20, opt.weightDecay or 0
   cfg.colnorm_max = opt.colnormconstr and (opt.colnorm_max or 1) or 0
   local gn = gradnoise or {eta = 0, gamma = 0.55, t = 0}
   cfg.gradnoise_eta, cfg.gradnoise_gamma = gn.eta or 0, gn.gamma or 0.55
   cfg.gradnoise_seed = gn.seed or 0x5EED
   if cfg.gradnoise_eta ~= 0 then
      M.check(C.s2s_optim_set_noise_step(ctx, stream, vptr(state), n, gn.t or 0))
      gn.t = (gn.t or 0) + 1
   end
   M.check(C.s2s_optim_adadelta_step(ctx, stream, cfg, dptr(params), dptr(grads), n, vptr(state), M._mats,
                                     M._nmats, gradnorm and dptr(gradnorm) or nil))
end

-- nn.TemporalConvolution(Din, Dout, kW) on a (L x Din) or (B x L x Din) CudaTensor, as the conv + BiLSTM
-- encoder's convlayer uses it (timit/timit.lua:113-121); relu = true fuses the nn.ReLU that follows.
function M.tconv_forward(ctx, stream, m, x, relu, output)
   local x3 = as3d(x)
   local B, L, Din = x3:size(1), x3:size(2), x3:size(3)
   output:resize(B, L - m.kW + 1, m.outputFrameSize)
   M.check(C.s2s_tconv_fwd(ctx, stream, B, L, Din, m.outputFrameSize, m.kW, relu and 1 or 0, dptr(x3),
                           dptr(m.weight), dptr(m.bias), dptr(output)))
   return output
end

-- updateGradInput + accGradParameters(scale) of the same module (gradInput overwritten)
function M.tconv_backward(ctx, stream, m, x, relu, output, gradOutput, gradInput, scale, scratch)
   local x3 = as3d(x)
   local B, L, Din = x3:size(1), x3:size(2), x3:size(3)
   gradInput:resizeAs(x3)
   scratch:resize(tonumber(C.s2s_tconv_scratch_bytes(B, L, Din, m.outputFrameSize, m.kW)))
   M.check(C.s2s_tconv_bwd(ctx, stream, B, L, Din, m.outputFrameSize, m.kW, relu and 1 or 0, dptr(x3), dptr(m.weight),
                           dptr(output), dptr(gradOutput), dptr(gradInput), 0, dptr(m.gradWeight), dptr(m.gradBias),
                           scale or 1, vptr(scratch), scratch:nElement()))
   return gradInput
end

return M
