-- LuaJIT FFI binding of libs2s_hip.so for the reference's Torch7 host (see INTEGRATION.md).
-- Untested in this repo: no LuaJIT/Torch7 exists in the build image or on the GPU box; the same
-- ABI is exercised through Python ctypes by tests/ and bench.py.
local ffi = require 'ffi'

ffi.cdef[[
typedef struct s2s_ctx s2s_ctx;
int s2s_version(void);
const char* s2s_last_error(void);
int s2s_ctx_create(int device, s2s_ctx** out);
void s2s_ctx_destroy(s2s_ctx* ctx);
int s2s_ctx_set_flags(s2s_ctx* ctx, int flags);
size_t s2s_gru_saved_bytes(int B, int L, int H);
size_t s2s_gru_scratch_bytes(int ndir, int B, int L, int D, int H);
int s2s_gru_fwd(s2s_ctx*, void* stream, int ndir, int B, int L, int D, int H, const int* reverse,
                const float* x, long ldx, const float* const* W, float* const* y, long ldy,
                void* const* saved, void* scratch, size_t scratch_bytes);
int s2s_gru_bwd(s2s_ctx*, void* stream, int ndir, int B, int L, int D, int H, const int* reverse,
                const float* x, long ldx, const float* const* W, void* const* saved,
                const float* const* dy, long lddy, float* dx, long lddx, int dx_accumulate,
                float* const* dW, float scale, void* scratch, size_t scratch_bytes);
typedef struct { int B, L, T; int annotationDepth, scoreDepth, stateDepth, outputDepth, mlpDepth, maxoutWindow;
                 float penalty; float dropout; unsigned long long dropout_seed; const float* dropout_mask;
                 int hybridAttendFilterSize, hybridAttendFeatureMaps; int external_mlp; int decoder_lstm; } s2s_attn_dims;
const float* s2s_attn_mlp_input(const s2s_attn_dims* d, const void* saved);
size_t s2s_attn_saved_bytes(const s2s_attn_dims* d);
size_t s2s_attn_scratch_bytes(const s2s_attn_dims* d);
int s2s_attn_fwd(s2s_ctx*, void* stream, const s2s_attn_dims* d, const float* h, const int* labels,
                 const float* const* params, float* logp, void* saved, void* scratch, size_t scratch_bytes);
int s2s_attn_bwd(s2s_ctx*, void* stream, const s2s_attn_dims* d, const float* h, const int* labels,
                 const float* const* params, const void* saved, const float* dlogp, float* dh, int dh_accumulate,
                 float* const* grads, float scale, void* scratch, size_t scratch_bytes);
const float* s2s_attn_alpha(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_mono_ind(const s2s_attn_dims* d, const void* saved);
const float* s2s_attn_dropout_mask(const s2s_attn_dims* d, const void* saved);
int s2s_nll_seed(s2s_ctx*, void* stream, int B, int T, int O, const float* logp, const int* labels, int normalize,
                 float* nll, float* dlogp);
int s2s_comm_unique_id(void* out_bytes);
int s2s_comm_init(s2s_ctx* ctx, const void* id_bytes, int nranks, int rank);
int s2s_allreduce_sum(s2s_ctx* ctx, void* stream, float* buf, size_t count);
int s2s_stream_wait_bucket(s2s_ctx* ctx, void* stream, int i);
size_t s2s_attn_beam_workspace_bytes(const s2s_attn_dims* d, int K, int maxseqlength);
int s2s_attn_beam_search(s2s_ctx* ctx, void* stream, const s2s_attn_dims* d, const float* h,
                         const float* const* params, int eos, int K, int maxseqlength, int* out, int ldo, int* out_len,
                         float* out_score, void* workspace, size_t workspace_bytes);
int s2s_edit_distance(s2s_ctx* ctx, void* stream, int n, const int* a, const int* alen, int lda, const int* b,
                      const int* blen, int ldb, int* out);
typedef struct { float rho, eps, maxnorm, weightDecay, colnorm_max; } s2s_optim_config;
size_t s2s_optim_state_bytes(size_t n);
int s2s_optim_reset(s2s_ctx* ctx, void* stream, void* state, size_t n);
int s2s_optim_adadelta_step(s2s_ctx* ctx, void* stream, const s2s_optim_config* cfg, float* params,
                            float* grads, size_t n, void* state, const long* mats, int n_mats, float* gradnorm);
size_t s2s_tconv_scratch_bytes(int B, int L, int Din, int Dout, int kW);
int s2s_tconv_fwd(s2s_ctx*, void* stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x,
                  const float* W, const float* b, float* y);
int s2s_tconv_bwd(s2s_ctx*, void* stream, int B, int L, int Din, int Dout, int kW, int relu, const float* x,
                  const float* W, const float* y, const float* dy, float* dx, int dx_accumulate, float* dW, float* db,
                  float scale, void* scratch, size_t scratch_bytes);
int s2s_tmaxpool_fwd(s2s_ctx*, void* stream, int B, int L, int D, int kW, int dW, const float* x, float* y, int* idx);
int s2s_tmaxpool_bwd(s2s_ctx*, void* stream, int B, int L, int D, int kW, int dW, const int* idx, const float* dy,
                     float* dx);
size_t s2s_sconv_scratch_bytes(int B, int Cin, int H, int W, int Cout, int kH, int kW);
int s2s_sconv_fwd(s2s_ctx*, void* stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu,
                  const float* x, const float* weight, const float* bias, float* y, void* scratch, size_t scratch_bytes);
int s2s_sconv_bwd(s2s_ctx*, void* stream, int B, int Cin, int H, int W, int Cout, int kH, int kW, int relu,
                  const float* x, const float* weight, const float* y, const float* dy, float* dx, int dx_accumulate,
                  float* dweight, float* dbias, float scale, void* scratch, size_t scratch_bytes,
                  int col_from_fwd);
int s2s_smaxpool_fwd(s2s_ctx*, void* stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH,
                     const float* x, float* y, int* idx);
int s2s_smaxpool_bwd(s2s_ctx*, void* stream, int B, int C, int H, int W, int kW, int kH, int dW, int dH,
                     const int* idx, const float* dy, float* dx);
int s2s_swap12(s2s_ctx*, void* stream, int B, int D1, int D2, int D3, const float* x, float* y);
int s2s_relu_fwd(s2s_ctx*, void* stream, long n, const float* x, float* y);
int s2s_relu_bwd(s2s_ctx*, void* stream, long n, const float* x, const float* dy, float* dx);
int s2s_logsoftmax_fwd(s2s_ctx*, void* stream, long rows, int n, const float* x, float* y);
int s2s_logsoftmax_bwd(s2s_ctx*, void* stream, long rows, int n, const float* y, const float* dy, float* dx);
]]

local C = ffi.load('s2s_hip')
local M = {C = C}

function M.check(rc)
   if rc ~= 0 then error(ffi.string(C.s2s_last_error())) end
end

function M.context(device)
   local out = ffi.new('s2s_ctx*[1]')
   M.check(C.s2s_ctx_create(device or 0, out))
   return ffi.gc(out[0], C.s2s_ctx_destroy)
end

-- device pointer of a contiguous CudaTensor
local function dptr(t) return ffi.cast('float*', torch.data(t)) end
M.dptr = dptr

-- nn.RNN(nn.GRU(D,H), reverse) forward/backward for a (L x D) or (B x L x D) input.
-- W = {Wz, Wr, Wh}: the three LinearZeroBias weights of the cell (GRU.lua:23-26).
function M.gru_forward(ctx, stream, x, W, H, reverse, output, saved, scratch)
   assert(x:nDimension() == 2 or x:nDimension() == 3, 'input dimension must be 2D or 3D')
   local x3 = x:nDimension() == 2 and x:view(1, x:size(1), x:size(2)) or x
   local B, L, D = x3:size(1), x3:size(2), x3:size(3)
   output:resize(B, L, H)
   saved:resize(tonumber(C.s2s_gru_saved_bytes(B, L, H)))
   scratch:resize(tonumber(C.s2s_gru_scratch_bytes(1, B, L, D, H)))
   local w = ffi.new('const float*[3]', {dptr(W[1]), dptr(W[2]), dptr(W[3])})
   local y = ffi.new('float*[1]', {dptr(output)})
   local sv = ffi.new('void*[1]', {ffi.cast('void*', torch.data(saved))})
   M.check(C.s2s_gru_fwd(ctx, stream, 1, B, L, D, H, ffi.new('int[1]', {reverse and 1 or 0}), dptr(x3), D, w, y, H,
                         sv, ffi.cast('void*', torch.data(scratch)), scratch:nElement()))
   return output
end

-- nn.TemporalConvolution(Din, Dout, kW) on a (L x Din) or (B x L x Din) CudaTensor, as the conv + BiLSTM
-- encoder's convlayer uses it (timit/timit.lua:113-121); relu = true fuses the nn.ReLU that follows.
function M.tconv_forward(ctx, stream, m, x, relu, output)
   local x3 = x:nDimension() == 2 and x:view(1, x:size(1), x:size(2)) or x
   local B, L, Din = x3:size(1), x3:size(2), x3:size(3)
   output:resize(B, L - m.kW + 1, m.outputFrameSize)
   M.check(C.s2s_tconv_fwd(ctx, stream, B, L, Din, m.outputFrameSize, m.kW, relu and 1 or 0, dptr(x3),
                           dptr(m.weight), dptr(m.bias), dptr(output)))
   return output
end

-- updateGradInput + accGradParameters(scale) of the same module (gradInput overwritten)
function M.tconv_backward(ctx, stream, m, x, relu, output, gradOutput, gradInput, scale, scratch)
   local x3 = x:nDimension() == 2 and x:view(1, x:size(1), x:size(2)) or x
   local B, L, Din = x3:size(1), x3:size(2), x3:size(3)
   gradInput:resizeAs(x3)
   scratch:resize(tonumber(C.s2s_tconv_scratch_bytes(B, L, Din, m.outputFrameSize, m.kW)))
   M.check(C.s2s_tconv_bwd(ctx, stream, B, L, Din, m.outputFrameSize, m.kW, relu and 1 or 0, dptr(x3), dptr(m.weight),
                           dptr(output), dptr(gradOutput), dptr(gradInput), 0, dptr(m.gradWeight), dptr(m.gradBias),
                           scale or 1, ffi.cast('void*', torch.data(scratch)), scratch:nElement()))
   return gradInput
end

return M
