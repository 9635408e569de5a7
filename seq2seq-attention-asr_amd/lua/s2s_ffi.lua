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
                 int hybridAttendFilterSize, hybridAttendFeatureMaps; } s2s_attn_dims;
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

return M
