// In-launch hand-offs between workgroups of a persistent kernel (MI355X guide §6 Guideline 16,
// form R2 "the data is the flag"): every handed-off fp32 value is ONE 8-byte granule
// {value, tag} stored write-through (sc1); consumers re-read the granules they need with sc1
// loads until every tag equals the expected epoch.  Buffers are zeroed (memset node) before each
// launch; epochs are 1-based step counters within the launch.  Every wait is bounded: on timeout
// (or when another wave already gave up) the abort word is raised and the wait returns false; the
// call's harvest launch reports it to the owning context (s2s_ctx_status; every later call fails).
#pragma once
#include "s2s_common.h"

#include <algorithm>

namespace s2s {

constexpr unsigned kSpinLimit = 1u << 21;
typedef unsigned long long granule_t;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc_of(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// local = every consumer runs on this workgroup's XCD (chain_is_local): the granule may then stay
// in that XCD's L2 (plain store, sc0) -- the consumers' sc1 loads are served from the same L2, one
// hop ~0.22 us instead of ~0.55 us through the fabric with write-through (sc1) stores (measured on
// MI355X, tools/pingpong.hip).  Cross-XCD consumers need local = false.
__device__ __forceinline__ void put_granule(granule_t* g, float v, unsigned tag, bool local = false) {
  const granule_t x = ((granule_t)tag << 32) | (granule_t)__float_as_uint(v);
  if (local) __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  else __hip_atomic_store(g, x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Publish granule base[idx] of this lane when `active` (base is wave-uniform).  Lanes l and l^1
// own adjacent granules j, j+1 (j even at the even lane) at every call site, so
// S2S_PAIRED_GRANULES=1 lets the even lane write both in one 16-byte sc1 buffer store after a
// lane shuffle (every lane must then call it).  Measured on MI355X (same-box A/B): slower than
// one 8-byte global sc1 store per lane, and buffer-form 8-byte stores are slower than the
// global form -- so the default is put_granule's global_store_dwordx2 sc1.
#ifndef S2S_PAIRED_GRANULES
#define S2S_PAIRED_GRANULES 0
#endif
__device__ __forceinline__ void put_granule_pair(granule_t* base, long idx, float v, unsigned tag, bool active,
                                                 bool local = false) {
#if S2S_PAIRED_GRANULES
  const float vn = __shfl_xor(v, 1, 64);
  if (active && (threadIdx.x & 1) == 0) {
    typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 d = {__float_as_uint(v), tag, __float_as_uint(vn), tag};
    __builtin_amdgcn_raw_buffer_store_b128(d, rsrc_of(base), (int)(8 * idx), 0, 16);
  }
#else
  if (active) put_granule(base + idx, v, tag, local);
#endif
}
// two adjacent granules j, j+1 of one lane (j % 2 == 0) as one 16-byte store
__device__ __forceinline__ void put_granule2(__amdgpu_buffer_rsrc_t rs, long byte_off, float v0, float v1, unsigned tag,
                                             bool local = false) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 d = {__float_as_uint(v0), tag, __float_as_uint(v1), tag};
  if (local) __builtin_amdgcn_raw_buffer_store_b128(d, rs, (int)byte_off, 0, 1);
  else __builtin_amdgcn_raw_buffer_store_b128(d, rs, (int)byte_off, 0, 16);
}
// four adjacent granules j..j+3 of one lane (j % 2 == 0) as two 16-byte write-through stores
__device__ __forceinline__ void put_granule4(__amdgpu_buffer_rsrc_t rs, long byte_off, float v0, float v1, float v2,
                                             float v3, unsigned tag, bool local = false) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 d0 = {__float_as_uint(v0), tag, __float_as_uint(v1), tag};
  const u32x4 d1 = {__float_as_uint(v2), tag, __float_as_uint(v3), tag};
  if (local) {
    __builtin_amdgcn_raw_buffer_store_b128(d0, rs, (int)byte_off, 0, 1);
    __builtin_amdgcn_raw_buffer_store_b128(d1, rs, (int)byte_off + 16, 0, 1);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(d0, rs, (int)byte_off, 0, 16);
    __builtin_amdgcn_raw_buffer_store_b128(d1, rs, (int)byte_off + 16, 0, 16);
  }
}
// value of a granule already known to carry the right tag (validated by a sweep of this workgroup)
__device__ __forceinline__ float peek_granule(const granule_t* g) {
  return __uint_as_float((unsigned)__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// ---- sync-region header (256 bytes in front of every persistent launch's hand-off region)
//   u32 word 0: abort word (0 = running; 1 = a wave gave up a wait; 2 = started aborted: the
//               s2s_debug_inject_abort test knob)
//   u32 word 16 (byte 64): launch epoch (tags = (epoch << 16) + step)
//   u32 word 48 (byte 192): sticky failure bits of the region's earlier launches since the last harvest: a
//               launch that prepares the region for the next one (prep_next_sync) ORs the abort word into it
//               before resetting the abort word
// The failure is reported OFF the hand-off path: a harvest launch at the end of every call (sync_harvest,
// stream-ordered after the call's persistent launches) ORs each region's abort word and sticky bits into the
// owning context's host-visible status words and clears them.  (Reporting from inside the waits, even on the
// give-up path only, changed the waits' code generation: +0.19 ms per config-2 step, same-box A/B.)
constexpr int kEpochWord = 16;   // u32 index of the epoch in the sync header
constexpr int kStickyWord = 48;  // u32 index of the sticky failure bits

// abort_word is the sync header's word 0
__device__ __forceinline__ bool spin_give_up(unsigned& spins, unsigned* abort_word, unsigned limit = kSpinLimit) {
  ++spins;
  if ((spins & 63u) == 0) {
    if (spins > limit || __hip_atomic_load(abort_word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) {
      __hip_atomic_store(abort_word, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
  }
  // Polls run back to back (no s_sleep between passes): a poll pass is already one L2 round trip, and the
  // sleep delayed the pass that sees the value -- measured (same box, config-2 step): 3.308 -> 3.278 ms without
  // the sleep, the GRU forward step 2.62 -> 2.50 us; sleeping only after the first 16 / 64 passes was slower
  // (3.33 ms).  S2S_SPIN_SLEEP=1 (a build flag) restores the sleep.
#if defined(S2S_SPIN_SLEEP) && S2S_SPIN_SLEEP
  __builtin_amdgcn_s_sleep(1);
#endif
  return false;
}

// ---- launch epochs
// Granule tags are (epoch << 16) + step, with a fresh epoch per launch: granules a previous launch
// left at the same addresses (same steps, so the same step tags) can never satisfy a wait, even if
// a cache still holds them (measured: without epochs a repeated decoder launch with new weights
// consumed the previous launch's values).  sync_prep (one launch replacing the memset) zeroes the
// granule region past the 256-byte header and, in block 0, draws the epoch from a device counter,
// resets the abort word (or raises it: the s2s_debug_inject_abort test knob) and the sticky bits (the
// previous call's harvest has reported them) -- with memory-side atomics; every workgroup reads the epoch
// with a memory-side atomic too (launch_tagbase).
static __device__ unsigned g_s2s_epoch_ctr;
static __global__ __launch_bounds__(256) void sync_prep(char* sync, size_t bytes, unsigned abort0, char* clear,
                                                         char* hdr_at) {
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if (clear) {  // the other (idle) region of a hand-over pair: its words may still be uninitialised memory
      unsigned* c = reinterpret_cast<unsigned*>(clear);
      __hip_atomic_exchange(c + kStickyWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_exchange(c, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    unsigned* hdr = reinterpret_cast<unsigned*>(hdr_at ? hdr_at : sync);
    const unsigned e = __hip_atomic_fetch_add(&g_s2s_epoch_ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
    __hip_atomic_exchange(hdr + kEpochWord, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(hdr + kStickyWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_exchange(hdr, abort0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  const size_t n16 = (bytes - 256) / 16;
  uint4* p = reinterpret_cast<uint4*>(sync + 256);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_uint4(0u, 0u, 0u, 0u);
}
// clear (optional): the header of the region the launch behind this prep will prepare for the next launch
// (prep_next_sync folds that region's abort word into its sticky bits, which must not be stale memory);
// hdr (optional): the region's header lives there instead of at `sync` (whose first 256 bytes are then unused)
inline int launch_sync_prep(hipStream_t st, void* sync, size_t bytes, void* clear = nullptr, void* hdr = nullptr) {
  // bytes - 256 is a multiple of 8 (granules) and of 4 (census words); round the tail up is not
  // allowed, so clear the last partial 16-byte piece with zero_async only when present
  const size_t n16 = (bytes - 256) / 16;
  int blocks = (int)std::min<size_t>(1024, (n16 + 255) / 256);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(sync_prep, dim3(blocks), dim3(256), 0, st, static_cast<char*>(sync), bytes,
                     inject_abort_take() ? 2u : 0u, static_cast<char*>(clear), static_cast<char*>(hdr));
  if ((bytes - 256) % 16)
    S2S_TRY(zero_async(st, static_cast<char*>(sync) + 256 + n16 * 16, (bytes - 256) % 16));
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}
// a launch that prepares `hdr`'s region for the next launch: keep its previous launch's failure (sticky)
__device__ __forceinline__ void rearm_abort_word(unsigned* hdr) {
  const unsigned old = __hip_atomic_exchange(hdr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (old) __hip_atomic_fetch_or(hdr + kStickyWord, old, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// harvest: region i's abort word | sticky bits -> the context's status words ([0] a wait timed out, [1] a
// launch started on an aborted region), then cleared.  One thread per region.
constexpr int kMaxHarvest = 8;
struct HarvestArgs {
  char* region[kMaxHarvest];
  int n;
  unsigned* status;
};
static __global__ __launch_bounds__(64) void sync_harvest(HarvestArgs h) {
  const int i = threadIdx.x;
  if (i >= h.n) return;
  unsigned* hdr = reinterpret_cast<unsigned*>(h.region[i]);
  const unsigned v = __hip_atomic_exchange(hdr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) |
                     __hip_atomic_exchange(hdr + kStickyWord, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (v) __hip_atomic_store(h.status + 4 + i, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);  // diagnostic: raw bits
  if (v & 1u) __hip_atomic_store(h.status, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (v & 2u) __hip_atomic_store(h.status + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
// status null: nothing reported (no launch)
inline int launch_sync_harvest(hipStream_t st, void* const* regions, int n, unsigned* status) {
  if (!status || n <= 0) return 0;
  HarvestArgs h{};
  S2S_REQUIRE(n <= kMaxHarvest, "harvest: too many regions");
  for (int i = 0; i < n; ++i) h.region[i] = static_cast<char*>(regions[i]);
  h.n = n;
  h.status = status;
  hipLaunchKernelGGL(sync_harvest, dim3(1), dim3(64), 0, st, h);
  S2S_CHECK_HIP(hipGetLastError());
  return 0;
}
// tag base of this launch (all threads call; one barrier)
__device__ __forceinline__ unsigned launch_tagbase(const unsigned* sync_hdr, unsigned* lds) {
  if (threadIdx.x == 0)
    *lds = __hip_atomic_fetch_add(const_cast<unsigned*>(sync_hdr) + kEpochWord, 0u, __ATOMIC_RELAXED,
                                  __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  return (*lds & 0xffffu) << 16;
}

// ---- XCD-local chains
// A chain = the workgroups that hand data to each other (independent of other chains).  Launches
// place chain c's members at blockIdx = 8 * (member + nmem * (c / 8)) + c % 8, which the MI355X
// dispatcher deals to ONE XCD (blocks b and b + 8 share an XCD; speed only, never assumed):
// chain_is_local() checks it at run time -- every member publishes HW_REG_XCC_ID and reads all of
// its chain's -- so a chain uses L2-resident hand-offs only when it really shares one L2.
constexpr int kXccIdHwreg = 20 | (0 << 6) | (3 << 11);  // hwreg(HW_REG_XCC_ID, 0, 4)
struct ChainSlot {
  int chain, member;
};
__device__ __forceinline__ ChainSlot chain_slot(int nmem) {
  const int x = blockIdx.x & 7, j = blockIdx.x >> 3;
  return ChainSlot{x + 8 * (j / nmem), j % nmem};
}
__host__ __device__ constexpr int chain_grid(int nchains, int nmem) { return 8 * nmem * ((nchains + 7) / 8); }
// census: zeroed u32 per (chain, member); flag: a __shared__ int; all 256 threads call it
__device__ __forceinline__ bool chain_is_local(unsigned* census, int chain, int nmem, int member, bool allow,
                                               unsigned* abort_word, int* flag, unsigned tb) {
  const unsigned me = tb | 0x100u | (__builtin_amdgcn_s_getreg(kXccIdHwreg) & 15u);
  unsigned* row = census + (long)chain * nmem;
  if (threadIdx.x == 0) {
    *flag = allow ? 1 : 0;
    __hip_atomic_store(row + member, me, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if ((int)threadIdx.x < nmem) {
    unsigned spins = 0, v;
    while (((v = __hip_atomic_load(row + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) & 0xffff0100u) !=
           (tb | 0x100u))
      if (spin_give_up(spins, abort_word)) break;
    if (v != me) *flag = 0;
  }
  __syncthreads();
  return *flag != 0;
}

// ---- sentinel hand-offs (XCD-local chains)
// A granule is 8 bytes to carry 4 bytes of payload; a sweep reads every handed-off value of its
// rows (16 rows x K per workgroup and phase), so the tag halves the useful rate of the per-CU L2
// path that bounds a recurrence step (measured: half the swept bytes took a GRU layer from 1.55
// to 1.15 ms).  Where every slot is written once per launch, the plain fp32 value can be its own
// flag: the slot is re-armed to kSent (an all-ones NaN pattern no finite computation produces)
// before the launch's first publication, and a consumer polls until no word equals kSent.
// Re-arming is done by the slot's own producer at launch start with plain stores into its XCD's
// L2 -- the L2 every consumer of a local chain reads -- drained (vmcnt(0)) before the producer's
// census word (chain_is_local), which every member waits for before its first poll; a chain that
// turns out not to be XCD-local uses tagged granules instead (stale lines of an earlier launch in
// another XCD's L2 could otherwise pass for fresh values).
constexpr unsigned kSent = 0xffffffffu;
__device__ __forceinline__ void put_sent(float* p, float v) {
  __hip_atomic_store(reinterpret_cast<unsigned*>(p), __float_as_uint(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_WORKGROUP);  // plain store: stays in this XCD's L2
}
// re-arm rows [r0, r0 + nr) x columns [c0, c0 + nc) (nc % 4 == 0, 16-byte aligned) of slots
// 0..nslots-1 (slot stride `slot`, row stride ld floats); all 256 threads call it; the producer's
// re-arms end with rearm_done() before its census word
// rearm_rect over a chain-interleaved slot (the XCD decoder's 4 x 4 form, dec_xcd.inc ilv): a chain's rows b0 ..
// b0 + nU - 1 of a [B][W] slot are stored quad-major, element (b0 + r, n) at b0 W + (n / 4) 4 nU + 4 r + n % 4, so
// one k-quad of all its rows is 16 nU contiguous bytes; rows r0 .. r0 + nr - 1, columns [c0, c0 + nc) re-armed
__device__ __forceinline__ void rearm_ilv(float* base, long slot, int nslots, long W, int b0, int nU, int r0, int nr,
                                          int c0, int nc) {
  const float4 sv = make_float4(__uint_as_float(kSent), __uint_as_float(kSent), __uint_as_float(kSent),
                                __uint_as_float(kSent));
  const int n4 = nc / 4, per = nr * n4;
  if (per <= 0) return;
  for (int i = threadIdx.x; i < nslots * per; i += 256) {
    const int s = i / per, rem = i - s * per, r = rem / n4, c = rem - r * n4;
    *reinterpret_cast<float4*>(base + s * slot + (long)b0 * W + (long)(c0 / 4 + c) * 4 * nU + 4 * (r0 + r)) = sv;
  }
}
__device__ __forceinline__ void rearm_rect(float* base, long slot, int nslots, long ld, int r0, int nr, int c0,
                                           int nc) {
  const float4 sv = make_float4(__uint_as_float(kSent), __uint_as_float(kSent), __uint_as_float(kSent),
                                __uint_as_float(kSent));
  const int n4 = nc / 4, per = nr * n4;
  if (per <= 0) return;
  if (256 % per == 0) {  // every thread keeps one (row, column) and strides over the slots
    const int spp = 256 / per, s0 = threadIdx.x / per, rem = threadIdx.x - s0 * per, r = rem / n4, c = rem - r * n4;
    float* p = base + (long)(r0 + r) * ld + c0 + 4 * c;
    for (int s = s0; s < nslots; s += spp) *reinterpret_cast<float4*>(p + s * slot) = sv;
    return;
  }
  for (int i = threadIdx.x; i < nslots * per; i += 256) {
    const int s = i / per, rem = i - s * per, r = rem / n4, c = rem - r * n4;
    *reinterpret_cast<float4*>(base + s * slot + (long)(r0 + r) * ld + c0 + 4 * c) = sv;
  }
}
__device__ __forceinline__ void rearm_done() {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
}
// sweep_skinny's operand layout over a sentinel row (row_off in bytes): one 16-byte load per chunk
template <int NC>
__device__ __forceinline__ bool sweep_sent(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long row_off, int wave,
                                           int lane, unsigned* abort_word, int kmul = 1) {
  const long kq = 4 * (lane >> 4);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = row_off + 4L * kmul * (wave * 16 + 64 * i + kq);
      const uint4 p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
      a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// Tile-major sentinel slots: a slot is [row tile][H / 16 column tiles][16 rows][16 columns] (row tiles of 16
// utterances), so the 16 x 16 tile one chain member publishes per step is 1 KB contiguous -- every 128-B line has
// one writer -- and chunk i of a sweeping wave (columns wave * 16 + 64 i .. + 15 = column tile wave + 4 i) is
// one wave instruction over that 1-KB tile instead of 64 B of each of 16 rows.  Measured (tools/sweepbench.hip:
// 16 members, H = 256, one seam per step): 1.18-1.20 -> 1.00-1.04 us per seam.
// Inside a 16 x 16 tile the floats are quad-major (S2S_TILE_QUAD, default): element (r, c) at (c / 4) 64 + 4 r + c % 4,
// so the float4 a sweeping lane loads (row r, k-quad c / 4) sits next to its neighbour lanes' rows: each quad of
// lanes reads one 64-byte run (one line) instead of four rows 64 bytes apart (two lines) -- the per-instruction
// line count that bounds a sweep pass (the XCD decoder's interleaved slots, dec_xcd.inc, measured the effect).
#ifndef S2S_TILE_QUAD
#define S2S_TILE_QUAD 1
#endif
__device__ __forceinline__ int tile_in(int r, int c) { return S2S_TILE_QUAD ? (c >> 2) * 64 + r * 4 + (c & 3) : r * 16 + c; }
// float offset of the float4 a lane loads from a tile: row rowt, k-quad lane >> 4
__device__ __forceinline__ int tile_lane(int rowt, int lane) {
  return S2S_TILE_QUAD ? (lane >> 4) * 64 + rowt * 4 : rowt * 16 + 4 * (lane >> 4);
}
__device__ __forceinline__ long tile_off(int row, int col, int H) {
  return (long)(row >> 4) * 16 * H + (long)(col >> 4) * 256 + tile_in(row & 15, col & 15);
}
// sweep_sent's operand layout over a tile-major slot: tbase = byte offset of the slot's row tile, rowt = this
// lane's row within it
template <int NC>
__device__ __forceinline__ bool sweep_sent_tile(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long tbase, int rowt,
                                                int wave, int lane, unsigned* abort_word) {
  const long lo = tbase + 4 * tile_lane(rowt, lane);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = lo + 4L * 256 * (wave + 4 * i);
      const uint4 p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
      a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// sweep_sent_tile's first pass split in two: sent_tile_issue loads the tile (no check, so nothing waits for the
// loads), sent_tile_check later tests and converts what arrived (false: some value is still a sentinel -- the
// caller then polls with sweep_sent_tile).  Work placed between the two (behind a sched_barrier) runs while the
// loads are in flight.
template <int NC>
__device__ __forceinline__ void sent_tile_issue(uint4 (&raw)[NC], __amdgpu_buffer_rsrc_t rs, long tbase, int rowt,
                                                int wave, int lane) {
  const long lo = tbase + 4 * tile_lane(rowt, lane);
#pragma unroll
  for (int i = 0; i < NC; ++i)
    raw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + 4L * 256 * (wave + 4 * i)), 0, 16));
}
template <int NC>
__device__ __forceinline__ bool sent_tile_check(const uint4 (&raw)[NC], float4 (&a)[NC]) {
  bool ok = true;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    const uint4 p = raw[i];
    ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
    a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
  }
  return __all(ok);
}

// sweep_sent_tile fused with its product, over loads already issued by sent_tile_issue: chunk i is checked (and
// polled on its own until published) and multiplied in order, so the MFMAs of the chunks that arrived first run
// while the later ones are still in flight.  Chunk i accumulates into acc0 (i even) / acc1 (i odd) in x, y, z, w
// order -- the per-accumulator sequences of mfma_chunks / mfma_pairs, so the sums are bitwise the same; acc0 / acc1
// come in initialised (zero, or a previous half's partials).  a receives the operands (false: gave up, abort).
template <int NC>
__device__ __forceinline__ bool sent_tile_mfma(uint4 (&raw)[NC], float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs,
                                               long tbase, int rowt, int wave, int lane, const float4* w,
                                               floatx4& acc0, floatx4& acc1, unsigned* abort_word) {
  const long lo = tbase + 4 * tile_lane(rowt, lane);
  unsigned spins = 0;
  bool ok = true;
#pragma unroll
  for (int i = 0; i < NC; ++i) {
    while (true) {
      const uint4 p = raw[i];
      if (__all(p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent)) break;
      if (spin_give_up(spins, abort_word)) {
        ok = false;
        break;
      }
      raw[i] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(lo + 4L * 256 * (wave + 4 * i)), 0, 16));
    }
    a[i] = make_float4(__uint_as_float(raw[i].x), __uint_as_float(raw[i].y), __uint_as_float(raw[i].z),
                       __uint_as_float(raw[i].w));
    floatx4& acc = (i & 1) ? acc1 : acc0;
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, w[i].x, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, w[i].y, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, w[i].z, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, w[i].w, acc, 0, 0, 0);
    __builtin_amdgcn_sched_barrier(0);  // chunk i's MFMAs stay ahead of chunk i + 1's check
  }
  return ok;
}
template <int NC>
__device__ __forceinline__ bool sweep_sent_mfma(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long tbase, int rowt,
                                                int wave, int lane, const float4* w, floatx4& acc0, floatx4& acc1,
                                                unsigned* abort_word) {
  uint4 raw[NC];
  sent_tile_issue<NC>(raw, rs, tbase, rowt, wave, lane);
  return sent_tile_mfma<NC>(raw, a, rs, tbase, rowt, wave, lane, w, acc0, acc1, abort_word);
}

// sweep_skinny_rows over sentinel rows: all R * NC loads of a pass issued before any check
template <int NC, int R>
__device__ __forceinline__ bool sweep_sent_rows(float4 (&a)[R][NC], const __amdgpu_buffer_rsrc_t (&rs)[R],
                                                const long (&row_off)[R], int wave, int lane, unsigned* abort_word,
                                                int kmul = 1) {
  const long kq = 4 * (lane >> 4);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const long off = row_off[r] + 4L * kmul * (wave * 16 + 64 * i + kq);
        const uint4 p = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs[r], (int)off, 0, 16));
        ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
        a[r][i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
      }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}
// sweep_vec over a sentinel row (row_off in bytes): float4 c4 = lane + 64 i, lanes with c4 >= n4 idle
template <int NV>
__device__ __forceinline__ bool sweep_vec_sent(float4 (&a)[NV], __amdgpu_buffer_rsrc_t rs, long row_off, int n4,
                                               int lane, unsigned* abort_word) {
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < n4) {
        const uint4 p =
            __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(row_off + 16L * c4), 0, 16));
        ok = ok && p.x != kSent && p.y != kSent && p.z != kSent && p.w != kSent;
        a[i] = make_float4(__uint_as_float(p.x), __uint_as_float(p.y), __uint_as_float(p.z), __uint_as_float(p.w));
      }
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// one thread waits for one granule
__device__ __forceinline__ float wait_granule(const granule_t* g, unsigned tag, unsigned* abort_word, bool& ok) {
  unsigned spins = 0;
  while (true) {
    const granule_t x = __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if ((unsigned)(x >> 32) == tag) return __uint_as_float((unsigned)x);
    if (spin_give_up(spins, abort_word)) {
      ok = false;
      return 0.f;
    }
  }
}

// one thread waits for n <= N granules base[j * stride], j < n: all loads are issued before any
// tag is checked (one round trip per pass instead of n dependent ones)
template <int N>
__device__ __forceinline__ bool wait_granules(const granule_t* base, long stride, int n, unsigned tag, float (&v)[N],
                                              unsigned* abort_word) {
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      if (j < n) {
        const granule_t x = __hip_atomic_load(base + j * stride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = ok && (unsigned)(x >> 32) == tag;
        v[j] = __uint_as_float((unsigned)x);
      }
    }
    if (ok) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// Skinny-operand sweep: this lane's NC chunks (chunk i = k in [wave*16 + 64 i + 4*(lane>>4), +4))
// of one granule row starting at byte offset row_off.  Matches skinny_wave's operand layout.
template <int NC>
__device__ __forceinline__ bool sweep_skinny(float4 (&a)[NC], __amdgpu_buffer_rsrc_t rs, long row_off, unsigned tag,
                                             int wave, int lane, unsigned* abort_word) {
  const long kq = 4 * (lane >> 4);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NC; ++i) {
      const long off = row_off + 8 * (wave * 16 + 64 * i + kq);
      const uint4 p0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
      const uint4 p1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off + 16, 0, 16));
      ok = ok && p0.y == tag && p0.w == tag && p1.y == tag && p1.w == tag;
      a[i] = make_float4(__uint_as_float(p0.x), __uint_as_float(p0.z), __uint_as_float(p1.x), __uint_as_float(p1.z));
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// Several granule rows (R of them, each NC chunks in sweep_skinny's layout) polled in ONE loop:
// every pass issues all R * NC * 2 loads before any tag check, so a phase that consumes R
// hand-offs pays one round trip, not R.  a[r][i] = chunk i of row r.
template <int NC, int R>
__device__ __forceinline__ bool sweep_skinny_rows(float4 (&a)[R][NC], const __amdgpu_buffer_rsrc_t (&rs)[R],
                                                  const long (&row_off)[R], const unsigned (&tag)[R], int wave,
                                                  int lane, unsigned* abort_word) {
  const long kq = 4 * (lane >> 4);
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int i = 0; i < NC; ++i) {
        const long off = row_off[r] + 8 * (wave * 16 + 64 * i + kq);
        const uint4 p0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs[r], (int)off, 0, 16));
        const uint4 p1 =
            __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs[r], (int)off + 16, 0, 16));
        ok = ok && p0.y == tag[r] && p0.w == tag[r] && p1.y == tag[r] && p1.w == tag[r];
        a[r][i] = make_float4(__uint_as_float(p0.x), __uint_as_float(p0.z), __uint_as_float(p1.x),
                              __uint_as_float(p1.z));
      }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// Vector sweep: float4 index c4 = lane + 64 i (i < NV) of one granule row (row_off bytes);
// lanes with c4 >= n4 read nothing.  Matches the "for (c4 = lane; c4 < n4; c4 += 64)" loops.
template <int NV>
__device__ __forceinline__ bool sweep_vec(float4 (&a)[NV], __amdgpu_buffer_rsrc_t rs, long row_off, int n4,
                                          unsigned tag, int lane, unsigned* abort_word) {
  unsigned spins = 0;
  while (true) {
    bool ok = true;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c4 = lane + 64 * i;
      if (c4 < n4) {
        const long off = row_off + 32L * c4;
        const uint4 p0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off, 0, 16));
        const uint4 p1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)off + 16, 0, 16));
        ok = ok && p0.y == tag && p0.w == tag && p1.y == tag && p1.w == tag;
        a[i] = make_float4(__uint_as_float(p0.x), __uint_as_float(p0.z), __uint_as_float(p1.x),
                           __uint_as_float(p1.z));
      }
    }
    if (__all(ok)) return true;
    if (spin_give_up(spins, abort_word)) return false;
  }
}

// same chunk order / accumulator split as skinny_wave (bitwise-equal sums)
template <int NC>
__device__ __forceinline__ floatx4 mfma_chunks(const float4 (&a)[NC], const float4 (&w)[NC]) {
  floatx4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i + 1 < NC; i += 2) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, w[i].x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].x, w[i + 1].x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, w[i].y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].y, w[i + 1].y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, w[i].z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].z, w[i + 1].z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, w[i].w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].w, w[i + 1].w, acc1, 0, 0, 0);
  }
  if (NC & 1) {
    constexpr int i = NC - 1;
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, w[i].x, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, w[i].y, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, w[i].z, acc0, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, w[i].w, acc0, 0, 0, 0);
  }
  return acc0 + acc1;
}

// mfma_chunks' pairs of chunks accumulated into (acc0, acc1): a K split into two operand halves of NC chunks
// (NC even) runs as mfma_pairs(first half, w) then mfma_pairs(second half, w + NC) -- mfma_chunks<2 NC> on the
// concatenation, instruction for instruction (bitwise-equal sums), with the first half's MFMAs free to run before
// the second half's operands have arrived
template <int NC>
__device__ __forceinline__ void mfma_pairs(const float4 (&a)[NC], const float4* w, floatx4& acc0, floatx4& acc1) {
  static_assert(NC % 2 == 0, "mfma_pairs: NC even");
#pragma unroll
  for (int i = 0; i < NC; i += 2) {
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].x, w[i].x, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].x, w[i + 1].x, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].y, w[i].y, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].y, w[i + 1].y, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].z, w[i].z, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].z, w[i + 1].z, acc1, 0, 0, 0);
    acc0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i].w, w[i].w, acc0, 0, 0, 0);
    acc1 = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i + 1].w, w[i + 1].w, acc1, 0, 0, 0);
  }
}

// mfma_chunks with the W fragments held in AGPRs, the accumulator half of gfx950's unified register file: an
// MFMA may read its A / B operands from AGPRs (cdna_hip_programming.md §3), so a kernel that keeps 100+ floats of
// weight fragments per lane for a whole launch leaves its 256 VGPRs to the code between the products -- the
// decoder kernels' attention loops otherwise run on one or two free VGPRs, every tanh chain serialised.  The
// same instruction sequence and accumulator split as mfma_chunks (bitwise-equal sums).  Inline asm, so its wait
// states are explicit: s_nop 1 before each MFMA (a just-written VGPR / AGPR operand), the first product of each
// accumulator takes C = 0 (no VALU-written C), and s_nop 11 after the chain before anything reads the
// accumulators (8-pass XDL result -> reader), tied to them so the readers stay below it.
template <int NC>
__device__ __forceinline__ floatx4 mfma_chunks_aw(const float4 (&a)[NC], const float4 (&w)[NC]) {
  floatx4 acc0, acc1;
#define S2S_MFMA_AW0(acc, x, y) asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=&v"(acc) : "v"(x), "a"(y))
#define S2S_MFMA_AW(acc, x, y) asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "a"(y))
  static_assert(NC >= 1, "mfma_chunks_aw");
  S2S_MFMA_AW0(acc0, a[0].x, w[0].x);
  if (NC >= 2) S2S_MFMA_AW0(acc1, a[1].x, w[1].x);
  else acc1 = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int i = 0; i + 1 < NC; i += 2) {
    if (i > 0) {
      S2S_MFMA_AW(acc0, a[i].x, w[i].x);
      S2S_MFMA_AW(acc1, a[i + 1].x, w[i + 1].x);
    }
    S2S_MFMA_AW(acc0, a[i].y, w[i].y);
    S2S_MFMA_AW(acc1, a[i + 1].y, w[i + 1].y);
    S2S_MFMA_AW(acc0, a[i].z, w[i].z);
    S2S_MFMA_AW(acc1, a[i + 1].z, w[i + 1].z);
    S2S_MFMA_AW(acc0, a[i].w, w[i].w);
    S2S_MFMA_AW(acc1, a[i + 1].w, w[i + 1].w);
  }
  if (NC & 1) {
    constexpr int i = NC - 1;
    if (NC > 1) S2S_MFMA_AW(acc0, a[i].x, w[i].x);
    S2S_MFMA_AW(acc0, a[i].y, w[i].y);
    S2S_MFMA_AW(acc0, a[i].z, w[i].z);
    S2S_MFMA_AW(acc0, a[i].w, w[i].w);
  }
#undef S2S_MFMA_AW0
#undef S2S_MFMA_AW
  asm volatile("s_nop 11" : "+v"(acc0), "+v"(acc1));
  return acc0 + acc1;
}

// mfma_chunks_aw split across operand groups (concatenated K): each call accumulates one group's chunks (pairs
// into acc0 / acc1, an odd tail into acc0) with its W fragments from AGPRs; the first call of a product passes init
// (its first product of each accumulator takes C = 0).  mfma_aw_done closes the chain (the XDL result wait) and
// returns acc0 + acc1.
template <int NC>
__device__ __forceinline__ void mfma_aw_acc(const float4 (&a)[NC], const float4 (&w)[NC], floatx4& acc0,
                                            floatx4& acc1, bool init) {
#define S2S_MFMA_AW0(acc, x, y) asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, 0" : "=&v"(acc) : "v"(x), "a"(y))
#define S2S_MFMA_AW(acc, x, y) asm volatile("s_nop 1\n\tv_mfma_f32_16x16x4_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "a"(y))
#pragma unroll
  for (int i = 0; i + 1 < NC; i += 2) {
    if (init && i == 0) {
      S2S_MFMA_AW0(acc0, a[0].x, w[0].x);
      S2S_MFMA_AW0(acc1, a[1].x, w[1].x);
    } else {
      S2S_MFMA_AW(acc0, a[i].x, w[i].x);
      S2S_MFMA_AW(acc1, a[i + 1].x, w[i + 1].x);
    }
    S2S_MFMA_AW(acc0, a[i].y, w[i].y);
    S2S_MFMA_AW(acc1, a[i + 1].y, w[i + 1].y);
    S2S_MFMA_AW(acc0, a[i].z, w[i].z);
    S2S_MFMA_AW(acc1, a[i + 1].z, w[i + 1].z);
    S2S_MFMA_AW(acc0, a[i].w, w[i].w);
    S2S_MFMA_AW(acc1, a[i + 1].w, w[i + 1].w);
  }
  if (NC & 1) {
    constexpr int i = NC - 1;
    if (init && NC == 1) {
      S2S_MFMA_AW0(acc0, a[i].x, w[i].x);
      acc1 = floatx4{0.f, 0.f, 0.f, 0.f};
    } else {
      S2S_MFMA_AW(acc0, a[i].x, w[i].x);
    }
    S2S_MFMA_AW(acc0, a[i].y, w[i].y);
    S2S_MFMA_AW(acc0, a[i].z, w[i].z);
    S2S_MFMA_AW(acc0, a[i].w, w[i].w);
  }
#undef S2S_MFMA_AW0
#undef S2S_MFMA_AW
}
__device__ __forceinline__ floatx4 mfma_aw_done(floatx4 acc0, floatx4 acc1) {
  asm volatile("s_nop 11" : "+v"(acc0), "+v"(acc1));
  return acc0 + acc1;
}

// The same products for a chain of at most 4 live rows on v_mfma_f32_4x4x1_16b_f32 (16 blocks of 4 x 4 x 1: 9.3
// cycles against the 16 x 16 x 4 form's 32.5 for a quarter of its multiply-adds, all of them live instead of 4 of 16
// rows; tools/mfma4_probe.hip).  The operand registers are the 16 x 16 x 4 form's, with the activation rows dealt
// by lane & 3 instead of lane & 15: lane l = 16 q + 4 g + j holds row j (A) and unit 4 g + j (B) of k-quad q, so
// block b = g + 4 q multiplies rows 0..3 by units 4g..4g+3 over k-quad q, and lane l's result register i is row i,
// unit l & 15, summed over k-quad q only.  mfma4_fold adds the four k-quads (lanes l, l ^ 16, l ^ 32, l ^ 48; the
// same order in every lane) and leaves the 16 x 16 form's layout: lanes 0..15 rows 0..3, every other row 0 -- so
// skinny_reduce / dec_sync sum the waves exactly as before.
template <int NC>
__device__ __forceinline__ void mfma4_aw_acc(const float4 (&a)[NC], const float4 (&w)[NC], floatx4& acc0,
                                             floatx4& acc1, bool init) {
#define S2S_MFMA4_AW0(acc, x, y) asm volatile("s_nop 1\n\tv_mfma_f32_4x4x1_16b_f32 %0, %1, %2, 0" : "=&v"(acc) : "v"(x), "a"(y))
#define S2S_MFMA4_AW(acc, x, y) asm volatile("s_nop 1\n\tv_mfma_f32_4x4x1_16b_f32 %0, %1, %2, %0" : "+v"(acc) : "v"(x), "a"(y))
#pragma unroll
  for (int i = 0; i + 1 < NC; i += 2) {
    if (init && i == 0) {
      S2S_MFMA4_AW0(acc0, a[0].x, w[0].x);
      S2S_MFMA4_AW0(acc1, a[1].x, w[1].x);
    } else {
      S2S_MFMA4_AW(acc0, a[i].x, w[i].x);
      S2S_MFMA4_AW(acc1, a[i + 1].x, w[i + 1].x);
    }
    S2S_MFMA4_AW(acc0, a[i].y, w[i].y);
    S2S_MFMA4_AW(acc1, a[i + 1].y, w[i + 1].y);
    S2S_MFMA4_AW(acc0, a[i].z, w[i].z);
    S2S_MFMA4_AW(acc1, a[i + 1].z, w[i + 1].z);
    S2S_MFMA4_AW(acc0, a[i].w, w[i].w);
    S2S_MFMA4_AW(acc1, a[i + 1].w, w[i + 1].w);
  }
  if (NC & 1) {
    constexpr int i = NC - 1;
    if (init && NC == 1) {
      S2S_MFMA4_AW0(acc0, a[i].x, w[i].x);
      acc1 = floatx4{0.f, 0.f, 0.f, 0.f};
    } else {
      S2S_MFMA4_AW(acc0, a[i].x, w[i].x);
    }
    S2S_MFMA4_AW(acc0, a[i].y, w[i].y);
    S2S_MFMA4_AW(acc0, a[i].z, w[i].z);
    S2S_MFMA4_AW(acc0, a[i].w, w[i].w);
  }
#undef S2S_MFMA4_AW0
#undef S2S_MFMA4_AW
}
__device__ __forceinline__ floatx4 mfma4_fold(floatx4 acc0, floatx4 acc1, int lane) {
  asm volatile("s_nop 11" : "+v"(acc0), "+v"(acc1));
  const floatx4 s = acc0 + acc1;
  floatx4 r;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const unsigned x = __float_as_uint(s[e]);
    const auto p = __builtin_amdgcn_permlane32_swap(x, x, false, false);  // {lanes' low-half value, high-half value}
    const float y = __uint_as_float(p[0]) + __uint_as_float(p[1]);      // k-quads q + (q ^ 2)
    const unsigned yu = __float_as_uint(y);
    const auto q = __builtin_amdgcn_permlane16_swap(yu, yu, false, false);
    r[e] = lane < 16 ? __uint_as_float(q[0]) + __uint_as_float(q[1]) : 0.f;
  }
  return r;
}
// mfma_chunks_aw / mfma_aw_acc + mfma_aw_done in the 16 x 16 form, or (R4) the 4 x 4 form + fold
template <bool R4, int NC>
__device__ __forceinline__ floatx4 mfma_rows_aw(const float4 (&a)[NC], const float4 (&w)[NC], int lane) {
  if constexpr (R4) {
    floatx4 acc0, acc1;
    mfma4_aw_acc<NC>(a, w, acc0, acc1, true);
    return mfma4_fold(acc0, acc1, lane);
  } else {
    return mfma_chunks_aw<NC>(a, w);
  }
}
template <bool R4, int NC>
__device__ __forceinline__ void mfma_rows_acc(const float4 (&a)[NC], const float4 (&w)[NC], floatx4& acc0,
                                              floatx4& acc1, bool init) {
  if constexpr (R4) mfma4_aw_acc<NC>(a, w, acc0, acc1, init);
  else mfma_aw_acc<NC>(a, w, acc0, acc1, init);
}
template <bool R4>
__device__ __forceinline__ floatx4 mfma_rows_done(floatx4 acc0, floatx4 acc1, int lane) {
  if constexpr (R4) return mfma4_fold(acc0, acc1, lane);
  else return mfma_aw_done(acc0, acc1);
}

// sweep_sent's first pass, loads only (its layout; checked with sent_tile_check, polled further with sweep_sent)
template <int NC>
__device__ __forceinline__ void sent_row_issue(uint4 (&raw)[NC], __amdgpu_buffer_rsrc_t rs, long row_off, int wave,
                                               int lane, int kmul = 1) {
  const long kq = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < NC; ++i)
    raw[i] = __builtin_bit_cast(
        uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(row_off + 4L * kmul * (wave * 16 + 64 * i + kq)), 0, 16));
}

// W operand fragments of one output-unit row (chunk i at wave*16 + 64 i), kept in VGPRs
template <int NC>
__device__ __forceinline__ void load_wfrag(float4 (&w)[NC], const float* row, int wave, int lane) {
#pragma unroll
  for (int i = 0; i < NC; ++i)
    w[i] = *reinterpret_cast<const float4*>(row + wave * 16 + 64 * i + 4 * (lane >> 4));
}

}  // namespace s2s
