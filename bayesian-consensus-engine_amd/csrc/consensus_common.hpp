// consensus_common.hpp -- declarations shared by the consensus translation units
// (consensus.hip: list / long-market kernels, launchers and the C ABI; consensus_tab.hip:
// the LDS-table kernel for contiguous short markets; consensus_wide.hip: 64 < n <= 4096).
#pragma once
#pragma clang fp contract(off)

#include "bce_device.hpp"
#include "bce_internal.hpp"

namespace bce {

struct ConsArgs {
  const int64_t* offsets;
  const int32_t* sid;
  const double* prob;
  const double2* relconf;    // [S] interleaved {reliability, confidence}: one 16-B row
  const uint32_t* pbits;     // [ceil(S/32)] present bitmask (bit s%32 of word s/32)
  int32_t n_sources;
  int64_t n_signals;
  const int32_t* list;  // nullable
  int64_t n_list;       // number of markets to process
  // consensus_wide_kernel only: positions li < n_hi come from list_hi[li], the rest from
  // list[li - n_hi] (EXACT's merged launch: the longer bin's markets first, longest-first overall)
  const int32_t* list_hi;
  int64_t n_hi;
  double* consensus;
  double* confidence;
  double* total_weight;
  int32_t* n_unique;
  int32_t* err_idx;   // nullable
  int32_t* usid;      // nullable
  double* weight;     // nullable
  double* nweight;    // nullable
  int32_t mode;
  void* scratch;      // long kernel, global variant
  int64_t scratch_stride;  // elements (keys) per workgroup slice
  int* fault;         // device word: set to a kFault* code by a wave that gave up
  int spin_cap;       // bounded waits of the persistent pipe kernel (polls before giving up)
  int32_t tab_rows;   // tab kernel, hybrid table: rows [0, tab_rows) staged in LDS, the rest read from relconf
  // Device-driven planned launch (bce_consensus_planned_device): the bin boundaries live on the
  // device (int64[BCE_NBINS + 1]); the kernel takes plan positions [dev_bins[dev_b0],
  // dev_bins[dev_b1 + 1]) of `list` (the whole plan order), bin dev_b1's markets first when
  // dev_b0 < dev_b1 (a merged launch, as list_hi / n_hi).  NULL: list / n_list as given.
  const int64_t* dev_bins;
  int32_t dev_b0, dev_b1;
};

// Resolve a device-driven launch's market range at kernel entry (uniform scalar loads).
__device__ __forceinline__ void dev_range(ConsArgs& a) {
  if (a.dev_bins) {
    const int64_t lo = a.dev_bins[a.dev_b0], mid = a.dev_bins[a.dev_b1], hi = a.dev_bins[a.dev_b1 + 1];
    const int32_t* order = a.list;
    a.list = order + lo;
    a.n_list = hi - lo;
    if (a.dev_b0 != a.dev_b1) {
      a.list_hi = order + mid;
      a.n_hi = hi - mid;
    }
  }
}

// Device fault codes (bce_fault_check reports them).
constexpr int kFaultSpinLoader = 1;   // pipe kernel: loader never saw a slot released
constexpr int kFaultSpinCompute = 2;  // pipe kernel: compute wave never saw its slot loaded
constexpr int kFaultSid = 3;          // a sid >= n_sources (the row read was clamped)
constexpr int kFaultTooLong = 4;      // a market longer than the launch's max_len (skipped)
constexpr int kFaultSpinChain = 5;    // wide kernel, exact mode: chain / producer wait timed out
constexpr int kFaultOffsets = 7;      // device planner: offsets decrease somewhere

constexpr int kBitsLds = 512;  // present bitmask words staged in LDS (S <= 16384)

__device__ __forceinline__ bool is_present(const uint32_t* bits, int s) {
  return ((bits[s >> 5] >> (s & 31)) & 1u) != 0;
}

// Batcher odd-even merge sort network for N (power of two) keys, generated at compile
// time; with full unrolling every key index is a constant, so the keys live in VGPRs.
template <int N>
struct OemNet {
  static constexpr int count() {
    int c = 0;
    for (int p = 1; p < N; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < N; j += 2 * k)
          for (int i = 0; i < k && i + j + k < N; ++i)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) ++c;
    return c;
  }
  static constexpr int C = count();
  struct Pairs {
    int a[C > 0 ? C : 1];
    int b[C > 0 ? C : 1];
  };
  static constexpr Pairs make() {
    Pairs r{};
    int c = 0;
    for (int p = 1; p < N; p <<= 1)
      for (int k = p; k >= 1; k >>= 1)
        for (int j = k % p; j + k < N; j += 2 * k)
          for (int i = 0; i < k && i + j + k < N; ++i)
            if ((i + j) / (2 * p) == (i + j + k) / (2 * p)) {
              r.a[c] = i + j;
              r.b[c] = i + j + k;
              ++c;
            }
    return r;
  }
};

template <int N>
__device__ __forceinline__ void oem_sort(unsigned (&key)[N]) {
  constexpr auto P = OemNet<N>::make();
#pragma unroll
  for (int c = 0; c < OemNet<N>::C; ++c) {
    const unsigned x = key[P.a[c]], y = key[P.b[c]];
    key[P.a[c]] = x < y ? x : y;
    key[P.b[c]] = x < y ? y : x;
  }
}

// Same network carrying a payload (the probability) with each key.
template <int N>
__device__ __forceinline__ void oem_sort_kv(unsigned (&key)[N], double (&val)[N]) {
  constexpr auto P = OemNet<N>::make();
#pragma unroll
  for (int c = 0; c < OemNet<N>::C; ++c) {
    const unsigned x = key[P.a[c]], y = key[P.b[c]];
    const double vx = val[P.a[c]], vy = val[P.b[c]];
    const bool sw = y < x;
    key[P.a[c]] = sw ? y : x;
    key[P.b[c]] = sw ? x : y;
    val[P.a[c]] = sw ? vy : vx;
    val[P.b[c]] = sw ? vx : vy;
  }
}

// Cross-lane LDS hand-off inside ONE wave (waves of a workgroup run independently): the
// wave's LDS instructions execute in order, so draining lgkmcnt behind a compiler
// barrier orders every earlier ds_write before every later ds_read / LDS-DMA.
__device__ __forceinline__ void wave_sync_lds() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Acquire-load of an LDS flag, broadcast to a wave-uniform (SGPR) value: every spin and
// branch on a flag is then scalar control flow (a per-lane view of the same word makes
// the compiler build divergent loop exits around it).
__device__ __forceinline__ int ldsflag(int* f) {
  const int v = __hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
  return __builtin_amdgcn_readfirstlane(v);
}

// A wave that gives up on a wait records why (first code wins) with a vector atomic.
__device__ __forceinline__ void raise_fault(int* fault, int code) {
  if (fault && lane_id() == 0) atomicCAS(fault, 0, code);
}

// LDS-DMA issued from inline asm.  The compiler's wait-count pass treats every LDS
// access after a *builtin* LDS-DMA as a possible alias and drains vmcnt(0) in front of
// it; the kernels that use these order their images themselves.  M0 is reserved to the
// compiler (an "m0" clobber is ignored), so the helpers save it into an SGPR, point it at
// the LDS destination for the DMA and restore it before returning: whatever M0 value the
// compiler keeps live across the call survives.
__device__ __forceinline__ void dma_b128(const void* g, const void* lds) {
  const uint32_t l = (uint32_t)(uintptr_t)lds;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %2, off\n\t"
               "s_mov_b32 m0, %0\n\ts_nop 0"
               : "=&s"(keep) : "s"(l), "v"(g) : "memory");
}
__device__ __forceinline__ void dma_b32(const void* g, const void* lds) {
  const uint32_t l = (uint32_t)(uintptr_t)lds;
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %2, off\n\t"
               "s_mov_b32 m0, %0\n\ts_nop 0"
               : "=&s"(keep) : "s"(l), "v"(g) : "memory");
}

// ---- host side -------------------------------------------------------------------------
// The device fault word of the current device (allocated once, zeroed).
int* fault_word();
// Polls a persistent wave makes before it gives up (bce_debug_set_spin_cap; default 2^22).
int spin_cap();

// LDS-table kernel (consensus_tab.hip): contiguous markets with n <= 32 and
// n_sources <= kTabMaxSources.
constexpr int kTabMaxSources = 10112;  // 16 B per source + the bitmask fit the 160 KiB LDS
// Larger tables (up to kTabHybMaxSources): the first rows that fit beside the whole present
// bitmask are staged in LDS, the rest are gathered from the global table (hybrid mode).
constexpr int kTabHybMaxSources = 1 << 18;
constexpr int kTabLdsBytes = 160 * 1024;
int launch_tab32(const ConsArgs& a, hipStream_t st);

// Register-sort kernel (consensus_wide.hip) for 64 < n <= 4096: keys (sid << ib) | index with
// ib = log2 of the bin's padded size (7..12), 32 bits while n_sources <= 2^(32 - ib), else 64.
int launch_wide_len(int64_t max_len, const ConsArgs& a, hipStream_t st);
// Resident workgroups (every CU's share) of the wide kernel launch_wide_len would pick.
int64_t wide_resident(int64_t max_len, int32_t mode, int32_t n_sources);
// kSplitWords words (one per wave of the grid) for a tie-break FULL/rest launch pair
// (tiebreak.hip; written with a per-launch ticket)
constexpr int kSplitWords = 4096;
int* split_slot(int ticket, hipStream_t st);  // clears the slot on `st` when the ticket counter wrapped

}  // namespace bce
