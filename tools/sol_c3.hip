// sol_c3.hip -- speed-of-light probes for the config-3 traffic (experiment tooling, not product
// code; driven by tools/sol_c3.py on the GPU box with the real C3 batch).
//
// Every probe moves exactly what one consensus step must move at C3 -- sid + prob per signal,
// offsets + 5 outputs per market, and per unique source of every market: its row of the
// `relconf` table (one random 16-B gather), its present-bitmask word (one 4-B gather), and the
// usid / weight / nweight outputs -- but replaces the sort + dedup by READING the unique ranks
// the real kernel produced (ulist, 4 B per unique: the only extra traffic) and does trivial
// arithmetic.  So their times bound what any design with these gathers can reach:
//   flat      grid-stride over all signals, then over all uniques (no market structure): the
//             traffic floor of the mix, gathers included
//   market<NT, WPE>  one workgroup of NT threads per market (persistent, plan order), the same
//             per-market phases as consensus_wide_kernel (load the market's signals, then its
//             uniques' gathers + stores, then the market's outputs); WPE = the waves-per-EU
//             budget (the wide kernels run 4, i.e. 16 waves per CU)
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/sol_c3.hip -o tools/bin/libsol_c3.so
#include <hip/hip_runtime.h>
#include <stdint.h>

struct SolArgs {
  const int64_t* offsets;    // [M+1] CSR of the signals
  const int32_t* sid;        // [N]
  const double* prob;        // [N]
  const int32_t* order;      // [M] plan order (market of list position li)
  int64_t n_markets;
  const int64_t* uoff;       // [M+1] CSR of the uniques (compact)
  const int32_t* ulist;      // [U] unique ranks (the real kernel's usid & 0x7fffffff)
  int64_t n_uniques;
  const double2* relconf;    // [S]
  const uint32_t* bits;      // [ceil(S/32)]
  int32_t* usid;             // [N] outputs at the market's signal offsets
  double* weight;
  double* nweight;
  double* cons;              // [M] x 3 + 2 int32
  double* conf;
  double* tw;
  int32_t* nu;
  int32_t* err;
  double* sink;
};

namespace {

__device__ __forceinline__ double gather_unique(const SolArgs& a, int32_t s) {
  const double2 rc = a.relconf[s];
  const uint32_t w = a.bits[s >> 5];
  return rc.x + rc.y + (double)((w >> (s & 31)) & 1u);
}

__global__ __launch_bounds__(256) void flat_signals(SolArgs a, int64_t n) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  double acc = 0.0;
  for (int64_t i = g; i < n; i += st) acc += (double)a.sid[i] + a.prob[i];
  if (acc == -1.0) a.sink[0] = acc;
}

// uniques of all markets, flat: unique j of market m lands at offsets[m] + (j - uoff[m]); the
// market of a unique is found from a per-unique market index built on the host (umk)
__global__ __launch_bounds__(256) void flat_uniques(SolArgs a, const int32_t* umk) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  for (int64_t j = g; j < a.n_uniques; j += st) {
    const int32_t s = a.ulist[j];
    const int32_t m = umk[j];
    const int64_t dst = a.offsets[m] + (j - a.uoff[m]);
    const double v = gather_unique(a, s);
    __builtin_nontemporal_store(s, &a.usid[dst]);
    __builtin_nontemporal_store(v, &a.weight[dst]);
    __builtin_nontemporal_store(v * 0.5, &a.nweight[dst]);
  }
}

__global__ __launch_bounds__(256) void flat_markets(SolArgs a) {
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x, st = (int64_t)gridDim.x * 256;
  for (int64_t m = g; m < a.n_markets; m += st) {
    const double x = (double)(a.offsets[m + 1] - a.offsets[m]);
    a.cons[m] = x; a.conf[m] = x; a.tw[m] = x;
    a.nu[m] = (int32_t)x; a.err[m] = -1;
  }
}

template <int NT, int WPE>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void market_probe(SolArgs a) {
  __shared__ double red[NT / 64];
  const int t = threadIdx.x;
  for (int64_t li = blockIdx.x; li < a.n_markets; li += gridDim.x) {
    const int32_t m = a.order[li];
    const int64_t o0 = a.offsets[m], n = a.offsets[m + 1] - o0;
    const int64_t u0 = a.uoff[m], u = a.uoff[m + 1] - u0;
    double acc = 0.0;
    for (int64_t i = t; i < n; i += NT) acc += (double)a.sid[o0 + i] + a.prob[o0 + i];
    for (int64_t j = t; j < u; j += NT) {
      const int32_t s = a.ulist[u0 + j];
      const double v = gather_unique(a, s);
      acc += v;
      __builtin_nontemporal_store(s, &a.usid[o0 + j]);
      __builtin_nontemporal_store(v, &a.weight[o0 + j]);
      __builtin_nontemporal_store(v * 0.5, &a.nweight[o0 + j]);
    }
    // a workgroup reduction, as the real kernel's totals
#pragma unroll
    for (int k = 32; k >= 1; k >>= 1) acc += __shfl_xor(acc, k);
    if ((t & 63) == 0) red[t >> 6] = acc;
    __syncthreads();
    if (t == 0) {
      double s = 0.0;
      for (int w = 0; w < NT / 64; ++w) s += red[w];
      a.cons[m] = s; a.conf[m] = s; a.tw[m] = s;
      a.nu[m] = (int32_t)u; a.err[m] = -1;
    }
    __syncthreads();
  }
}

template <int NT, int WPE>
void launch_market(const SolArgs& a, int per_cu, hipStream_t st) {
  int dev = 0, cus = 256;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  hipLaunchKernelGGL((market_probe<NT, WPE>), dim3(cus * per_cu), dim3(NT), 0, st, a);
}

}  // namespace

extern "C" int sol_c3_run(const SolArgs* a, const int32_t* umk, int variant, int n_signals_lo, int n_signals_hi,
                          void* stream) {
  hipStream_t st = reinterpret_cast<hipStream_t>(stream);
  const int64_t n = ((int64_t)n_signals_hi << 32) | (uint32_t)n_signals_lo;
  switch (variant) {
    case 0:  // flat: signals, uniques, markets
      hipLaunchKernelGGL(flat_signals, dim3(256 * 16), dim3(256), 0, st, *a, n);
      hipLaunchKernelGGL(flat_uniques, dim3(256 * 16), dim3(256), 0, st, *a, umk);
      hipLaunchKernelGGL(flat_markets, dim3(256 * 4), dim3(256), 0, st, *a);
      break;
    case 1: launch_market<512, 4>(*a, 2, st); break;   // the <8,8> wide kernel's shape: 2 x 8 waves per CU
    case 2: launch_market<256, 4>(*a, 4, st); break;   // 4 x 4 waves per CU
    case 3: launch_market<256, 8>(*a, 8, st); break;   // 8 waves per SIMD
    case 4: launch_market<64, 8>(*a, 32, st); break;   // one wave per market, 8 per SIMD
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
