// elementwise.hip -- fused elementwise kernels over the dense source table.
//
//   decay_view     get_reliability(apply_decay=True)  (reliability.py:110-131,
//                  decay.py:61-145): view = max(m, min(1, m + (r-m)*2^(-days/h)))
//   outcome_update compute_update / update_reliability (reliability.py:142-183)
//   replay_step    config 4: both in one pass (view at `now`, then the update)
//
// HBM-bound: each thread owns two consecutive sources so every table stream is read
// and written with 16-byte accesses.  FP contraction off (CPython rounding).
#include "bce_device.hpp"
#include "bce_internal.hpp"
#include "glibc_pow.hpp"

#pragma clang fp contract(off)

namespace bce {

struct DecayConst {
  int64_t now_us;
  double half_life;
  double min_rel;
  double default_rel;
  double default_conf;
};

// decay.py:52-58 and 90-100, with days from decay.py:140-145.
__device__ __forceinline__ double decayed(double r, int64_t t_us, const DecayConst& k,
                                          const unsigned long long* tab = kExpTab) {
  if (t_us == BCE_NO_TIMESTAMP) return r;
  const double secs = (double)(k.now_us - t_us) / 1e6;  // timedelta.total_seconds()
  const double days = py_max(0.0, secs / 86400.0);
  if (!(days > 0.0)) return r;
  const double f = bce_pow::pow_base2(-days / k.half_life, tab);  // 2.0 ** x as libm pow (glibc_pow.hpp)
  const double d = k.min_rel + (r - k.min_rel) * f;
  return py_max(k.min_rel, py_min(1.0, d));
}

// reliability.py:163-173 for one participant.
__device__ __forceinline__ void update_one(double& r, double& c, bool correct) {
  const double direction = correct ? 1.0 : -1.0;
  const double raw = 0.15 * direction;                      // _BASE_LEARNING_RATE
  const double capped = py_max(-0.10, py_min(0.10, raw));   // MAX_UPDATE_STEP
  r = py_max(0.0, py_min(1.0, r + capped));
  c = py_min(1.0, c + (1.0 - c) * 0.10);
}

__global__ __launch_bounds__(256) void decay_view_kernel(int64_t n, const double* __restrict__ rel,
                                                         const int64_t* __restrict__ t_us,
                                                         const uint8_t* __restrict__ present,
                                                         DecayConst k, double* __restrict__ view) {
  __shared__ unsigned long long sExp[256];  // the exp table in LDS (see replay_step_kernel)
  sExp[threadIdx.x] = kExpTab[threadIdx.x];
  __syncthreads();
  const int64_t npair = n >> 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npair;
       i += (int64_t)gridDim.x * blockDim.x) {
    const double2 r = reinterpret_cast<const double2*>(rel)[i];
    const longlong2 t = reinterpret_cast<const longlong2*>(t_us)[i];
    double v0 = decayed(r.x, t.x, k, sExp), v1 = decayed(r.y, t.y, k, sExp);
    if (present) {
      const uchar2 p = reinterpret_cast<const uchar2*>(present)[i];
      if (!p.x) v0 = k.default_rel;
      if (!p.y) v1 = k.default_rel;
    }
    reinterpret_cast<double2*>(view)[i] = make_double2(v0, v1);
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t s = n - 1;
    double v = decayed(rel[s], t_us[s], k, sExp);
    if (present && !present[s]) v = k.default_rel;
    view[s] = v;
  }
}

// decay.compute_decay_factor / apply_reliability_decay on elapsed-day arrays
// (decay.py:52-58, 90-100).
__global__ __launch_bounds__(256) void decay_apply_kernel(int64_t n, const double* __restrict__ rel,
                                                          const double* __restrict__ days, double h,
                                                          double mn, double* __restrict__ out,
                                                          double* __restrict__ factor) {
  __shared__ unsigned long long sExp[256];  // the exp table in LDS (see replay_step_kernel)
  sExp[threadIdx.x] = kExpTab[threadIdx.x];
  __syncthreads();
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const double e = days[s];
    const double f = (e <= 0) ? 1.0 : bce_pow::pow_base2(-e / h, sExp);  // 2.0 ** x as libm pow
    if (factor) factor[s] = f;
    if (out) {
      const double r = rel[s];
      if (e <= 0) {
        out[s] = r;
      } else {
        const double d = mn + (r - mn) * f;
        out[s] = py_max(mn, py_min(1.0, d));
      }
    }
  }
}

__global__ __launch_bounds__(256) void outcome_update_kernel(int64_t n, double* rel, double* conf,
                                                             int64_t* t_us, uint8_t* present,
                                                             const uint8_t* __restrict__ flags,
                                                             DecayConst k) {
  for (int64_t s = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; s < n;
       s += (int64_t)gridDim.x * blockDim.x) {
    const uint8_t f = flags[s];
    if (!(f & 1)) continue;
    const bool pres = present ? present[s] != 0 : true;
    double r = pres ? rel[s] : k.default_rel;   // reliability.py:133-140 cold start
    double c = pres ? conf[s] : k.default_conf;
    update_one(r, c, (f & 2) != 0);
    rel[s] = r;
    conf[s] = c;
    t_us[s] = k.now_us;  // reliability.py:175
    if (present) present[s] = 1;
  }
}

// Nontemporal rel / t loads (C4 0.085 -> 0.080 ms); nt view stores and an nt conf load
// measured slower (measurements/c3_c4_nt_variants_r02.jsonl).
typedef double ew_d2v __attribute__((ext_vector_type(2)));
typedef long long ew_l2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 ew_ld(const double2* p) {
  const ew_d2v v = __builtin_nontemporal_load(reinterpret_cast<const ew_d2v*>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ longlong2 ew_ld(const longlong2* p) {
  const ew_l2v v = __builtin_nontemporal_load(reinterpret_cast<const ew_l2v*>(p));
  return make_longlong2(v.x, v.y);
}
__device__ __forceinline__ void ew_st_view(double2* p, double x0, double x1) { *p = make_double2(x0, x1); }

// Grids are one thread per work item (C4 -4%, f3 -5.5% against 16 workgroups per CU).

// Config-4 step.  Absent rows must carry the baked cold-start values
// (rel = default_rel, conf = default_conf, t = BCE_NO_TIMESTAMP), so the view needs no
// `present` read; `present` is only written (rows that now exist).
__global__ __launch_bounds__(256) void replay_step_kernel(int64_t n, double* __restrict__ rel,
                                                          double* __restrict__ conf,
                                                          int64_t* __restrict__ t_us,
                                                          uint8_t* __restrict__ present,
                                                          const uint8_t* __restrict__ flags2,
                                                          DecayConst k, double* __restrict__ view) {
  // the exp table (2 KB) staged in LDS: one ds_read per decay factor instead of a per-lane
  // gather from the constant table beside the streaming loads (C4 0.0827 -> 0.0741 ms,
  // profiles/r03ah/)
  __shared__ unsigned long long sExp[256];
  sExp[threadIdx.x] = kExpTab[threadIdx.x];
  __syncthreads();
  const int64_t npair = n >> 1;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < npair;
       i += (int64_t)gridDim.x * blockDim.x) {
    double2 r = ew_ld(reinterpret_cast<const double2*>(rel) + i);
    longlong2 t = ew_ld(reinterpret_cast<const longlong2*>(t_us) + i);
    const uint8_t fb = flags2[i >> 1];
    const unsigned f = (fb >> ((i & 1) * 4)) & 0xF;  // 2 bits per source, sources 2i, 2i+1
    ew_st_view(reinterpret_cast<double2*>(view) + i, decayed(r.x, t.x, k, sExp), decayed(r.y, t.y, k, sExp));
    if (f & 0x5) {  // any participant in the pair
      double2 c = reinterpret_cast<const double2*>(conf)[i];
      if (f & 1) {
        update_one(r.x, c.x, (f & 2) != 0);
        t.x = k.now_us;
        present[2 * i] = 1;
      }
      if (f & 4) {
        update_one(r.y, c.y, (f & 8) != 0);
        t.y = k.now_us;
        present[2 * i + 1] = 1;
      }
      reinterpret_cast<double2*>(rel)[i] = r;
      reinterpret_cast<double2*>(conf)[i] = c;
      reinterpret_cast<longlong2*>(t_us)[i] = t;
    }
  }
  if ((n & 1) && blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t s = n - 1;
    const unsigned f = (flags2[s >> 2] >> (2 * (s & 3))) & 3;
    double r = rel[s];
    view[s] = decayed(r, t_us[s], k, sExp);
    if (f & 1) {
      double c = conf[s];
      update_one(r, c, (f & 2) != 0);
      rel[s] = r;
      conf[s] = c;
      t_us[s] = k.now_us;
      present[s] = 1;
    }
  }
}

// NamespacedReliabilityStore.get_reliability for every source at once
// (reliability_abstraction.py:119-188): the first scope (market, domain, global) whose row
// has a truthy updated_at supplies the record -- decayed as
// SQLiteReliabilityStore.get_reliability does (reliability.py:110-131) -- else the
// cold-start defaults (:177-186).  One pass writes the packed consensus table directly.
struct NsScope {
  const double* rel;
  const double* conf;
  const int64_t* t_us;
  const uint8_t* has;
};
struct NsArgs {
  NsScope sc[3];
  int n_scopes;  // leading non-NULL scopes after compaction (host)
  uint8_t scope_code[3];
  int apply_decay;
  int mark_cold;
  DecayConst k;
  double2* relconf;
  uint32_t* bits;
  uint8_t* scope;
};

// nontemporal hints on the namespace pass (every byte is read / written once): both on 0.1665
// ms, off 0.1752 (10M sources x 3 scopes, profiles/archive/r04t/)
constexpr bool kNsNtLoad = true;
constexpr int kNsGridCap = 8192;  // workgroups of namespace_resolve_kernel (32 per CU)
constexpr bool kNsNtStore = true;
template <typename T>
__device__ __forceinline__ T ns_ld(const T* p) {
  if constexpr (kNsNtLoad) return __builtin_nontemporal_load(p);
  else return *p;
}

__global__ __launch_bounds__(256) void namespace_resolve_kernel(int64_t n, NsArgs a) {
  __shared__ unsigned long long sExp[256];  // the exp table in LDS (see replay_step_kernel)
  sExp[threadIdx.x] = kExpTab[threadIdx.x];
  __syncthreads();
  // whole waves walk 64 consecutive sources so the present bits come from one ballot
  for (int64_t base = (int64_t)blockIdx.x * 256; base < n; base += (int64_t)gridDim.x * 256) {
    const int64_t s = base + threadIdx.x;
    const bool in = s < n;
    double r = a.k.default_rel, c = a.k.default_conf;
    int code = 3;  // cold start
    if (in) {
      // the `has` bytes of every scope are independent loads: issue them together
      uint8_t h[3] = {0, 0, 0};
#pragma unroll
      for (int q = 0; q < 3; ++q)
        if (q < a.n_scopes) h[q] = ns_ld(a.sc[q].has + s);
      int pick = -1;
#pragma unroll
      for (int q = 2; q >= 0; --q)
        if (q < a.n_scopes && h[q]) pick = q;
      if (pick >= 0) {
        const NsScope& sc = a.sc[pick];
        r = ns_ld(sc.rel + s);
        c = ns_ld(sc.conf + s);
        if (a.apply_decay) r = decayed(r, ns_ld(sc.t_us + s), a.k, sExp);
        code = a.scope_code[pick];
      }
      if constexpr (kNsNtStore) {
        typedef double d2v __attribute__((ext_vector_type(2)));
        d2v v;
        v.x = r;
        v.y = c;
        if (a.relconf) __builtin_nontemporal_store(v, reinterpret_cast<d2v*>(a.relconf + s));
        if (a.scope) __builtin_nontemporal_store((uint8_t)code, a.scope + s);
      } else {
        if (a.relconf) a.relconf[s] = make_double2(r, c);
        if (a.scope) a.scope[s] = (uint8_t)code;
      }
    }
    if (a.bits) {
      const unsigned long long m = __ballot(in && (!a.mark_cold || code != 3));
      const int ln = (int)(threadIdx.x & 63);
      const int64_t w0 = (base + (threadIdx.x & ~63)) >> 5;
      const int64_t nw = (n + 31) >> 5;
      if (ln < 2 && w0 + ln < nw) a.bits[w0 + ln] = (uint32_t)(m >> (32 * ln));
    }
  }
}

static int grid_for(int64_t work, int threads) {
  int64_t g = (work + threads - 1) / threads;
  // one thread per work item (the grid-stride loops run once)
  const int64_t cap = (int64_t)1 << 30;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

}  // namespace bce

using namespace bce;

extern "C" int bce_decay_view(int64_t n, const double* rel, const int64_t* t_us,
                              const uint8_t* present, int64_t now_us, double half_life_days,
                              double min_rel, double default_rel, double* view, void* stream) {
  BCE_REQUIRE(n >= 0, "decay_view: n < 0");
  if (n == 0) return BCE_OK;
  BCE_REQUIRE(rel && t_us && view, "decay_view: NULL array");
  BCE_REQUIRE(((uintptr_t)rel | (uintptr_t)t_us | (uintptr_t)view) % 16 == 0,
              "decay_view: arrays must be 16-byte aligned");
  BCE_REQUIRE(present == nullptr || (uintptr_t)present % 2 == 0, "decay_view: present alignment");
  DecayConst k{now_us, half_life_days, min_rel, default_rel, 0.25};
  hipLaunchKernelGGL(decay_view_kernel, dim3(grid_for(n / 2 + 1, 256)), dim3(256), 0,
                     as_stream(stream), n, rel, t_us, present, k, view);
  return check_launch("decay_view_kernel");
}

extern "C" int bce_decay_apply(int64_t n, const double* rel, const double* elapsed_days,
                               double half_life_days, double min_rel, double* out, double* factor,
                               void* stream) {
  BCE_REQUIRE(n >= 0, "decay_apply: n < 0");
  if (n == 0) return BCE_OK;
  BCE_REQUIRE(elapsed_days && (out == nullptr || rel) && (out || factor), "decay_apply: NULL array");
  hipLaunchKernelGGL(decay_apply_kernel, dim3(grid_for(n, 256)), dim3(256), 0, as_stream(stream), n,
                     rel, elapsed_days, half_life_days, min_rel, out, factor);
  return check_launch("decay_apply_kernel");
}

extern "C" int bce_outcome_update(int64_t n, double* rel, double* conf, int64_t* t_us,
                                  uint8_t* present, const uint8_t* flags, int64_t now_us,
                                  double default_rel, double default_conf, void* stream) {
  BCE_REQUIRE(n >= 0, "outcome_update: n < 0");
  if (n == 0) return BCE_OK;
  BCE_REQUIRE(rel && conf && t_us && flags, "outcome_update: NULL array");
  DecayConst k{now_us, 30.0, 0.1, default_rel, default_conf};
  hipLaunchKernelGGL(outcome_update_kernel, dim3(grid_for(n, 256)), dim3(256), 0,
                     as_stream(stream), n, rel, conf, t_us, present, flags, k);
  return check_launch("outcome_update_kernel");
}

extern "C" int bce_replay_step(int64_t n, double* rel, double* conf, int64_t* t_us,
                               uint8_t* present, const uint8_t* flags2, int64_t now_us,
                               double half_life_days, double min_rel, double default_rel,
                               double default_conf, double* view, void* stream) {
  BCE_REQUIRE(n >= 0, "replay_step: n < 0");
  if (n == 0) return BCE_OK;
  BCE_REQUIRE(rel && conf && t_us && present && flags2 && view, "replay_step: NULL array");
  BCE_REQUIRE(((uintptr_t)rel | (uintptr_t)conf | (uintptr_t)t_us | (uintptr_t)view) % 16 == 0,
              "replay_step: arrays must be 16-byte aligned");
  DecayConst k{now_us, half_life_days, min_rel, default_rel, default_conf};
  hipLaunchKernelGGL(replay_step_kernel, dim3(grid_for(n / 2 + 1, 256)), dim3(256), 0,
                     as_stream(stream), n, rel, conf, t_us, present, flags2, k, view);
  return check_launch("replay_step_kernel");
}

extern "C" int bce_namespace_resolve(int64_t n, const double* rel0, const double* conf0,
                                     const int64_t* t0, const uint8_t* has0, const double* rel1,
                                     const double* conf1, const int64_t* t1, const uint8_t* has1,
                                     const double* rel2, const double* conf2, const int64_t* t2,
                                     const uint8_t* has2, int apply_decay, int64_t now_us,
                                     double half_life_days, double min_rel, double default_rel,
                                     double default_conf, int mark_cold, double* relconf,
                                     uint32_t* present_bits, uint8_t* scope, void* stream) {
  BCE_REQUIRE(n >= 0, "namespace_resolve: n < 0");
  if (n == 0) return BCE_OK;
  BCE_REQUIRE(relconf || present_bits || scope, "namespace_resolve: no output");
  BCE_REQUIRE(relconf == nullptr || (uintptr_t)relconf % 16 == 0,
              "namespace_resolve: relconf must be 16-byte aligned");
  NsArgs a{};
  const NsScope in[3] = {{rel0, conf0, t0, has0}, {rel1, conf1, t1, has1}, {rel2, conf2, t2, has2}};
  for (int q = 0; q < 3; ++q) {
    if (in[q].rel == nullptr) continue;  // scope not requested (falsy market_id / domain)
    BCE_REQUIRE(in[q].conf && in[q].has && (in[q].t_us || !apply_decay),
                "namespace_resolve: scope %d: NULL array", q);
    a.scope_code[a.n_scopes] = (uint8_t)q;
    a.sc[a.n_scopes++] = in[q];
  }
  a.apply_decay = apply_decay;
  a.mark_cold = mark_cold;
  a.k = DecayConst{now_us, half_life_days, min_rel, default_rel, default_conf};
  a.relconf = reinterpret_cast<double2*>(relconf);
  a.bits = present_bits;
  a.scope = scope;
  // a capped grid striding over the sources (the LDS exp table staged once per workgroup, not
  // once per 256 sources): 0.1605-0.1610 vs 0.1662-0.1673 ms at 10M sources x 3 scopes, three
  // interleaved reps (profiles/r06ew/, r06ns/; the C4 replay step measured slower capped: one thread
  // per source stays there)
  const int g = grid_for(n, 256);
  hipLaunchKernelGGL(namespace_resolve_kernel, dim3(g < kNsGridCap ? g : kNsGridCap), dim3(256), 0,
                     as_stream(stream), n, a);
  return check_launch("namespace_resolve_kernel");
}
