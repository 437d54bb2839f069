// capi.hip -- library-level C ABI: version, errors, device queries.
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include <atomic>
#include <map>
#include <mutex>
#include <set>
#include <tuple>

#include "bce_internal.hpp"
#include "consensus_common.hpp"

namespace bce {

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    set_error("%s launch failed: %s", what, hipGetErrorString(e));
    return BCE_EHIP;
  }
  return BCE_OK;
}

// ---- per-device context -------------------------------------------------------------
// Everything the launchers cache is keyed by the calling thread's current device and
// initialised under a once-flag / mutex: one process may drive several GPUs from several
// host threads (ctypes releases the GIL), and lazily created device objects must not race.
namespace {
constexpr int kMaxDev = 64;

struct DevCtx {
  std::once_flag once;
  int cus = 256;
  int* fault = nullptr;
  hipError_t init_err = hipSuccess;
  std::mutex side_mu;  // held from the plan's fork to its join (bce_consensus_planned)
  hipStream_t side[kSideStreams] = {};  // side[0]: the short-market bins' stream
  hipEvent_t ev_fork = nullptr, ev_join[kSideStreams] = {};
  int* split = nullptr;               // kQueueSlots blocks of kSplitWords tie-break ticket words
  std::atomic<unsigned> split_next{0};
  std::atomic<int> split_last[64] = {};  // per slot: the ticket of the last pair that took it
};
constexpr int kQueueSlots = 64;
DevCtx g_dev[kMaxDev];

DevCtx* dev_ctx() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= kMaxDev) return nullptr;
  DevCtx* c = &g_dev[dev];
  std::call_once(c->once, [c, dev] {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0) c->cus = n;
    int* p = nullptr;
    hipError_t e = hipMalloc((void**)&p, sizeof(int));
    if (e == hipSuccess) e = hipMemset(p, 0, sizeof(int));  // synchronous: done before first use
    // the fork / join events only order the side streams against the caller's stream on this
    // device: no system-scope fence (each shard step 1.3% shorter, profiles/r06y/)
    const unsigned evf = hipEventDisableTiming | hipEventDisableSystemFence;
    for (int k = 0; k < kSideStreams; ++k) {
      if (e == hipSuccess) e = hipStreamCreateWithFlags(&c->side[k], hipStreamNonBlocking);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_join[k], evf);
    }
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->ev_fork, evf);
    int* sw = nullptr;
    if (e == hipSuccess) e = hipMalloc((void**)&sw, (size_t)kQueueSlots * kSplitWords * sizeof(int));
    if (e == hipSuccess) e = hipMemset(sw, 0, (size_t)kQueueSlots * kSplitWords * sizeof(int));
    if (e == hipSuccess) c->split = sw;
    c->init_err = e;
    if (e == hipSuccess) c->fault = p;
  });
  return c;
}

struct OccKey {
  int dev;
  const void* fn;
  int threads;
  size_t lds;
  bool operator<(const OccKey& o) const {
    return std::tie(dev, fn, threads, lds) < std::tie(o.dev, o.fn, o.threads, o.lds);
  }
};
std::mutex g_occ_mu;
std::map<OccKey, int> g_occ;
std::set<std::pair<int, const void*>> g_attr;
}  // namespace

int cu_count() {
  DevCtx* c = dev_ctx();
  return c ? c->cus : 256;
}

int* split_slot(int ticket, hipStream_t st) {
  DevCtx* c = dev_ctx();
  if (!c || !c->split) return nullptr;
  static_assert(kQueueSlots == 64, "split_last size");
  // tickets make reuse safe, on any stream: PART 1 raises a word to its ticket (atomicMax) and
  // PART 2 runs whenever the word holds its own or a newer pair's ticket (tiebreak.hip)
  const unsigned k = c->split_next.fetch_add(1) % kQueueSlots;
  int* w = c->split + (size_t)k * kSplitWords;
  // After the 30-bit ticket counter wraps, the slot's words still hold the old, larger tickets
  // and would make every later PART 2 launch run all its waves: clear the slot on
  // this stream, ahead of this pair's PART 1, once per wrap.
  if (ticket < c->split_last[k].exchange(ticket) && hipMemsetAsync(w, 0, kSplitWords * sizeof(int), st) != hipSuccess)
    return nullptr;
  return w;
}

int* fault_word() {
  DevCtx* c = dev_ctx();
  return c ? c->fault : nullptr;
}

int blocks_per_cu(const void* fn, int threads, size_t lds, int fallback, const char* name) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return fallback;
  std::lock_guard<std::mutex> lk(g_occ_mu);
  const OccKey k{dev, fn, threads, lds};
  auto it = g_occ.find(k);
  if (it != g_occ.end()) return it->second;
  int nb = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, fn, threads, lds) != hipSuccess || nb <= 0) nb = fallback;
  g_occ[k] = nb;
  if (name && getenv("BCE_DEBUG_LAUNCH"))
    fprintf(stderr, "[bce] %s: %d blocks/CU x %d CUs (dev %d, %zu B dynamic LDS)\n", name, nb, cu_count(), dev, lds);
  return nb;
}

int ensure_dynamic_lds(const void* fn, int bytes) {
  int dev = 0;
  BCE_HIP(hipGetDevice(&dev));
  std::lock_guard<std::mutex> lk(g_occ_mu);
  if (g_attr.count({dev, fn})) return BCE_OK;
  BCE_HIP(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, bytes));
  g_attr.insert({dev, fn});
  return BCE_OK;
}

int side_fork(hipStream_t st, int k, hipStream_t* sides, std::unique_lock<std::mutex>* lock) {
  DevCtx* c = dev_ctx();
  if (k == 0) return BCE_OK;
  if (!c || !c->side[0] || k < 0 || k > kSideStreams) {
    set_error("side stream unavailable: %s", c ? hipGetErrorString(c->init_err) : "no device");
    return BCE_EHIP;
  }
  *lock = std::unique_lock<std::mutex>(c->side_mu);
  BCE_HIP(hipEventRecord(c->ev_fork, st));
  for (int i = 0; i < k; ++i) {
    BCE_HIP(hipStreamWaitEvent(c->side[i], c->ev_fork, 0));
    sides[i] = c->side[i];
  }
  return BCE_OK;
}

int side_join(hipStream_t st, int k) {
  DevCtx* c = dev_ctx();
  for (int i = 0; i < k; ++i) {
    BCE_HIP(hipEventRecord(c->ev_join[i], c->side[i]));
    BCE_HIP(hipStreamWaitEvent(st, c->ev_join[i], 0));
  }
  return BCE_OK;
}

static int g_spin_cap = 1 << 22;
int spin_cap() { return g_spin_cap; }

static const char* fault_text(int code) {
  switch (code) {
    case kFaultSpinLoader: return "consensus_pipe_kernel: loader wave timed out waiting for a free slot";
    case kFaultSpinCompute: return "consensus_pipe_kernel: compute wave timed out waiting for its tile";
    case kFaultSid: return "consensus: a sid is >= n_sources (its row read was clamped)";
    case kFaultTooLong: return "consensus: a market is longer than the launch's max_len (left unprocessed)";
    case kFaultSpinChain: return "consensus_wide_kernel: exact-mode chain hand-off timed out";
    case 6: return "tiebreak round(): rounded value too large to represent";
    case kFaultOffsets: return "plan_bins: offsets not monotone (device planner; nothing was computed)";
    default: return "unknown device fault";
  }
}

}  // namespace bce

extern "C" int bce_fault_check(void* stream) {
  int* w = bce::fault_word();
  if (!w) {
    bce::set_error("bce_fault_check: no fault word on this device");
    return BCE_EHIP;
  }
  hipStream_t st = bce::as_stream(stream);
  int h = 0;
  BCE_HIP(hipMemcpyAsync(&h, w, sizeof h, hipMemcpyDeviceToHost, st));
  BCE_HIP(hipStreamSynchronize(st));
  if (h == 0) return BCE_OK;
  BCE_HIP(hipMemsetAsync(w, 0, sizeof(int), st));
  BCE_HIP(hipStreamSynchronize(st));
  bce::set_error("device fault %d: %s", h, bce::fault_text(h));
  return BCE_EHIP;
}

extern "C" int bce_debug_set_spin_cap(int cap) {
  bce::g_spin_cap = (cap > 0) ? cap : (1 << 22);
  return BCE_OK;
}

extern "C" int bce_abi_version(void) { return BCE_ABI_VERSION; }
extern "C" int bce_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}
