// mh_api.hip — the C ABI (include/mitty_hip.h): context, buffers, argument checks, dispatch to the subsystems.
#include <sys/mman.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cctype>
#include <cstdio>
#include <unordered_map>
#include <chrono>
#include <cmath>
#include <condition_variable>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>

#include "mh_bgzf.h"
#include <vector>

#include "mh_corrupt.h"
#include "mh_internal.h"
#include "mh_scan.h"
#include "mh_sort.h"

namespace mh {
namespace jump {
void window_at(uint32_t seed, uint64_t J, uint32_t *out624);
}

static std::mutex g_err_mu;   // the splice's second lane (a host thread) may report an error beside the first

int32_t hip_fail(mh_ctx *ctx, hipError_t e, const char *what, const char *file, int line) {
  if (ctx) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    ctx->err = std::string("HIP error ") + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ") in " + what + " at " +
               file + ":" + std::to_string(line);
  }
  return e == hipErrorOutOfMemory ? MH_E_OOM : MH_E_HIP;
}

int32_t arg_fail(mh_ctx *ctx, int32_t code, const std::string &msg) {
  if (ctx) {
    std::lock_guard<std::mutex> lk(g_err_mu);
    ctx->err = msg;
  }
  return code;
}

bool scan_fault_pending(const mh_ctx *ctx) {
  const uint32_t *h = scan_fault_host();
  return h && __atomic_load_n(h + (ctx ? ctx->fault_slot : 0), __ATOMIC_ACQUIRE) != 0;
}

// a library thread working for ctx (the splice's second lane): its look-back scans report to ctx's fault word, which
// its synchronisations (SYNCCHK) check — the entry-point guard sets this only for the calling thread
void lane_thread_enter(mh_ctx *ctx) { scan_fault_slot = ctx->fault_slot; }

int32_t scan_fault_fail(mh_ctx *ctx) {
  const uint32_t v = scan_fault_take(ctx ? ctx->fault_slot : 0);
  // bits 2 and 4: the single-pass FASTQ writer (k_emit_fused) found a read's qname part past the splice's bound, or
  // a tile past the arena it was given; it stored nothing wrong there, but the unit's output is incomplete
  if (v & 2u) return arg_fail(ctx, MH_E_STATE, "single-pass writer: a qname part exceeded the splice's bound (internal)");
  if (v & 4u) return arg_fail(ctx, MH_E_STATE, "single-pass writer: the arena reservation was too small (internal)");
  return arg_fail(ctx, MH_E_STATE, "a look-back scan's wait timed out (a broken ticket base or scratch): its offsets "
                                   "are wrong");
}

// Device memory cache, process-wide and per device: the blocks the library frees are kept and handed to later
// requests (best fit), so a context created after an earlier one closed — a generate-reads command after a whole-
// genome job in one process — reuses blocks allocated while device memory was unfragmented.  Measured (round 4,
// scripts/e2e_fresh.py): the chr1 arenas allocated after 200 GB had been allocated and freed were copied out at
// 28 GB/s against 55 GB/s in a fresh process.  A block is cached only after the device is idle (hipFree's own
// synchronisation); an allocation that fails empties the cache and tries again; mh_device_cache_trim frees it.
namespace {
struct CachedBlock {
  void *p;
  int dev;
};
std::mutex g_cache_mu;
std::multimap<size_t, CachedBlock> g_cache;   // by capacity
// bytes of the library's device blocks in use (handed out, not in the cache), and their peak (mh_device_live_bytes)
std::atomic<int64_t> g_live{0}, g_live_peak{0};

void live_add(int64_t d) {
  const int64_t v = g_live.fetch_add(d) + d;
  int64_t pk = g_live_peak.load();
  while (v > pk && !g_live_peak.compare_exchange_weak(pk, v)) {
  }
}

void cache_put(void *p, size_t cap) {
  live_add(-(int64_t)cap);
  int dev = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceSynchronize();   // (what hipFree does: no kernel still reads or writes the block)
  std::lock_guard<std::mutex> lk(g_cache_mu);
  g_cache.insert({cap, CachedBlock{p, dev}});
}

// a cached block of this device with capacity >= bytes (the smallest), or nullptr
void *cache_take(size_t bytes, size_t *cap) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(g_cache_mu);
  for (auto it = g_cache.lower_bound(bytes); it != g_cache.end(); ++it)
    if (it->second.dev == dev) {
      void *p = it->second.p;
      *cap = it->first;
      g_cache.erase(it);
      return p;
    }
  return nullptr;
}

int64_t cache_trim(int dev) {   // dev < 0: every device's blocks
  std::vector<std::pair<void *, int>> out;
  int64_t freed = 0;
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    for (auto it = g_cache.begin(); it != g_cache.end();)
      if (dev < 0 || it->second.dev == dev) {
        out.push_back({it->second.p, it->second.dev});
        freed += (int64_t)it->first;
        it = g_cache.erase(it);
      } else {
        ++it;
      }
  }
  int cur = 0;
  (void)hipGetDevice(&cur);
  for (auto &b : out) {
    if (b.second != cur) (void)hipSetDevice(b.second);
    (void)hipFree(b.first);
    if (b.second != cur) (void)hipSetDevice(cur);
  }
  return freed;
}

hipError_t dev_alloc(void **p, size_t bytes, size_t *cap) {
  if ((*p = cache_take(bytes, cap))) {
    live_add((int64_t)*cap);
    return hipSuccess;
  }
  hipError_t e = hipMalloc(p, bytes);
  if (e != hipSuccess) {   // the cache's blocks back to the device, then once more
    (void)hipGetLastError();
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (cache_trim(dev) > 0) e = hipMalloc(p, bytes);
  }
  if (e == hipSuccess) {
    *cap = bytes;
    live_add((int64_t)bytes);
  } else {
    *p = nullptr;
  }
  return e;
}
}  // namespace

int32_t ensure(mh_ctx *ctx, DevBuf &b, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (b.cap >= bytes) return MH_OK;
  if (b.p) {
    MH_TRY(sync_writers(ctx));   // a queued FASTQ writer (or corruption pass) may still read or write it
    SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
    lb_forget(b.p);
    cache_put(b.p, b.cap);
    b.p = nullptr;
    b.cap = 0;
  }
  size_t c = bytes + bytes / 8 + 256;
  hipError_t e = dev_alloc(&b.p, c, &c);
  if (e != hipSuccess) {
    b.p = nullptr;
    (void)hipGetLastError();
    return arg_fail(ctx, MH_E_OOM, "device allocation of " + std::to_string(c) + " bytes failed");
  }
  b.cap = c;
  return MH_OK;
}

int32_t ensure_keep(mh_ctx *ctx, DevBuf &b, size_t bytes, size_t keep, int32_t grow_shift) {
  if (b.cap >= bytes) return MH_OK;
  DevBuf nb;
  MH_TRY(ensure(ctx, nb, bytes + (bytes >> grow_shift)));
  MH_TRY(sync_writers(ctx));   // the old buffer's queued writers finish first
  if (b.p && keep) HIPCHK(ctx, hipMemcpyAsync(nb.p, b.p, keep, hipMemcpyDeviceToDevice, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  lb_forget(b.p);
  if (b.p) cache_put(b.p, b.cap);
  b = nb;
  return MH_OK;
}

void release(DevBuf &b) {
  lb_forget(b.p);
  if (b.p) cache_put(b.p, b.cap);
  b.p = nullptr;
  b.cap = 0;
}

void release_hap(Hap &h) {
  release(h.hap); release(h.rc); release(h.nd); release(h.bkt); release(h.keys); release(h.ps); release(h.pr);
  release(h.op); release(h.oplen); release(h.nrun_s); release(h.nrun_e);
  if (h.used) (void)hipEventDestroy(h.used);
  h.used = nullptr;
  h.used_set = false;
}

int32_t mark_used(mh_ctx *ctx, hipEvent_t &ev, bool &set) {
  if (!ev) HIPCHK(ctx, hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  HIPCHK(ctx, hipEventRecord(ev, ctx->wstream));
  set = true;
  return MH_OK;
}

int32_t wait_unused(mh_ctx *ctx, hipEvent_t ev, bool set, hipStream_t st) {
  if (set) HIPCHK(ctx, hipStreamWaitEvent(st ? st : ctx->stream, ev, 0));
  return MH_OK;
}

// the prefetch thread joined (its failure reported here) and the main stream after the prefetched splices
// (mh_prefetch_haplotypes_vset): before any use of a prefetched Hap
int32_t join_prefetch(mh_ctx *ctx) {
  if (ctx->pf_thread.joinable()) {
    ctx->pf_thread.join();
    if (ctx->pf_rc != MH_OK) {   // (its message is in ctx->err)
      const int32_t rc = ctx->pf_rc;
      ctx->pf_rc = MH_OK;
      ctx->prefetch_pending = false;
      for (auto &kv : ctx->haps) kv.second.prefetched = false;
      return rc;
    }
  }
  if (!ctx->prefetch_pending) return MH_OK;
  HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_prefetch, 0));
  for (auto &kv : ctx->haps) kv.second.prefetched = false;
  ctx->prefetch_pending = false;
  return MH_OK;
}

int32_t sync_writers(mh_ctx *ctx) {
  SYNCCHK(ctx, hipStreamSynchronize(ctx->wstream));
  return MH_OK;
}

// the NUMA node of device dev's PCI function (sysfs), -1 when unknown
int gpu_numa_node(int dev) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), dev) != hipSuccess) return -1;
  for (char *c = bus; *c; c++) *c = (char)tolower(*c);
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
  FILE *fp = fopen(path.c_str(), "r");
  if (!fp) return -1;
  int node = -1;
  if (fscanf(fp, "%d", &node) != 1) node = -1;
  fclose(fp);
  return node;
}
std::mutex &host_allocs_mu() {
  static std::mutex m;
  return m;
}
std::unordered_map<void *, size_t> &host_allocs() {
  static std::unordered_map<void *, size_t> m;
  return m;
}

int64_t *pinned_small(mh_ctx *ctx) {
  if (!ctx->h_small && hipHostMalloc((void **)&ctx->h_small, 4096, hipHostMallocDefault) != hipSuccess)
    ctx->h_small = nullptr;
  return ctx->h_small;
}

int32_t join_writer(mh_ctx *ctx) {
  if (!ctx->writer_pending) return MH_OK;
  HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_writer, 0));
  ctx->writer_pending = false;
  return MH_OK;
}

void stage_begin(mh_ctx *ctx, const char *name) {
  if (!ctx->timing) return;
  StageTime s{name, nullptr, nullptr};
  (void)hipEventCreate(&s.a);
  (void)hipEventCreate(&s.b);
  (void)hipEventRecord(s.a, ctx->stage_stream ? ctx->stage_stream : ctx->stream);
  ctx->stages.push_back(s);
}

void stage_end(mh_ctx *ctx) {
  if (!ctx->timing || ctx->stages.empty()) return;
  StageTime s = ctx->stages.back();
  ctx->stages.pop_back();
  (void)hipEventRecord(s.b, ctx->stage_stream ? ctx->stage_stream : ctx->stream);   // resolved by stages_collect
  ctx->pending.push_back(s);
}

void stages_collect(mh_ctx *ctx) {
  for (auto &s : ctx->pending) {
    (void)hipEventSynchronize(s.b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, s.a, s.b);
    ctx->last_times.emplace_back(s.name, (double)ms);
    (void)hipEventDestroy(s.a);
    (void)hipEventDestroy(s.b);
  }
  ctx->pending.clear();
}

}  // namespace mh

using namespace mh;

// the emission entry points: they run beside a batch's asynchronous tail (their template set was resolved by
// mh_use_templates; their scratch is not the tail's)
#define CTX_GUARD_EMIT(ctx)                                                \
  do {                                                                     \
    if (!(ctx)) return MH_E_ARG;                                           \
    scan_fault_slot = (ctx)->fault_slot;                                   \
    hipError_t _e = hipSetDevice((ctx)->device);                           \
    if (_e != hipSuccess) return hip_fail((ctx), _e, "hipSetDevice", __FILE__, __LINE__); \
  } while (0)
// every other entry point first resolves a pending asynchronous tail (it may share the batch scratch)
#define CTX_GUARD_NOJOIN(ctx)                                              \
  do {                                                                     \
    CTX_GUARD_EMIT(ctx);                                                   \
    MH_TRY(tpl_resolve_all(ctx));                                          \
    MH_TRY(join_prefetch(ctx));                                            \
  } while (0)
// every entry point but the emission ones: the main stream first waits for the last queued FASTQ writer
#define CTX_GUARD(ctx)                                                     \
  do {                                                                     \
    CTX_GUARD_NOJOIN(ctx);                                                 \
    MH_TRY(join_writer(ctx));                                              \
  } while (0)

namespace mh {
CorruptCfg corrupt_cfg(const mh_ctx *ctx, uint64_t unit_key, int64_t t_base) {
  CorruptCfg cc{1, (const double *)ctx->corrupt_cum.p, (const double *)ctx->corrupt_phred.p, ctx->corrupt_max_bp,
                ctx->corrupt_n_bq, (uint32_t)ctx->corrupt_seed, (uint32_t)unit_key,
                (uint32_t)(ctx->corrupt_seed >> 32) ^ (uint32_t)(unit_key >> 32) ^ 0x636f7272u, t_base};
  const char *base = (const char *)ctx->corrupt_cum.p;
  cc.guide = (const uint16_t *)(base + ctx->corrupt_guide_off);
  cc.bk = (const uint8_t *)(base + ctx->corrupt_bk_off);
  cc.T16 = (const uint16_t *)(base + ctx->corrupt_T16_off);
  cc.Fp16 = (const uint16_t *)(base + ctx->corrupt_Fp16_off);
  cc.bkf = (const uint8_t *)(base + ctx->corrupt_bkf_off);
  return cc;
}
}  // namespace mh

extern "C" {

int32_t mh_version(void) { return 1; }

int32_t mh_device_count(int32_t *out) {
  int n = 0;
  hipError_t e = hipGetDeviceCount(&n);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  *out = n;
  return MH_OK;
}

int32_t mh_create(int32_t device, mh_ctx **out) {
  if (!out) return MH_E_ARG;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    (void)hipGetLastError();
    return MH_E_NO_DEVICE;
  }
  if (device < 0 || device >= n) return MH_E_ARG;
  mh_ctx *ctx = new mh_ctx();
  ctx->device = device;
  {   // its own scan-fault word (slots 1 .. SCAN_FAULT_SLOTS - 1, reused round-robin past that many contexts)
    static std::atomic<int> next{0};
    ctx->fault_slot = 1 + next++ % (SCAN_FAULT_SLOTS - 1);
    (void)scan_fault_take(ctx->fault_slot);
  }
  // the FASTQ writers (bandwidth-bound, long) yield to the main stream's latency-bound sampling kernels
  int prio_lo = 0, prio_hi = 0;
  (void)hipSetDevice(device);
  (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
  if (hipSetDevice(device) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->stream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->stream2, hipStreamNonBlocking, prio_hi) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_fork, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_join, hipEventDisableTiming) != hipSuccess ||
      hipStreamCreateWithPriority(&ctx->wstream, hipStreamNonBlocking, prio_lo) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_ready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&ctx->ev_writer, hipEventDisableTiming) != hipSuccess ||
      [&] {
        for (auto &e : ctx->eset)
          if (hipEventCreateWithFlags(&e.done, hipEventDisableTiming) != hipSuccess ||
              hipEventCreateWithFlags(&e.rb, hipEventDisableTiming) != hipSuccess ||
              hipHostMalloc((void **)&e.h_stat, 64 + 8192, hipHostMallocDefault) != hipSuccess)
            return true;
        return false;
      }()) {
    delete ctx;
    return MH_E_HIP;
  }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, device) == hipSuccess) ctx->max_cu = prop.multiProcessorCount;
  *out = ctx;
  return MH_OK;
}

int32_t mh_destroy(mh_ctx *ctx) {
  if (!ctx) return MH_OK;
  if (ctx->pf_thread.joinable()) ctx->pf_thread.join();
  (void)hipSetDevice(ctx->device);
  (void)hipStreamSynchronize(ctx->wstream);
  (void)hipStreamSynchronize(ctx->stream);
  if (ctx->stream2) (void)hipStreamSynchronize(ctx->stream2);
  if (ctx->pstream) (void)hipStreamSynchronize(ctx->pstream);
  for (auto x : ctx->xstream)
    if (x) (void)hipStreamSynchronize(x);
  for (auto &kv : ctx->contigs) release(kv.second.seq);
  for (auto &kv : ctx->haps) release_hap(kv.second);
  for (auto &h : ctx->hap_spare) release_hap(h);
  for (auto &kv : ctx->vsets) release_vars(kv.second);
  for (auto &kv : ctx->tsets) {
    release(kv.second.fo0); release(kv.second.pos0); release(kv.second.pos1); release(kv.second.n0);
    if (kv.second.used) (void)hipEventDestroy(kv.second.used);
  }
  release(ctx->jump_polys); release(ctx->perm_tmp); release(ctx->nrun_tmp); release(ctx->dec_buf);
  for (auto &b : ctx->pb) release(b);
  release(ctx->pb_tmp);
  release(ctx->gz_slots); release(ctx->gz_tok); release(ctx->gz_info); release(ctx->gz_off); release(ctx->gz_scan); release(ctx->gz_out);
  release(ctx->gz_in);
  for (auto &b : ctx->s) release(b);
  for (auto &b : ctx->lane2) release(b);
  for (auto &l : ctx->xlane)
    for (auto &b : l) release(b);
  for (auto &b : ctx->xscan) release(b);
  release(ctx->scan_partials); release(ctx->scan_partials2); release(ctx->d_small);
  release(ctx->corrupt_cum); release(ctx->corrupt_phred);
  release(ctx->out1); release(ctx->out2);
  release(ctx->cr_rows);
  release(ctx->cr_codes);
  release(ctx->scan_partials_w);
  for (auto &b : ctx->sl2) release(b);
  for (auto &b : ctx->sl3) release(b);
  ctx->tail_state.reset();
  for (hipEvent_t e : ctx->ev_gz)
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : ctx->ev_fetch)
    if (e) (void)hipEventDestroy(e);
  if (ctx->h_small) (void)hipHostFree(ctx->h_small);
  if (ctx->h_small3) (void)hipHostFree(ctx->h_small3);
  if (ctx->h_units) (void)hipHostFree(ctx->h_units);
  for (uint8_t *p : ctx->h_bam_pin)
    if (p) (void)hipHostFree(p);
  for (auto &e : ctx->eset) {
    release(e.recs); release(e.off); release(e.tsum); release(e.tpre); release(e.stat); release(e.crrec);
    (void)hipEventDestroy(e.done);
    if (e.rb) (void)hipEventDestroy(e.rb);
    if (e.h_stat) (void)hipHostFree(e.h_stat);
  }
  (void)hipEventDestroy(ctx->ev_ready);
  (void)hipEventDestroy(ctx->ev_writer);
  (void)hipStreamDestroy(ctx->wstream);
  bam_release(ctx->bam);
  if (ctx->ev_fork) (void)hipEventDestroy(ctx->ev_fork);
  if (ctx->ev_join) (void)hipEventDestroy(ctx->ev_join);
  if (ctx->stream2) (void)hipStreamDestroy(ctx->stream2);
  if (ctx->ev_prefetch) (void)hipEventDestroy(ctx->ev_prefetch);
  if (ctx->pstream) (void)hipStreamDestroy(ctx->pstream);
  for (int l = 0; l < 2; l++) {
    if (ctx->xstream[l]) (void)hipStreamDestroy(ctx->xstream[l]);
    if (ctx->ev_xjoin[l]) (void)hipEventDestroy(ctx->ev_xjoin[l]);
  }
  (void)hipStreamDestroy(ctx->stream);
  delete ctx;
  return MH_OK;
}

const char *mh_last_error(const mh_ctx *ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int32_t mh_sync(mh_ctx *ctx) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

namespace {
struct LoadOne {
  __device__ int64_t operator()(int64_t) const { return 1; }
};
struct StoreCheck {   // element i's exclusive prefix must be i
  int32_t *bad;
  __device__ void operator()(int64_t i, int64_t, int64_t ex) const {
    if (ex != i) atomicOr(bad, 1);
  }
};
}  // namespace

// A look-back scan whose tile 0 never runs (device_scan_sum's skip_tile0): every waiting tile times out, the fault
// word is set, and the synchronisation after it fails with MH_E_STATE — the expected result.  A correct scan after it
// then succeeds (the word was cleared).
int32_t mh_selftest_sort(mh_ctx *ctx, const uint32_t *keys, int64_t n, int32_t end_bit, uint32_t *keys_out,
                         uint32_t *vals_out) {
  CTX_GUARD(ctx);
  if (n < 0 || (n > 0 && (!keys || !keys_out || !vals_out)) || end_bit < 0 || end_bit > 32)
    return arg_fail(ctx, MH_E_ARG, "bad sort arguments");
  hipStream_t st = ctx->stream;
  size_t tmp = 0;
  HIPCHK(ctx, lsd_sort_pairs_iota(nullptr, tmp, nullptr, nullptr, nullptr, n, (unsigned)end_bit, st));
  DevBuf b;
  const size_t kb = (4 * (size_t)n + 255) & ~(size_t)255;
  MH_TRY(ensure(ctx, b, 3 * kb + tmp + 256));
  uint32_t *dk = (uint32_t *)b.p, *ko = (uint32_t *)((char *)b.p + kb), *vo = (uint32_t *)((char *)b.p + 2 * kb);
  const int32_t rc = [&]() -> int32_t {
    if (n) HIPCHK(ctx, hipMemcpyAsync(dk, keys, 4 * (size_t)n, hipMemcpyHostToDevice, st));
    HIPCHK(ctx, lsd_sort_pairs_iota((char *)b.p + 3 * kb, tmp, dk, ko, vo, n, (unsigned)end_bit, st));
    if (n) {
      HIPCHK(ctx, hipMemcpyAsync(keys_out, ko, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
      HIPCHK(ctx, hipMemcpyAsync(vals_out, vo, 4 * (size_t)n, hipMemcpyDeviceToHost, st));
    }
    SYNCCHK(ctx, hipStreamSynchronize(st));
    return MH_OK;
  }();
  release(b);
  return rc;
}

int32_t mh_selftest_scan_fault(mh_ctx *ctx) {
  CTX_GUARD(ctx);
  hipStream_t st = ctx->stream;
  const int64_t n = 2 * (int64_t)LB_TILE + 5;
  MH_TRY(ensure(ctx, ctx->scan_partials, scan_lb_scratch_bytes<int64_t>(n)));
  MH_TRY(ensure(ctx, ctx->scan_partials2, scan_lb_scratch_bytes<int64_t>(n)));
  MH_TRY(ensure(ctx, ctx->d_small, 8192 + 256));
  int64_t *tot = (int64_t *)((char *)ctx->d_small.p + 160);
  int32_t *bad = (int32_t *)((char *)ctx->d_small.p + 168);
  // the faulting scan on `s`, then its synchronisation: MH_E_STATE expected
  auto fault_once = [&](hipStream_t s, void *scratch) -> int32_t {
    HIPCHK(ctx, hipMemsetAsync(bad, 0, 4, s));
    HIPCHK(ctx, device_scan_sum<int64_t>(s, n, LoadOne{}, StoreCheck{bad}, scratch, tot, true));
    SYNCCHK(ctx, hipStreamSynchronize(s));
    return MH_OK;
  };
  // 1. from a lane thread (as the splice's second lane, mh_build_haplotypes_vset): its launches must report to this
  // context's fault word, not to slot 0
  int32_t rc_lane = MH_OK;
  std::thread t1([&]() {
    lane_thread_enter(ctx);
    if (hipSetDevice(ctx->device) != hipSuccess) {
      rc_lane = MH_E_HIP;
      return;
    }
    rc_lane = fault_once(ctx->stream2, ctx->scan_partials2.p);
  });
  t1.join();
  if (rc_lane != MH_E_STATE) return arg_fail(ctx, MH_E_HIP, "the timed-out scan of a lane thread was not reported");
  // 2. from the calling thread
  const int32_t rc = fault_once(st, ctx->scan_partials.p);
  if (rc != MH_E_STATE) return arg_fail(ctx, MH_E_HIP, "the timed-out scan was not reported");
  const std::string msg = ctx->err;
  HIPCHK(ctx, hipMemsetAsync(bad, 0, 4, st));
  HIPCHK(ctx, device_scan_sum<int64_t>(st, n, LoadOne{}, StoreCheck{bad}, ctx->scan_partials.p, tot));
  int32_t hb = 0;
  HIPCHK(ctx, hipMemcpyAsync(&hb, bad, 4, hipMemcpyDeviceToHost, st));
  SYNCCHK(ctx, hipStreamSynchronize(st));
  if (hb) return arg_fail(ctx, MH_E_HIP, "the scan after the fault is wrong");
  arg_fail(ctx, MH_E_STATE, msg);
  return MH_E_STATE;
}

// illumina.read_model_params (illumina.py:12-40)
int32_t mh_read_model_params(int64_t mean_rlen, double coverage, double *p_out, int64_t *passes_out) {
  if (!p_out || !passes_out || mean_rlen <= 0) return MH_E_ARG;
  double p = 1.0;
  int64_t passes = 1;
  while (p > 0.1) {
    passes *= 2;
    p = 0.5 * coverage / (double)(2 * mean_rlen * passes);
  }
  *p_out = p;
  *passes_out = passes;
  return MH_OK;
}

// readgenerate.get_data_for_workers (readgenerate.py:129-159)
int32_t mh_work_units(uint64_t seed, const int32_t *ploidy, int64_t n_regions, int64_t passes, int32_t *out_region,
                      int32_t *out_cpy, uint32_t *out_seed, int64_t *out_n) {
  if (seed > 0xffffffffull) return MH_E_SEED;
  if (n_regions < 0 || passes < 0 || (n_regions && !ploidy)) return MH_E_ARG;
  HostMT s;
  s.seed((uint32_t)seed);
  uint32_t shuffle_seed = (uint32_t)s.interval(0xfffffffeull);
  int64_t n = 0;
  for (int64_t r = 0; r < n_regions; r++)
    for (int32_t c = 0; c < ploidy[r]; c++)
      for (int64_t k = 0; k < passes; k++) {
        out_region[n] = (int32_t)r;
        out_cpy[n] = c;
        out_seed[n] = (uint32_t)s.interval(0xfffffffeull);
        n++;
      }
  HostMT sh;
  sh.seed(shuffle_seed);
  for (int64_t i = n - 1; i >= 1; i--) {
    int64_t j = (int64_t)sh.interval((uint64_t)i);
    std::swap(out_region[i], out_region[j]);
    std::swap(out_cpy[i], out_cpy[j]);
    std::swap(out_seed[i], out_seed[j]);
  }
  *out_n = n;
  return MH_OK;
}

int32_t mh_upload_contig(mh_ctx *ctx, int32_t contig_id, const char *seq, int64_t len) {
  CTX_GUARD(ctx);
  if (len < 0 || (len > 0 && !seq)) return arg_fail(ctx, MH_E_ARG, "bad contig");
  Contig &c = ctx->contigs[contig_id];
  MH_TRY(ensure(ctx, c.seq, len + 16));
  if (len) HIPCHK(ctx, hipMemcpyAsync(c.seq.p, seq, len, hipMemcpyHostToDevice, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  c.len = len;
  return MH_OK;
}

// the slot's Hap for a (re)build: released haplotypes' buffers when one is free (no queued writer still reads it) —
// the smallest whose haplotype buffer holds `need` bytes, else the largest (grown by the build) — else fresh ones
// (the pool grows to the generations a pipelined job needs); the main stream waits for the slot's last writer.  Best
// fit keeps a whole genome's haplotypes (50 of very different lengths) rebuilding without a hipMalloc / hipFree.
static int32_t hap_for_build(mh_ctx *ctx, int32_t slot, int64_t need, Hap **out, hipStream_t st = nullptr) {
  if (!ctx->haps.count(slot)) {
    int best = -1, big = -1;
    for (int i = 0; i < (int)ctx->hap_spare.size(); i++) {
      const Hap &s = ctx->hap_spare[i];
      if (s.used_set && hipEventQuery(s.used) != hipSuccess) continue;   // a queued writer still reads it
      if (s.hap.cap >= (size_t)need && (best < 0 || s.hap.cap < ctx->hap_spare[best].hap.cap)) best = i;
      if (big < 0 || s.hap.cap > ctx->hap_spare[big].hap.cap) big = i;
    }
    if (best < 0) best = big;
    if (best >= 0) {
      Hap r{};
      const Hap &s = ctx->hap_spare[best];
      r.hap = s.hap; r.rc = s.rc; r.keys = s.keys; r.ps = s.ps; r.pr = s.pr; r.op = s.op; r.oplen = s.oplen;
      r.nrun_s = s.nrun_s; r.nrun_e = s.nrun_e; r.nd = s.nd; r.bkt = s.bkt;
      r.used = s.used; r.used_set = s.used_set;
      ctx->hap_spare.erase(ctx->hap_spare.begin() + best);
      ctx->haps[slot] = r;
    }
  }
  Hap &h = ctx->haps[slot];
  MH_TRY(wait_unused(ctx, h.used, h.used_set, st));   // a queued writer may still read the old bytes
  h.valid = false;
  *out = &h;
  return MH_OK;
}

static int32_t build_from(mh_ctx *ctx, int32_t slot, int32_t contig_id, int64_t ref_start_pos, const VarSet &v,
                          int64_t *out_n_nodes, int64_t *out_p_min, int64_t *out_p_max) {
  auto it = ctx->contigs.find(contig_id);
  if (it == ctx->contigs.end()) return arg_fail(ctx, MH_E_STATE, "unknown contig id");
  Hap *hp = nullptr;
  MH_TRY(hap_for_build(ctx, slot, it->second.len + (it->second.len >> 6) + (1 << 20), &hp));
  Hap &h = *hp;
  MH_TRY(splice_build(ctx, h, it->second, ref_start_pos, v));
  if (out_n_nodes) *out_n_nodes = h.n_nodes;
  if (out_p_min) *out_p_min = h.p_min;
  if (out_p_max) *out_p_max = h.p_max;
  return MH_OK;
}

int32_t mh_build_haplotype(mh_ctx *ctx, int32_t slot, int32_t contig_id, int64_t ref_start_pos, const int64_t *v_pos,
                           const uint8_t *v_op, const int64_t *v_oplen, const int64_t *v_alt_off,
                           const int64_t *v_alt_len, const char *alt_pool, int64_t alt_pool_len, int64_t n_var,
                           int64_t *out_n_nodes, int64_t *out_p_min, int64_t *out_p_max) {
  CTX_GUARD_NOJOIN(ctx);   // orders itself against queued writers (Hap/TplSet used events)
  if (!ctx->contigs.count(contig_id)) return arg_fail(ctx, MH_E_STATE, "unknown contig id");
  if (n_var < 0 || (n_var > 0 && (!v_pos || !v_op || !v_oplen || !v_alt_off || !v_alt_len)))
    return arg_fail(ctx, MH_E_ARG, "bad variant arrays");
  VarSet &v = ctx->vsets[-1];   // scratch set, replaced by every call
  MH_TRY(var_upload(ctx, v, v_pos, v_op, v_oplen, v_alt_off, v_alt_len, alt_pool, alt_pool_len, n_var));
  return build_from(ctx, slot, contig_id, ref_start_pos, v, out_n_nodes, out_p_min, out_p_max);
}

int32_t mh_upload_variants(mh_ctx *ctx, int32_t vset, const int64_t *v_pos, const uint8_t *v_op,
                           const int64_t *v_oplen, const int64_t *v_alt_off, const int64_t *v_alt_len,
                           const char *alt_pool, int64_t alt_pool_len, int64_t n_var) {
  CTX_GUARD(ctx);
  if (vset < 0) return arg_fail(ctx, MH_E_ARG, "variant set ids are >= 0");
  if (n_var < 0 || (n_var > 0 && (!v_pos || !v_op || !v_oplen || !v_alt_off || !v_alt_len)))
    return arg_fail(ctx, MH_E_ARG, "bad variant arrays");
  const int32_t rc = var_upload(ctx, ctx->vsets[vset], v_pos, v_op, v_oplen, v_alt_off, v_alt_len, alt_pool,
                                alt_pool_len, n_var);
  if (rc != MH_OK) {
    release_vars(ctx->vsets[vset]);
    ctx->vsets.erase(vset);
  }
  return rc;
}

int32_t mh_build_haplotype_vset(mh_ctx *ctx, int32_t slot, int32_t contig_id, int64_t ref_start_pos, int32_t vset,
                                int64_t *out_n_nodes, int64_t *out_p_min, int64_t *out_p_max) {
  CTX_GUARD_NOJOIN(ctx);   // orders itself against queued writers (Hap/TplSet used events)
  auto it = ctx->vsets.find(vset);
  if (vset < 0 || it == ctx->vsets.end()) return arg_fail(ctx, MH_E_STATE, "unknown variant set id");
  return build_from(ctx, slot, contig_id, ref_start_pos, it->second, out_n_nodes, out_p_min, out_p_max);
}

int32_t mh_build_haplotypes_vset(mh_ctx *ctx, int32_t n, const int32_t *slots, const int32_t *contig_ids,
                                 const int64_t *ref_starts, const int32_t *vsets, int64_t *out_n_nodes,
                                 int64_t *out_p_min, int64_t *out_p_max) {
  CTX_GUARD_NOJOIN(ctx);
  if (n < 0 || (n > 0 && (!slots || !contig_ids || !ref_starts || !vsets))) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  for (int32_t i = 0; i < n; i++) {
    if (!ctx->contigs.count(contig_ids[i])) return arg_fail(ctx, MH_E_STATE, "unknown contig id");
    if (vsets[i] < 0 || !ctx->vsets.count(vsets[i])) return arg_fail(ctx, MH_E_STATE, "unknown variant set id");
    for (int32_t j = 0; j < i; j++)
      if (slots[j] == slots[i]) return arg_fail(ctx, MH_E_ARG, "a slot appears twice");
  }
  if (!pinned_small(ctx)) return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  for (int32_t i0 = 0; i0 < n; i0 += 2) {   // two copies at a time: the second on its own stream and host thread
    const int32_t k = n - i0 < 2 ? n - i0 : 2;
    Hap *hp[2] = {nullptr, nullptr};
    for (int32_t j = 0; j < k; j++) {
      const int64_t L = ctx->contigs[contig_ids[i0 + j]].len;
      MH_TRY(hap_for_build(ctx, slots[i0 + j], L + (L >> 6) + (1 << 20), &hp[j]));
    }
    if (k == 1) {
      MH_TRY(splice_build(ctx, *hp[0], ctx->contigs[contig_ids[i0]], ref_starts[i0], ctx->vsets[vsets[i0]]));
    } else {
      HIPCHK(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));   // lane 1 after everything the main stream waits for
      HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
      const Contig &c1 = ctx->contigs[contig_ids[i0 + 1]];
      const VarSet &v1 = ctx->vsets[vsets[i0 + 1]];
      int32_t rc1 = MH_OK;
      std::thread t1([&]() {   // nothing may escape the lane's thread (std::terminate): errors become codes
        lane_thread_enter(ctx);
        try {
          const hipError_t e = hipSetDevice(ctx->device);
          if (e != hipSuccess) {
            rc1 = hip_fail(ctx, e, "hipSetDevice (splice lane 1)", __FILE__, __LINE__);
            return;
          }
          rc1 = splice_build(ctx, *hp[1], c1, ref_starts[i0 + 1], v1, 1);
        } catch (const std::bad_alloc &) {
          rc1 = arg_fail(ctx, MH_E_OOM, "host memory (splice lane 1)");
        } catch (const std::exception &x) {
          rc1 = arg_fail(ctx, MH_E_STATE, std::string("splice lane 1: ") + x.what());
        } catch (...) {
          rc1 = arg_fail(ctx, MH_E_STATE, "splice lane 1: unknown exception");
        }
      });
      const int32_t rc0 = splice_build(ctx, *hp[0], ctx->contigs[contig_ids[i0]], ref_starts[i0],
                                       ctx->vsets[vsets[i0]]);
      t1.join();
      HIPCHK(ctx, hipEventRecord(ctx->ev_join, ctx->stream2));
      HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
      if (rc0 != MH_OK) return rc0;
      if (rc1 != MH_OK) return rc1;
    }
    for (int32_t j = 0; j < k; j++) {
      if (out_n_nodes) out_n_nodes[i0 + j] = hp[j]->n_nodes;
      if (out_p_min) out_p_min[i0 + j] = hp[j]->p_min;
      if (out_p_max) out_p_max[i0 + j] = hp[j]->p_max;
    }
  }
  return MH_OK;
}

// The next batch's haplotypes — and, given its units, its MT19937 word streams — while the current batch's sampling
// tails, measure passes and FASTQ writers run (the splice and the word generation off the batch boundary's critical
// path).  On the calling thread: each slot's buffers (hap_for_build, the
// prefetch stream waiting for the writer that last read a reused buffer); then a host thread of the context issues
// the splices one after the other on the prefetch stream (created on first use, the context's fourth) with scratch
// and a pinned readback block of their own, and waits on their readbacks, so the call returns at once and neither
// waits for the pending sampling tail nor for the main stream's queued measure passes.  join_prefetch (every entry
// point that resolves the sampling tail, and emission from a prefetched slot) joins that thread and makes the main
// stream wait for the splices.  The slots must be free (a live slot may be read by queued work).
int32_t mh_prefetch_haplotypes_vset(mh_ctx *ctx, int32_t n, const int32_t *slots, const int32_t *contig_ids,
                                    const int64_t *ref_starts, const int32_t *vsets, int32_t n_units,
                                    const int32_t *unit_slots, const uint64_t *unit_seeds, double p) {
  CTX_GUARD_EMIT(ctx);
  MH_TRY(join_prefetch(ctx));   // (an earlier prefetch's thread)
  if (n < 0 || (n > 0 && (!slots || !contig_ids || !ref_starts || !vsets))) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  if (n_units < 0 || (n_units > 0 && (!unit_slots || !unit_seeds || !(p > 0.0 && p <= 1.0))))
    return arg_fail(ctx, MH_E_ARG, "bad unit arguments");
  for (int32_t i = 0; i < n; i++) {
    if (!ctx->contigs.count(contig_ids[i])) return arg_fail(ctx, MH_E_STATE, "unknown contig id");
    if (vsets[i] < 0 || !ctx->vsets.count(vsets[i])) return arg_fail(ctx, MH_E_STATE, "unknown variant set id");
    if (ctx->haps.count(slots[i])) return arg_fail(ctx, MH_E_ARG, "prefetch into a live haplotype slot");
    for (int32_t j = 0; j < i; j++)
      if (slots[j] == slots[i]) return arg_fail(ctx, MH_E_ARG, "a slot appears twice");
  }
  if (n == 0 && n_units == 0) return MH_OK;
  if (!ctx->pstream) {
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    HIPCHK(ctx, hipStreamCreateWithPriority(&ctx->pstream, hipStreamNonBlocking, hi));
    HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_prefetch, hipEventDisableTiming));
  }
  if (!ctx->h_small3 && hipHostMalloc((void **)&ctx->h_small3, 4096, hipHostMallocDefault) != hipSuccess) {
    ctx->h_small3 = nullptr;
    return arg_fail(ctx, MH_E_OOM, "pinned host memory");
  }
  struct Job {
    Hap *h;
    const Contig *c;
    int64_t rs;
    const VarSet *v;
  };
  std::vector<Job> jobs;
  for (int32_t i = 0; i < n; i++) {
    const Contig &c = ctx->contigs[contig_ids[i]];
    Hap *hp = nullptr;
    MH_TRY(hap_for_build(ctx, slots[i], c.len + (c.len >> 6) + (1 << 20), &hp, ctx->pstream));
    hp->prefetched = true;   // (Hap references stay valid while other slots are inserted: node-based map)
    jobs.push_back(Job{hp, &c, ref_starts[i], &ctx->vsets[vsets[i]]});
  }
  // the units' haplotypes: prefetched above (spans known once spliced) or live
  std::vector<const Hap *> uh(n_units);
  for (int32_t u = 0; u < n_units; u++) {
    auto it = ctx->haps.find(unit_slots[u]);
    if (it == ctx->haps.end() || (!it->second.valid && !it->second.prefetched))
      return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
    uh[u] = &it->second;
  }
  std::vector<uint64_t> useeds(unit_seeds, unit_seeds + n_units);
  ctx->pf_words.valid = false;
  ctx->prefetch_pending = true;
  ctx->pf_rc = MH_OK;
  ctx->pf_thread = std::thread([ctx, jobs, uh, useeds, p]() {   // nothing may escape the thread: errors become codes
    int32_t rc = MH_OK;
    lane_thread_enter(ctx);
    try {
      const hipError_t e = hipSetDevice(ctx->device);
      if (e != hipSuccess) rc = hip_fail(ctx, e, "hipSetDevice (prefetch)", __FILE__, __LINE__);
      for (size_t k = 0; k < jobs.size() && rc == MH_OK; k++)
        rc = splice_build(ctx, *jobs[k].h, *jobs[k].c, jobs[k].rs, *jobs[k].v, 2);
      if (rc == MH_OK && !uh.empty()) {   // the next batch's word streams (sample_head takes them when it matches)
        std::vector<int64_t> pmin(uh.size()), pmax(uh.size());
        for (size_t u = 0; u < uh.size(); u++) {
          pmin[u] = uh[u]->p_min;
          pmax[u] = uh[u]->p_max;
        }
        rc = prefetch_words(ctx, ctx->pstream, (int32_t)uh.size(), pmin.data(), pmax.data(), useeds.data(), p);
      }
      const hipError_t e2 = hipEventRecord(ctx->ev_prefetch, ctx->pstream);
      if (rc == MH_OK && e2 != hipSuccess) rc = hip_fail(ctx, e2, "hipEventRecord (prefetch)", __FILE__, __LINE__);
    } catch (const std::bad_alloc &) {
      rc = arg_fail(ctx, MH_E_OOM, "host memory (prefetch)");
    } catch (const std::exception &x) {
      rc = arg_fail(ctx, MH_E_STATE, std::string("prefetch: ") + x.what());
    } catch (...) {
      rc = arg_fail(ctx, MH_E_STATE, "prefetch: unknown exception");
    }
    ctx->pf_rc = rc;
  });
  return MH_OK;
}

int32_t mh_release_variants(mh_ctx *ctx, int32_t vset) {
  CTX_GUARD(ctx);
  auto it = ctx->vsets.find(vset);
  if (it == ctx->vsets.end()) return MH_OK;
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  release_vars(it->second);
  ctx->vsets.erase(it);
  return MH_OK;
}

int32_t mh_get_nodes(mh_ctx *ctx, int32_t slot, int64_t *ps, int64_t *pr, uint8_t *op, int64_t *oplen, char *hap,
                     int64_t hap_cap, int64_t *hap_len) {
  CTX_GUARD(ctx);
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  Hap &h = it->second;
  hipStream_t st = ctx->stream;
  size_t n = (size_t)h.n_nodes;
  if (ps) HIPCHK(ctx, hipMemcpyAsync(ps, h.ps.p, 8 * n, hipMemcpyDeviceToHost, st));
  if (pr) HIPCHK(ctx, hipMemcpyAsync(pr, h.pr.p, 8 * n, hipMemcpyDeviceToHost, st));
  if (op) HIPCHK(ctx, hipMemcpyAsync(op, h.op.p, n, hipMemcpyDeviceToHost, st));
  if (oplen) HIPCHK(ctx, hipMemcpyAsync(oplen, h.oplen.p, 8 * n, hipMemcpyDeviceToHost, st));
  if (hap_len) *hap_len = h.hap_len;
  if (hap) {
    if (hap_cap < h.hap_len) {
      SYNCCHK(ctx, hipStreamSynchronize(st));
      return arg_fail(ctx, MH_E_CAPACITY, "haplotype buffer too small");
    }
    if (h.hap_len) HIPCHK(ctx, hipMemcpyAsync(hap, h.hap.p, h.hap_len, hipMemcpyDeviceToHost, st));
  }
  SYNCCHK(ctx, hipStreamSynchronize(st));
  return MH_OK;
}

int32_t mh_release_haplotype(mh_ctx *ctx, int32_t slot) {
  CTX_GUARD_NOJOIN(ctx);   // orders itself against queued writers (Hap/TplSet used events)
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end()) return MH_OK;
  Hap &h = it->second;
  // keep the buffers for the next build (stream order protects them: every later user is on ctx->stream)
  // a whole genome's haplotypes (25 regions x 2 copies) plus the generation the queued writers still read
  constexpr size_t SPARE_MAX = 128;
  if (ctx->hap_spare.size() < SPARE_MAX) {
    h.valid = false;
    ctx->hap_spare.push_back(h);
  } else {
    MH_TRY(sync_writers(ctx));
    SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
    release_hap(h);
  }
  ctx->haps.erase(it);
  return MH_OK;
}

int32_t mh_sample_templates(mh_ctx *ctx, int32_t slot, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                            uint64_t seed, int32_t rng_mode, int64_t *out_n) {
  CTX_GUARD_NOJOIN(ctx);   // orders itself against queued writers (Hap/TplSet used events)
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (!cum_tlen || !out_n || rlen <= 0 || !(p > 0.0 && p <= 1.0)) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  const int32_t id = -1;
  const NodeIdx ni = node_idx_of(it->second);
  MH_TRY(sample_units(ctx, 1, &id, &it->second.p_min, &it->second.p_max, &seed, p, rlen, cum_tlen, n_tlen, rng_mode,
                      out_n, &ni));
  ctx->cur_tpl = id;
  return MH_OK;
}

int32_t mh_sample_templates_span(mh_ctx *ctx, int64_t p_min, int64_t p_max, double p, int32_t rlen,
                                 const double *cum_tlen, int32_t n_tlen, uint64_t seed, int32_t rng_mode,
                                 int64_t *out_n) {
  CTX_GUARD_NOJOIN(ctx);   // orders itself against queued writers (Hap/TplSet used events)
  if (!cum_tlen || !out_n || rlen <= 0 || !(p > 0.0 && p <= 1.0) || p_max < p_min)
    return arg_fail(ctx, MH_E_ARG, "bad arguments");
  const int32_t id = -1;
  MH_TRY(sample_units(ctx, 1, &id, &p_min, &p_max, &seed, p, rlen, cum_tlen, n_tlen, rng_mode, out_n));
  ctx->cur_tpl = id;
  return MH_OK;
}

static int32_t unit_spans(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int32_t *slots,
                          const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen,
                          std::vector<int64_t> &pmin, std::vector<int64_t> &pmax, std::vector<NodeIdx> &nidx) {
  if (n_units < 0 || (n_units > 0 && (!tpl_ids || !slots || !seeds)) || !cum_tlen || rlen <= 0 ||
      !(p > 0.0 && p <= 1.0))
    return arg_fail(ctx, MH_E_ARG, "bad arguments");
  pmin.resize(n_units);
  pmax.resize(n_units);
  nidx.resize(n_units);
  for (int32_t u = 0; u < n_units; u++) {
    if (tpl_ids[u] < 0) return arg_fail(ctx, MH_E_ARG, "template set ids must be >= 0");
    for (int32_t v = 0; v < u; v++)
      if (tpl_ids[v] == tpl_ids[u]) return arg_fail(ctx, MH_E_ARG, "duplicate template set id");
    auto it = ctx->haps.find(slots[u]);
    if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
    pmin[u] = it->second.p_min;
    pmax[u] = it->second.p_max;
    nidx[u] = node_idx_of(it->second);
  }
  return MH_OK;
}

int32_t mh_sample_units(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int32_t *slots,
                        const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                        int32_t rng_mode, int64_t *out_n) {
  CTX_GUARD_NOJOIN(ctx);   // orders itself against queued writers (Hap/TplSet used events)
  std::vector<int64_t> pmin, pmax;
  std::vector<NodeIdx> nidx;
  MH_TRY(unit_spans(ctx, n_units, tpl_ids, slots, seeds, p, rlen, cum_tlen, pmin, pmax, nidx));
  return sample_units(ctx, n_units, tpl_ids, pmin.data(), pmax.data(), seeds, p, rlen, cum_tlen, n_tlen, rng_mode,
                      out_n, nidx.data());
}

int32_t mh_sample_units_async(mh_ctx *ctx, int32_t n_units, const int32_t *tpl_ids, const int32_t *slots,
                              const uint64_t *seeds, double p, int32_t rlen, const double *cum_tlen, int32_t n_tlen,
                              int32_t rng_mode) {
  CTX_GUARD_NOJOIN(ctx);
  std::vector<int64_t> pmin, pmax;
  std::vector<NodeIdx> nidx;
  MH_TRY(unit_spans(ctx, n_units, tpl_ids, slots, seeds, p, rlen, cum_tlen, pmin, pmax, nidx));
  return sample_units_async(ctx, n_units, tpl_ids, pmin.data(), pmax.data(), seeds, p, rlen, cum_tlen, n_tlen,
                            rng_mode, nidx.data());
}

int32_t mh_templates_count(mh_ctx *ctx, int32_t tpl_id, int64_t *n) {
  CTX_GUARD_EMIT(ctx);
  auto it = ctx->tsets.find(tpl_id);
  if (it == ctx->tsets.end()) return arg_fail(ctx, MH_E_STATE, "unknown template set");
  MH_TRY(tpl_resolve(ctx, it->second));
  if (!it->second.valid) return arg_fail(ctx, MH_E_STATE, "unknown template set");
  if (n) *n = it->second.n;
  return MH_OK;
}

int32_t mh_use_templates(mh_ctx *ctx, int32_t tpl_id) {
  CTX_GUARD_EMIT(ctx);
  auto it = ctx->tsets.find(tpl_id);
  if (it == ctx->tsets.end()) return arg_fail(ctx, MH_E_STATE, "unknown template set");
  MH_TRY(tpl_resolve(ctx, it->second));
  if (!it->second.valid) return arg_fail(ctx, MH_E_STATE, "unknown template set");
  ctx->cur_tpl = tpl_id;
  return MH_OK;
}

int32_t mh_release_templates(mh_ctx *ctx, int32_t tpl_id) {
  CTX_GUARD(ctx);
  auto it = ctx->tsets.find(tpl_id);
  if (it == ctx->tsets.end()) return MH_OK;
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  release(it->second.fo0); release(it->second.pos0); release(it->second.pos1); release(it->second.n0);
  if (it->second.used) (void)hipEventDestroy(it->second.used);
  ctx->tsets.erase(it);
  if (ctx->cur_tpl == tpl_id) ctx->cur_tpl = -1;
  return MH_OK;
}

int32_t mh_set_templates(mh_ctx *ctx, const int8_t *fo0, const int64_t *pos0, const int64_t *pos1, int64_t n,
                         int32_t rlen) {
  CTX_GUARD(ctx);
  if (n < 0 || rlen <= 0 || (n > 0 && (!fo0 || !pos0 || !pos1))) return arg_fail(ctx, MH_E_ARG, "bad templates");
  for (int64_t i = 0; i < n; i++)
    if (fo0[i] != 0 && fo0[i] != 1) return arg_fail(ctx, MH_E_ARG, "file_order must be 0/1");
  TplSet &ts = ctx->tsets[-1];
  MH_TRY(ensure(ctx, ts.fo0, n + 1));
  MH_TRY(ensure(ctx, ts.pos0, 8 * (n + 1)));
  ts.has_n0 = false;   // (no start nodes: the measure pass searches)
  MH_TRY(ensure(ctx, ts.pos1, 8 * (n + 1)));
  if (n) {
    HIPCHK(ctx, hipMemcpyAsync(ts.fo0.p, fo0, n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ts.pos0.p, pos0, 8 * n, hipMemcpyHostToDevice, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ts.pos1.p, pos1, 8 * n, hipMemcpyHostToDevice, ctx->stream));
  }
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  ts.n = n;
  ts.rlen = rlen;
  ts.valid = true;
  ctx->cur_tpl = -1;
  return MH_OK;
}

int32_t mh_get_templates(mh_ctx *ctx, int8_t *fo0, int64_t *pos0, int64_t *pos1, int64_t cap, int64_t *n) {
  CTX_GUARD(ctx);
  auto it = ctx->tsets.find(ctx->cur_tpl);
  if (it == ctx->tsets.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "no templates");
  const TplSet &ts = it->second;
  if (n) *n = ts.n;
  if (cap < ts.n) return arg_fail(ctx, MH_E_CAPACITY, "template buffers too small");
  size_t m = (size_t)ts.n;
  if (m) {
    if (fo0) HIPCHK(ctx, hipMemcpyAsync(fo0, ts.fo0.p, m, hipMemcpyDeviceToHost, ctx->stream));
    if (pos0) HIPCHK(ctx, hipMemcpyAsync(pos0, ts.pos0.p, 8 * m, hipMemcpyDeviceToHost, ctx->stream));
    if (pos1) HIPCHK(ctx, hipMemcpyAsync(pos1, ts.pos1.p, 8 * m, hipMemcpyDeviceToHost, ctx->stream));
  }
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

int32_t mh_expand_variant(int64_t samp_pos, int64_t ref_pos, int64_t ref_start_pos, int64_t v_pos, int32_t op,
                          int64_t oplen, int64_t *out, int32_t *n_nodes, int64_t *samp_next, int64_t *ref_next) {
  if (!out || !n_nodes || !samp_next || !ref_next || (op != 'X' && op != 'I' && op != 'D') || oplen < 0)
    return MH_E_ARG;
  VarNode v[2];
  const int n = expand_variant((uint8_t)op, v_pos, oplen, ref_pos, samp_pos, ref_start_pos, v, samp_next, ref_next);
  for (int j = 0; j < n; j++) {
    out[5 * j] = v[j].ps;
    out[5 * j + 1] = v[j].pr;
    out[5 * j + 2] = v[j].op;
    out[5 * j + 3] = v[j].oplen;
    out[5 * j + 4] = v[j].src;
  }
  *n_nodes = n;
  return MH_OK;
}

int32_t mh_templates_export(mh_ctx *ctx, int32_t tpl_id, int32_t on_device, int8_t *fo0, int64_t *pos0,
                            int64_t *pos1, int64_t cap, int64_t *n) {
  CTX_GUARD(ctx);
  auto it = ctx->tsets.find(tpl_id);
  if (it == ctx->tsets.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "unknown template set");
  const TplSet &ts = it->second;
  if (n) *n = ts.n;
  if (cap < ts.n) return arg_fail(ctx, MH_E_CAPACITY, "template buffers too small");
  const size_t m = (size_t)ts.n;
  const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
  if (m) {
    if (fo0) HIPCHK(ctx, hipMemcpyAsync(fo0, ts.fo0.p, m, k, ctx->stream));
    if (pos0) HIPCHK(ctx, hipMemcpyAsync(pos0, ts.pos0.p, 8 * m, k, ctx->stream));
    if (pos1) HIPCHK(ctx, hipMemcpyAsync(pos1, ts.pos1.p, 8 * m, k, ctx->stream));
  }
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

int32_t mh_templates_import(mh_ctx *ctx, int32_t tpl_id, int32_t on_device, const int8_t *fo0, const int64_t *pos0,
                            const int64_t *pos1, int64_t n, int32_t rlen) {
  CTX_GUARD(ctx);
  if (n < 0 || rlen <= 0 || (n > 0 && (!fo0 || !pos0 || !pos1))) return arg_fail(ctx, MH_E_ARG, "bad templates");
  if (!on_device)
    for (int64_t i = 0; i < n; i++)
      if (fo0[i] != 0 && fo0[i] != 1) return arg_fail(ctx, MH_E_ARG, "file_order must be 0/1");
  TplSet &ts = ctx->tsets[tpl_id];
  MH_TRY(wait_unused(ctx, ts.used, ts.used_set));   // a queued FASTQ writer may still read the old templates
  ts.valid = false;
  MH_TRY(ensure(ctx, ts.fo0, n + 16));
  MH_TRY(ensure(ctx, ts.pos0, 8 * (n + 16)));
  ts.has_n0 = false;   // (no start nodes: the measure pass searches)
  MH_TRY(ensure(ctx, ts.pos1, 8 * (n + 16)));
  const hipMemcpyKind k = on_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice;
  if (n) {
    HIPCHK(ctx, hipMemcpyAsync(ts.fo0.p, fo0, n, k, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ts.pos0.p, pos0, 8 * n, k, ctx->stream));
    HIPCHK(ctx, hipMemcpyAsync(ts.pos1.p, pos1, 8 * n, k, ctx->stream));
  }
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  if (ts.prep.valid) ctx->eset[ts.prep.set].prepared = false;   // the buffer set of a measure pass made for the old set
  ts.prep.valid = false;
  ts.n = n;
  ts.rlen = rlen;
  ts.valid = true;
  return MH_OK;
}

int32_t mh_emit_reads(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                      int32_t write_fastq2, uint64_t unit_key, int64_t *out_kept, int64_t *out_b1, int64_t *out_b2) {
  CTX_GUARD_EMIT(ctx);
  MH_TRY(lazy_resolve(ctx));   // (appends at the arenas' exact ends)
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (it->second.prefetched) MH_TRY(join_prefetch(ctx));   // (its splice was queued on the prefetch stream)
  if (!serial_stub || !chrom || !out_kept || !out_b1 || !out_b2) return arg_fail(ctx, MH_E_ARG, "null argument");
  return emit_reads(ctx, it->second, slot, serial_stub, chrom, cpy, write_fastq2, unit_key, 0, -1, 0, false, out_kept,
                    out_b1, out_b2);
}

int32_t mh_emit_prepare(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                        int32_t write_fastq2, uint64_t unit_key, int64_t *out_kept, int64_t *out_b1, int64_t *out_b2) {
  CTX_GUARD_EMIT(ctx);
  MH_TRY(lazy_resolve(ctx));   // (appends at the arenas' exact ends)
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (it->second.prefetched) MH_TRY(join_prefetch(ctx));   // (its splice was queued on the prefetch stream)
  if (!serial_stub || !chrom || (!out_kept) != (!out_b1) || (!out_kept) != (!out_b2))
    return arg_fail(ctx, MH_E_ARG, "null argument");
  return emit_reads(ctx, it->second, slot, serial_stub, chrom, cpy, write_fastq2, unit_key, 0, -1, 0, true, out_kept,
                    out_b1, out_b2);
}

int32_t mh_emit_reads_range(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                            int32_t write_fastq2, uint64_t unit_key, int64_t t_begin, int64_t t_end,
                            int64_t cnt_base, int64_t *out_kept, int64_t *out_b1, int64_t *out_b2) {
  CTX_GUARD_EMIT(ctx);
  MH_TRY(lazy_resolve(ctx));   // (appends at the arenas' exact ends)
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (it->second.prefetched) MH_TRY(join_prefetch(ctx));   // (its splice was queued on the prefetch stream)
  if (!serial_stub || !chrom || !out_kept || !out_b1 || !out_b2) return arg_fail(ctx, MH_E_ARG, "null argument");
  if (t_begin < 0 || t_end < t_begin || cnt_base < 0) return arg_fail(ctx, MH_E_ARG, "bad template range");
  return emit_reads(ctx, it->second, slot, serial_stub, chrom, cpy, write_fastq2, unit_key, t_begin, t_end, cnt_base,
                    false, out_kept, out_b1, out_b2);
}

int32_t mh_emit_reads_async(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                            int32_t write_fastq2, uint64_t unit_key) {
  CTX_GUARD_EMIT(ctx);
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (it->second.prefetched) MH_TRY(join_prefetch(ctx));   // (its splice was queued on the prefetch stream)
  if (!serial_stub || !chrom) return arg_fail(ctx, MH_E_ARG, "null argument");
  bool queued = false;
  MH_TRY(emit_unit_async(ctx, it->second, serial_stub, chrom, cpy, write_fastq2, unit_key, &queued));
  if (queued) return MH_OK;
  // a unit the single-pass writer does not cover: the two-pass path at the arenas' exact ends, its totals queued
  // in order with the others
  MH_TRY(lazy_resolve(ctx));
  int64_t k = 0, b1 = 0, b2 = 0;
  MH_TRY(emit_reads(ctx, it->second, slot, serial_stub, chrom, cpy, write_fastq2, unit_key, 0, -1, 0, false, &k, &b1,
                    &b2));
  ctx->lazy.push_back(mh_ctx::LazyUnit{-1, ctx->lazy_gen, {k, b1, b2}});
  return MH_OK;
}

int32_t mh_emit_collect(mh_ctx *ctx, int64_t *out, int64_t cap, int64_t *n_units) {
  CTX_GUARD_EMIT(ctx);
  if (!n_units) return arg_fail(ctx, MH_E_ARG, "null argument");
  MH_TRY(lazy_resolve(ctx));
  const int64_t n = (int64_t)ctx->lazy_done.size() / 3;
  *n_units = n;
  if (!out) return MH_OK;   // (the count only: the totals stay for the next call)
  if (cap < n) return arg_fail(ctx, MH_E_CAPACITY, "mh_emit_collect: room for " + std::to_string(n) + " units needed");
  std::memcpy(out, ctx->lazy_done.data(), sizeof(int64_t) * 3 * (size_t)n);
  ctx->lazy_done.clear();
  return MH_OK;
}

int32_t mh_emit_measure(mh_ctx *ctx, int32_t slot, const char *serial_stub, const char *chrom, int64_t cpy,
                        int32_t write_fastq2, uint64_t unit_key, int64_t t_begin, int64_t t_end, int64_t cnt_base,
                        int64_t *out_kept, int64_t *out_b1, int64_t *out_b2) {
  CTX_GUARD_EMIT(ctx);
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (it->second.prefetched) MH_TRY(join_prefetch(ctx));   // (its splice was queued on the prefetch stream)
  if (!serial_stub || !chrom || !out_kept || !out_b1 || !out_b2) return arg_fail(ctx, MH_E_ARG, "null argument");
  if (t_begin < 0 || (t_end >= 0 && t_end < t_begin) || cnt_base < 0) return arg_fail(ctx, MH_E_ARG, "bad template range");
  MH_TRY(emit_reads(ctx, it->second, slot, serial_stub, chrom, cpy, write_fastq2, unit_key, t_begin, t_end, cnt_base,
                    true, out_kept, out_b1, out_b2));
  auto tit = ctx->tsets.find(ctx->cur_tpl);   // the preparation is dropped: its buffer set is free again
  if (tit != ctx->tsets.end() && tit->second.prep.valid) {
    ctx->eset[tit->second.prep.set].prepared = false;
    tit->second.prep.valid = false;
  }
  return MH_OK;
}

int32_t mh_count_kept(mh_ctx *ctx, int32_t slot, int64_t t_begin, int64_t t_end, int64_t *out_kept) {
  CTX_GUARD(ctx);
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (!out_kept) return arg_fail(ctx, MH_E_ARG, "null argument");
  if (t_begin < 0 || t_end < t_begin) return arg_fail(ctx, MH_E_ARG, "bad template range");
  return count_kept(ctx, it->second, t_begin, t_end, out_kept);
}

int32_t mh_output_size(mh_ctx *ctx, int64_t *b1, int64_t *b2) {
  CTX_GUARD_EMIT(ctx);
  MH_TRY(lazy_resolve(ctx));
  if (b1) *b1 = ctx->used1;
  if (b2) *b2 = ctx->used2;
  return MH_OK;
}

int32_t mh_output_fetch(mh_ctx *ctx, int64_t off1, char *fq1, int64_t len1, int64_t off2, char *fq2, int64_t len2) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if ((fq1 && (off1 < 0 || len1 < 0 || off1 + len1 > ctx->used1)) ||
      (fq2 && (off2 < 0 || len2 < 0 || off2 + len2 > ctx->used2)))
    return arg_fail(ctx, MH_E_ARG, "fetch range outside the arena");
  // the two files' copies on two streams (two DMA engines side by side), file 2's after everything the main stream
  // waits for (the writers)
  const bool both = fq1 && len1 && fq2 && len2;
  stage_begin(ctx, "output_d2h");
  if (both) {
    HIPCHK(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
  }
  if (fq1 && len1) HIPCHK(ctx, hipMemcpyAsync(fq1, (char *)ctx->out1.p + off1, len1, hipMemcpyDeviceToHost, ctx->stream));
  if (fq2 && len2)
    HIPCHK(ctx, hipMemcpyAsync(fq2, (char *)ctx->out2.p + off2, len2, hipMemcpyDeviceToHost,
                               both ? ctx->stream2 : ctx->stream));
  if (both) {
    HIPCHK(ctx, hipEventRecord(ctx->ev_join, ctx->stream2));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
  }
  stage_end(ctx);
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

int32_t mh_output_fetch_async(mh_ctx *ctx, int64_t off1, char *fq1, int64_t len1, int64_t off2, char *fq2,
                              int64_t len2, int32_t *ticket) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if (!ticket || (fq1 && (off1 < 0 || len1 < 0 || off1 + len1 > ctx->used1)) ||
      (fq2 && (off2 < 0 || len2 < 0 || off2 + len2 > ctx->used2)))
    return arg_fail(ctx, MH_E_ARG, "fetch range outside the arena");
  for (int t = 0; t < 2; t++)
    if (!ctx->ev_fetch[t]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_fetch[t], hipEventDisableTiming));
  const int t = ctx->fetch_next;
  if (ctx->fetch_pending[t]) return arg_fail(ctx, MH_E_STATE, "two fetches in flight: wait for one first");
  // file 1 on the main stream (after the writers it waits for), file 2 on the second stream behind the same point
  stage_begin(ctx, "output_d2h");
  HIPCHK(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
  if (fq1 && len1) HIPCHK(ctx, hipMemcpyAsync(fq1, (char *)ctx->out1.p + off1, len1, hipMemcpyDeviceToHost, ctx->stream));
  if (fq2 && len2) HIPCHK(ctx, hipMemcpyAsync(fq2, (char *)ctx->out2.p + off2, len2, hipMemcpyDeviceToHost, ctx->stream2));
  HIPCHK(ctx, hipEventRecord(ctx->ev_join, ctx->stream2));
  HIPCHK(ctx, hipStreamWaitEvent(ctx->stream, ctx->ev_join, 0));
  stage_end(ctx);
  HIPCHK(ctx, hipEventRecord(ctx->ev_fetch[t], ctx->stream));
  ctx->fetch_pending[t] = true;
  ctx->fetch_next = t ^ 1;
  *ticket = t;
  return MH_OK;
}

int32_t mh_output_fetch_wait(mh_ctx *ctx, int32_t ticket) {
  CTX_GUARD_EMIT(ctx);
  if (ticket < 0) return MH_OK;
  if (ticket > 1) return arg_fail(ctx, MH_E_ARG, "bad ticket");
  if (ctx->fetch_pending[ticket]) {
    SYNCCHK(ctx, hipEventSynchronize(ctx->ev_fetch[ticket]));
    ctx->fetch_pending[ticket] = false;
  }
  return MH_OK;
}

int32_t mh_output_reset(mh_ctx *ctx) {
  CTX_GUARD_EMIT(ctx);
  for (int t = 0; t < 2; t++)   // copies still reading the arenas finish before they are refilled
    if (ctx->fetch_pending[t]) {
      SYNCCHK(ctx, hipEventSynchronize(ctx->ev_fetch[t]));
      ctx->fetch_pending[t] = false;
    }
  ctx->used1 = ctx->used2 = 0;
  // the single-pass chain starts again from the empty arenas; units still queued keep their totals for
  // mh_emit_collect but no longer move the arenas
  ctx->chain_open = false;
  ctx->lazy_gen++;
  ctx->used_ub1 = ctx->used_ub2 = 0;
  return MH_OK;
}

int32_t mh_read_batch(mh_ctx *ctx, int32_t slot, const int64_t *p, const int64_t *l, int64_t n, int64_t *out_pos,
                      int64_t *out_n0, int64_t *out_n1, char *cigar, int64_t cigar_cap, int64_t *cigar_off,
                      int64_t *cigar_used, char *vlist, int64_t vlist_cap, int64_t *vlist_off, int64_t *vlist_used,
                      char *seq, int64_t seq_cap, int64_t *seq_off, int64_t *seq_used) {
  CTX_GUARD(ctx);
  auto it = ctx->haps.find(slot);
  if (it == ctx->haps.end() || !it->second.valid) return arg_fail(ctx, MH_E_STATE, "empty haplotype slot");
  if (n < 0 || !cigar_used || !vlist_used || !seq_used) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  return read_batch(ctx, it->second, p, l, n, out_pos, out_n0, out_n1, cigar, cigar_cap, cigar_off, cigar_used, vlist,
                    vlist_cap, vlist_off, vlist_used, seq, seq_cap, seq_off, seq_used);
}

int32_t mh_set_corruption(mh_ctx *ctx, int32_t enable, const double *cum_bq, int32_t max_bp, int32_t n_bq,
                          const double *phred_p, uint64_t seed) {
  CTX_GUARD(ctx);
  if (!enable) {
    ctx->corrupt_on = false;
    return MH_OK;
  }
  if (!cum_bq || !phred_p || max_bp <= 0 || n_bq <= 0 || n_bq > 4096)
    return arg_fail(ctx, MH_E_ARG, "bad corruption model");
  if (seed > 0xffffffffull) return arg_fail(ctx, MH_E_SEED, "Seed value out of range 0 - 4294967295");
  if (max_bp > 16384) return arg_fail(ctx, MH_E_ARG, "BQ model longer than 16384 positions");
  const size_t nt = (size_t)2 * max_bp * n_bq;
  // u16 tables of the Philox mode: T = min(floor(x * 2^16), 65535) (exact: x * 2^16 is exact in f64); a NaN entry
  // counts as larger than any draw, as numpy's searchsorted orders it
  auto fix16 = [](double x) -> uint16_t {
    if (!(x > 0.0)) return x != x ? 0xffff : 0;
    const double y = std::floor(x * 65536.0);
    return y >= 65535.0 ? 0xffff : (uint16_t)y;
  };
  std::vector<uint16_t> T16(nt), Fp16(100);
  for (size_t i = 0; i < nt; i++) T16[i] = fix16(cum_bq[i]);
  for (int i = 0; i < 100; i++) Fp16[i] = fix16(phred_p[i]);
  // per row: the f64 search guide g[k] = entries below k / CG_BUCKETS (a lower bound for any draw in bucket k,
  // g[k + 1] an upper one), and the Philox-mode bucket table bk[k] = min(g[k], 93) | 0x80 when an entry lies in
  // [k, k + 1) / 256 and g[k] < 93 (CB_ROW = CG_BUCKETS buckets of the 16-bit draw)
  static_assert(mh::CB_ROW == mh::CG_BUCKETS, "bucket table and guide share their buckets");
  std::vector<uint16_t> guide((size_t)2 * max_bp * (mh::CG_BUCKETS + 1));
  std::vector<uint8_t> bk((size_t)2 * max_bp * mh::CB_ROW), bkf((size_t)2 * max_bp * mh::CF_ROW);
  for (size_t r = 0; r < (size_t)2 * max_bp; r++) {
    const uint16_t *row = T16.data() + r * n_bq;
    uint16_t *g = guide.data() + r * (mh::CG_BUCKETS + 1);
    int64_t c = 0;
    for (int k = 0; k <= mh::CG_BUCKETS; k++) {
      while (c < n_bq && (uint32_t)row[c] < ((uint32_t)k << 8)) c++;
      g[k] = (uint16_t)c;
    }
    for (int k = 0; k < mh::CB_ROW; k++) {
      const int lo = g[k];
      bk[r * mh::CB_ROW + k] = (uint8_t)((lo < 93 ? lo : 93) | (lo < 93 && g[k + 1] > lo ? 0x80 : 0));
    }
    // the fine table: the same entry over buckets of 32 draw values
    c = 0;
    int64_t c1 = 0;
    for (int k = 0; k < mh::CF_ROW; k++) {
      while (c < n_bq && (uint32_t)row[c] < ((uint32_t)k << mh::CF_SHIFT)) c++;
      if (c1 < c) c1 = c;
      while (c1 < n_bq && (uint32_t)row[c1] < ((uint32_t)(k + 1) << mh::CF_SHIFT)) c1++;
      bkf[r * mh::CF_ROW + k] = (uint8_t)((c < 93 ? c : 93) | (c < 93 && c1 > c ? 0x80 : 0));
    }
  }
  auto al16 = [](size_t x) { return ((x + 15) / 16) * 16; };
  ctx->corrupt_guide_off = al16(8 * nt);
  ctx->corrupt_bk_off = al16(ctx->corrupt_guide_off + 2 * guide.size());
  ctx->corrupt_T16_off = al16(ctx->corrupt_bk_off + bk.size());
  ctx->corrupt_Fp16_off = al16(ctx->corrupt_T16_off + 2 * nt);
  ctx->corrupt_bkf_off = al16(ctx->corrupt_Fp16_off + 2 * 100);
  MH_TRY(sync_writers(ctx));   // queued writers and row passes may still read the previous tables
  MH_TRY(ensure(ctx, ctx->corrupt_cum, ctx->corrupt_bkf_off + bkf.size() + 64));
  MH_TRY(ensure(ctx, ctx->corrupt_phred, 8 * 100));
  char *base = (char *)ctx->corrupt_cum.p;
  HIPCHK(ctx, hipMemcpyAsync(base, cum_bq, 8 * nt, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(base + ctx->corrupt_guide_off, guide.data(), 2 * guide.size(), hipMemcpyHostToDevice,
                             ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(base + ctx->corrupt_bk_off, bk.data(), bk.size(), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(base + ctx->corrupt_T16_off, T16.data(), 2 * nt, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(base + ctx->corrupt_Fp16_off, Fp16.data(), 2 * 100, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(base + ctx->corrupt_bkf_off, bkf.data(), bkf.size(), hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemcpyAsync(ctx->corrupt_phred.p, phred_p, 8 * 100, hipMemcpyHostToDevice, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  ctx->corrupt_on = true;
  ctx->corrupt_max_bp = max_bp;
  ctx->corrupt_n_bq = n_bq;
  ctx->corrupt_seed = seed;
  return MH_OK;
}

int32_t mh_set_corruption_stream(mh_ctx *ctx, int32_t rng_mode, uint64_t seed, const uint32_t *key624, int32_t pos) {
  CTX_GUARD(ctx);
  if (rng_mode == MH_RNG_PHILOX) {
    ctx->cx_mode = 0;
    return MH_OK;
  }
  if (rng_mode != MH_RNG_MITTY) return arg_fail(ctx, MH_E_ARG, "unknown rng mode");
  if (key624) {
    if (pos < 0 || pos > 624) return arg_fail(ctx, MH_E_ARG, "MT19937 state position outside 0..624");
    std::copy(key624, key624 + 624, ctx->cx_key);
    ctx->cx_kpos = pos;
    ctx->cx_mode = 2;
    return MH_OK;
  }
  if (seed > 0xffffffffull) return arg_fail(ctx, MH_E_SEED, "Seed value out of range 0 - 4294967295");
  ctx->cx_seed = (uint32_t)seed;
  ctx->cx_pos = 0;
  ctx->cx_mode = 1;
  return MH_OK;
}

int32_t mh_get_corruption_stream(mh_ctx *ctx, uint32_t *key624, int32_t *pos, int64_t *words) {
  CTX_GUARD(ctx);
  if (ctx->cx_mode == 0) return arg_fail(ctx, MH_E_STATE, "corruption stream is Philox (no MT19937 state)");
  if (words) *words = ctx->cx_mode == 1 ? ctx->cx_pos : -1;
  if (!key624 && !pos) return MH_OK;
  HostMT h;
  if (ctx->cx_mode == 1) {   // RandomState(seed) advanced by the words consumed (twists only)
    h.seed(ctx->cx_seed);
    for (int64_t left = ctx->cx_pos; left > 0;) {
      if (h.pos == 624) {
        h.next();
        left--;
        continue;
      }
      const int64_t take = std::min<int64_t>(624 - h.pos, left);
      h.pos += (int)take;
      left -= take;
    }
  } else {
    std::copy(ctx->cx_key, ctx->cx_key + 624, h.key);
    h.pos = ctx->cx_kpos;
  }
  if (key624) std::copy(h.key, h.key + 624, key624);
  if (pos) *pos = h.pos;
  return MH_OK;
}

int32_t mh_host_alloc(int64_t bytes, void **out) {
  if (!out || bytes < 0) return MH_E_ARG;
  *out = nullptr;
  const size_t n = (size_t)(bytes > 0 ? bytes : 1);
  // on the current GPU's NUMA node: the same chunked D2H ran at 28 GB/s into staging the allocating thread had
  // placed on the far socket, 55-56 GB/s into near memory (round 4).  Anonymous pages bound to that node, then
  // page-locked and mapped for the GPU; hipHostMalloc when the node is unknown or the binding fails.
  int dev = 0;
  const int node = hipGetDevice(&dev) == hipSuccess ? mh::gpu_numa_node(dev) : -1;
  if (node >= 0 && node < 1024) {
    void *p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p != MAP_FAILED) {
      unsigned long mask[1024 / (8 * sizeof(unsigned long))] = {0};
      mask[node / (8 * sizeof(unsigned long))] |= 1ul << (node % (8 * sizeof(unsigned long)));
      const long rc = syscall(SYS_mbind, p, n, 2 /* MPOL_BIND */, mask, (unsigned long)1024, 0u);
      if (rc == 0 && hipHostRegister(p, n, hipHostRegisterDefault) == hipSuccess) {
        std::lock_guard<std::mutex> lk(mh::host_allocs_mu());
        mh::host_allocs()[p] = n;
        *out = p;
        return MH_OK;
      }
      (void)hipGetLastError();
      munmap(p, n);
    }
  }
  if (hipHostMalloc(out, n, hipHostMallocDefault) != hipSuccess) return MH_E_OOM;
  return MH_OK;
}

int32_t mh_device_cache_trim(int64_t *freed_bytes) {
  const int64_t f = mh::cache_trim(-1);
  if (freed_bytes) *freed_bytes = f;
  return MH_OK;
}

int32_t mh_device_live_bytes(int64_t *live, int64_t *peak, int32_t reset_peak) {
  if (live) *live = mh::g_live.load();
  if (peak) *peak = mh::g_live_peak.load();
  if (reset_peak) mh::g_live_peak.store(mh::g_live.load());
  return MH_OK;
}

int32_t mh_host_free(void *p) {
  if (!p) return MH_OK;
  size_t n = 0;
  {
    std::lock_guard<std::mutex> lk(mh::host_allocs_mu());
    auto it = mh::host_allocs().find(p);
    if (it != mh::host_allocs().end()) {
      n = it->second;
      mh::host_allocs().erase(it);
    }
  }
  if (n) {   // a node-bound registration
    const hipError_t e = hipHostUnregister(p);
    munmap(p, n);
    return e == hipSuccess ? MH_OK : MH_E_HIP;
  }
  if (hipHostFree(p) != hipSuccess) return MH_E_HIP;
  return MH_OK;
}

int32_t mh_mt_window_at(uint32_t seed, uint64_t offset, uint32_t *out624) {
  if (!out624) return MH_E_ARG;
  try {
    mh::jump::window_at(seed, offset, out624);
  } catch (...) {
    return MH_E_ARG;
  }
  return MH_OK;
}

int32_t mh_set_emit_mode(mh_ctx *ctx, int32_t mode) {
  if (!ctx || mode < 0 || mode > 3) return MH_E_ARG;
  ctx->emit_lds_only = mode == 1;
  ctx->emit_two_pass = mode == 2;
  ctx->emit_single = mode == 3;
  return MH_OK;
}

int32_t mh_set_decode_mode(mh_ctx *ctx, int32_t mode) {
  if (!ctx || mode < 0 || mode > (MH_DEC_SEQUENTIAL | MH_DEC_FORCE_FIXUP | MH_DEC_FORCE_GEO)) return MH_E_ARG;
  ctx->decode_sequential = (mode & MH_DEC_SEQUENTIAL) != 0;
  ctx->force_fixup = (mode & MH_DEC_FORCE_FIXUP) != 0;
  ctx->force_geo = (mode & MH_DEC_FORCE_GEO) != 0;
  return MH_OK;
}

int32_t mh_fixup_count(mh_ctx *ctx, int64_t *n) {
  if (!ctx || !n) return MH_E_ARG;
  *n = ctx->fixups;
  return MH_OK;
}

int32_t mh_enable_timing(mh_ctx *ctx, int32_t on) {
  if (!ctx) return MH_E_ARG;
  (void)hipSetDevice(ctx->device);
  stages_collect(ctx);
  ctx->timing = on != 0;
  ctx->last_times.clear();
  return MH_OK;
}

int32_t mh_stage_times(mh_ctx *ctx, const char **names, double *ms, int32_t cap, int32_t *n) {
  if (!ctx || !n) return MH_E_ARG;
  (void)hipSetDevice(ctx->device);
  stages_collect(ctx);
  int32_t k = 0;
  for (auto &t : ctx->last_times) {
    if (k < cap) {
      if (names) names[k] = t.first;
      if (ms) ms[k] = t.second;
    }
    k++;
  }
  *n = k;
  if (names || ms) ctx->last_times.clear();   // a size query (both NULL) keeps them
  return MH_OK;
}

// ---- god-aligner BAM (mh_bam.hip, mh_bgzf.cpp) ----------------------------------------------------------------
int32_t mh_bam_set_refs(mh_ctx *ctx, int32_t n_refs, const char *names, const int64_t *lengths) {
  CTX_GUARD(ctx);
  if (n_refs < 0 || (n_refs > 0 && (!names || !lengths))) return arg_fail(ctx, MH_E_ARG, "bad reference list");
  // a new store (counts reset by bam_set_refs); the device buffers stay for the next job, as everything else does
  // (freeing and reallocating GBs of them per job stretched a 10-step configs[4] bench from 47 to 481 ms per step)
  return bam_set_refs(ctx, n_refs, names, lengths);
}

static int32_t stage_in(mh_ctx *ctx, DevBuf &b, const char *src, int64_t len) {
  MH_TRY(ensure(ctx, b, (size_t)len + 64));
  if (len) HIPCHK(ctx, hipMemcpyAsync(b.p, src, len, hipMemcpyHostToDevice, ctx->stream));
  HIPCHK(ctx, hipMemsetAsync((char *)b.p + len, 0, 64, ctx->stream));
  return MH_OK;
}

int32_t mh_bam_add_fastq(mh_ctx *ctx, const char *fq1, int64_t len1, const char *fq2, int64_t len2,
                         int64_t max_templates, int64_t *used1, int64_t *used2, int64_t *templates) {
  CTX_GUARD(ctx);
  if (!fq1 || len1 < 0 || (fq2 && len2 < 0) || !used1 || !used2 || !templates)
    return arg_fail(ctx, MH_E_ARG, "null argument");
  MH_TRY(stage_in(ctx, ctx->bam.in1, fq1, len1));
  if (fq2) MH_TRY(stage_in(ctx, ctx->bam.in2, fq2, len2));
  return bam_add(ctx, (const uint8_t *)ctx->bam.in1.p, len1, fq2 ? (const uint8_t *)ctx->bam.in2.p : nullptr,
                 fq2 ? len2 : 0, max_templates, used1, used2, templates);
}

int32_t mh_bam_add_output(mh_ctx *ctx, int64_t max_templates, int64_t *templates) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if (!templates) return arg_fail(ctx, MH_E_ARG, "null argument");
  int64_t u1 = 0, u2 = 0;
  const bool two = ctx->used2 > 0;
  const uint8_t *a1 = (const uint8_t *)ctx->out1.p, *a2 = two ? (const uint8_t *)ctx->out2.p : nullptr;
  if (ctx->bam.cap <= 0)
    return bam_add(ctx, a1, ctx->used1, a2, two ? ctx->used2 : 0, max_templates, &u1, &u2, templates, true);
  // bounded HBM (mh_bam_set_capacity): the arenas in pieces of cap / 2048 templates (a template's records are well
  // under 2 KiB: 2x250 reads with their qnames ~1 KiB), so the store spills between pieces and stays near the bound
  const int64_t per = std::max<int64_t>(1, ctx->bam.cap / 2048);
  int64_t o1 = 0, o2 = 0, tot = 0;
  // each piece indexes a byte window of about its own records (4 KiB per template, doubled when a window holds no
  // whole template), not the whole rest of the arenas: the newline index of every piece over the remainder made the
  // bounded add quadratic in arena / piece
  int64_t win = per * 4096;
  while (max_templates < 0 || tot < max_templates) {
    const int64_t lim = max_templates < 0 ? per : std::min(per, max_templates - tot);
    const int64_t r1 = ctx->used1 - o1, r2 = two ? ctx->used2 - o2 : 0;
    const int64_t l1 = std::min(r1, win), l2 = std::min(r2, win);
    int64_t t = 0;
    MH_TRY(bam_add(ctx, a1 + o1, l1, two ? a2 + o2 : nullptr, l2, lim, &u1, &u2, &t, false));
    if (t == 0 && (l1 < r1 || l2 < r2)) {   // (a template longer than the window: a wider one)
      win *= 2;
      continue;
    }
    if (t == 0) break;
    o1 += u1;
    o2 += u2;
    tot += t;
  }
  *templates = tot;
  return MH_OK;
}

int32_t mh_bam_records(mh_ctx *ctx, int64_t *n_records, int64_t *bytes) {
  if (!ctx) return MH_E_ARG;
  if (n_records) *n_records = ctx->bam.n_rec;
  if (bytes) *bytes = ctx->bam.bytes;
  return MH_OK;
}

int32_t mh_bam_export(mh_ctx *ctx, int64_t r0, int64_t r1, uint8_t *recs, int64_t *roff, uint64_t *keys,
                      int32_t *info) {
  CTX_GUARD(ctx);
  return bam_export(ctx, r0, r1, recs, roff, keys, info);
}

int32_t mh_bam_import(mh_ctx *ctx, const uint8_t *recs, const int64_t *roff, const uint64_t *keys, const int32_t *info,
                      int64_t n) {
  CTX_GUARD(ctx);
  if (n < 0 || (n > 0 && (!roff || !keys || !info))) return arg_fail(ctx, MH_E_ARG, "null argument");
  return bam_import(ctx, recs, roff, keys, info, n);
}

int32_t mh_bam_spilled(mh_ctx *ctx, int64_t *bytes, int64_t *blocks) {
  if (!ctx) return MH_E_ARG;
  if (bytes) *bytes = ctx->bam.spilled;
  if (blocks) *blocks = (int64_t)ctx->bam.spill.size();
  return MH_OK;
}

int32_t mh_bam_write(mh_ctx *ctx, const char *bam_path, const char *header_text, int64_t header_len, int32_t level,
                     int32_t threads, const char *bai_path, int64_t *out_records, int64_t *out_bytes) {
  CTX_GUARD(ctx);
  BamStore &B = ctx->bam;
  if (!bam_path || (header_len > 0 && !header_text)) return arg_fail(ctx, MH_E_ARG, "null argument");
  if (!B.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  if (level < 0 || level > 9) return arg_fail(ctx, MH_E_ARG, "compression level must be 0..9");
  MH_TRY(bam_sort(ctx));
  const int64_t n = B.n_rec;
  std::vector<uint8_t> recs((size_t)B.bytes + 1);
  std::vector<int64_t> soff((size_t)n + 1, 0);
  std::vector<BaiRec> info((size_t)n + 1);
  MH_TRY(bam_fetch_sorted(ctx, recs.data(), soff.data(), (int32_t *)info.data()));
  const std::string hdr = bam_header_bytes(std::string(header_text ? header_text : "", (size_t)header_len),
                                           B.ref_names, B.ref_len);
  std::vector<int64_t> coff;
  std::string err;
  if (!bgzf_write(bam_path, hdr, recs.data(), B.bytes, level, threads, coff, err))
    return arg_fail(ctx, MH_E_ARG, err);
  if (bai_path && !bai_write(bai_path, (int32_t)B.ref_names.size(), n, info.data(), soff.data(), coff, err))
    return arg_fail(ctx, MH_E_ARG, err);
  if (out_records) *out_records = n;
  if (out_bytes) *out_bytes = B.bytes;
  return MH_OK;
}

}  // extern "C"

// copies that mh_output_bgzf_pair left in flight out of gz_out's halves: done before anything else rewrites gz_out
static int32_t gz_drain(mh_ctx *ctx) {
  for (int h = 0; h < 2; h++)
    if (ctx->gz_pending[h]) {
      SYNCCHK(ctx, hipEventSynchronize(ctx->ev_gz[h]));
      ctx->gz_pending[h] = false;
    }
  return MH_OK;
}

// Window of a spilled store's deflate: a quarter of the store's capacity (two staging windows in HBM and two ring
// slots of compressed output, each about a window: together about the capacity), whole BGZF blocks, at most 8192
// blocks (535 MB)
static int64_t spill_window(const BamStore &B) {
  const int64_t cap_blocks = B.cap > 0 ? B.cap / 4 / BGZF_BLOCK : 8192;
  return std::max<int64_t>(1, std::min<int64_t>(8192, cap_blocks)) * BGZF_BLOCK;
}

// A spilled store's sorted record stream deflated on the device window by window: the host assembles window i + 1
// (bam_assemble, a thread of its own) while window i goes H2D and through bgzf_device into ring slot i & 1 of
// ctx->gz_out (ring bytes per slot; pieces are reported at their ring offsets, the block offsets in `boff` are the
// stream's).  Before window i overwrites its slot, slot_free(i) returns once the compressed pieces of window i - 2 have
// left the device.  Windows are whole numbers of BGZF blocks, so the blocks — and the file — are the ones one deflate
// of the whole stream makes.  The stream deflated is the sorted stream from byte `skip`, then `tail` (a range's part
// of a file, mh_bam_write_part).
static int32_t bam_deflate_spilled(mh_ctx *ctx, int64_t ring, int64_t skip, const uint8_t *tail, int64_t tail_len,
                                   int64_t *nz, std::vector<int64_t> *boff,
                                   const std::function<void(int64_t, int64_t)> &on_piece,
                                   const std::function<int32_t(int64_t)> &slot_free) {
  BamStore &B = ctx->bam;
  MH_TRY(bam_spill(ctx));   // (the records still in HBM: every record is then on the host)
  MH_TRY(bam_sort(ctx));    // (a no-op unless the spill undid a direct write's order)
  BamHostOrder o;
  MH_TRY(bam_host_order(ctx, o));
  const int64_t W = spill_window(B);
  const int64_t nb = B.bytes - skip, L = nb + tail_len;   // the stream: sorted [skip, bytes), then the tail
  const int64_t n_win = (L + W - 1) / W;
  uint8_t *pin[2] = {nullptr, nullptr};
  struct PinGuard {
    uint8_t **p;
    ~PinGuard() {
      for (int s = 0; s < 2; s++)
        if (p[s]) (void)hipHostFree(p[s]);
    }
  } pguard{pin};
  for (int s = 0; s < 2; s++) HIPCHK(ctx, hipHostMalloc((void **)&pin[s], (size_t)W, hipHostMallocDefault));
  MH_TRY(ensure(ctx, B.in1, (size_t)W + 64));
  MH_TRY(ensure(ctx, B.in2, (size_t)W + 64));
  uint8_t *dwin[2] = {(uint8_t *)B.in1.p, (uint8_t *)B.in2.p};
  std::mutex mu;
  std::condition_variable cv;
  int64_t ready = 0;            // windows assembled
  int64_t freed = 2;            // windows whose staging slot may be refilled (slot of window i: i & 1)
  bool stop = false;
  std::thread asm_th([&]() {
    for (int64_t i = 0; i < n_win; i++) {
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || i < freed; });
        if (stop) return;
      }
      const int64_t v0 = i * W, v1 = std::min(L, v0 + W);
      if (std::min(v1, nb) > v0) bam_assemble(B, o, skip + v0, skip + std::min(v1, nb), pin[i & 1], 16);
      if (v1 > nb) {
        const int64_t t0 = std::max(v0, nb);
        std::memcpy(pin[i & 1] + (t0 - v0), tail + (t0 - nb), (size_t)(v1 - t0));
      }
      std::lock_guard<std::mutex> lk(mu);
      ready = i + 1;
      cv.notify_all();
    }
  });
  struct Join {
    std::thread *t;
    std::mutex *m;
    std::condition_variable *c;
    bool *stop;
    ~Join() {
      {
        std::lock_guard<std::mutex> lk(*m);
        *stop = true;
        c->notify_all();
      }
      t->join();
    }
  } join{&asm_th, &mu, &cv, &stop};
  boff->assign(1, 0);
  int64_t zpos = 0;
  std::vector<int64_t> bw;
  for (int64_t i = 0; i < n_win; i++) {
    {
      std::unique_lock<std::mutex> lk(mu);
      cv.wait(lk, [&] { return ready > i; });
    }
    const int s = (int)(i & 1);
    const int64_t len = std::min(L, (i + 1) * W) - i * W;
    HIPCHK(ctx, hipMemcpyAsync(dwin[s], pin[s], (size_t)len, hipMemcpyHostToDevice, ctx->stream));
    MH_TRY(slot_free(i));   // ring slot s: window i - 2's compressed pieces copied out
    const int64_t zb = s * ring;
    const std::function<void(int64_t, int64_t)> piece = [&](int64_t off, int64_t bytes) { on_piece(zb + off, bytes); };
    int64_t used = 0;
    MH_TRY(bgzf_device(ctx, ctx->stream, dwin[s], len, (uint8_t *)ctx->gz_out.p + zb, ring, &used, &bw,
                       &piece));   // (returns with the stream drained)
    {
      std::lock_guard<std::mutex> lk(mu);
      freed = i + 3;   // slot s (its H2D is done) takes window i + 2
      cv.notify_all();
    }
    boff->pop_back();
    for (int64_t x : bw) boff->push_back(zpos + x);
    zpos += used;
  }
  *nz = zpos;
  return MH_OK;
}

// The sorted store's record stream deflated on the device and written to `path`: the header's block(s) first (hdr
// null: none), the stream from byte `skip` followed by `tail` (tail_len bytes, host memory) cut into 0xff00-byte BGZF
// blocks, the EOF marker when `eof`.  A writer thread copies each packed piece out (stream2, two page-locked 64 MiB
// slots) and writes it while the next piece deflates.  boff: the data blocks' offsets from data_pos (nblocks + 1).
struct BamPart {
  int64_t data_pos = 0, end_pos = 0, nz = 0;
  std::vector<int64_t> boff;
};
static int32_t bam_write_gpu_impl(mh_ctx *ctx, const char *path, const std::string *hdr, int64_t skip,
                                  const uint8_t *tail, int64_t tail_len, bool eof, BamPart &P) {
  BamStore &B = ctx->bam;
  MH_TRY(bam_sort(ctx));
  if (skip < 0 || skip > B.bytes || tail_len < 0 || (tail_len > 0 && !tail))
    return arg_fail(ctx, MH_E_ARG, "BAM part: skip or tail out of range");
  std::vector<int64_t> &boff = P.boff;
  int64_t nz = 0;
  struct Piece {
    int64_t off, len;
    hipEvent_t ev;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::vector<Piece> pieces;
  bool fin = false;
  // gz_out is sized for the whole BAM (GBs): released on every exit into the device block cache (the next job's
  // buffers, or the next file's gz_out, take it from there)
  struct Guard {
    mh_ctx *c;
    std::vector<Piece> *pc;
    ~Guard() {
      for (Piece &x : *pc)
        if (x.ev) (void)hipEventDestroy(x.ev);
      release(c->gz_out);   // (to the device block cache: the next file's output buffer)
    }
  } guard{ctx, &pieces};
  MH_TRY(gz_drain(ctx));
  const int64_t L = B.bytes - skip + tail_len;
  // a spilled (bounded) store deflates window by window into two ring slots; otherwise one buffer for the whole file
  const int64_t ring = B.spilled > 0 ? bgzf_device_bound(spill_window(B)) : 0;
  MH_TRY(ensure(ctx, ctx->gz_out, (size_t)(ring ? 2 * ring : bgzf_device_bound(L))));
  const int64_t SLOT_B = (int64_t)1 << 26;
  for (auto &p : ctx->h_bam_pin)
    if (!p) HIPCHK(ctx, hipHostMalloc((void **)&p, (size_t)SLOT_B, hipHostMallocDefault));
  uint8_t *const pin[2] = {ctx->h_bam_pin[0], ctx->h_bam_pin[1]};
  const uint8_t *z = (const uint8_t *)ctx->gz_out.p;
  std::atomic<int> werr{(int)hipSuccess};   // (set by either thread)
  std::string err;
  bool wrote = false, writer_done = false;
  size_t pieces_out = 0;   // pieces whose bytes have all been copied off the device (the ring's slots reuse them)
  int64_t data_pos = 0, end_pos = 0;
  const std::string no_header;
  std::thread writer([&]() {
    (void)hipSetDevice(ctx->device);
    size_t item = 0;
    int64_t in_item = 0;
    size_t slot_piece[2] = {0, 0};   // per staging slot: 1 + the piece its sub-piece ends, or 0
    // the next sub-piece (<= 64 MiB) of the queued pieces, waiting for the deflate to queue it
    auto take = [&](int64_t *o, int64_t *m, hipEvent_t *ev, size_t *ends) -> bool {
      std::unique_lock<std::mutex> lk(mu);
      for (;;) {
        while (item < pieces.size() && in_item >= pieces[item].len) {
          item++;
          in_item = 0;
        }
        if (item < pieces.size()) break;
        if (fin) return false;
        cv.wait(lk);
      }
      const Piece &p = pieces[item];
      *o = p.off + in_item;
      *m = std::min(SLOT_B, p.len - in_item);
      *ev = p.ev;
      in_item += *m;
      *ends = in_item >= p.len ? item + 1 : 0;
      return true;
    };
    auto issue = [&](int s, int64_t *len) -> bool {   // a copy into slot s on stream2, behind its piece's pack
      int64_t o, m;
      hipEvent_t ev;
      if (!take(&o, &m, &ev, &slot_piece[s])) return false;
      hipError_t e = hipStreamWaitEvent(ctx->stream2, ev, 0);
      if (e == hipSuccess) e = hipMemcpyAsync(pin[s], z + o, (size_t)m, hipMemcpyDeviceToHost, ctx->stream2);
      if (e != hipSuccess) {
        werr = (int)e;
        return false;
      }
      *len = m;
      return true;
    };
    int cur = 0;
    int64_t len_cur = 0, len_next = 0;
    bool have = issue(0, &len_cur);
    auto next = [&](const uint8_t **buf, int64_t *len) -> bool {
      if (!have || werr.load() != (int)hipSuccess) return false;
      hipError_t e = hipStreamSynchronize(ctx->stream2);   // slot cur is in (and nothing else is in flight)
      if (e != hipSuccess) {
        werr = (int)e;
        return false;
      }
      const int s = cur;
      if (slot_piece[s]) {   // that piece's last bytes are off the device: its ring space may be refilled
        std::lock_guard<std::mutex> lk(mu);
        pieces_out = std::max(pieces_out, slot_piece[s]);
        cv.notify_all();
      }
      *buf = pin[s];
      *len = len_cur;
      have = issue(s ^ 1, &len_next);   // the following sub-piece into the other slot, while this one is written
      len_cur = len_next;
      cur = s ^ 1;
      return true;
    };
    wrote = bgzf_write_stream(path, hdr ? *hdr : no_header, 6, next, &data_pos, &end_pos, err, eof);
    if (!wrote) {   // drain what is in flight before the slots go
      (void)hipStreamSynchronize(ctx->stream2);
    }
    std::lock_guard<std::mutex> lk(mu);
    writer_done = true;
    cv.notify_all();
  });
  const std::function<void(int64_t, int64_t)> on_piece = [&](int64_t off, int64_t bytes) {
    hipEvent_t ev = nullptr;
    if (hipEventCreateWithFlags(&ev, hipEventDisableTiming) != hipSuccess ||
        hipEventRecord(ev, ctx->stream) != hipSuccess) {
      if (ev) (void)hipEventDestroy(ev);
      ev = nullptr;
    }
    std::lock_guard<std::mutex> lk(mu);
    pieces.push_back(Piece{off, ev ? bytes : 0, ev});
    if (!ev) werr = (int)hipErrorUnknown;
    cv.notify_all();
  };
  std::vector<size_t> win_end;   // win_end[i]: pieces queued before window i
  const std::function<int32_t(int64_t)> slot_free = [&](int64_t i) -> int32_t {
    std::unique_lock<std::mutex> lk(mu);
    win_end.push_back(pieces.size());
    if (i < 2) return MH_OK;
    const size_t need = win_end[(size_t)i - 1];   // every piece of windows <= i - 2
    cv.wait(lk, [&] { return pieces_out >= need || writer_done || werr.load() != (int)hipSuccess; });
    if (pieces_out < need) return arg_fail(ctx, MH_E_STATE, "BAM writer stopped before the deflate ring drained");
    return MH_OK;
  };
  int32_t rc = MH_OK;
  if (B.spilled > 0) {
    rc = bam_deflate_spilled(ctx, ring, skip, tail, tail_len, &nz, &boff, on_piece, slot_free);
  } else {
    // the tail after the sorted records (srecs keeps its bytes), then one deflate of [skip, bytes + tail_len)
    if (tail_len > 0) {
      rc = ensure_keep(ctx, B.srecs, (size_t)(B.bytes + tail_len + 64), (size_t)B.bytes);
      if (rc == MH_OK &&
          hipMemcpyAsync((uint8_t *)B.srecs.p + B.bytes, tail, (size_t)tail_len, hipMemcpyHostToDevice, ctx->stream) !=
              hipSuccess)
        rc = hip_fail(ctx, hipGetLastError(), "BAM part tail H2D", __FILE__, __LINE__);
    }
    if (rc == MH_OK)
      rc = bgzf_device(ctx, ctx->stream, (const uint8_t *)B.srecs.p + skip, L, (uint8_t *)ctx->gz_out.p,
                       (int64_t)ctx->gz_out.cap, &nz, &boff, &on_piece);
  }
  {
    std::lock_guard<std::mutex> lk(mu);
    fin = true;
    cv.notify_all();
  }
  writer.join();
  if (rc != MH_OK) return rc;
  if (werr.load() != (int)hipSuccess) return hip_fail(ctx, (hipError_t)werr.load(), "BAM D2H", __FILE__, __LINE__);
  if (!wrote) return arg_fail(ctx, MH_E_ARG, err);
  if (end_pos - data_pos != nz) return arg_fail(ctx, MH_E_STATE, "BAM: compressed bytes written differ (internal)");
  P.data_pos = data_pos;
  P.end_pos = end_pos;
  P.nz = nz;
  return MH_OK;
}

extern "C" {

int32_t mh_bam_write_gpu(mh_ctx *ctx, const char *bam_path, const char *header_text, int64_t header_len,
                         const char *bai_path, int64_t *out_records, int64_t *out_bytes, int64_t *out_file_bytes) {
  CTX_GUARD(ctx);
  BamStore &B = ctx->bam;
  if (!bam_path || (header_len > 0 && !header_text)) return arg_fail(ctx, MH_E_ARG, "null argument");
  if (!B.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  MH_TRY(bam_sort(ctx));
  const int64_t n = B.n_rec;
  // the BAI's per-record half on the device (chunks and linear windows; only their offsets cross PCIe)
  BaiPlan plan;
  std::vector<int64_t> offs;
  bool dev_plan = false;
  if (bai_path) MH_TRY(bam_bai_plan(ctx, plan, offs, &dev_plan));
  const std::string hdr = bam_header_bytes(std::string(header_text ? header_text : "", (size_t)header_len),
                                           B.ref_names, B.ref_len);
  BamPart P;
  MH_TRY(bam_write_gpu_impl(ctx, bam_path, &hdr, 0, nullptr, 0, true, P));
  std::vector<int64_t> coff(P.boff.size());
  for (size_t b = 0; b < P.boff.size(); b++) coff[b] = P.data_pos + P.boff[b];
  std::string err;
  if (bai_path) {
    if (dev_plan) {
      if (!bai_emit(bai_path, plan, offs.data(), coff, err)) return arg_fail(ctx, MH_E_ARG, err);
    } else {   // outside the device plan's checks: the host plan (and its errors)
      std::vector<int64_t> soff((size_t)n + 1, 0);
      std::vector<BaiRec> info((size_t)n + 1);
      MH_TRY(bam_fetch_sorted(ctx, nullptr, soff.data(), (int32_t *)info.data()));
      if (!bai_write(bai_path, (int32_t)B.ref_names.size(), n, info.data(), soff.data(), coff, err))
        return arg_fail(ctx, MH_E_ARG, err);
    }
  }
  if (out_records) *out_records = n;
  if (out_bytes) *out_bytes = B.bytes;
  if (out_file_bytes) *out_file_bytes = P.end_pos + 28;
  return MH_OK;
}

int32_t mh_bam_write_part(mh_ctx *ctx, const char *path, const char *header_text, int64_t header_len, int64_t skip,
                          const uint8_t *tail, int64_t tail_len, int32_t eof, int64_t *out_blocks, int64_t *out_data_pos,
                          int64_t *out_bytes, int64_t *boff, int64_t boff_cap) {
  CTX_GUARD(ctx);
  BamStore &B = ctx->bam;
  if (!path || !out_blocks || !out_data_pos || !out_bytes || (header_len > 0 && !header_text))
    return arg_fail(ctx, MH_E_ARG, "null argument");
  if (!B.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  std::string hdr;
  if (header_len >= 0)
    hdr = bam_header_bytes(std::string(header_text ? header_text : "", (size_t)header_len), B.ref_names, B.ref_len);
  BamPart P;
  MH_TRY(bam_write_gpu_impl(ctx, path, header_len >= 0 ? &hdr : nullptr, skip, tail, tail_len, eof != 0, P));
  const int64_t nb = (int64_t)P.boff.size() - 1;
  *out_blocks = nb;
  *out_data_pos = P.data_pos;
  *out_bytes = P.end_pos + (eof ? 28 : 0);
  if (boff) {
    if (boff_cap < nb + 1) return arg_fail(ctx, MH_E_CAPACITY, "block offset array too small");
    std::memcpy(boff, P.boff.data(), 8 * (size_t)(nb + 1));
  }
  return MH_OK;
}

int32_t mh_bam_partition(mh_ctx *ctx, const uint64_t *splitters, int32_t n_dest, uint64_t tie_base, int64_t *seg_off,
                         int64_t *seg_n, int64_t *seg_bytes) {
  CTX_GUARD(ctx);
  if (n_dest < 1 || (n_dest > 1 && !splitters) || !seg_off || !seg_n || !seg_bytes)
    return arg_fail(ctx, MH_E_ARG, "null argument");
  if (!ctx->bam.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  return bam_partition(ctx, splitters, n_dest, tie_base, seg_off, seg_n, seg_bytes);
}

int32_t mh_bam_partition_fetch(mh_ctx *ctx, void *out, int64_t cap) {
  CTX_GUARD(ctx);
  BamStore &B = ctx->bam;
  if ((!out && B.send_bytes > 0) || cap < B.send_bytes) return arg_fail(ctx, MH_E_CAPACITY, "partition buffer too small");
  if (B.send_bytes > 0) HIPCHK(ctx, hipMemcpyAsync(out, B.send.p, (size_t)B.send_bytes, hipMemcpyDefault, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

int32_t mh_bam_import_tie(mh_ctx *ctx, const uint8_t *recs, const int64_t *roff, const uint64_t *keys,
                          const int32_t *info, const uint64_t *ties, int64_t n) {
  CTX_GUARD(ctx);
  if (n < 0 || (n > 0 && (!roff || !keys || !info || !ties))) return arg_fail(ctx, MH_E_ARG, "null argument");
  return bam_import(ctx, recs, roff, keys, info, n, ties);
}

int32_t mh_bam_sorted_head(mh_ctx *ctx, int64_t len, uint8_t *out) {
  CTX_GUARD(ctx);
  BamStore &B = ctx->bam;
  if (len < 0 || len > B.bytes || (len > 0 && !out)) return arg_fail(ctx, MH_E_ARG, "bad head length");
  MH_TRY(bam_sort(ctx));
  if (len == 0) return MH_OK;
  if (B.spilled > 0) {
    MH_TRY(bam_spill(ctx));
    MH_TRY(bam_sort(ctx));
    BamHostOrder o;
    MH_TRY(bam_host_order(ctx, o));
    bam_assemble(B, o, 0, len, out, 4);
    return MH_OK;
  }
  HIPCHK(ctx, hipMemcpyAsync(out, B.srecs.p, (size_t)len, hipMemcpyDeviceToHost, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

int32_t mh_bam_bai_runs(mh_ctx *ctx, int64_t *n_runs, int64_t *runs, int64_t runs_cap, int64_t *n_win, int64_t *win,
                        int64_t win_cap, int64_t *ref_nwin) {
  CTX_GUARD(ctx);
  BamStore &B = ctx->bam;
  if (!n_runs || !n_win) return arg_fail(ctx, MH_E_ARG, "null argument");
  MH_TRY(bam_sort(ctx));
  std::vector<int64_t> hr, hw, woff;
  std::vector<uint32_t> hn;
  bool ok = false;
  MH_TRY(bam_bai_raw(ctx, hr, hw, hn, woff, &ok));
  if (!ok) return arg_fail(ctx, MH_E_STATE, "BAI plan: records outside the references' lengths or not sorted");
  *n_runs = (int64_t)hr.size() / 4;
  *n_win = (int64_t)hw.size();
  if (!runs || !win || !ref_nwin) return MH_OK;   // (the sizes only)
  if (runs_cap < (int64_t)hr.size() || win_cap < (int64_t)hw.size()) return arg_fail(ctx, MH_E_CAPACITY, "BAI arrays");
  std::memcpy(runs, hr.data(), 8 * hr.size());
  std::memcpy(win, hw.data(), 8 * hw.size());
  for (size_t t = 0; t < hn.size(); t++) ref_nwin[t] = hn[t];
  (void)B;
  return MH_OK;
}

int32_t mh_corrupt_fastq(mh_ctx *ctx, const char *fq1, int64_t len1, const char *fq2, int64_t len2, int64_t t_base,
                         int64_t *used1, int64_t *used2, int64_t *templates) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if (!fq1 || len1 < 0 || (fq2 && len2 < 0) || t_base < 0 || !used1 || !used2 || !templates)
    return arg_fail(ctx, MH_E_ARG, "null argument");
  MH_TRY(stage_in(ctx, ctx->bam.in1, fq1, len1));
  if (fq2) MH_TRY(stage_in(ctx, ctx->bam.in2, fq2, len2));
  return corrupt_fastq(ctx, (const uint8_t *)ctx->bam.in1.p, len1, fq2 ? (const uint8_t *)ctx->bam.in2.p : nullptr,
                       fq2 ? len2 : 0, t_base, used1, used2, templates);
}

int32_t mh_bam_sort(mh_ctx *ctx) {
  CTX_GUARD(ctx);
  if (!ctx->bam.refs_set) return arg_fail(ctx, MH_E_STATE, "call mh_bam_set_refs first");
  return bam_sort(ctx);
}

int32_t mh_bam_set_spill_dir(mh_ctx *ctx, const char *dir) {
  if (!ctx) return MH_E_ARG;
  ctx->bam.spill_dir = dir ? dir : "";
  return MH_OK;
}

int32_t mh_bam_set_capacity(mh_ctx *ctx, int64_t bytes) {
  if (!ctx) return MH_E_ARG;
  if (bytes < 0) return arg_fail(ctx, MH_E_ARG, "capacity must be >= 0");
  ctx->bam.cap = bytes;
  return MH_OK;
}

int32_t mh_bam_reset(mh_ctx *ctx) {
  if (!ctx) return MH_E_ARG;
  bam_free_spill(ctx->bam);
  ctx->bam.n_rec = ctx->bam.bytes = 0;
  ctx->bam.n_files = 0;
  ctx->bam.sorted = false;
  ctx->bam.direct = false;
  ctx->bam.use_tie = false;
  return MH_OK;
}

}  // extern "C"

// ---- device BGZF (mh_deflate.hip) ----
int32_t mh_bgzf_compress_device(mh_ctx *ctx, const void *d_in, int64_t len, void *d_out, int64_t cap,
                                int64_t *used) {
  CTX_GUARD(ctx);
  if ((!d_in && len > 0) || len < 0 || !d_out || !used) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  return bgzf_device(ctx, ctx->stream, (const uint8_t *)d_in, len, (uint8_t *)d_out, cap, used);
}

int32_t mh_bgzf_compress_gpu(mh_ctx *ctx, const char *in, int64_t len, char *out, int64_t cap, int64_t *used) {
  CTX_GUARD(ctx);
  if ((!in && len > 0) || len < 0 || !out || !used) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  *used = 0;
  if (len == 0) return MH_OK;
  MH_TRY(gz_drain(ctx));
  MH_TRY(ensure(ctx, ctx->gz_in, (size_t)len + 64));
  MH_TRY(ensure(ctx, ctx->gz_out, (size_t)bgzf_device_bound(len)));
  HIPCHK(ctx, hipMemcpyAsync(ctx->gz_in.p, in, len, hipMemcpyHostToDevice, ctx->stream));
  int64_t u = 0;
  MH_TRY(bgzf_device(ctx, ctx->stream, (const uint8_t *)ctx->gz_in.p, len, (uint8_t *)ctx->gz_out.p,
                     (int64_t)ctx->gz_out.cap, &u));
  if (u > cap) {
    *used = u;
    return arg_fail(ctx, MH_E_CAPACITY, "output buffer too small");
  }
  HIPCHK(ctx, hipMemcpyAsync(out, ctx->gz_out.p, u, hipMemcpyDeviceToHost, ctx->stream));
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  *used = u;
  return MH_OK;
}

int32_t mh_output_bgzf_range(mh_ctx *ctx, int32_t file, int64_t offset, int64_t len, char *out, int64_t cap,
                             int64_t *used) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if ((file != 0 && file != 1) || !used || offset < 0 || len < 0) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  MH_TRY(sync_writers(ctx));   // the writers (and corruption passes) of the arena's last units
  const int64_t n = file ? ctx->used2 : ctx->used1;
  if (offset > n || len > n - offset) return arg_fail(ctx, MH_E_ARG, "range outside the arena");
  const uint8_t *src = (const uint8_t *)(file ? ctx->out2.p : ctx->out1.p) + offset;
  *used = 0;
  if (len == 0) return MH_OK;
  MH_TRY(gz_drain(ctx));
  MH_TRY(ensure(ctx, ctx->gz_out, (size_t)bgzf_device_bound(len)));
  int64_t u = 0;
  stage_begin(ctx, "bgzf_deflate");
  MH_TRY(bgzf_device(ctx, ctx->stream, src, len, (uint8_t *)ctx->gz_out.p, (int64_t)ctx->gz_out.cap, &u));
  stage_end(ctx);
  *used = u;
  if (!out) return MH_OK;   // (the size only)
  if (u > cap) return arg_fail(ctx, MH_E_CAPACITY, "output buffer too small");
  stage_begin(ctx, "bgzf_d2h");
  HIPCHK(ctx, hipMemcpyAsync(out, ctx->gz_out.p, u, hipMemcpyDeviceToHost, ctx->stream));
  stage_end(ctx);
  SYNCCHK(ctx, hipStreamSynchronize(ctx->stream));
  return MH_OK;
}

int32_t mh_output_bgzf_pair(mh_ctx *ctx, int64_t offset, int64_t n1, int64_t n2, char *out1, int64_t cap1,
                            char *out2, int64_t cap2, int64_t *used1, int64_t *used2, int32_t *ticket) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if (!used1 || !used2 || !ticket || offset < 0 || n1 < 0 || n2 < 0 || (n1 && !out1) || (n2 && !out2))
    return arg_fail(ctx, MH_E_ARG, "bad arguments");
  MH_TRY(sync_writers(ctx));   // the writers (and corruption passes) of the arena's last units
  if ((n1 && offset + n1 > ctx->used1) || (n2 && offset + n2 > ctx->used2))
    return arg_fail(ctx, MH_E_ARG, "range outside the arena");
  *used1 = *used2 = 0;
  *ticket = -1;
  const int64_t b1 = n1 ? bgzf_device_bound(n1) : 0, b2 = n2 ? bgzf_device_bound(n2) : 0;
  const int64_t need = (b1 + b2 + 255) & ~(int64_t)255;
  if (need == 0) return MH_OK;
  for (int h = 0; h < 2; h++)
    if (!ctx->ev_gz[h]) HIPCHK(ctx, hipEventCreateWithFlags(&ctx->ev_gz[h], hipEventDisableTiming));
  if ((int64_t)ctx->gz_out.cap / 2 < need) {   // (growing frees the old halves: their copies first)
    SYNCCHK(ctx, hipStreamSynchronize(ctx->stream2));
    ctx->gz_pending[0] = ctx->gz_pending[1] = false;
    MH_TRY(ensure(ctx, ctx->gz_out, 2 * (size_t)need));
  }
  const int h = ctx->gz_half;
  if (ctx->gz_pending[h]) {   // the call two back copied out of this half
    SYNCCHK(ctx, hipEventSynchronize(ctx->ev_gz[h]));
    ctx->gz_pending[h] = false;
  }
  uint8_t *base = (uint8_t *)ctx->gz_out.p + (size_t)h * (ctx->gz_out.cap / 2);
  const uint8_t *src[2] = {(const uint8_t *)ctx->out1.p + offset, (const uint8_t *)ctx->out2.p + offset};
  const int64_t nn[2] = {n1, n2}, cap[2] = {cap1, cap2}, off[2] = {0, b1};
  char *out[2] = {out1, out2};
  int64_t *used[2] = {used1, used2};
  for (int f = 0; f < 2; f++) {
    if (nn[f] == 0) continue;
    int64_t u = 0;
    stage_begin(ctx, "bgzf_deflate");
    MH_TRY(bgzf_device(ctx, ctx->stream, src[f], nn[f], base + off[f], f ? b2 : b1, &u));
    stage_end(ctx);
    if (u > cap[f]) {
      SYNCCHK(ctx, hipStreamSynchronize(ctx->stream2));
      return arg_fail(ctx, MH_E_CAPACITY, "output buffer too small");
    }
    *used[f] = u;
    // the copy behind the deflate on the second stream: it overlaps the next deflate
    HIPCHK(ctx, hipEventRecord(ctx->ev_fork, ctx->stream));
    HIPCHK(ctx, hipStreamWaitEvent(ctx->stream2, ctx->ev_fork, 0));
    ctx->stage_stream = ctx->stream2;
    stage_begin(ctx, "bgzf_d2h");
    HIPCHK(ctx, hipMemcpyAsync(out[f], base + off[f], (size_t)u, hipMemcpyDeviceToHost, ctx->stream2));
    stage_end(ctx);
    ctx->stage_stream = nullptr;
  }
  HIPCHK(ctx, hipEventRecord(ctx->ev_gz[h], ctx->stream2));
  ctx->gz_pending[h] = true;
  ctx->gz_half = h ^ 1;
  *ticket = h;
  return MH_OK;
}

int32_t mh_output_bgzf_wait(mh_ctx *ctx, int32_t ticket) {
  CTX_GUARD_EMIT(ctx);
  if (ticket < 0) return MH_OK;
  if (ticket > 1) return arg_fail(ctx, MH_E_ARG, "bad ticket");
  if (ctx->gz_pending[ticket]) {
    SYNCCHK(ctx, hipEventSynchronize(ctx->ev_gz[ticket]));
    ctx->gz_pending[ticket] = false;
  }
  return MH_OK;
}

int32_t mh_output_bgzf(mh_ctx *ctx, int32_t file, char *out, int64_t cap, int64_t *used) {
  CTX_GUARD(ctx);
  MH_TRY(lazy_resolve(ctx));
  if ((file != 0 && file != 1) || !used) return arg_fail(ctx, MH_E_ARG, "bad arguments");
  return mh_output_bgzf_range(ctx, file, 0, file ? ctx->used2 : ctx->used1, out, cap, used);
}
