// api.hip — libbrickrec C-ABI: index handle, uploads, batched search, cross-shard finalize.
//
// Search pipeline per query chunk (all stream-ordered, no host sync unless results are host):
//   prep (normalise / gather / copy query rows)
//   for each side (content/semantic = cosine over the item matrix; CF = u·F):
//     for each item slab:  gemm (MFMA score slab) -> select (exact top-K_int, carried list)
//   finalize (rank-0 drop, truncation, hybrid union-blend) -> scores / ids / counts
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_set>
#include <vector>

#include "../../include/brickrec.h"
#include "common.h"
#include "list_epi.h"
#include "sq.h"

#include <cmath>
#include <cstdlib>

using namespace bb;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define BB_HIP(expr)                                                                         \
  do {                                                                                       \
    hipError_t e__ = (expr);                                                                 \
    if (e__ != hipSuccess)                                                                   \
      return fail(BB_E_HIP, std::string(#expr) + ": " + hipGetErrorString(e__));           \
  } while (0)

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }
size_t elem_size(int dtype) { return dtype == F64 ? 8 : dtype == BF16 ? 2 : 4; }

// K_RERUN counts searches the streaming path handed back to the slab path (no kernel time)
enum Kfam { K_PREP = 0, K_GEMM = 1, K_SELECT = 2, K_FIN = 3, K_MASK = 4, K_RERUN = 5, K_RERANK = 6, K_PACK = 7, K_NFAM = 8 };
const char* kFamNames[K_NFAM] = {"prep", "gemm", "select", "finalize", "mask", "rerun", "rerank", "pack"};

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  bool owned = true;  // false: an alias of another handle's buffer (bb_create_view)
  int ensure(size_t bytes) {
    if (bytes <= cap) return BB_OK;
    if (!owned) return fail(BB_E_STATE, "a view cannot resize its base's buffers");
    // a plan being recorded keeps every pointer it captured: no buffer may move under it
    if (p && tl_capture) return fail(BB_E_STATE, "bb_plan_create: a workspace buffer regrew within the search");
    if (p) {
      hipError_t e = hipFree(p);
      if (e != hipSuccess) return fail(BB_E_HIP, std::string("hipFree: ") + hipGetErrorString(e));
      p = nullptr;
      cap = 0;
    }
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {
      p = nullptr;
      return fail(BB_E_NOMEM, "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    }
    cap = bytes;
    return BB_OK;
  }
  void release() {
    if (p && owned) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    owned = true;
  }
};

// Live handles (bb_create / bb_create_view / bb_plan_create add, bb_destroy / bb_plan_destroy
// remove): every entry point checks its handle here before touching it, so a destroyed, foreign
// or corrupted pointer returns BB_E_ARG instead of crashing the caller's process (ADVICE / VERDICT
// r04: a use-after-free reached bb_search from a dropped Python view).  The magic word is
// checked only after the set says the pointer is ours (a freed pointer is never dereferenced).
constexpr uint64_t kIndexMagic = 0x3130786469626262ull;  // "bbbidx01"
constexpr uint64_t kPlanMagic = 0x31306e616c706262ull;   // "bbplan01"
std::mutex g_live_mu;
std::unordered_set<const void*> g_live;

void live_add(const void* p) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  g_live.insert(p);
}
bool live_del(const void* p) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  return g_live.erase(p) != 0;
}
template <typename H>
bool live_has_magic(const H* p, uint64_t magic) {
  std::lock_guard<std::mutex> lk(g_live_mu);
  return g_live.count(p) != 0 && p->magic == magic;
}

}  // namespace

struct bb_index {
  uint64_t magic = kIndexMagic;
  int device = 0;
  int dtype = F32;
  int64_t id_offset = 0;
  int64_t ws_cap = 512ll << 20;
  bool ws_set = false;                 // ws_cap set by the caller (desc / BB_OPT_WORKSPACE_BYTES)
  int stream_opt = -1;                 // BB_OPT_STREAM
  int64_t stream_min_items = 100000;   // BB_OPT_STREAM_MIN_ITEMS
  int refine_opt = -1;                 // BB_OPT_STREAM_REFINE
  int lists_opt = -1;                  // BB_OPT_RR_LISTS
  int sq_opt = -1;                     // BB_OPT_SMALL_BATCH
  int prefilter_opt = -1;              // BB_OPT_PREFILTER
  bb_index* base = nullptr;            // a view (bb_create_view): the handle owning the rows
  std::atomic<int> n_views{0};         // views of this handle still alive
  hipStream_t stream = nullptr;
  std::mutex mu;
  // Cross-stream ordering of the shared workspace: every call records `done` on the stream it
  // ran on; a call arriving on a different stream first waits for that event, so two calls
  // on two streams never overlap on the same scratch buffers.
  hipEvent_t done = nullptr;
  hipStream_t last_stream = nullptr;
  bool has_last = false;

  int64_t n = 0, Npad = 0;
  int d = 0, Dpad = 0;
  DevBuf items, items_present;
  DevBuf ones, zeros;  // all-ones / all-zeros bitsets standing in for 'no mask' / 'no exclusions'
  int r = 0, Rpad = 0;
  DevBuf cf, cf_present;
  DevBuf items3, cf3;  // f32 index: the same rows as three bf16 planes (split scan, scan3)
  // f32 index: one-product bf16 copies for the approximate scan of the exact re-rank path
  // ([Npad][Dpad_b] / [Npad][Rpad_b]) and their error statistics (rr_prepare_kernel)
  DevBuf items_bf, cf_bf, rr_stats;
  int Dpad_b = 0, Rpad_b = 0;
  DevBuf parts, year, theme;

  // workspace
  DevBuf qn, qcf, S, tmax, keys, maxk, stage_in, out_sc, out_id, out_cnt, tmp;
  DevBuf qf32, qeps, qcf32, qcfeps;  // re-rank: f32 query rows and per-query bounds
  DevBuf qh, qcfh;                   // re-rank: per-query quanta of the int16 score image
  DevBuf rr_out, rr_cnt, rr_thr, rr_r0, rr_r0n;  // re-rank: select -> rerank hand-off
  // streaming top-K (large indexes): pilot lists, candidate regions, overflow flag
  DevBuf pilot, cand, cand_cnt, cand_pmax;
  DevBuf pilot_top;  // kScanPilot scans: per lane the top-m half-tile maxima of the pilot rows
  DevBuf trace;        // BB_SELECT_TRACE probe stamps
  DevBuf rr_flags;     // one-wave re-rank select: rows left to the block select
  DevBuf list1, max1;  // two-level streaming: exact top-K_int (+ rank-0 key) of items [0, n1)
  DevBuf lists, r0lists;  // bounded candidate lists of the list scans (list_epi.h), both sides
  DevBuf sq_top, sq_ptop, sq_ords;  // small-batch exact search (sq.hip)
  uint32_t* ovf_host = nullptr;  // pinned
  // constraint-first search (compact.hip): the rank-0 key of every item's own row (its
  // unmasked arg-max, :217; [n] = a zero row's), built at upload for f32 indexes of up to
  // 65,536 rows, and the packed shadow index a selective mask's rows are gathered into
  DevBuf r0key;
  bool r0_ready = false;
  bb_index* cx = nullptr;          // the shadow (owned; not a live handle)
  bool shadow = false;             // this index is a shadow: no rank-0 drop, final ids via idmap
  DevBuf idmap, cexcl0, cexcl1;           // shadow: slot -> id, content / CF exclusions
  const uint32_t* cur_cexcl = nullptr;    // shadow: the content exclusions of this search
  bb::CompactArgs cjob{};                 // shadow: the packing launch, issued in place of its prep
  bool cjob_set = false;
  size_t filled_words = 0;                // shadow: words of ones / zeros filled

  bool prof = false;
  struct Pending {
    int fam;
    hipEvent_t a, b;
  };
  std::vector<Pending> pending;
  double ms[K_NFAM] = {0};
  int64_t launches[K_NFAM] = {0};
};

// A prepared search (bb_plan_create): the launches of one recorded search, replayed as they
// are.  It owns a private view of the index (own stream, own workspace) so no other call can
// move or overwrite the buffers its launches were recorded with.
struct bb_plan {
  uint64_t magic = kPlanMagic;
  bb_index* view = nullptr;
  int device = 0;
  hipStream_t s = nullptr;
  // launches of one plan from several threads are serialised by mu (two replays'
  // launches interleaved on one stream would let one overwrite the other's scratch between
  // producer and consumer).  Destroy waits for the plan's stream s only (the caller keeps it
  // valid until then, include/brickrec.h), not for the device.  (An event recorded after each
  // replay instead cost +2.7 us per one-query plan, r06g: similar_k10 19.8 -> 22.4 us.)
  std::mutex mu;
  std::vector<bb::CapturedOp> ops;
  std::vector<std::vector<void*>> argv;  // per launch: pointers into its argument blob
};

namespace {

// Every device buffer and profiling event of a handle (bb_destroy; a shadow index's too).
void free_buffers(bb_index* x) {
  for (auto& p : x->pending) {
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  x->pending.clear();
  for (DevBuf* b : {&x->items, &x->items_present, &x->ones, &x->zeros, &x->cf, &x->cf_present, &x->parts, &x->year, &x->theme, &x->qn, &x->qcf, &x->S, &x->tmax,
                    &x->keys, &x->maxk, &x->stage_in, &x->out_sc, &x->out_id, &x->out_cnt, &x->tmp, &x->pilot, &x->list1, &x->max1,
                    &x->cand, &x->cand_cnt, &x->cand_pmax, &x->items3, &x->cf3, &x->items_bf, &x->cf_bf,
                    &x->rr_stats, &x->qf32, &x->qeps, &x->qcf32, &x->qcfeps, &x->qh, &x->qcfh, &x->rr_out, &x->rr_cnt,
                    &x->rr_thr, &x->rr_r0, &x->rr_r0n, &x->trace, &x->rr_flags, &x->lists, &x->r0lists, &x->pilot_top,
                    &x->sq_top, &x->sq_ptop, &x->sq_ords, &x->r0key, &x->idmap, &x->cexcl0, &x->cexcl1})
    b->release();
  if (x->ovf_host) (void)hipHostFree(x->ovf_host);
  x->ovf_host = nullptr;
}

// Handle checks of the entry points (see g_live above).
// The magic word is read while g_live_mu is held (a destroy removes the handle under the same
// lock before it frees anything).
int check_index(const bb_index* x, const char* fn) {
  if (!x) return fail(BB_E_ARG, std::string(fn) + ": null index");
  if (!live_has_magic(x, kIndexMagic))
    return fail(BB_E_ARG, std::string(fn) + ": stale or foreign index handle (destroyed, or not from bb_create)");
  return BB_OK;
}
#define BB_CHECK_INDEX(x, fn)                \
  do {                                       \
    const int rc__ = check_index((x), (fn)); \
    if (rc__) return rc__;                   \
  } while (0)

// Stream operations of a search: while a plan is recorded (tl_capture) the copies and fills
// join the record and a host synchronisation fails the plan (the streaming top-K reads its
// overflow flag on the host; host buffers are synchronised) — such searches stay bb_search's.
int s_memset(void* p, int v, size_t bytes, hipStream_t s) {
  if (tl_capture) {
    CapturedOp op;
    op.kind = 1;
    op.dst = p;
    op.value = v;
    op.bytes = bytes;
    tl_capture->push_back(std::move(op));
    return BB_OK;
  }
  BB_HIP(hipMemsetAsync(p, v, bytes, s));
  return BB_OK;
}
int s_copy(void* dst, const void* src, size_t bytes, hipMemcpyKind kind, hipStream_t s) {
  if (tl_capture) {
    if (kind != hipMemcpyDeviceToDevice) return fail(BB_E_HOSTSYNC, "bb_plan_create: the search copies to the host");
    CapturedOp op;
    op.kind = 2;
    op.dst = dst;
    op.src = src;
    op.bytes = bytes;
    tl_capture->push_back(std::move(op));
    return BB_OK;
  }
  BB_HIP(hipMemcpyAsync(dst, src, bytes, kind, s));
  return BB_OK;
}
// Host wait for the work queued on s.  BB_SPIN_WAIT (A/B): 1 polls hipStreamQuery, 2 polls
// and yields between polls, instead of hipStreamSynchronize's blocking wait.
hipError_t host_wait(hipStream_t s) {
  static const int mode = ab_env("BB_SPIN_WAIT") ? atoi(ab_env("BB_SPIN_WAIT")) : 0;
  if (!mode) return hipStreamSynchronize(s);
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    if (mode == 2) std::this_thread::yield();
  }
}

int s_sync(hipStream_t s) {
  if (tl_capture)
    return fail(BB_E_HOSTSYNC, "bb_plan_create: this search synchronises with the host (the streaming top-K of a large "
                            "index): use bb_search");
  BB_HIP(host_wait(s));
  return BB_OK;
}

struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev >= 0 && dev != prev) (void)hipSetDevice(dev);
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

// Order this call after the handle's previous call when that one ran on another stream.
int enter_stream(bb_index* x, hipStream_t s) {
  if (x->has_last && x->last_stream != s) BB_HIP(hipStreamWaitEvent(s, x->done, 0));
  return BB_OK;
}
// Mark the end of this call's work on s (the next call on another stream waits for it).
int leave_stream(bb_index* x, hipStream_t s) {
  BB_HIP(hipEventRecord(x->done, s));
  x->last_stream = s;
  x->has_last = true;
  return BB_OK;
}
// Entered stream of one call: leave() on success; on an early error return the destructor
// still records `done` on s, so work already queued there is covered and a later call on
// another stream waits for it.
struct StreamScope {
  bb_index* x = nullptr;
  hipStream_t s = nullptr;
  int enter(bb_index* xi, hipStream_t si) {
    const int rc = enter_stream(xi, si);
    if (rc == BB_OK) x = xi, s = si;
    return rc;
  }
  int leave() {
    bb_index* xi = x;
    x = nullptr;
    return xi ? leave_stream(xi, s) : BB_OK;
  }
  ~StreamScope() {
    if (x) (void)leave_stream(x, s);
  }
};

// Run a launcher with optional event bracketing for the profiler.
template <typename F>
int timed(bb_index* x, int fam, hipStream_t s, F&& launch) {
  hipEvent_t a = nullptr, b = nullptr;
  if (x->prof) {  // the family's kernels carry the events themselves (bb_launch, common.h)
    BB_HIP(hipEventCreate(&a));
    BB_HIP(hipEventCreate(&b));
    tl_launch_prof = LaunchProf{a, b};
  }
  hipError_t e = launch();
  const bool none = tl_launch_prof.start != nullptr;  // no kernel went out (a copy, or nothing)
  tl_launch_prof = LaunchProf{};
  if (e != hipSuccess) {
    if (a) (void)hipEventDestroy(a);
    if (b) (void)hipEventDestroy(b);
    return fail(BB_E_HIP, std::string("launch ") + kFamNames[fam] + ": " + hipGetErrorString(e));
  }
  if (x->prof) {
    if (none) {  // a zero-length interval, so the pair still reads
      BB_HIP(hipEventRecord(a, s));
      BB_HIP(hipEventRecord(b, s));
    }
    x->pending.push_back({fam, a, b});
    x->launches[fam] += 1;
  }
  return BB_OK;
}

// Copy `bytes` of a caller buffer to the device when it is a host pointer; returns the
// device-side pointer to use.
int to_device(bb_index* x, DevBuf& buf, size_t off, const void* src, size_t bytes, int where, hipStream_t s,
              const void** out) {
  if (!src || bytes == 0) {
    *out = src;
    return BB_OK;
  }
  if (where == BB_DEVICE) {
    *out = src;
    return BB_OK;
  }
  BB_HIP(hipMemcpyAsync((char*)buf.p + off, src, bytes, hipMemcpyHostToDevice, s));
  *out = (char*)buf.p + off;
  return BB_OK;
}

hipStream_t call_stream(bb_index* x, const bb_query* q) {
  return (q->flags & BB_Q_NULL_STREAM) ? (hipStream_t)0 : q->stream ? (hipStream_t)q->stream : x->stream;
}

int side_k_int(const bb_query* q, int32_t* sides, int32_t* k_int) {
  if (!q) return fail(BB_E_ARG, "null query");
  if (q->k <= 0) return fail(BB_E_ARG, "k must be > 0");
  const int ks = q->k_side > 0 ? q->k_side : 2 * q->k;
  switch (q->mode) {
    case BB_MODE_SEMANTIC:
    case BB_MODE_CF:
      *sides = 1;
      *k_int = q->k;
      break;
    case BB_MODE_SIMILAR:
      *sides = 1;
      *k_int = q->k + 1;
      break;
    case BB_MODE_HYBRID:
      *sides = 2;
      *k_int = ks + 1;
      break;
    default:
      return fail(BB_E_ARG, "unknown mode " + std::to_string(q->mode));
  }
  if (*k_int > kMaxKInt) return fail(BB_E_ARG, "k too large (internal list " + std::to_string(*k_int) +
                                                    " > " + std::to_string(kMaxKInt) + ")");
  return BB_OK;
}

}  // namespace

extern "C" {

const char* bb_last_error(void) { return g_err.c_str(); }
int bb_abi_version(void) { return BB_ABI_VERSION; }

int bb_create(const bb_desc* desc, bb_index** out) {
  if (!out) return fail(BB_E_ARG, "null out");
  *out = nullptr;
  int dev = desc ? desc->device : -1;
  if (dev < 0) BB_HIP(hipGetDevice(&dev));
  int ndev = 0;
  BB_HIP(hipGetDeviceCount(&ndev));
  if (dev >= ndev) return fail(BB_E_ARG, "device " + std::to_string(dev) + " out of range");
  const int dtype = desc ? desc->dtype : F32;
  if (dtype != F32 && dtype != BF16) return fail(BB_E_ARG, "index dtype must be BB_F32 or BB_BF16");
  DeviceGuard g(dev);
  bb_index* x = new bb_index();
  x->device = dev;
  x->dtype = dtype;
  x->id_offset = desc ? desc->id_offset : 0;
  if (desc && desc->workspace_bytes > 0) x->ws_cap = desc->workspace_bytes, x->ws_set = true;
  hipError_t e = hipStreamCreateWithFlags(&x->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    delete x;
    return fail(BB_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  e = hipEventCreateWithFlags(&x->done, hipEventDisableTiming);
  if (e != hipSuccess) {
    (void)hipStreamDestroy(x->stream);
    delete x;
    return fail(BB_E_HIP, std::string("hipEventCreate: ") + hipGetErrorString(e));
  }
  live_add(x);
  *out = x;
  return BB_OK;
}

int bb_create_view(bb_index* b, bb_index** out) {
  BB_CHECK_INDEX(b, "bb_create_view");
  if (!out) return fail(BB_E_ARG, "bb_create_view: null argument");
  *out = nullptr;
  if (b->base) return fail(BB_E_ARG, "bb_create_view: the base is itself a view");
  std::lock_guard<std::mutex> lk(b->mu);
  DeviceGuard g(b->device);
  BB_HIP(hipStreamSynchronize(b->stream));  // the base's uploads are complete
  bb_desc desc{b->device, b->dtype, b->id_offset, b->ws_set ? b->ws_cap : 0};
  bb_index* x = nullptr;
  int rc = bb_create(&desc, &x);
  if (rc) return rc;
  x->stream_opt = b->stream_opt;
  x->stream_min_items = b->stream_min_items;
  x->refine_opt = b->refine_opt;
  x->lists_opt = b->lists_opt;
  x->sq_opt = b->sq_opt;
  x->prefilter_opt = b->prefilter_opt;
  x->r0_ready = b->r0_ready;
  x->n = b->n;
  x->Npad = b->Npad;
  x->d = b->d;
  x->Dpad = b->Dpad;
  x->r = b->r;
  x->Rpad = b->Rpad;
  x->Dpad_b = b->Dpad_b;
  x->Rpad_b = b->Rpad_b;
  for (auto pr : {std::make_pair(&x->items, &b->items), std::make_pair(&x->items_present, &b->items_present),
                  std::make_pair(&x->ones, &b->ones), std::make_pair(&x->zeros, &b->zeros),
                  std::make_pair(&x->cf, &b->cf), std::make_pair(&x->cf_present, &b->cf_present),
                  std::make_pair(&x->items3, &b->items3), std::make_pair(&x->cf3, &b->cf3),
                  std::make_pair(&x->items_bf, &b->items_bf), std::make_pair(&x->cf_bf, &b->cf_bf),
                  std::make_pair(&x->rr_stats, &b->rr_stats), std::make_pair(&x->parts, &b->parts),
                  std::make_pair(&x->year, &b->year), std::make_pair(&x->theme, &b->theme),
                  std::make_pair(&x->r0key, &b->r0key)}) {
    pr.first->p = pr.second->p;
    pr.first->cap = pr.second->cap;
    pr.first->owned = false;
  }
  x->base = b;
  ++b->n_views;
  *out = x;
  return BB_OK;
}

int bb_destroy(bb_index* x) {
  if (!x) return BB_OK;
  // removal from the live set is the point of truth: of two concurrent destroys
  // one removes the handle and the other fails here without touching it
  if (!live_del(x))
    return fail(BB_E_ARG, "bb_destroy: stale or foreign index handle (destroyed, or not from bb_create)");
  {
    std::lock_guard<std::mutex> lk(x->mu);  // bb_create_view counts views under it
    if (x->n_views > 0) {
      live_add(x);
      return fail(BB_E_STATE, "bb_destroy: destroy the index's views (and plans) first");
    }
  }
  {
    DeviceGuard g(x->device);
    // a view's kernels read its base's rows: they finish before the base may be destroyed
    (void)hipStreamSynchronize(x->stream);
    if (x->has_last) (void)hipEventSynchronize(x->done);
  }
  if (x->base) {
    std::lock_guard<std::mutex> lk(x->base->mu);
    --x->base->n_views;
  }
  {
    DeviceGuard g(x->device);
    free_buffers(x);
    if (x->cx) {  // the shadow's kernels ran on x's streams, synchronised above
      free_buffers(x->cx);
      delete x->cx;
      x->cx = nullptr;
    }
    if (x->has_last) (void)hipEventSynchronize(x->done);
    (void)hipEventDestroy(x->done);
    (void)hipStreamDestroy(x->stream);
  }
  x->magic = 0;  // poisoned (the allocator may hand the memory out again)
  delete x;
  return BB_OK;
}

int bb_info(bb_index* x, int64_t* n_items, int32_t* d, int32_t* d_pad, int32_t* r) {
  BB_CHECK_INDEX(x, "bb_info");
  if (n_items) *n_items = x->n;
  if (d) *d = x->d;
  if (d_pad) *d_pad = x->Dpad;
  if (r) *r = x->r;
  return BB_OK;
}

int bb_get_rows(bb_index* x, const int64_t* ids, int32_t B, void* out, int32_t where) {
  BB_CHECK_INDEX(x, "bb_get_rows");
  if (!ids || !out || B <= 0) return fail(BB_E_ARG, "bb_get_rows: bad arguments");
  if (x->n <= 0) return fail(BB_E_STATE, "no items uploaded");
  std::lock_guard<std::mutex> lk(x->mu);
  DeviceGuard g(x->device);
  const size_t es = elem_size(x->dtype);
  const int bpad = (int)round_up(B, kTileRows);
  int rc;
  StreamScope scope;
  if ((rc = scope.enter(x, x->stream))) return rc;
  if ((rc = x->tmp.ensure((size_t)bpad * x->Dpad * es + (size_t)B * 8 + 256))) return rc;
  char* rows = (char*)x->tmp.p;
  const int64_t* d_ids = ids;
  if (where != BB_DEVICE) {
    int64_t* staged = (int64_t*)(rows + round_up((int64_t)bpad * x->Dpad * es, 256));
    BB_HIP(hipMemcpyAsync(staged, ids, (size_t)B * 8, hipMemcpyHostToDevice, x->stream));
    d_ids = staged;
  }
  PrepArgs pa{};
  pa.Bpad = bpad;
  pa.B = B;
  pa.d = x->d;
  pa.Dpad = x->Dpad;
  pa.out = rows;
  pa.out_dtype = x->dtype;
  pa.items = x->items.p;
  pa.n_items = x->n;
  pa.id_offset = x->id_offset;
  pa.item_ids = d_ids;
  BB_HIP(launch_prep(pa, x->stream));
  BB_HIP(hipMemcpy2DAsync(out, (size_t)x->d * es, rows, (size_t)x->Dpad * es, (size_t)x->d * es, B,
                          where == BB_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, x->stream));
  BB_HIP(hipStreamSynchronize(x->stream));
  return scope.leave();
}

// Upload rows (host or device) in chunks through the staging buffer and convert them into
// dst (Npad × ldst, index dtype), normalising when asked.
static int upload_rows(bb_index* x, const void* rows, int64_t n, int32_t d, int32_t in_dtype, int normalize,
                       int where, void* dst, int64_t ldst) {
  const size_t es = elem_size(in_dtype);
  const size_t row_bytes = (size_t)d * es;
  const int64_t chunk = std::max<int64_t>(1, (int64_t)((256ull << 20) / row_bytes));
  if (where == BB_HOST) {
    int rc = x->tmp.ensure(std::min<int64_t>(chunk, n) * row_bytes);
    if (rc) return rc;
  }
  for (int64_t r0 = 0; r0 < n; r0 += chunk) {
    const int64_t nr = std::min(chunk, n - r0);
    const void* src = (const char*)rows + (size_t)r0 * row_bytes;
    if (where == BB_HOST) {
      BB_HIP(hipMemcpyAsync(x->tmp.p, src, nr * row_bytes, hipMemcpyHostToDevice, x->stream));
      src = x->tmp.p;
    }
    char* d0 = (char*)dst + (size_t)r0 * ldst * elem_size(x->dtype);
    BB_HIP(launch_convert_rows(src, in_dtype, nr, d, normalize, d0, x->dtype, ldst, x->stream));
  }
  BB_HIP(hipStreamSynchronize(x->stream));
  return BB_OK;
}

// f32 index: keep a three-plane bf16 copy of the rows for the split-precision scan
// (scan3_kernel.h) when its width is supported; the f32 rows stay for everything else.
static int make_planes(bb_index* x, DevBuf& rows, DevBuf& planes, int ld) {
  if (x->dtype != F32 || !scan3_supported(kTileRows, ld)) {
    planes.release();
    return BB_OK;
  }
  int rc = planes.ensure((size_t)x->Npad * 3 * ld * 2);
  if (rc) return rc;
  BB_HIP(launch_split_planes((const float*)rows.p, x->Npad, ld, (uint16_t*)planes.p, x->stream));
  BB_HIP(hipStreamSynchronize(x->stream));
  return BB_OK;
}

// f32 index: the one-product f16 copy + error statistics for the exact re-rank path (the
// approximate f16 MFMA scan, then the f32 rescoring of the candidates within its bound; f16
// keeps 11 significant bits to bf16's 8, so the bound and the candidate windows are ~1/8 as
// wide: at configs[1] ~55 rescored rows per query for K = 51 instead of ~92).  stat_off: 0 =
// item rows, 4 = CF factors.  Widths the 16-bit scan or the re-rank cannot take leave the
// copy unset (those searches run the split-precision scan instead).
static int make_rr(bb_index* x, DevBuf& rows, DevBuf& bf, int ld, int& ld_b, int stat_off) {
  ld_b = (int)round_up(ld, 64);
  if (x->dtype != F32 || ld > kRrMaxD || !gemm_uses_scan(BF16, kTileRows, ld_b)) {
    bf.release();
    ld_b = 0;
    return BB_OK;
  }
  int rc;
  if ((rc = bf.ensure((size_t)x->Npad * ld_b * 2)) || (rc = x->rr_stats.ensure(64))) return rc;
  BB_HIP(hipMemsetAsync((float*)x->rr_stats.p + stat_off, 0, 16, x->stream));
  BB_HIP(launch_rr_prepare((const float*)rows.p, x->Npad, ld, (uint16_t*)bf.p, ld_b, (float*)x->rr_stats.p + stat_off,
                           x->stream));
  BB_HIP(hipStreamSynchronize(x->stream));
  return BB_OK;
}

}  // extern "C"

namespace {
int search_locked(bb_index* x, const bb_query* q, bb_result* res, bool allow_stream);

// The rank-0 table of the constraint-first search (compact.hip): every item's own stored row
// searched as a similar-sets query (k = 1, key lists out) over this index — its max key is
// the arg-max of the unmasked ranking that get_similar_sets drops (:217), the same key the
// full search's list select finds — plus one zero row (an id outside the index, as the
// gather treats it).  Built once per upload; read by the packed searches of similar / hybrid
// queries, whose packed rows no longer hold the unmasked ranking.
int build_r0(bb_index* x) {
  x->r0_ready = false;
  const int64_t n = x->n, B = n + 1;
  int rc;
  if ((rc = x->r0key.ensure((size_t)B * 8))) return rc;
  DevBuf ids, keys;
  std::vector<int64_t> h((size_t)B);
  for (int64_t i = 0; i < n; ++i) h[(size_t)i] = x->id_offset + i;
  h[(size_t)n] = x->id_offset - 1;
  bb_query q{};
  q.mode = BB_MODE_SIMILAR;
  q.flags = BB_Q_OUT_KEYS;
  q.B = (int32_t)B;
  q.k = 1;
  q.where = BB_DEVICE;
  q.stream = x->stream;
  bb_result r{};
  r.where = BB_DEVICE;
  r.max_keys = (uint64_t*)x->r0key.p;
  if ((rc = ids.ensure((size_t)B * 8)) || (rc = keys.ensure((size_t)B * 2 * 8))) return rc;
  q.q_items = (const int64_t*)ids.p;
  r.keys = (uint64_t*)keys.p;
  hipError_t e = hipMemcpyAsync(ids.p, h.data(), (size_t)B * 8, hipMemcpyHostToDevice, x->stream);
  if (e == hipSuccess) {
    const bool prof = x->prof;  // (not a caller's search: nothing joins the profile)
    x->prof = false;
    rc = search_locked(x, &q, &r, false);
    x->prof = prof;
    e = hipStreamSynchronize(x->stream);
  }
  ids.release();
  keys.release();
  if (e != hipSuccess) return fail(BB_E_HIP, std::string("rank-0 table: ") + hipGetErrorString(e));
  if (rc) return rc;
  x->r0_ready = true;
  return BB_OK;
}
}  // namespace

extern "C" {

int bb_upload_items(bb_index* x, const void* rows, int64_t n, int32_t d, int32_t in_dtype, int32_t prenormalized,
                    int32_t where, const uint32_t* present_bits) {
  BB_CHECK_INDEX(x, "bb_upload_items");
  if (x->base) return fail(BB_E_STATE, "a view shares its base's rows: upload to the base");
  if (!rows || n <= 0 || d <= 0) return fail(BB_E_ARG, "bb_upload_items: bad arguments");
  if (in_dtype != F32 && in_dtype != BF16 && in_dtype != F64) return fail(BB_E_ARG, "bad input dtype");
  if (n >= 0xFFFFFFFFll - x->id_offset) return fail(BB_E_ARG, "too many items for 32-bit ids");
  std::lock_guard<std::mutex> lk(x->mu);  // bb_create_view takes it too
  if (x->n_views > 0) return fail(BB_E_STATE, "the index has live views: destroy them before uploading");
  DeviceGuard g(x->device);
  StreamScope scope;
  if (int rc0 = scope.enter(x, x->stream)) return rc0;
  x->n = n;
  x->d = d;
  x->Npad = round_up(n, kTileRows);
  x->Dpad = (int)round_up(d, gemm_tile_k(x->dtype));
  const size_t bytes = (size_t)x->Npad * x->Dpad * elem_size(x->dtype);
  int rc = x->items.ensure(bytes);
  if (rc) return rc;
  BB_HIP(hipMemsetAsync(x->items.p, 0, bytes, x->stream));
  const size_t wbytes = (size_t)(x->Npad / 32) * 4;
  if ((rc = x->items_present.ensure(wbytes))) return rc;
  if (present_bits) {
    BB_HIP(hipMemsetAsync(x->items_present.p, 0, wbytes, x->stream));
    BB_HIP(hipMemcpyAsync(x->items_present.p, present_bits, (size_t)((n + 31) / 32) * 4, hipMemcpyHostToDevice,
                          x->stream));
  } else {
    BB_HIP(hipMemsetAsync(x->items_present.p, 0xFF, wbytes, x->stream));
  }
  if ((rc = x->ones.ensure(wbytes)) || (rc = x->zeros.ensure(wbytes))) return rc;
  BB_HIP(hipMemsetAsync(x->ones.p, 0xFF, wbytes, x->stream));
  BB_HIP(hipMemsetAsync(x->zeros.p, 0, wbytes, x->stream));
  if ((rc = upload_rows(x, rows, n, d, in_dtype, prenormalized ? 0 : 1, where, x->items.p, x->Dpad))) return rc;
  if ((rc = make_planes(x, x->items, x->items3, x->Dpad))) return rc;
  if ((rc = make_rr(x, x->items, x->items_bf, x->Dpad, x->Dpad_b, 0))) return rc;
  x->r0_ready = false;
  if (x->dtype == F32 && x->items_bf.p && n <= (int64_t)kCompactMaxWords * 32 && (rc = build_r0(x))) return rc;
  return scope.leave();
}

int bb_upload_cf(bb_index* x, const void* f, int32_t r, int32_t in_dtype, const uint32_t* present_bits) {
  BB_CHECK_INDEX(x, "bb_upload_cf");
  if (x->base) return fail(BB_E_STATE, "a view shares its base's rows: upload to the base");
  if (!f || r <= 0) return fail(BB_E_ARG, "bb_upload_cf: bad arguments");
  if (x->n <= 0) return fail(BB_E_STATE, "upload items before CF factors");
  std::lock_guard<std::mutex> lk(x->mu);  // bb_create_view takes it too
  if (x->n_views > 0) return fail(BB_E_STATE, "the index has live views: destroy them before uploading");
  DeviceGuard g(x->device);
  StreamScope scope;
  if (int rc0 = scope.enter(x, x->stream)) return rc0;
  x->r = r;
  x->Rpad = (int)round_up(r, gemm_tile_k(x->dtype));
  const size_t bytes = (size_t)x->Npad * x->Rpad * elem_size(x->dtype);
  int rc = x->cf.ensure(bytes);
  if (rc) return rc;
  BB_HIP(hipMemsetAsync(x->cf.p, 0, bytes, x->stream));
  const size_t wbytes = (size_t)(x->Npad / 32) * 4;
  if ((rc = x->cf_present.ensure(wbytes))) return rc;
  if (present_bits) {
    BB_HIP(hipMemsetAsync(x->cf_present.p, 0, wbytes, x->stream));
    BB_HIP(hipMemcpyAsync(x->cf_present.p, present_bits, (size_t)((x->n + 31) / 32) * 4, hipMemcpyHostToDevice,
                          x->stream));
  } else {
    BB_HIP(hipMemsetAsync(x->cf_present.p, 0xFF, wbytes, x->stream));
  }
  if ((rc = upload_rows(x, f, x->n, r, in_dtype, 0, BB_HOST, x->cf.p, x->Rpad))) return rc;
  if ((rc = make_planes(x, x->cf, x->cf3, x->Rpad))) return rc;
  if ((rc = make_rr(x, x->cf, x->cf_bf, x->Rpad, x->Rpad_b, 4))) return rc;
  return scope.leave();
}

int bb_upload_attrs(bb_index* x, const int32_t* num_parts, const int16_t* year, const int32_t* theme_id) {
  BB_CHECK_INDEX(x, "bb_upload_attrs");
  if (x->base) return fail(BB_E_STATE, "a view shares its base's rows: upload to the base");
  if (!num_parts || !year || !theme_id) return fail(BB_E_ARG, "bb_upload_attrs: bad arguments");
  if (x->n <= 0) return fail(BB_E_STATE, "upload items before attributes");
  std::lock_guard<std::mutex> lk(x->mu);  // bb_create_view takes it too
  if (x->n_views > 0) return fail(BB_E_STATE, "the index has live views: destroy them before uploading");
  DeviceGuard g(x->device);
  int rc;
  StreamScope scope;
  if ((rc = scope.enter(x, x->stream))) return rc;
  if ((rc = x->parts.ensure(x->n * 4)) || (rc = x->year.ensure(x->n * 2)) || (rc = x->theme.ensure(x->n * 4)))
    return rc;
  BB_HIP(hipMemcpyAsync(x->parts.p, num_parts, x->n * 4, hipMemcpyHostToDevice, x->stream));
  BB_HIP(hipMemcpyAsync(x->year.p, year, x->n * 2, hipMemcpyHostToDevice, x->stream));
  BB_HIP(hipMemcpyAsync(x->theme.p, theme_id, x->n * 4, hipMemcpyHostToDevice, x->stream));
  BB_HIP(hipStreamSynchronize(x->stream));
  return scope.leave();
}

int bb_eval_mask(bb_index* x, const bb_predicate* p, uint32_t* out_bits, int32_t where) {
  BB_CHECK_INDEX(x, "bb_eval_mask");
  if (!p || !out_bits) return fail(BB_E_ARG, "bb_eval_mask: bad arguments");
  if (!x->parts.p) return fail(BB_E_STATE, "upload attributes before evaluating masks");
  std::lock_guard<std::mutex> lk(x->mu);
  DeviceGuard g(x->device);
  const int64_t nw = (x->n + 31) / 32;
  const size_t tb = (size_t)((std::max(p->n_theme_bits, 0) + 31) / 32) * 4;
  const size_t ib = (size_t)std::max<int64_t>(p->n_excluded, 0) * 8;
  StreamScope scope;
  int rc = scope.enter(x, x->stream);
  if (rc) return rc;
  if ((rc = x->stage_in.ensure(nw * 4 + tb + ib + 64))) return rc;
  char* base = (char*)x->stage_in.p;
  uint32_t* dout = where == BB_DEVICE ? out_bits : (uint32_t*)base;
  uint32_t* dtheme = (uint32_t*)(base + round_up(nw * 4, 16));
  int64_t* dids = (int64_t*)(base + round_up(nw * 4, 16) + round_up(tb, 16));
  if (p->theme_mode && tb && p->theme_bits)
    BB_HIP(hipMemcpyAsync(dtheme, p->theme_bits, tb, hipMemcpyHostToDevice, x->stream));
  MaskArgs m{};
  m.parts = (const int32_t*)x->parts.p;
  m.year = (const int16_t*)x->year.p;
  m.theme = (const int32_t*)x->theme.p;
  m.n = x->n;
  m.parts_min = p->parts_min;
  m.parts_max = p->parts_max;
  m.year_min = p->year_min;
  m.year_max = p->year_max;
  m.theme_mode = (p->theme_mode && p->theme_bits) || p->theme_mode == 1 ? p->theme_mode : 0;
  m.n_theme_bits = p->theme_bits ? p->n_theme_bits : 0;
  m.theme_bits = dtheme;
  m.out = dout;
  if ((rc = timed(x, K_MASK, x->stream, [&] { return launch_mask(m, x->stream); }))) return rc;
  if (p->n_excluded > 0 && p->excluded_items) {
    std::vector<int64_t> local(p->n_excluded);
    for (int64_t i = 0; i < p->n_excluded; ++i) local[i] = p->excluded_items[i] - x->id_offset;
    BB_HIP(hipMemcpyAsync(dids, local.data(), ib, hipMemcpyHostToDevice, x->stream));
    BB_HIP(launch_clear_bits(dout, dids, p->n_excluded, x->n, x->stream));
    BB_HIP(hipStreamSynchronize(x->stream));  // `local` goes out of scope
  }
  if (where != BB_DEVICE) {
    BB_HIP(hipMemcpyAsync(out_bits, dout, nw * 4, hipMemcpyDeviceToHost, x->stream));
  }
  BB_HIP(hipStreamSynchronize(x->stream));
  return scope.leave();
}

int bb_key_lens(const bb_query* q, int32_t* sides, int32_t* k_int) { return side_k_int(q, sides, k_int); }

}  // extern "C"

namespace {

constexpr int kRetrySlab = 1;  // search_locked: a streaming candidate region overflowed
constexpr int kNoCompact = 2;  // search_locked of a shadow: its shapes leave the list path (nothing launched)

// Constraint-first search (compact.hip, the reference's "apply hard constraints first",
// recommendation_system.py:628-656): the `cnt` rows mask d_mask allows are packed into the
// shadow index x->cx (positions in ascending id order, so ties still break by id), with the
// liked sets' rows, their rank-0 exclusions and the per-query exclusions re-indexed, in ONE
// launch; the unchanged search then runs over the packed rows and writes idmap[position] as
// each id.  Returns kNoCompact (having launched only the packing kernel) when the shadow's
// shapes would leave the list path, whose writers map the ids.
int compact_search(bb_index* x, const bb_query* q, bb_result* res, hipStream_t s, const void* d_rows,
                   const void* d_items, const void* d_cf, const void* d_mask, const void* d_excl, int64_t cnt) {
  const bool need_content = q->mode != BB_MODE_CF;
  const bool need_cf = q->mode == BB_MODE_CF || q->mode == BB_MODE_HYBRID;
  const bool liked = need_content && q->mode != BB_MODE_SEMANTIC;
  const int B = q->B;
  bb_index* c = x->cx;
  if (!c) {
    c = new bb_index();
    c->magic = 0;  // never a caller's handle
    c->shadow = true;
    c->device = x->device;
    c->dtype = F32;
    x->cx = c;
  }
  // the list path (BB_PF_LISTS=0, A/B runs: the int16-image selects — one wave per query
  // rescoring its candidates, 111 vs 48 us at configs[2], r06d)
  static const int pf_lists = ab_env("BB_PF_LISTS") ? atoi(ab_env("BB_PF_LISTS")) : -1;
  c->lists_opt = pf_lists == 0 ? 0 : x->lists_opt;
  c->sq_opt = 0;       // the packed search is the list path (B > kSqMaxB anyway)
  c->stream_opt = 0;
  c->refine_opt = 0;
  c->ws_cap = x->ws_cap;
  c->ws_set = x->ws_set;
  c->prof = x->prof;
  // slot stride: allowed item p sits in slot p·stride, so a lane half's top-5 list of one
  // tile covers at most 16 / stride allowed items — stride 4 when the top-K_int is a large
  // share of the allowed rows (no list can overflow), 2 or 1 as it shrinks (compact.hip)
  int32_t sides_q = 0, K_int = 0;
  int rc = side_k_int(q, &sides_q, &K_int);
  if (rc) return rc;
  const int64_t e1 = std::max<int64_t>(cnt, 1);  // (no allowed item: one padding slot, never present)
  static const int pf_stride = ab_env("BB_PF_STRIDE") ? atoi(ab_env("BB_PF_STRIDE")) : 0;
  const int stride = pf_stride == 1 || pf_stride == 2 || pf_stride == 4 ? pf_stride
                     : (int64_t)K_int * 4 >= e1                     ? 4
                     : (int64_t)K_int * 16 >= e1                    ? 2
                                                                    : 1;
  const int64_t cap = round_up(e1 * stride, kTileRows);
  if (cap > kCompactMaxSlots) return kNoCompact;  // (forced on a dense mask: the full search)
  const int cnw = (int)(cap / 32);
  c->n = e1 * stride;
  c->Npad = cap;
  c->d = x->d;
  c->Dpad = x->Dpad;
  c->Dpad_b = x->Dpad_b;
  c->r = x->r;
  c->Rpad = x->Rpad;
  c->Rpad_b = x->Rpad_b;
  c->id_offset = 0;
  c->rr_stats.p = x->rr_stats.p;  // bounds over every row hold for any subset of them
  c->rr_stats.cap = x->rr_stats.cap;
  c->rr_stats.owned = false;
  const size_t wb = (size_t)cnw * 4;
  if ((rc = c->ones.ensure(wb)) || (rc = c->zeros.ensure(wb)) || (rc = c->idmap.ensure((size_t)cap * 4))) return rc;
  if (c->filled_words < (size_t)cnw) {  // constant fills, once per size (outside any plan record)
    BB_HIP(hipMemsetAsync(c->ones.p, 0xFF, c->ones.cap, s));
    BB_HIP(hipMemsetAsync(c->zeros.p, 0, c->zeros.cap, s));
    c->filled_words = c->ones.cap / 4;
  }
  if (need_content &&
      ((rc = c->items.ensure((size_t)cap * x->Dpad * 4)) || (rc = c->items_bf.ensure((size_t)cap * x->Dpad_b * 2)) ||
       (rc = c->items_present.ensure(wb))))
    return rc;
  if (need_cf && ((rc = c->cf.ensure((size_t)cap * x->Rpad * 4)) || (rc = c->cf_bf.ensure((size_t)cap * x->Rpad_b * 2)) ||
                  (rc = c->cf_present.ensure(wb))))
    return rc;
  if (liked && (rc = c->cexcl0.ensure((size_t)B * wb))) return rc;
  if (need_cf && d_excl && (rc = c->cexcl1.ensure((size_t)B * wb))) return rc;
  CompactArgs a{};
  a.mask = (const uint32_t*)d_mask;
  a.n = x->n;
  a.nw = (int32_t)((x->n + 31) / 32);
  a.id_offset = (uint32_t)x->id_offset;
  if (need_content) {
    a.items = (const float*)x->items.p;
    a.ld = x->Dpad;
    a.items_bf = (const uint16_t*)x->items_bf.p;
    a.ld_b = x->Dpad_b;
    a.items_present = (const uint32_t*)x->items_present.p;
    a.c_items = (float*)c->items.p;
    a.c_items_bf = (uint16_t*)c->items_bf.p;
    a.c_present = (uint32_t*)c->items_present.p;
  }
  if (need_cf) {
    a.cf = (const float*)x->cf.p;
    a.ldc = x->Rpad;
    a.cf_bf = (const uint16_t*)x->cf_bf.p;
    a.ldc_b = x->Rpad_b;
    a.cf_present = (const uint32_t*)x->cf_present.p;
    a.c_cf = (float*)c->cf.p;
    a.c_cf_bf = (uint16_t*)c->cf_bf.p;
    a.c_cf_present = (uint32_t*)c->cf_present.p;
  }
  a.cap = (int32_t)cap;
  a.stride = stride;
  a.cap_pos = (int32_t)(cap / stride);
  a.cnw = cnw;
  a.xnw = (int32_t)((c->n + 31) / 32);  // the shadow search's exclusion row stride (its nw)
  a.n_word_wg = cnw;
  a.ch_items = need_content ? x->Dpad / 4 : 0;
  a.ch_items_b = need_content ? x->Dpad_b / 8 : 0;
  a.ch_cf = need_cf ? x->Rpad / 4 : 0;
  a.ch_cf_b = need_cf ? x->Rpad_b / 8 : 0;
  a.n_copy_wg = (int32_t)((a.cap_pos * (a.ch_items + a.ch_cf) + cap * (a.ch_items_b + a.ch_cf_b) + 1023) / 1024);
  a.idmap = (uint32_t*)c->idmap.p;
  const bool per_query = liked || (need_cf && d_excl);
  a.B = per_query ? B : 0;
  if (liked) {
    a.q_items = (const int64_t*)d_items;
    a.r0key = (const uint64_t*)x->r0key.p;
    a.c_excl0 = (uint32_t*)c->cexcl0.p;
  }
  if (need_cf && d_excl) {
    a.excl = (const uint32_t*)d_excl;
    a.excl_ld = a.nw;
    a.c_excl1 = (uint32_t*)c->cexcl1.p;
  }
  // launched by the shadow's search in place of its prep launch, with that prep's arguments
  // (so the packing and the query prep are one launch, and nothing runs if the shadow's
  // shapes leave the list / image paths)
  c->cjob = a;
  c->cjob_set = true;
  bb_query q2 = *q;
  q2.where = BB_DEVICE;
  q2.stream = s;
  q2.flags = (q->flags & ~BB_Q_NULL_STREAM) | (s ? 0 : BB_Q_NULL_STREAM);
  q2.mask_bits = nullptr;
  q2.mask_count = 0;
  q2.excl_bits = need_cf && d_excl ? (const uint32_t*)c->cexcl1.p : nullptr;
  // (liked sets: the ORIGINAL ids — the packing launch's prep gathers their rows from the full
  // index; the shadow itself never reads them)
  q2.q_items = liked ? (const int64_t*)d_items : nullptr;
  q2.q_rows = liked ? nullptr : d_rows;
  q2.q_cf = d_cf;
  c->cur_cexcl = liked ? (const uint32_t*)c->cexcl0.p : nullptr;
  rc = search_locked(c, &q2, res, false);
  c->cjob_set = false;
  // the shadow's kernels count as this handle's
  for (auto& pe : c->pending) x->pending.push_back(pe);
  c->pending.clear();
  for (int i = 0; i < K_NFAM; ++i) {
    x->launches[i] += c->launches[i];
    c->launches[i] = 0;
  }
  return rc;
}

int search_locked(bb_index* x, const bb_query* q, bb_result* res, bool allow_stream) {
  int32_t sides, K_int;
  int rc = side_k_int(q, &sides, &K_int);
  if (rc) return rc;
  const int B = q->B;
  if (B <= 0) return fail(BB_E_ARG, "B must be > 0");
  if (x->n <= 0) return fail(BB_E_STATE, "no items uploaded");
  const bool need_content = q->mode != BB_MODE_CF;
  const bool need_cf = q->mode == BB_MODE_CF || q->mode == BB_MODE_HYBRID;
  // (a shadow's packed rows drop the rank-0 item through its content exclusions instead)
  const bool drop = (q->mode == BB_MODE_SIMILAR || q->mode == BB_MODE_HYBRID) && !x->shadow;
  if (need_cf && !x->cf.p) return fail(BB_E_STATE, "CF mode needs bb_upload_cf");
  if (need_content && q->mode != BB_MODE_SEMANTIC && !q->q_items && !q->q_rows)
    return fail(BB_E_ARG, "similar/hybrid mode needs q_items (or pre-normalised q_rows)");
  if (q->mode == BB_MODE_SEMANTIC && !q->q_rows) return fail(BB_E_ARG, "semantic mode needs q_rows");
  if (need_cf && !q->q_cf) return fail(BB_E_ARG, "cf/hybrid mode needs q_cf");
  const bool out_keys = (q->flags & BB_Q_OUT_KEYS) != 0;
  if (out_keys && (!res->keys || !res->max_keys)) return fail(BB_E_ARG, "BB_Q_OUT_KEYS needs keys/max_keys");
  if (!out_keys && (!res->scores || !res->ids)) return fail(BB_E_ARG, "null result buffers");

  const hipStream_t s = call_stream(x, q);
  const int where = q->where;
  const int64_t nw = (x->n + 31) / 32;

  // query-row padding: 128-query groups, or whole 256-query groups where the bf16 scan
  // holds 64 queries per wave (scan4_kernel.h) — any query chunk taller than one group
  const int64_t rq = x->dtype == BF16 && B > kTileRows ? 2 * kTileRows : kTileRows;
  auto pad_rows = [&](int64_t b) { return round_up(b, b > kTileRows ? rq : kTileRows); };
  // BB_OPT_STREAM (or the BB_STREAM environment variable, for A/B runs) forces it off / on
  static const int stream_env = ab_env("BB_STREAM") ? atoi(ab_env("BB_STREAM")) : -1;
  const int stream_sel = x->stream_opt >= 0 ? x->stream_opt : stream_env;
  // (the streaming epilogue lives in the query-resident scan kernels only)
  auto scan_ok = [&](int kp, bool planes) { return planes ? scan3_supported(128, kp) : gemm_uses_scan(x->dtype, 128, kp); };
  const bool stream = allow_stream && (stream_sel == 1 || (stream_sel != 0 && x->n >= x->stream_min_items)) &&
                      (!need_content || scan_ok(x->Dpad, x->items3.p != nullptr)) &&
                      (!need_cf || scan_ok(x->Rpad, x->cf3.p != nullptr));

  // slab / chunk geometry
  // Slab path: a slab is as many item columns as the score workspace holds for a query chunk
  // of up to 1024 queries; queries beyond the chunk loop over the same slabs again.
  // Streaming path (below): the workspace only holds the pilot slab [0, n0), so query chunks
  // grow to 8192 rows — every staged item tile then serves that many queries per launch.
  // Unless the caller capped the workspace, streaming may use up to 4 GiB of it.
  const int64_t ws = stream && !x->ws_set ? std::max<int64_t>(x->ws_cap, 4ll << 30) : x->ws_cap;
  int64_t n0 = 0, lds, Bc;
  if (stream) {
    // pilot rows: n/16, or n/8 below the two-level bound's range (< 500K rows) for batches of
    // 256+, where the candidate select dominates: 125K x 768, B = 4096 appends ~K_int·n/n0
    // keys per query, and T(n0) ≈ pilot + select is minimal near n/8 (BB_PILOT_DIV, A/B runs)
    static const int pilot_div_env = ab_env("BB_PILOT_DIV") ? atoi(ab_env("BB_PILOT_DIV")) : 0;
    const int64_t pilot_div = pilot_div_env > 0 ? pilot_div_env : (x->n < 500000 && B >= 256 ? 8 : 16);
    const int64_t n0_target =
        std::min<int64_t>(round_up(std::max<int64_t>(x->n / pilot_div, 64ll * K_int), kTileRows), x->Npad);
    const int64_t n0_min = std::min<int64_t>(n0_target, 8192);
    Bc = std::min<int64_t>(pad_rows(B), 8192);
    while (Bc > rq && Bc * n0_min * 4 > ws) Bc = std::max<int64_t>(rq, Bc / 2 / rq * rq);
    n0 = std::max<int64_t>(kTileRows, std::min<int64_t>(n0_target, ws / (Bc * 4) / kTileRows * kTileRows));
    lds = n0;
  } else {
    const int64_t Bt = std::min<int64_t>(pad_rows(B), 1024);
    lds = std::min<int64_t>(x->Npad, std::max<int64_t>(kTileRows, (ws / (Bt * 4)) / kTileRows * kTileRows));
    Bc = std::max<int64_t>(rq, (ws / (lds * 4)) / rq * rq);
    Bc = std::min<int64_t>(Bc, pad_rows(B));
  }
  const int64_t slab = lds;        // multiple of kTileRows
  const int64_t n_slabs = (x->n + slab - 1) / slab;
  const int64_t ldt = slab / 32;   // per-tile maxima per query row
  // exact re-rank path (f32 index, one slab): the one-product bf16 MFMA scan writes
  // approximate scores, the select rescores the candidates within their error bound from
  // the f32 rows.  BB_NO_RR (A/B runs) forces the split-precision scan instead.
  static const bool no_rr = ab_env("BB_NO_RR") != nullptr;
  const bool rr_c = !no_rr && !stream && n_slabs == 1 && need_content && x->items_bf.p;
  const bool rr_f = !no_rr && !stream && n_slabs == 1 && need_cf && x->cf_bf.p;
  // Bounded candidate lists (list_epi.h, select_list.hip) on the re-rank scans: no score
  // image; per lane the top-5 keys of every period of G <= 8 tiles.  Geometry of a query
  // chunk of bpad_c rows: item chunks of the scan launch (scan2 or scan4), periods per chunk
  // (enough lists that a list expects <= 1/3 of a top-K member: 2·chunks·periods >= 3·K_int),
  // tiles per period.
  auto list_geom = [&](int bpad_c, int ku, int& nch, int& np, int& G) -> bool {
    if (x->lists_opt == 0) return false;
    const int tiles = (int)(round_up(x->n, kTileRows) / 32);
    nch = scan_chunks(BF16, bpad_c, tiles, false, ku);
    const int tpc = (tiles + nch - 1) / nch;
    if (nch > 256) return false;
    np = (tpc + kListMaxPeriod - 1) / kListMaxPeriod;
    // BB_LIST_DENSE (A/B runs): as many periods as the per-row cap allows (shorter periods:
    // fewer overflowed lists, and fewer items to enumerate when one overflows)
    static const bool dense = ab_env("BB_LIST_DENSE") && atoi(ab_env("BB_LIST_DENSE")) != 0;
    const int np_goal = dense ? kListMaxPerRow : 3 * K_int;
    while (2 * nch * np < np_goal && 2 * nch * (np + 1) <= kListMaxPerRow && np < tpc) ++np;
    G = (tpc + np - 1) / np;
    np = (tpc + G - 1) / G;
    return G <= kListMaxPeriod && 2 * nch * np <= kListMaxPerRow;
  };

  // stage host inputs
  const size_t es_q = elem_size(q->q_dtype), es_cf = elem_size(q->q_cf_dtype);
  const size_t b_rows = q->q_rows ? (size_t)B * x->d * es_q : 0;
  const size_t b_items = q->q_items ? (size_t)B * 8 : 0;
  const size_t b_cf = q->q_cf && need_cf ? (size_t)B * x->r * es_cf : 0;
  const size_t b_mask = q->mask_bits ? (size_t)nw * 4 : 0;
  const size_t b_excl = q->excl_bits ? (size_t)B * nw * 4 : 0;
  size_t off_rows = 0, off_items = round_up(b_rows, 256), off_cf = off_items + round_up(b_items, 256),
         off_mask = off_cf + round_up(b_cf, 256), off_excl = off_mask + round_up(b_mask, 256),
         stage_total = off_excl + round_up(b_excl, 256);
  if (where == BB_HOST && (rc = x->stage_in.ensure(std::max<size_t>(stage_total, 256)))) return rc;
  const void *d_rows, *d_items, *d_cf, *d_mask, *d_excl;
  if ((rc = to_device(x, x->stage_in, off_rows, q->q_rows, b_rows, where, s, &d_rows)) ||
      (rc = to_device(x, x->stage_in, off_items, q->q_items, b_items, where, s, &d_items)) ||
      (rc = to_device(x, x->stage_in, off_cf, q->q_cf, b_cf, where, s, &d_cf)) ||
      (rc = to_device(x, x->stage_in, off_mask, q->mask_bits, b_mask, where, s, &d_mask)) ||
      (rc = to_device(x, x->stage_in, off_excl, q->excl_bits, b_excl, where, s, &d_excl)))
    return rc;

  // ---- constraint-first search: a selective mask with a known count (host masks are counted
  // here; device masks carry bb_query.mask_count) on a one-slab f32 index packs its allowed
  // rows and searches only them (compact_search).  BB_OPT_PREFILTER: -1 auto (allowed rows
  // <= n/4), 0 off, 1 whenever the count is known. ----
  if (!x->shadow && d_mask && !out_keys && B > kSqMaxB && x->prefilter_opt != 0 && x->dtype == F32 &&
      x->n <= (int64_t)kCompactMaxWords * 32 && x->lists_opt != 0 && x->stream_opt != 1 &&
      (!need_content || (x->items_bf.p && x->Dpad <= kRrMaxD && x->d <= kRrMaxD)) && (!need_cf || x->cf_bf.p) &&
      (q->mode == BB_MODE_SEMANTIC || q->mode == BB_MODE_CF || (d_items && x->r0_ready))) {
    int64_t cnt = -1;
    if (where == BB_HOST) {
      cnt = 0;
      for (int64_t w = 0; w < nw; ++w) {
        uint32_t v = q->mask_bits[w];
        if ((w + 1) * 32 > x->n) v &= (1u << (x->n & 31)) - 1u;
        cnt += __builtin_popcount(v);
      }
    } else if (q->mask_count > 0) {
      cnt = std::min<int64_t>(q->mask_count, x->n);
    }
    if (cnt >= 0 && (x->prefilter_opt == 1 || cnt * 4 <= x->n)) {
      rc = compact_search(x, q, res, s, d_rows, d_items, d_cf, d_mask, d_excl, cnt);
      if (rc != kNoCompact) return rc;
    }
  }

  // ---- small batches (the reference's request shape: one target row, one user, one
  // retriever query, one HybridRecommender request): one approximate pass over the bf16 copy
  // per side and an exact rescore of the candidates within its bound (sq.hip) instead of the
  // MFMA scan + lists + list select; a hybrid search then blends the two sides' key lists in
  // finalize1 as the large-batch path does.  BB_OPT_SMALL_BATCH / BB_SQ (A/B runs): 0 off,
  // 1 on, -1 auto (on). ----
  static const int sq_env = ab_env("BB_SQ") ? atoi(ab_env("BB_SQ")) : -1;
  const int sq_sel = x->sq_opt >= 0 ? x->sq_opt : sq_env;
  const bool sq_sides = (!need_content || (x->items_bf.p && x->Dpad <= kRrMaxD && x->d <= kRrMaxD && x->Dpad_b <= 512)) &&
                        (!need_cf || (x->cf_bf.p && x->Rpad <= kRrMaxD && x->r <= kRrMaxD && x->Rpad_b <= 512));
  if (sq_sel != 0 && x->dtype == F32 && B <= kSqMaxB && K_int <= kSqMaxK && sq_sides &&
      x->n <= (int64_t)kSqMaxWg * kSqMaxRows) {
    static const int sq_wg_env = ab_env("BB_SQ_WG") ? atoi(ab_env("BB_SQ_WG")) : 256;
    const bool hyb = sides == 2;
    const int64_t wg_goal = std::max(1, std::min(sq_wg_env, kSqMaxWg));
    const int32_t rpw = (int32_t)std::min<int64_t>(kSqMaxRows, std::max<int64_t>(4, round_up((x->n + wg_goal - 1) / wg_goal, 4)));
    const int32_t nwg = (int32_t)((x->n + rpw - 1) / rpw);
    const size_t top_side = (size_t)B * nwg * kSqM, ord_side = (size_t)B * x->n * 2;
    if ((rc = x->sq_top.ensure(top_side * 8 * sides)) || (rc = x->sq_ptop.ensure(top_side * 8)) ||
        (rc = x->sq_ords.ensure(ord_side * 4 * sides)) ||
        (rc = x->keys.ensure((size_t)sides * B * K_int * 8)) || (rc = x->maxk.ensure((size_t)B * 8)))
      return rc;
    const bool host_res = !out_keys && res->where != BB_DEVICE;
    if (host_res && ((rc = x->out_sc.ensure((size_t)B * q->k * 4)) || (rc = x->out_id.ensure((size_t)B * q->k * 8)) ||
                     (rc = x->out_cnt.ensure((size_t)B * 4))))
      return rc;
    float* f_sc = host_res ? (float*)x->out_sc.p : res->scores;
    int64_t* f_id = host_res ? (int64_t*)x->out_id.p : res->ids;
    int32_t* f_cnt = host_res ? (int32_t*)x->out_cnt.p : res->counts;
    static const int sq_mopt = ab_env("BB_SQ_MOPT") ? atoi(ab_env("BB_SQ_MOPT")) : 3;
    // one side's pass: the content side (semantic / similar / hybrid side 0) or the CF side
    auto side_args = [&](int side) {
      const bool cf_side = q->mode == BB_MODE_CF || side == 1;
      SqArgs a{};
      a.Xb = (const uint16_t*)(cf_side ? x->cf_bf.p : x->items_bf.p);
      a.ldb = cf_side ? x->Rpad_b : x->Dpad_b;
      a.X = (const float*)(cf_side ? x->cf.p : x->items.p);
      a.ldx = cf_side ? x->Rpad : x->Dpad;
      a.stats = (const float*)x->rr_stats.p + (cf_side ? 4 : 0);
      a.n = (int32_t)x->n;
      a.gid0 = (uint32_t)x->id_offset;
      a.present = (const uint32_t*)(cf_side ? x->cf_present.p : x->items_present.p);
      a.mask = (const uint32_t*)(d_mask ? d_mask : x->ones.p);
      // rated items: the CF side only (as the scans)
      a.excl = (const uint32_t*)(cf_side && d_excl ? d_excl : x->zeros.p);
      a.excl_ld = cf_side && d_excl ? nw : 0;
      a.drop = drop && side == 0;
      a.B = B;
      if (q->mode == BB_MODE_SEMANTIC || cf_side || !d_items) {
        a.q_kind = q->mode == BB_MODE_SEMANTIC ? 0 : 2;
        a.q_src = cf_side ? d_cf : d_rows;
        a.q_dtype = cf_side ? q->q_cf_dtype : q->q_dtype;
        a.q_ld = a.q_d = cf_side ? x->r : x->d;
      } else {
        a.q_kind = 1;
        a.q_ids = (const int64_t*)d_items;
        a.q_id_offset = x->id_offset;
      }
      a.rpw = rpw;
      a.nwg = nwg;
      a.K = K_int;
      a.mopt = sq_mopt;
      a.wg_top = (uint64_t*)x->sq_top.p + side * top_side;
      a.wg_ptop = (uint64_t*)x->sq_ptop.p;  // (the rank-0 side only)
      a.ords = (uint32_t*)x->sq_ords.p + side * ord_side;
      a.ords_p = a.ords + (size_t)B * x->n;
      a.ords_ld = x->n;
      if (out_keys || hyb) {  // key lists (+ the present maximum) for a cross-shard merge or the blend
        a.keys_out = (uint64_t*)x->keys.p + (size_t)side * B * K_int;
        a.max_out = side == 0 ? (uint64_t*)x->maxk.p : nullptr;
      } else {
        a.k_final = q->k;
        a.out_scores = f_sc;
        a.out_ids = f_id;
        a.out_counts = f_cnt;
      }
      return a;
    };
    SqArgs a0 = side_args(0);
    SqArgs a1 = hyb ? side_args(1) : a0;
    // BB_SQ_TRACE (probe runs): phase stamps of side 0's pass workgroups and merge rows
    static const bool sq_trace = kProbes && ab_env("BB_SQ_TRACE") != nullptr;
    if (sq_trace) {
      if ((rc = x->trace.ensure((size_t)(nwg + B) * 8 * 8))) return rc;
      BB_HIP(hipMemsetAsync(x->trace.p, 0, (size_t)(nwg + B) * 64, s));
      a0.trace = (uint64_t*)x->trace.p;
      a0.mtrace = a0.trace + (size_t)nwg * 8;
    }
    for (int side = 0; side < sides; ++side)
      if ((rc = timed(x, K_GEMM, s, [&] { return launch_sq_scan(side ? a1 : a0, s); }))) return rc;
    if ((rc = timed(x, K_SELECT, s, [&] { return launch_sq_merge(a0, hyb ? &a1 : nullptr, s); }))) return rc;
    if (sq_trace) {
      std::vector<uint64_t> tr((size_t)(nwg + B) * 8);
      BB_HIP(hipMemcpyAsync(tr.data(), x->trace.p, tr.size() * 8, hipMemcpyDeviceToHost, s));
      BB_HIP(hipStreamSynchronize(s));
      uint64_t t0 = ~0ull, tend = 0;
      double ph[6] = {0};
      for (int w2 = 0; w2 < nwg; ++w2) {
        const uint64_t* t = &tr[(size_t)w2 * 8];
        t0 = std::min(t0, t[0]);
        tend = std::max(tend, t[4]);
        for (int j = 1; j < 6; ++j) ph[j] += t[j] ? (double)(t[j] - t[0]) : 0.0;
      }
      uint64_t s_max = 0;
      for (int w2 = 0; w2 < nwg; ++w2) s_max = std::max<uint64_t>(s_max, tr[(size_t)w2 * 8] - t0);
      double mp[4] = {0}, ce = 0, cp = 0;
      uint64_t m0 = ~0ull, m1 = 0;
      for (int bq = 0; bq < B; ++bq) {
        const uint64_t* t = &tr[((size_t)nwg + bq) * 8];
        m0 = std::min(m0, t[0]);
        m1 = std::max(m1, t[3]);
        for (int j = 1; j < 4; ++j) mp[j] += (double)(t[j] - t[0]);
        ce += (double)(uint32_t)t[4];
        cp += (double)(t[4] >> 32);
      }
      fprintf(stderr, "[bb sq trace] B=%d nwg=%d rpw=%d pass (us from workgroup start): queries-loaded %.2f "
              "queries-normalised %.2f mfma-done %.2f order-images %.2f end %.2f | starts spread %.2f, span %.2f | merge: "
              "gathered %.2f rescored %.2f end %.2f, span %.2f, cands %.1f + r0 %.1f | pass end -> merge start %.2f\n",
              B, nwg, rpw, ph[1] / nwg / 100, ph[2] / nwg / 100, ph[3] / nwg / 100, ph[5] / nwg / 100, ph[4] / nwg / 100,
              (double)s_max / 100,
              (double)(tend - t0) / 100, mp[1] / B / 100, mp[2] / B / 100, mp[3] / B / 100, (double)(m1 - m0) / 100, ce / B,
              cp / B, ((double)m0 - (double)tend) / 100);
    }
    if (out_keys) {
      const hipMemcpyKind kind = res->where == BB_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
      if ((rc = s_copy(res->keys, x->keys.p, (size_t)sides * B * K_int * 8, kind, s))) return rc;
      if (drop) {
        if ((rc = s_copy(res->max_keys, x->maxk.p, (size_t)B * 8, kind, s))) return rc;
      } else if (res->where == BB_DEVICE) {
        if ((rc = s_memset(res->max_keys, 0, (size_t)B * 8, s))) return rc;
      }
      else memset(res->max_keys, 0, (size_t)B * 8);
    } else if (hyb) {  // the union blend of _combine_recommendations (:789-843), as the large-batch path
      FinalizeArgs fa{};
      fa.keys = (const uint64_t*)x->keys.p;
      fa.max_keys = (const uint64_t*)x->maxk.p;
      fa.P = 1;
      fa.sides = 2;
      fa.B = B;
      fa.K_int = K_int;
      fa.drop_rank0 = 1;
      fa.k = q->k;
      fa.k_side = q->k_side > 0 ? q->k_side : 2 * q->k;
      fa.hybrid = 1;
      fa.w_content = q->w_content;
      fa.w_cf = q->w_cf;
      fa.scores = f_sc;
      fa.ids = f_id;
      fa.counts = f_cnt;
      fa.n_rows = B;
      if ((rc = timed(x, K_FIN, s, [&] { return launch_finalize(fa, s); }))) return rc;
    }
    if (host_res) {
      BB_HIP(hipMemcpyAsync(res->scores, f_sc, (size_t)B * q->k * 4, hipMemcpyDeviceToHost, s));
      BB_HIP(hipMemcpyAsync(res->ids, f_id, (size_t)B * q->k * 8, hipMemcpyDeviceToHost, s));
      if (res->counts) BB_HIP(hipMemcpyAsync(res->counts, f_cnt, (size_t)B * 4, hipMemcpyDeviceToHost, s));
    }
    if (host_res || where == BB_HOST || (out_keys && res->where != BB_DEVICE))
      if ((rc = s_sync(s))) return rc;
    return BB_OK;
  }

  // workspace
  const size_t es = elem_size(x->dtype);
  if ((rc = x->S.ensure((size_t)Bc * lds * 4))) return rc;
  // tmax + pmax, twice for the dual hybrid launch (both sides' scans before both selects)
  if ((rc = x->tmax.ensure((size_t)Bc * ldt * 4 * 2 * (q->mode == BB_MODE_HYBRID ? 2 : 1)))) return rc;
  // query rows: index dtype, or three bf16 planes (6 B / element) for the split scan
  const size_t qes_c = x->items3.p ? std::max<size_t>(es, 6) : es, qes_f = x->cf3.p ? std::max<size_t>(es, 6) : es;
  if (need_content && (rc = x->qn.ensure(std::max((size_t)Bc * x->Dpad * qes_c, (size_t)Bc * x->Dpad_b * 2)))) return rc;
  if (need_cf && (rc = x->qcf.ensure(std::max((size_t)Bc * x->Rpad * qes_f, (size_t)Bc * x->Rpad_b * 2)))) return rc;
  if (rr_c && ((rc = x->qf32.ensure((size_t)Bc * x->Dpad * 4)) || (rc = x->qeps.ensure((size_t)Bc * 4)) ||
               (rc = x->qh.ensure((size_t)Bc * 4))))
    return rc;
  if (rr_f && ((rc = x->qcf32.ensure((size_t)Bc * x->Rpad * 4)) || (rc = x->qcfeps.ensure((size_t)Bc * 4)) ||
               (rc = x->qcfh.ensure((size_t)Bc * 4))))
    return rc;
  // re-rank scans write an int16 score image (2 B per score: half the slab traffic of f32;
  // the quantum is folded into ε, common.h rr_quantum).  BB_S16=0 (A/B runs) keeps f32.
  // BB_S16: 0 off, 1 every re-rank scan, 2 only scan4 (query chunks > 256 rows)
  static const int s16_env = ab_env("BB_S16") ? atoi(ab_env("BB_S16")) : 1;
  // The block select hands its candidates to a separate rerank_kernel launch; BB_RR_FUSED=1
  // makes the select kernel rescore them itself.  Measured on one box (r02zd, configs[1]):
  // fused serial p50 52.6 us vs 55.5 us split, but with three batches in flight split
  // 8.30 M q/s vs fused 7.66 M q/s — two shorter launches leave the CUs to the next batch's
  // scan sooner than one long one.  (The one-wave select of query chunks > 256 rows always
  // rescores in place.)
  static const bool rr_split = !(ab_env("BB_RR_FUSED") && atoi(ab_env("BB_RR_FUSED")) == 1);
  if ((rr_c || rr_f) && rr_split &&
      ((rc = x->rr_out.ensure((size_t)Bc * kRrCap * 8)) || (rc = x->rr_cnt.ensure((size_t)Bc * 4)) ||
       (rc = x->rr_thr.ensure((size_t)Bc * 8)) || (rc = x->rr_r0.ensure((size_t)Bc * kRrR0Cap * 4)) ||
       (rc = x->rr_r0n.ensure((size_t)Bc * 4))))
    return rc;
  const size_t side_keys = (size_t)Bc * K_int;
  if ((rc = x->keys.ensure(2 * sides * side_keys * 8))) return rc;
  if ((rc = x->maxk.ensure((size_t)Bc * 8))) return rc;
  const bool host_out = !out_keys && res->where != BB_DEVICE;
  if (host_out) {
    if ((rc = x->out_sc.ensure((size_t)B * q->k * 4)) || (rc = x->out_id.ensure((size_t)B * q->k * 8)) ||
        (rc = x->out_cnt.ensure((size_t)B * 4)))
      return rc;
  }
  float* o_sc = host_out ? (float*)x->out_sc.p : res->scores;
  int64_t* o_id = host_out ? (int64_t*)x->out_id.p : res->ids;
  int32_t* o_cnt = host_out ? (int32_t*)x->out_cnt.p : res->counts;
  uint64_t* keys = (uint64_t*)x->keys.p;
  uint64_t* maxk = (uint64_t*)x->maxk.p;
  // single-list modes (semantic / similar / CF) finish inside the last select launch
  const bool fuse_final = !out_keys && sides == 1;

  // ---- streaming top-K geometry (SURVEY.md §8d C4/C5 scale): a pilot slab of the first
  // n0 items gives each query an exact top-K_int over the sample, whose last key bounds the
  // K_int-th score from below; one scan over all items then appends every eligible score
  // reaching that bound to per-lane regions (~K_int·n/n0 per query) and a candidate select
  // finishes the exact top-K.  No B×n score slab is written. ----
  // Two-level bound (when the pilot is a small sample of the index): pass A streams items
  // [0, n1) against the pilot bound and a candidate select turns them into the exact
  // top-K_int of [0, n1); its last key bounds pass B over [n1, n), whose candidates join
  // that list in the final select.  Expected appends per query drop from K_int·n/n0 to
  // K_int·(n1/n0 + n/n1), minimal at n1 = sqrt(n·n0): 16 -> 7 K_int at n0 = n/16 (1M rows),
  // 76 -> 16 K_int at n0 = n/76 (10M rows).  Appends are what the streaming scan pays for.
  static const int refine_env = ab_env("BB_STREAM_REFINE") ? atoi(ab_env("BB_STREAM_REFINE")) : 1;
  // Auto (measured): from n >= 8·n0 on indexes of 500K+ rows with query chunks of 256+
  // (10M x 384, B=8192: 83 -> 71 ms; 1.25M: 12.4 -> 11.7 ms); on smaller indexes or batches
  // the extra candidate select costs more than the appends it saves (125K rows: 1.36 ->
  // 1.45 ms, B=1: +8 %).  BB_OPT_STREAM_REFINE forces it (tests) when n >= 2·n0.
  const int refine_sel = x->refine_opt >= 0 ? x->refine_opt : (refine_env == 0 ? 0 : -1);
  const bool refine = stream && refine_sel != 0 && x->n >= 2 * n0 &&
                      (refine_sel == 1 || (x->n >= 8 * n0 && x->n >= 500000 && Bc >= 256));
  const int64_t n1 = refine ? std::min<int64_t>(x->Npad - kTileRows,
                                                std::max<int64_t>(n0, round_up((int64_t)std::sqrt((double)x->n * (double)n0),
                                                                               kTileRows)))
                            : x->n;
  // streaming pass p (0 = A, 1 = B): item range and the appends expected per query
  auto pass_cols = [&](int p, int64_t& c0, int64_t& nc) {
    c0 = p == 0 ? 0 : n1;
    nc = p == 0 ? std::min<int64_t>(n1, x->n) : x->n - n1;
  };
  // regions per query and keys per region for a query chunk of bpad rows: ~4x the expected
  // candidates spread over the regions, plus slack
  auto stream_geom = [&](int bpad_c, int p, int& regions, int& cap) {
    int64_t c0, nc;
    pass_cols(p, c0, nc);
    regions = 2 * scan_chunks(x->dtype, bpad_c, (int)(round_up(nc, kTileRows) / 32), false);
    const double base = p == 0 ? (double)std::min<int64_t>(n0, x->n) : (double)n1;
    const double expect = (double)K_int * ((double)nc / base) + K_int;
    cap = (int)round_up((int64_t)(4.0 * expect / regions) + 32, 16);
  };
  if (stream) {
    size_t need_keys = 0, need_rg = 0;
    for (int bp : {(int)pad_rows(std::min<int64_t>(Bc, B)), (int)pad_rows(B - (B - 1) / Bc * Bc)})
      for (int p = 0; p < (refine ? 2 : 1); ++p) {
        int rg, cap;
        stream_geom(bp, p, rg, cap);
        need_keys = std::max(need_keys, (size_t)bp * rg * cap);
        need_rg = std::max(need_rg, (size_t)bp * rg);
      }
    if (refine && ((rc = x->list1.ensure((size_t)Bc * K_int * 8)) || (rc = x->max1.ensure((size_t)Bc * 8))))
      return rc;
    if ((rc = x->pilot.ensure((size_t)Bc * K_int * 8)) || (rc = x->cand.ensure(need_keys * 8)) ||
        (rc = x->cand_cnt.ensure(need_rg * 4)) || (rc = x->cand_pmax.ensure(need_rg * 8)))
      return rc;
    // the overflow flag: coherent pinned host memory the candidate selects store into, cleared
    // here by the host (every earlier search on this index has completed: the stream path
    // waits for its flag before returning) and read after the search's one wait — no fill or
    // copy launch on the path
    if (!x->ovf_host) BB_HIP(hipHostMalloc((void**)&x->ovf_host, 64, hipHostMallocCoherent));
    *(volatile uint32_t*)x->ovf_host = 0u;
  }

  for (int64_t b0 = 0; b0 < B; b0 += Bc) {
    const int bc = (int)std::min<int64_t>(Bc, B - b0);
    const int bpad = (int)pad_rows(bc);
    // ---- query prep: fused into the scan kernel's prologue when it runs (gathered item
    // rows; raw f32 rows with 16-B rows), otherwise a prep launch fills qn / qcf ----
    // split-precision scan (f32 index with bf16 planes): queries always come from a prep
    // launch writing the q3f plane image (coalesced query loads in the scan)
    const bool s3_c = !rr_c && need_content && x->items3.p && scan3_supported(bpad, x->Dpad);
    const bool s3_f = !rr_f && need_cf && x->cf3.p && scan3_supported(bpad, x->Rpad);
    const bool scan_c = !rr_c && !s3_c && gemm_uses_scan(x->dtype, bpad, x->Dpad);
    const bool scan_f = !rr_f && !s3_f && need_cf && gemm_uses_scan(x->dtype, bpad, x->Rpad);
    const bool gather_c = q->mode != BB_MODE_SEMANTIC && d_items;
    const float* rows_c = d_rows ? (const float*)((const char*)d_rows + (size_t)b0 * x->d * es_q) : nullptr;
    const float* rows_f = d_cf ? (const float*)((const char*)d_cf + (size_t)b0 * x->r * es_cf) : nullptr;
    static const bool no_fuse = ab_env("BB_NO_FUSE_PREP") != nullptr;
    const bool fuse_c = !no_fuse && need_content && scan_c &&
                        (gather_c || (x->dtype == F32 && q->q_dtype == F32 && x->d % 4 == 0 && rows_c &&
                                      ((uintptr_t)rows_c & 15) == 0));
    const bool fuse_f = !no_fuse && scan_f && x->dtype == F32 && q->q_cf_dtype == F32 && x->r % 4 == 0 && rows_f &&
                        ((uintptr_t)rows_f & 15) == 0;
    // exact re-rank on scan2 (query chunks <= 128 rows): the scan's prologue rounds the f32
    // query rows (raw, or the liked sets' stored rows) to the bf16 operand itself and its
    // chunk-0 workgroups write the f32 rows + ε the select needs — no prep launch
    // (opt-in, BB_RR_FUSE_PREP: the per-lane query loads of the prologue cost more than the
    // prep launch they replace — r02s: scan 20.8 -> 33.8 us vs prep 7.6 us at configs[1])
    static const bool rr_fuse_prep = ab_env("BB_RR_FUSE_PREP") != nullptr;
    const bool rrfuse_c = rr_fuse_prep && !no_fuse && rr_c && !scan4_used(BF16, bpad) &&
                          (gather_c || (q->q_dtype == F32 && x->d % 4 == 0 && rows_c && ((uintptr_t)rows_c & 15) == 0));
    const bool rrfuse_f = rr_fuse_prep && !no_fuse && rr_f && !scan4_used(BF16, bpad) && q->q_cf_dtype == F32 && x->r % 4 == 0 &&
                          rows_f && ((uintptr_t)rows_f & 15) == 0;
    // int16 score image on the re-rank scans (not with the fused re-rank prologue, whose
    // chunk-0 workgroups write the bound while the others already store scores)
    const bool s16_on = s16_env == 1 || (s16_env == 2 && scan4_used(BF16, bpad));
    // list geometry per side (the CF side's narrow rows take finer chunks: scan4_list_chunks)
    int l_nch[2] = {0, 0}, l_np[2] = {0, 0}, l_G[2] = {0, 0};
    const bool lgeo_c = rr_c && list_geom(bpad, x->Dpad_b * 2 / 16, l_nch[0], l_np[0], l_G[0]);
    const bool lgeo_f = rr_f && list_geom(bpad, x->Rpad_b * 2 / 16, l_nch[1], l_np[1], l_G[1]);
    const bool list_c = lgeo_c && rr_c && !rrfuse_c && gemm_uses_scan(BF16, bpad, x->Dpad_b);
    const bool list_f = lgeo_f && rr_f && !rrfuse_f && gemm_uses_scan(BF16, bpad, x->Rpad_b);
    // raw-query lists (semantic searches on scan2, f32 query rows, small chunks): the scan
    // rounds the RAW rows to its bf16 operand and the list select normalises them and derives
    // ε itself — no prep launch on the path.  Every item chunk's workgroups convert their
    // query rows again, so it pays only for small chunks: at 256 rows (configs[1]) the scan
    // grew 16.6 -> 20.4 us and three batches in flight served 8.8 instead of 10.2 M q/s,
    // while the serial search fell 48 -> 43 us (r03_raw); serial B = 1 / 16: 30.0 -> 28.8 /
    // 34.5 -> 33.0 us, B = 64 unchanged (r03_raw3).  BB_RR_RAW (A/B runs): 0 / 1 forces it
    // off / on; auto = chunks of at most kRrRawRows rows.
    static const int rr_raw_env = ab_env("BB_RR_RAW") ? atoi(ab_env("BB_RR_RAW")) : -1;
    const bool rr_raw_on = rr_raw_env >= 0 ? rr_raw_env != 0 : bc <= kRrRawRows;
    const bool rraw_c = rr_raw_on && list_c && q->mode == BB_MODE_SEMANTIC && !scan4_used(BF16, bpad) &&
                        q->q_dtype == F32 && x->d % 4 == 0 && x->d <= kRrMaxD && rows_c && ((uintptr_t)rows_c & 15) == 0;
    const bool s16_c = !list_c && s16_on && rr_c && !rrfuse_c && gemm_uses_scan(BF16, bpad, x->Dpad_b);
    const bool s16_f = !list_f && s16_on && rr_f && !rrfuse_f && gemm_uses_scan(BF16, bpad, x->Rpad_b);
    const size_t list_b[2] = {(size_t)l_nch[0] * l_np[0] * (bpad / 32) * 64 * 16,
                              (size_t)l_nch[1] * l_np[1] * (bpad / 32) * 64 * 16};
    if ((list_c || list_f) &&
        ((rc = x->lists.ensure(list_b[0] + list_b[1])) ||
         (list_c && drop && (rc = x->r0lists.ensure((size_t)l_nch[0] * (bpad / 32) * 64 * 8)))))
      return rc;
    // a shadow's ids are mapped by the list / int16-image selects and finalize1 only: any other
    // path leaves it before its first launch (the caller then runs the full search)
    if (x->shadow && (bc < B || (need_content && !list_c && !s16_c) || (need_cf && !list_f && !s16_f)))
      return b0 == 0 ? kNoCompact : fail(BB_E_STATE, "internal: a packed search's later query chunk left the list path");
    // the prep launches of both sides (hybrid) go out as one launch
    const bool prep_c = need_content && !fuse_c && !rrfuse_c && !rraw_c, prep_f = need_cf && !fuse_f && !rrfuse_f;
    PrepArgs pa_c{}, pa_f{};
    if (prep_c) {
      PrepArgs& pa = pa_c;
      pa.Bpad = bpad;
      pa.B = bc;
      pa.d = x->d;
      pa.Dpad = x->Dpad;
      pa.out = x->qn.p;
      pa.out_dtype = s3_c ? SPLIT3 : x->dtype;
      if (rr_c) {  // f16 operand + f32 row + bound
        pa.out_dtype = F16;
        pa.Dpad = x->Dpad_b;
        pa.out_f32 = (float*)x->qf32.p;
        pa.Dpad_f = x->Dpad;
        pa.eps_out = (float*)x->qeps.p;
        pa.istats = (const float*)x->rr_stats.p;
        pa.h_out = s16_c || list_c ? (float*)x->qh.p : nullptr;
      }
      pa.items = x->items.p;
      pa.n_items = x->n;
      pa.id_offset = x->id_offset;
      if (q->mode != BB_MODE_SEMANTIC && d_items) {
        pa.item_ids = (const int64_t*)d_items + b0;
      } else {
        pa.src = (const char*)d_rows + (size_t)b0 * x->d * es_q;
        pa.src_dtype = q->q_dtype;
        pa.src_ld = x->d;
        pa.normalize = q->mode == BB_MODE_SEMANTIC ? 1 : 0;
      }
    }
    if (prep_f) {
      PrepArgs& pa = pa_f;
      pa.Bpad = bpad;
      pa.B = bc;
      pa.d = x->r;
      pa.Dpad = x->Rpad;
      pa.out = x->qcf.p;
      pa.out_dtype = s3_f ? SPLIT3 : x->dtype;
      if (rr_f) {
        pa.out_dtype = F16;
        pa.Dpad = x->Rpad_b;
        pa.out_f32 = (float*)x->qcf32.p;
        pa.Dpad_f = x->Rpad;
        pa.eps_out = (float*)x->qcfeps.p;
        pa.istats = (const float*)x->rr_stats.p + 4;
        pa.h_out = s16_f || list_f ? (float*)x->qcfh.p : nullptr;
      }
      pa.src = (const char*)d_cf + (size_t)b0 * x->r * es_cf;
      pa.src_dtype = q->q_cf_dtype;
      pa.src_ld = x->r;
      pa.normalize = 0;
    }
    // the bf16 operand of a scan launch goes out in its lane order (scan4_q_offset /
    // scan2_q_offset): coalesced prologue loads (at 1,024 x 384 the row-major loads took ~8
    // of a 23 us scan4).  BB_QPERM2=0 (A/B runs) keeps scan2's row-major operand.
    static const bool qperm2_env = !(ab_env("BB_QPERM2") && atoi(ab_env("BB_QPERM2")) == 0);
    const int perm_kind = scan4_used(BF16, bpad) ? 1 : qperm2_env ? 2 : 0;
    const bool perm_c = perm_kind && prep_c && !s3_c &&
                        (rr_c ? gemm_uses_scan(BF16, bpad, x->Dpad_b) : x->dtype == BF16 && scan_c);
    const bool perm_f = perm_kind && prep_f && !s3_f &&
                        (rr_f ? gemm_uses_scan(BF16, bpad, x->Rpad_b) : x->dtype == BF16 && scan_f);
    pa_c.q_perm = perm_c ? perm_kind : 0;
    pa_f.q_perm = perm_f ? perm_kind : 0;
    if (x->shadow && x->cjob_set) {
      // a packed search: the packing launch (compact.hip) runs this prep in its query
      // workgroups; the liked sets' rows come from the full index by their original ids
      CompactArgs cj = x->cjob;
      if (prep_c) {
        cj.prep_c = pa_c;
        if (pa_c.item_ids) {
          cj.prep_c.items = cj.items;
          cj.prep_c.n_items = cj.n;
          cj.prep_c.id_offset = cj.id_offset;
        }
      }
      if (prep_f) cj.prep_f = pa_f;
      cj.n_query_wg = (cj.B + 3) / 4;
      x->cjob_set = false;
      if ((rc = timed(x, K_PACK, s, [&] { return launch_compact(cj, s); }))) return rc;
    } else if (prep_c && prep_f) {
      if ((rc = timed(x, K_PREP, s, [&] { return launch_prep2(pa_c, pa_f, s); }))) return rc;
    } else if (prep_c || prep_f) {
      if ((rc = timed(x, K_PREP, s, [&] { return launch_prep(prep_c ? pa_c : pa_f, s); }))) return rc;
    }
    // ---- per side: slabs of gemm + select ----
    // Hybrid on the exact re-rank path with both sides on scan4 + the one-wave select: the two
    // sides' scans go out as ONE launch and their selects as one (scan4_dual_kernel,
    // select_rr_wave_dual_kernel); each side keeps its own half of the int16 image and its own
    // maxima / flag rows.  Measured (r02za, configs[2]): serial p50 222 -> 173 us (scan 86 ->
    // 77 us, select 116 -> 62 us per step); with three batches in flight 6.6 -> 6.3 M q/s.
    // BB_DUAL=0 (A/B runs) keeps one launch per side.  The list scans (round 4) go out one per
    // side by default: the CF side's narrow rows now take twice the chunks at two workgroups per
    // CU (scan4_list_chunks), which one dual launch — held to one workgroup per CU by the
    // content side's registers — cannot give them (configs[2]: scans 54.1 us dual vs 48.5 us
    // per side, serial 0.126 vs 0.121 ms, r04p); BB_DUAL=1 forces the dual list scan.
    static const int dual_sel = ab_env("BB_DUAL") ? atoi(ab_env("BB_DUAL")) : -1;
    static const int sel_wave_env0 = ab_env("BB_SELECT_WAVE") ? atoi(ab_env("BB_SELECT_WAVE")) : -1;
    // (a packed constraint-first search's scans are a few tiles each: one launch for both
    // sides, serial 74 -> 69 us at configs[2], r06i)
    const bool dual = dual_sel != 0 && q->mode == BB_MODE_HYBRID && sides == 2 &&
                      ((s16_c && s16_f) || (list_c && list_f && (dual_sel == 1 || x->shadow))) &&
                      !stream &&
                      n_slabs == 1 && scan4_used(BF16, bpad) && scan4_dual_supported((int)x->Dpad_b / 8, (int)x->Rpad_b / 8) &&
                      std::min<int64_t>(slab, x->n) <= 32768 && K_int <= 256 && sel_wave_env0 != 0 && bc > 256;
    if (dual && (rc = x->rr_flags.ensure((size_t)Bc * 4 * 2))) return rc;
    GemmArgs ga_dual0{};
    SelectArgs sa_dual0{};
    int final_pp = 0;
    for (int side = 0; side < sides; ++side) {
      const bool cf_side = (q->mode == BB_MODE_CF) || (q->mode == BB_MODE_HYBRID && side == 1);
      const bool side_drop = drop && side == 0;
      bool pilot_topm = false;  // this side's pilot left one bound key per row (thr_ld 1)
      // stream: pass 0 = the pilot slab [0, n0) -> pilot lists, pass 1 = the streaming scan
      // (A: [0, n1)), pass 2 with the two-level bound (B: [n1, n))
      const int64_t n_pass = stream ? (refine ? 3 : 2) : n_slabs;
      for (int64_t sl = 0; sl < n_pass; ++sl) {
        const bool pilot = stream && sl == 0, spass = stream && sl >= 1;
        const int sp = (int)sl - 1;                       // streaming pass index
        const bool last_spass = spass && sl == n_pass - 1;
        int64_t c0 = stream ? 0 : sl * slab, nc_s = 0;
        if (spass) pass_cols(sp, c0, nc_s);
        const int ncols = (int)(spass ? nc_s : pilot ? std::min<int64_t>(n0, x->n) : std::min<int64_t>(slab, x->n - c0));
        const int ncols_pad = (int)round_up(ncols, kTileRows);
        GemmArgs ga{};
        ga.Q = cf_side ? x->qcf.p : x->qn.p;
        ga.q_perm = (cf_side ? perm_f : perm_c) ? perm_kind : 0;
        ga.ldq = cf_side ? x->Rpad : x->Dpad;
        ga.X = (const char*)(cf_side ? x->cf.p : x->items.p) + (size_t)c0 * ga.ldq * es;
        ga.ldx = ga.ldq;
        ga.S = (float*)x->S.p;
        ga.lds = lds;
        ga.Mpad = bpad;
        ga.Ncols = ncols_pad;
        ga.Kpad = (int)ga.ldq;
        ga.M_valid = bc;
        ga.n_valid = ncols;
        ga.slab_start = c0;
        // the scan epilogue is branch-free: every bitset pointer is valid
        // per-query exclusions: the CF side's rated items; in a shadow also the content side's
        // rank-0 item (x->cur_cexcl)
        const uint32_t* side_excl = cf_side ? (const uint32_t*)d_excl : x->cur_cexcl;
        const bool has_excl = side_excl != nullptr;
        ga.mask = d_mask ? (const uint32_t*)d_mask : (const uint32_t*)x->ones.p;
        ga.present = (const uint32_t*)(cf_side ? x->cf_present.p : x->items_present.p);
        ga.excl = has_excl ? side_excl + (size_t)b0 * nw : (const uint32_t*)x->zeros.p;
        ga.excl_ld = has_excl ? nw : 0;
        ga.tmax = (uint32_t*)x->tmax.p + (dual && side ? (size_t)Bc * ldt * 2 : 0);
        // present maxima only where a rank 0 is dropped (the content side of similar / hybrid):
        // the scans skip the half-wave of maxima stores otherwise (the dual scan always
        // stores both: a uniform store measured 2.6% faster there than the masked one)
        ga.pmax = side_drop || dual ? ga.tmax + (size_t)Bc * ldt : nullptr;
        if (dual && side) ga.S = (float*)((int16_t*)x->S.p + (size_t)Bc * lds);  // the image's second half
        ga.ldt = ldt;
        int regions = 0, cand_cap = 0;
        if (spass) {
          stream_geom(bpad, sp, regions, cand_cap);
          ga.thr_keys = (const uint64_t*)(sp == 0 ? x->pilot.p : x->list1.p);
          ga.thr_ld = sp == 0 && pilot_topm ? 1 : K_int;
          ga.cand = (uint64_t*)x->cand.p;
          ga.cand_cnt = (uint32_t*)x->cand_cnt.p;
          ga.cand_pmax = side_drop ? (uint64_t*)x->cand_pmax.p : nullptr;
          ga.cand_cap = cand_cap;
          ga.gid0 = (uint32_t)(x->id_offset + c0);
          if (scan_chunks(x->dtype, bpad, ncols_pad / 32, false) * 2 != regions)
            return fail(BB_E_STATE, "stream geometry mismatch");
        }
        if (cf_side ? fuse_f : fuse_c) {
          ga.q_d = cf_side ? x->r : x->d;
          if (!cf_side && gather_c) {
            ga.q_ids = (const int64_t*)d_items + b0;
            ga.q_id_offset = x->id_offset;
            ga.q_n_items = x->n;
            ga.q_items_base = x->items.p;
          } else {
            ga.q_src = cf_side ? rows_f : rows_c;
            ga.q_src_ld = ga.q_d;
            ga.q_normalize = !cf_side && q->mode == BB_MODE_SEMANTIC;
          }
        }
        if (cf_side ? rrfuse_f : rrfuse_c) {
          ga.q_istats = (const float*)x->rr_stats.p + (cf_side ? 4 : 0);
          ga.q_f32_out = (float*)(cf_side ? x->qcf32.p : x->qf32.p);
          ga.q_f32_ld = cf_side ? x->Rpad : x->Dpad;
          ga.q_eps_out = (float*)(cf_side ? x->qcfeps.p : x->qeps.p);
          if (!cf_side && gather_c) {  // the stored f32 rows (normalised, zero padded)
            ga.q_ids = (const int64_t*)d_items + b0;
            ga.q_id_offset = x->id_offset;
            ga.q_n_items = x->n;
            ga.q_items_base = x->items.p;
            ga.q_src_ld = x->Dpad;
            ga.q_d = x->Dpad;
          } else {
            ga.q_src = cf_side ? rows_f : rows_c;
            ga.q_d = cf_side ? x->r : x->d;
            ga.q_src_ld = ga.q_d;
            ga.q_normalize = !cf_side && q->mode == BB_MODE_SEMANTIC;
          }
        }
        DevBuf& planes = cf_side ? x->cf3 : x->items3;
        const bool rr_side = cf_side ? rr_f : rr_c;
        if (rr_side) {
          // approximate scan: f16 queries x the one-product f16 item copy
          const int64_t w = cf_side ? x->Rpad_b : x->Dpad_b;
          ga.f16 = 1;
          ga.X = (const char*)(cf_side ? x->cf_bf.p : x->items_bf.p) + (size_t)c0 * w * 2;
          ga.ldx = ga.ldq = w;
          ga.Kpad = (int)w;
          ga.s_h = (cf_side ? s16_f || list_f : s16_c || list_c) ? (const float*)(cf_side ? x->qcfh.p : x->qh.p)
                                                                   : nullptr;
          if (!cf_side && rraw_c) {
            ga.q_raw = 1;
            ga.q_src = rows_c;
            ga.q_src_ld = x->d;
            ga.q_d = x->d;
            ga.q_istats = (const float*)x->rr_stats.p;
            ga.q_h_out = (float*)x->qh.p;
            ga.q_eps_out = (float*)x->qeps.p;
          }
          if (cf_side ? list_f : list_c) {
            ga.lists = (uint32_t*)((char*)x->lists.p + (cf_side ? list_b[0] : 0));
            ga.r0lists = side_drop ? (uint32_t*)x->r0lists.p : nullptr;
            ga.l_period = l_G[cf_side];
            ga.l_np = l_np[cf_side];
          }
          if (dual && side == 0) {
            ga_dual0 = ga;  // launched with side 1's
          } else if (dual) {
            const char* why = nullptr;
            if (!scan4_dual_args_ok(ga_dual0, ga, &why)) return fail(BB_E_ARG, std::string("hybrid dual scan: ") + why);
            if ((rc = timed(x, K_GEMM, s, [&] { return launch_scan4_dual(ga_dual0, ga, s); }))) return rc;
          } else {
            // BB_SCAN_TRACE (probe runs): phase stamps of the list scan's workgroups (scan4)
            static const bool scan_trace = kProbes && ab_env("BB_SCAN_TRACE") != nullptr;
            const bool tr = scan_trace && ga.lists && scan4_used(BF16, bpad);
            if (tr) {
              if ((rc = x->trace.ensure((size_t)4096 * 64))) return rc;
              BB_HIP(hipMemsetAsync(x->trace.p, 0, (size_t)4096 * 64, s));
              ga.trace = (uint64_t*)x->trace.p;
            }
            if ((rc = timed(x, K_GEMM, s, [&] { return launch_gemm(BF16, ga, s); }))) return rc;
            if (tr) {
              std::vector<uint64_t> t((size_t)4096 * 8);
              BB_HIP(hipMemcpyAsync(t.data(), x->trace.p, t.size() * 8, hipMemcpyDeviceToHost, s));
              BB_HIP(hipStreamSynchronize(s));
              uint64_t t0 = ~0ull, t1 = 0;
              double acc[6] = {0}, tiles = 0, cyc = 0;
              int nwg = 0, n5 = 0;
              for (size_t w = 0; w < 4096; ++w) {
                const uint64_t* r = &t[w * 8];
                if (!r[0] || !r[5]) continue;
                ++nwg;
                t0 = std::min(t0, r[0]);
                t1 = std::max(t1, r[5]);
                for (int j = 1; j < 6; ++j)
                  if (j != 3 || r[3]) acc[j] += (double)(r[j] - r[0]);
                n5 += r[3] != 0;
                tiles += (double)r[6];
                cyc += (double)r[7];
              }
              double st = 0;
              for (size_t w = 0; w < 4096; ++w)
                if (t[w * 8] && t[w * 8 + 5]) st += (double)(t[w * 8] - t0);
              nwg = std::max(nwg, 1);
              fprintf(stderr, "[bb scan trace] side=%d wgs=%d tiles/wg=%.1f us-from-wg-start: prologue %.2f tile1 %.2f "
                      "tile5 %.2f loop %.2f end %.2f | start skew avg %.2f | span %.2f | shader clock %.2f GHz\n", (int)cf_side, nwg,
                      tiles / nwg, acc[1] / nwg / 100, acc[2] / nwg / 100, n5 ? acc[3] / n5 / 100 : 0.0,
                      acc[4] / nwg / 100, acc[5] / nwg / 100, st / nwg / 100, (double)(t1 - t0) / 100,
                      acc[5] > 0 ? cyc / (acc[5] / 100.0) / 1e3 : 0.0);
            }
          }
        } else if (cf_side ? s3_f : s3_c) {
          // split-precision scan: items, gathered rows and prepped queries are bf16 planes
          const int64_t w = ga.ldq;
          ga.X = (const char*)planes.p + (size_t)c0 * 3 * w * 2;
          ga.ldx = 3 * w;
          ga.ldq = 3 * w;
          if ((rc = timed(x, K_GEMM, s, [&] { return launch_scan3(ga, s); }))) return rc;
        } else {
          // Streaming pilot on scan4 (bf16 index): no B×n0 score image and no pilot select —
          // the scan keeps each lane's top-m eligible half-tile maxima and pilot_bound_kernel
          // turns them into one bound key per row (configs[3]: the image was 1.0 GB written
          // plus 0.7 GB of scattered maxima stores per batch)
          const int tiles_p = ncols_pad / 32;
          bool use_top = pilot && x->dtype == BF16 && scan4_used(BF16, bpad) && gemm_uses_scan(BF16, bpad, ga.Kpad);
          const int nch_p = use_top ? scan_chunks(BF16, bpad, tiles_p, false) : 0;
          const int m_p = use_top ? scan4_pilot_m(ga.Kpad) : 0;
          use_top = use_top && 2 * nch_p * m_p <= 16 * 256;
          if (pilot) pilot_topm = use_top;
          if (use_top) {
            if ((rc = x->pilot_top.ensure((size_t)nch_p * (bpad / 32) * 64 * m_p * 4))) return rc;
            ga.pilot_top = (uint32_t*)x->pilot_top.p;
            ga.pilot_m = m_p;
          }
          if ((rc = timed(x, K_GEMM, s, [&] { return launch_gemm(x->dtype, ga, s); }))) return rc;
          if (use_top) {
            if ((rc = timed(x, K_SELECT, s, [&] {
                   return launch_pilot_bound((const uint32_t*)x->pilot_top.p, nch_p, m_p, bpad / 32, K_int, bc,
                                             (uint64_t*)x->pilot.p, s);
                 })))
              return rc;
            continue;  // no pilot select
          }
        }
        if (spass) {
          // candidate select: exact top-K_int of the appended candidates of each query
          CandSelectArgs ca{};
          ca.cand = ga.cand;
          ca.cand_cnt = ga.cand_cnt;
          ca.cand_pmax = ga.cand_pmax;
          ca.regions = regions;
          ca.cap = cand_cap;
          ca.K = K_int;
          ca.overflow = x->ovf_host;
          if (!last_spass) {  // pass A of the two-level bound: the exact list of [0, n1)
            ca.keys_out = (uint64_t*)x->list1.p;
            ca.max_out = side_drop ? (uint64_t*)x->max1.p : nullptr;
            if ((rc = timed(x, K_SELECT, s, [&] { return launch_cand_select(ca, bc, s); }))) return rc;
            continue;
          }
          if (refine) {
            ca.carry_in = (const uint64_t*)x->list1.p;
            ca.max_in = side_drop ? (const uint64_t*)x->max1.p : nullptr;
          }
          ca.keys_out = keys + (size_t)side * side_keys;
          ca.max_out = side_drop ? maxk : nullptr;
          if (fuse_final) {
            ca.out_scores = o_sc + (size_t)b0 * q->k;
            ca.out_ids = o_id + (size_t)b0 * q->k;
            ca.out_counts = o_cnt ? o_cnt + b0 : nullptr;
            ca.k_final = q->k;
          }
          if ((rc = timed(x, K_SELECT, s, [&] { return launch_cand_select(ca, bc, s); }))) return rc;
          final_pp = 0;
          continue;
        }
        const int pp = (int)(sl & 1);
        SelectArgs sa{};
        sa.S = (const float*)x->S.p;
        sa.lds = lds;
        sa.tmax = ga.tmax;
        sa.pmax = side_drop ? ga.pmax : nullptr;
        sa.ldt = ldt;
        sa.n_cols = ncols;
        sa.slab_start = c0;
        sa.gid0 = (uint32_t)(x->id_offset + c0);
        sa.mask = (const uint32_t*)d_mask;
        sa.present = (const uint32_t*)(cf_side ? x->cf_present.p : x->items_present.p);
        sa.excl = has_excl ? side_excl + (size_t)b0 * nw : nullptr;
        sa.idmap = x->shadow ? (const uint32_t*)x->idmap.p : nullptr;
        sa.excl_ld = nw;
        sa.K = K_int;
        // blocked score image: the split scan, and the bf16 scan with 64 queries per wave
        // every scan kernel (scan2 / scan3 / scan4) writes the blocked image; the tiled
        // gemm_nt fallback writes row-major S
        sa.s_blocked = ((cf_side ? s3_f : s3_c) || (cf_side ? scan_f : scan_c) ||
                        (rr_side && gemm_uses_scan(BF16, bpad, cf_side ? x->Rpad_b : x->Dpad_b))) ? 1 : 0;
        if (rr_side) {
          sa.rr_eps = (const float*)(cf_side ? x->qcfeps.p : x->qeps.p);
          sa.s_h = (cf_side ? s16_f : s16_c) ? (const float*)(cf_side ? x->qcfh.p : x->qh.p) : nullptr;
          sa.rr_x = (const float*)(cf_side ? x->cf.p : x->items.p);
          sa.rr_q = (const float*)(cf_side ? x->qcf32.p : x->qf32.p);
          sa.rr_ld = cf_side ? x->Rpad : x->Dpad;
          sa.rr_d = (int)sa.rr_ld;
          sa.rr_gid_base = (uint32_t)x->id_offset;
        }
        sa.carry_in = sl && !stream ? keys + ((size_t)(pp ^ 1) * sides + side) * side_keys : nullptr;
        sa.keys_out = pilot ? (uint64_t*)x->pilot.p : keys + ((size_t)pp * sides + side) * side_keys;
        sa.max_inout = side_drop && !pilot ? maxk : nullptr;
        sa.pmax = sa.max_inout ? ga.pmax : nullptr;
        sa.first_slab = sl == 0;
        if (fuse_final && !stream && sl == n_slabs - 1) {  // single-list mode: select writes the results
          sa.out_scores = o_sc + (size_t)b0 * q->k;
          sa.out_ids = o_id + (size_t)b0 * q->k;
          sa.out_counts = o_cnt ? o_cnt + b0 : nullptr;
          sa.k_final = q->k;
        }
        if (cf_side ? list_f : list_c) {
          // bounded candidate lists: one select launch per search (both hybrid sides together)
          sa.s_h = ga.s_h;
          sa.lists = ga.lists;
          sa.r0lists = ga.r0lists;
          sa.l_chunks = l_nch[cf_side];
          sa.l_tiles = ncols_pad / 32;
          sa.l_np = l_np[cf_side];
          sa.l_period = l_G[cf_side];
          sa.l_nb = bpad / 32;
          if (!cf_side && rraw_c) {
            sa.rr_q_raw = rows_c;
            sa.rr_q_raw_ld = x->d;
            sa.rr_q_raw_d = x->d;
          }
          // BB_LS_ABLATE (probe runs) bit 0: one cache-resident rescore row; BB_LS_BITWISE (A/B
          // runs): the bitwise K-th code search instead of the two-level histogram (ablate bit 2)
          static const int ls_ablate = (ab_env("BB_LS_ABLATE") ? atoi(ab_env("BB_LS_ABLATE")) : 0) |
                                       (ab_env("BB_LS_BITWISE") ? 4 : 0);
          sa.ablate = ls_ablate;
          final_pp = pp;
          if (q->mode == BB_MODE_HYBRID && side == 0 && list_f) {
            sa_dual0 = sa;  // launched with side 1's
            continue;
          }
          const bool both = q->mode == BB_MODE_HYBRID && side == 1 && list_c;
          static const bool ls_trace = kProbes && ab_env("BB_SELECT_TRACE") != nullptr;
          if (ls_trace) {  // probe runs: phase stamps of side 0's rows (16 words per row)
            if ((rc = x->trace.ensure((size_t)bc * 16 * 8))) return rc;
            BB_HIP(hipMemsetAsync(x->trace.p, 0, (size_t)bc * 128, s));
            (both ? sa_dual0 : sa).trace = (uint64_t*)x->trace.p;
          }
          if ((rc = timed(x, K_SELECT, s, [&] { return launch_select_list(both ? sa_dual0 : sa, both ? &sa : nullptr, bc, s); })))
            return rc;
          if (ls_trace) {
            std::vector<uint64_t> tr((size_t)bc * 16);
            BB_HIP(hipMemcpyAsync(tr.data(), x->trace.p, tr.size() * 8, hipMemcpyDeviceToHost, s));
            BB_HIP(hipStreamSynchronize(s));
            double acc[8] = {0}, oacc[8] = {0}, nc = 0, ov_items = 0, r0_items = 0, st_max = 0, st_avg = 0;
            int rows = 0, ovf_rows = 0, fb_rows = 0;
            uint64_t t0 = ~0ull, t1 = 0;
            for (int i = 0; i < bc; ++i) t0 = std::min<uint64_t>(t0, tr[(size_t)i * 16] ? tr[(size_t)i * 16] : ~0ull);
            for (int i = 0; i < bc; ++i) {
              const uint64_t* t = &tr[(size_t)i * 16];
              if (t[10]) { ++fb_rows; continue; }
              if (!t[7]) continue;
              const bool ov = (t[8] >> 32) != 0;
              ++rows;
              ovf_rows += ov;
              for (int j = 1; j < 8; ++j) (ov ? oacc : acc)[j] += t[j] ? (double)(t[j] - t[0]) : 0.0;
              nc += (double)(uint32_t)t[8];
              ov_items += (double)(uint32_t)t[9];
              r0_items += (double)(t[9] >> 32);
              st_max = std::max(st_max, (double)(t[0] - t0));
              st_avg += (double)(t[0] - t0);
              t1 = std::max(t1, t[7]);
            }
            const int nr = std::max(rows - ovf_rows, 1), no = std::max(ovf_rows, 1), ra = std::max(rows, 1);
            fprintf(stderr, "[bb list select trace] rows=%d (overflowed %d, fallback %d) us-from-row-start: loaded %.2f "
                    "bound %.2f classified %.2f appended %.2f rescored %.2f gmax %.2f end %.2f | overflow rows: "
                    "appended %.2f rescored %.2f end %.2f | cands %.1f ovf items %.1f r0 items %.1f | row start "
                    "avg %.2f max %.2f  span %.2f us\n", rows, ovf_rows, fb_rows, acc[1] / nr / 100, acc[2] / nr / 100,
                    acc[3] / nr / 100, acc[4] / nr / 100, acc[5] / nr / 100, acc[6] / nr / 100, acc[7] / nr / 100,
                    oacc[4] / no / 100, oacc[5] / no / 100, oacc[7] / no / 100, nc / ra, ov_items / ra, r0_items / ra,
                    st_avg / ra / 100, st_max / 100, (double)(t1 - t0) / 100);
            std::vector<int> ord(bc);
            for (int i = 0; i < bc; ++i) ord[i] = i;
            std::sort(ord.begin(), ord.end(), [&](int u, int w) { return tr[(size_t)u * 16 + 7] > tr[(size_t)w * 16 + 7]; });
            for (int k = 0; k < std::min(bc, 4); ++k) {  // the slowest rows
              const uint64_t* t = &tr[(size_t)ord[k] * 16];
              if (!t[7]) break;
              fprintf(stderr, "   slow row %d: start %.2f end %.2f | loaded %.2f bound %.2f cls %.2f app %.2f resc %.2f "
                      "| cands %u lists-ovf %u ovf items %u r0 items %u\n", ord[k], (double)(t[0] - t0) / 100,
                      (double)(t[7] - t0) / 100, (double)(t[1] - t[0]) / 100, (double)(t[2] - t[0]) / 100,
                      (double)(t[3] - t[0]) / 100, (double)(t[4] - t[0]) / 100, (double)(t[5] - t[0]) / 100,
                      (uint32_t)t[8], (uint32_t)(t[8] >> 32), (uint32_t)t[9], (uint32_t)(t[9] >> 32));
            }
          }
          continue;
        }
        // BB_SELECT_TRACE (probe runs): per-phase s_memrealtime stamps of every query row,
        // averaged over the rows and printed to stderr
        static const bool sel_trace = kProbes && ab_env("BB_SELECT_TRACE") != nullptr;
        if (sel_trace) {
          if ((rc = x->trace.ensure((size_t)bc * 8 * 8))) return rc;
          BB_HIP(hipMemsetAsync(x->trace.p, 0, (size_t)bc * 64, s));
          sa.trace = (uint64_t*)x->trace.p;
        }
        // one-slab re-rank of query chunks > 256 rows: one wave per query (select_rr_wave_kernel;
        // the rows it leaves — caps overflowed — go to the block select, which skips the
        // others).  Measured (r02y): B=1024 10.2 -> 10.5 M q/s, B=4096 10.9 -> 11.9 M q/s in
        // flight; at B <= 256 the block select's four waves per query win on latency (19 vs
        // 34 us per query).  BB_SELECT_WAVE=0/1 (A/B runs) forces it off / on.
        static const int sel_wave_env = ab_env("BB_SELECT_WAVE") ? atoi(ab_env("BB_SELECT_WAVE")) : -1;
        const bool sel_wave = rr_side && !sa.carry_in && ncols <= 32768 && K_int <= 256 &&
                              (!sa.out_scores || q->k <= 256) &&
                              (sel_wave_env == 1 || (sel_wave_env != 0 && bc > 256));
        // block select of a re-rank search: hand-off buffers for the rerank_kernel launch
        const bool rr_handoff = rr_side && rr_split && !sel_wave;
        if (rr_handoff) {
          sa.rr_out = (uint64_t*)x->rr_out.p;
          sa.rr_cnt = (uint32_t*)x->rr_cnt.p;
          sa.rr_thr = (uint32_t*)x->rr_thr.p;
          sa.rr_r0 = (uint32_t*)x->rr_r0.p;
          sa.rr_r0n = (uint32_t*)x->rr_r0n.p;
        }
        if (dual) {
          sa.S = ga.S;
          sa.rr_flags = (uint32_t*)x->rr_flags.p + (side ? Bc : 0);
          if (side == 0) {
            sa_dual0 = sa;  // launched with side 1's
          } else if ((rc = timed(x, K_SELECT, s, [&] { return launch_select_rr_wave_dual(sa_dual0, sa, bc, s); }))) {
            return rc;
          }
          final_pp = pp;
          continue;
        }
        if (sel_wave) {
          if ((rc = x->rr_flags.ensure((size_t)Bc * 4))) return rc;
          sa.rr_flags = (uint32_t*)x->rr_flags.p;
          if ((rc = timed(x, K_SELECT, s, [&] { return launch_select_rr_wave(sa, bc, s); }))) return rc;
          if (sel_trace) {  // wave select phases: bound, tile list, gather, rescore, emit
            std::vector<uint64_t> tr((size_t)bc * 8);
            BB_HIP(hipMemcpyAsync(tr.data(), x->trace.p, tr.size() * 8, hipMemcpyDeviceToHost, s));
            BB_HIP(hipStreamSynchronize(s));
            double acc[8] = {0};
            int rows = 0;
            for (int i = 0; i < bc; ++i) {
              const uint64_t* t = &tr[(size_t)i * 8];
              if (!t[5]) continue;  // left to the block select
              ++rows;
              for (int j = 1; j < 6; ++j) acc[j] += (double)(t[j] - t[0]);
              acc[6] += (double)t[6];
              acc[7] += (double)t[7];
            }
            rows = std::max(rows, 1);
            fprintf(stderr, "[bb wave select trace] rows=%d us-from-start: bound %.2f tiles %.2f gather %.2f "
                    "rescore %.2f end %.2f  cands %.1f tiles %.1f\n", rows, acc[1] / rows / 100, acc[2] / rows / 100,
                    acc[3] / rows / 100, acc[4] / rows / 100, acc[5] / rows / 100, acc[6] / rows, acc[7] / rows);
            BB_HIP(hipMemsetAsync(x->trace.p, 0, (size_t)bc * 64, s));
          }
        }
        if ((rc = timed(x, K_SELECT, s, [&] { return launch_select(sa, bc, s); }))) return rc;
        if (sel_trace) {
          std::vector<uint64_t> tr((size_t)bc * 8);
          BB_HIP(hipMemcpyAsync(tr.data(), x->trace.p, tr.size() * 8, hipMemcpyDeviceToHost, s));
          BB_HIP(hipStreamSynchronize(s));
          double acc[8] = {0};
          uint64_t t0 = ~0ull, t1 = 0;
          for (int i = 0; i < bc; ++i) {
            const uint64_t* t = &tr[(size_t)i * 8];
            for (int j = 1; j < 6; ++j) acc[j] += t[j] ? (double)(t[j] - t[0]) : 0.0;
            acc[7] += t[7] ? (double)(t[7] - t[0]) : 0.0;
            acc[6] += t[6] ? (double)(t[6] - t[0]) : 0.0;
            t0 = std::min(t0, t[0]);
            t1 = std::max(t1, t[7] ? t[7] : t[5]);
          }
          fprintf(stderr, "[bb select trace] rows=%d us-from-start: maxima %.2f bound %.2f tiles %.2f gather %.2f "
                  "pre-finish %.2f rescored %.2f end %.2f  span %.2f us\n", bc, acc[1] / bc / 100, acc[2] / bc / 100,
                  acc[3] / bc / 100, acc[4] / bc / 100, acc[5] / bc / 100, acc[6] / bc / 100, acc[7] / bc / 100,
                  (double)(t1 - t0) / 100);
        }
        if (rr_handoff && (rc = timed(x, K_RERANK, s, [&] { return launch_rerank(sa, bc, s); }))) return rc;
        final_pp = pp;
      }
    }
    if (fuse_final) continue;
    const uint64_t* fin_keys = keys + (size_t)final_pp * sides * side_keys;
    if (out_keys) {  // key lists out: device buffers, or host buffers (copied, synchronised below)
      const hipMemcpyKind kind = res->where == BB_DEVICE ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost;
      for (int side = 0; side < sides; ++side)
        if ((rc = s_copy(res->keys + ((size_t)side * B + b0) * K_int, fin_keys + (size_t)side * side_keys,
                         (size_t)bc * K_int * 8, kind, s)))
          return rc;
      if (drop) {
        if ((rc = s_copy(res->max_keys + b0, maxk, (size_t)bc * 8, kind, s))) return rc;
      } else if (res->where == BB_DEVICE) {
        if ((rc = s_memset(res->max_keys + b0, 0, (size_t)bc * 8, s))) return rc;
      }
      else
        memset(res->max_keys + b0, 0, (size_t)bc * 8);
      continue;
    }
    FinalizeArgs fa{};
    fa.keys = fin_keys;
    fa.max_keys = drop ? maxk : nullptr;
    fa.P = 1;
    fa.sides = sides;
    fa.B = (int)Bc;  // row stride of the per-side key blocks
    fa.K_int = K_int;
    fa.drop_rank0 = drop;
    fa.k = q->k;
    fa.k_side = q->k_side > 0 ? q->k_side : 2 * q->k;
    fa.hybrid = q->mode == BB_MODE_HYBRID;
    fa.w_content = q->w_content;
    fa.w_cf = q->w_cf;
    fa.scores = o_sc + (size_t)b0 * q->k;
    fa.ids = o_id + (size_t)b0 * q->k;
    fa.counts = o_cnt ? o_cnt + b0 : nullptr;
    fa.n_rows = bc;
    fa.idmap = x->shadow ? (const uint32_t*)x->idmap.p : nullptr;
    static const bool fin_trace = kProbes && ab_env("BB_SELECT_TRACE") != nullptr;
    if (fin_trace) {
      if ((rc = x->trace.ensure((size_t)bc * 8 * 8))) return rc;
      BB_HIP(hipMemsetAsync(x->trace.p, 0, (size_t)bc * 64, s));
      fa.trace = (uint64_t*)x->trace.p;
    }
    if ((rc = timed(x, K_FIN, s, [&] { return launch_finalize(fa, s); }))) return rc;
    if (fin_trace) {  // finalize phases: keys loaded, table ready, content blended, CF-only, end
      std::vector<uint64_t> tr((size_t)bc * 8);
      BB_HIP(hipMemcpyAsync(tr.data(), x->trace.p, tr.size() * 8, hipMemcpyDeviceToHost, s));
      BB_HIP(hipStreamSynchronize(s));
      double acc[8] = {0};
      uint64_t t0 = ~0ull, t1 = 0;
      int rows = 0;
      for (int i = 0; i < bc; ++i) {
        const uint64_t* t = &tr[(size_t)i * 8];
        if (!t[5] || !t[4]) continue;
        ++rows;
        for (int j = 1; j < 6; ++j) acc[j] += (double)(t[j] - t[0]);
        t0 = std::min(t0, t[0]);
        t1 = std::max(t1, t[5]);
      }
      rows = std::max(rows, 1);
      fprintf(stderr, "[bb finalize trace] rows=%d us-from-start: keys %.2f table %.2f content %.2f cf-only %.2f end %.2f  "
              "span %.2f us\n", rows, acc[1] / rows / 100, acc[2] / rows / 100, acc[3] / rows / 100, acc[4] / rows / 100,
              acc[5] / rows / 100, (double)(t1 - t0) / 100);
    }
  }
  if (stream) {
    // a candidate region overflowed (masses of equal scores, a pilot sample unlike the rest):
    // the caller reruns the search on the exact slab path
    if (tl_capture) return s_sync(s);  // (fails the plan: the host reads the flag)
    BB_HIP(host_wait(s));
    const uint32_t overflowed = *(volatile uint32_t*)x->ovf_host;
    if (kProbes && overflowed && ab_env("BB_STREAM_DEBUG")) {
      int rg, cap;
      const int bpl = (int)pad_rows(B - (B - 1) / Bc * Bc);
      stream_geom(bpl, refine ? 1 : 0, rg, cap);
      std::vector<uint32_t> cnt((size_t)bpl * rg);
      BB_HIP(hipMemcpy(cnt.data(), x->cand_cnt.p, cnt.size() * 4, hipMemcpyDeviceToHost));
      uint32_t mx = 0;
      double sum = 0;
      size_t over = 0, arg = 0;
      for (size_t i = 0; i < cnt.size(); ++i) {
        if (cnt[i] > mx) mx = cnt[i], arg = i;
        sum += cnt[i];
        over += cnt[i] > (uint32_t)cap;
      }
      std::vector<uint64_t> pk((size_t)bpl * K_int);
      BB_HIP(hipMemcpy(pk.data(), x->pilot.p, pk.size() * 8, hipMemcpyDeviceToHost));
      int zero_rows = 0;
      for (int i = 0; i < bpl; ++i) zero_rows += pk[(size_t)i * K_int + K_int - 1] == 0;
      fprintf(stderr, "[bb stream] overflow n=%lld n0=%lld K_int=%d bpad=%d regions=%d cap=%d max=%u at region %zu "
              "(q=%zu) mean=%.1f over=%zu pilot_rows_with_zero_kth=%d key0[K-1]=%016llx\n", (long long)x->n,
              (long long)n0, K_int, bpl, rg, cap, mx, arg, arg / rg, sum / cnt.size(), over, zero_rows,
              (unsigned long long)pk[K_int - 1]);
    }
    if (overflowed) return kRetrySlab;
  }
  if (host_out) {
    BB_HIP(hipMemcpyAsync(res->scores, o_sc, (size_t)B * q->k * 4, hipMemcpyDeviceToHost, s));
    BB_HIP(hipMemcpyAsync(res->ids, o_id, (size_t)B * q->k * 8, hipMemcpyDeviceToHost, s));
    if (res->counts) BB_HIP(hipMemcpyAsync(res->counts, o_cnt, (size_t)B * 4, hipMemcpyDeviceToHost, s));
  }
  if (host_out || where == BB_HOST || (out_keys && res->where != BB_DEVICE))
    if ((rc = s_sync(s))) return rc;
  return BB_OK;
}

}  // namespace

extern "C" {

int bb_search(bb_index* x, const bb_query* q, bb_result* res) {
  BB_CHECK_INDEX(x, "bb_search");
  if (!q || !res) return fail(BB_E_ARG, "bb_search: null argument");
  std::lock_guard<std::mutex> lk(x->mu);
  DeviceGuard g(x->device);
  const hipStream_t s = call_stream(x, q);
  int rc = enter_stream(x, s);
  if (rc) return rc;
  rc = search_locked(x, q, res, true);
  if (rc == kRetrySlab) {
    if (x->prof) ++x->launches[K_RERUN];
    rc = search_locked(x, q, res, false);
  }
  // an error may leave work enqueued on s: the next call still orders after it
  const int rc2 = leave_stream(x, s);
  return rc ? rc : rc2;
}

int bb_finalize(bb_index* x, const bb_query* q, const uint64_t* keys, const uint64_t* max_keys, int32_t n_parts,
                bb_result* res) {
  BB_CHECK_INDEX(x, "bb_finalize");
  if (!q || !keys || !res || n_parts <= 0) return fail(BB_E_ARG, "bb_finalize: bad arguments");
  int32_t sides, K_int;
  int rc = side_k_int(q, &sides, &K_int);
  if (rc) return rc;
  if (n_parts * K_int > 4096) return fail(BB_E_ARG, "bb_finalize: n_parts * k_int > 4096");
  std::lock_guard<std::mutex> lk(x->mu);
  DeviceGuard g(x->device);
  const hipStream_t s = call_stream(x, q);
  StreamScope scope;
  if ((rc = scope.enter(x, s))) return rc;
  const int B = q->B;
  const bool host_out = res->where != BB_DEVICE;
  if (host_out) {
    if ((rc = x->out_sc.ensure((size_t)B * q->k * 4)) || (rc = x->out_id.ensure((size_t)B * q->k * 8)) ||
        (rc = x->out_cnt.ensure((size_t)B * 4)))
      return rc;
  }
  const bool drop = q->mode == BB_MODE_SIMILAR || q->mode == BB_MODE_HYBRID;
  if (q->where != BB_DEVICE) {  // host key lists (q->where): staged to the device
    const size_t kb = (size_t)n_parts * sides * B * K_int * 8, mb = drop ? (size_t)n_parts * B * 8 : 0;
    if ((rc = x->stage_in.ensure(kb + mb + 64))) return rc;
    BB_HIP(hipMemcpyAsync(x->stage_in.p, keys, kb, hipMemcpyHostToDevice, s));
    if (mb) BB_HIP(hipMemcpyAsync((char*)x->stage_in.p + kb, max_keys, mb, hipMemcpyHostToDevice, s));
    keys = (const uint64_t*)x->stage_in.p;
    max_keys = mb ? (const uint64_t*)((char*)x->stage_in.p + kb) : nullptr;
  }
  FinalizeArgs fa{};
  fa.keys = keys;
  fa.max_keys = drop ? max_keys : nullptr;
  fa.P = n_parts;
  fa.sides = sides;
  fa.B = B;
  fa.K_int = K_int;
  fa.drop_rank0 = drop;
  fa.k = q->k;
  fa.k_side = q->k_side > 0 ? q->k_side : 2 * q->k;
  fa.hybrid = q->mode == BB_MODE_HYBRID;
  fa.w_content = q->w_content;
  fa.w_cf = q->w_cf;
  fa.scores = host_out ? (float*)x->out_sc.p : res->scores;
  fa.ids = host_out ? (int64_t*)x->out_id.p : res->ids;
  fa.counts = host_out ? (int32_t*)x->out_cnt.p : res->counts;
  fa.n_rows = B;
  if ((rc = timed(x, K_FIN, s, [&] { return launch_finalize(fa, s); }))) return rc;
  if (host_out) {
    BB_HIP(hipMemcpyAsync(res->scores, x->out_sc.p, (size_t)B * q->k * 4, hipMemcpyDeviceToHost, s));
    BB_HIP(hipMemcpyAsync(res->ids, x->out_id.p, (size_t)B * q->k * 8, hipMemcpyDeviceToHost, s));
    if (res->counts) BB_HIP(hipMemcpyAsync(res->counts, x->out_cnt.p, (size_t)B * 4, hipMemcpyDeviceToHost, s));
    BB_HIP(host_wait(s));
  }
  return scope.leave();
}

int bb_set_option(bb_index* x, int32_t option, int64_t value) {
  BB_CHECK_INDEX(x, "bb_set_option");
  std::lock_guard<std::mutex> lk(x->mu);
  switch (option) {
    case BB_OPT_STREAM:
      if (value < -1 || value > 1) return fail(BB_E_ARG, "BB_OPT_STREAM must be -1, 0 or 1");
      x->stream_opt = (int)value;
      return BB_OK;
    case BB_OPT_STREAM_MIN_ITEMS:
      if (value < 0) return fail(BB_E_ARG, "BB_OPT_STREAM_MIN_ITEMS must be >= 0");
      x->stream_min_items = value;
      return BB_OK;
    case BB_OPT_STREAM_REFINE:
      if (value < -1 || value > 1) return fail(BB_E_ARG, "BB_OPT_STREAM_REFINE must be -1, 0 or 1");
      x->refine_opt = (int)value;
      return BB_OK;
    case BB_OPT_RR_LISTS:
      if (value < -1 || value > 1) return fail(BB_E_ARG, "BB_OPT_RR_LISTS must be -1, 0 or 1");
      x->lists_opt = (int)value;
      return BB_OK;
    case BB_OPT_SMALL_BATCH:
      if (value < -1 || value > 1) return fail(BB_E_ARG, "BB_OPT_SMALL_BATCH must be -1, 0 or 1");
      x->sq_opt = (int)value;
      return BB_OK;
    case BB_OPT_PREFILTER:
      if (value < -1 || value > 1) return fail(BB_E_ARG, "BB_OPT_PREFILTER must be -1, 0 or 1");
      x->prefilter_opt = (int)value;
      return BB_OK;
    case BB_OPT_WORKSPACE_BYTES:
      if (value < (1ll << 20)) return fail(BB_E_ARG, "BB_OPT_WORKSPACE_BYTES must be >= 1 MiB");
      x->ws_cap = value;
      x->ws_set = true;
      return BB_OK;
    default:
      return fail(BB_E_ARG, "unknown option " + std::to_string(option));
  }
}

int bb_set_profiling(bb_index* x, int32_t on) {
  BB_CHECK_INDEX(x, "bb_set_profiling");
  x->prof = on != 0;
  return BB_OK;
}

int bb_get_profile(bb_index* x, bb_profile* out) {
  BB_CHECK_INDEX(x, "bb_get_profile");
  if (!out) return fail(BB_E_ARG, "bb_get_profile: null argument");
  std::lock_guard<std::mutex> lk(x->mu);
  DeviceGuard g(x->device);
  for (auto& p : x->pending) {
    BB_HIP(hipEventSynchronize(p.b));
    float ms = 0.f;
    BB_HIP(hipEventElapsedTime(&ms, p.a, p.b));
    x->ms[p.fam] += ms;
    (void)hipEventDestroy(p.a);
    (void)hipEventDestroy(p.b);
  }
  x->pending.clear();
  std::memset(out, 0, sizeof(*out));
  out->n = K_NFAM;
  for (int i = 0; i < K_NFAM; ++i) {
    out->ms[i] = x->ms[i];
    out->launches[i] = x->launches[i];
    out->names[i] = kFamNames[i];
    x->ms[i] = 0;
    x->launches[i] = 0;
  }
  return BB_OK;
}

// ---- prepared searches ----------------------------------------------------------------------
// Diagnostics: the hybrid dual scan's shape rules on a configs[2]-shaped argument pair whose
// item row stride is `ldx` (both sides); no device call (the 24-bit DMA
// offset guard, tested on the CPU).
int bb_check_dual_scan_args(int64_t ldx) {
  GemmArgs a0{}, a1{};
  static float h[1];
  static char lists[16];
  for (GemmArgs* g : {&a0, &a1}) {
    g->ldx = ldx;
    g->Mpad = 1024;
    g->Ncols = 25216;
    g->s_h = h;
    g->f16 = 1;
    g->lists = (decltype(g->lists))lists;
    g->l_period = 4;
    g->l_np = 2;
  }
  a0.Kpad = 384;
  a1.Kpad = 64;
  const char* why = nullptr;
  if (!scan4_dual_args_ok(a0, a1, &why)) return fail(BB_E_ARG, std::string("bb_check_dual_scan_args: ") + why);
  return BB_OK;
}

int bb_plan_create(bb_index* x, const bb_query* q, const bb_result* res, bb_plan** out) {
  BB_CHECK_INDEX(x, "bb_plan_create");
  if (!q || !res || !out) return fail(BB_E_ARG, "bb_plan_create: null argument");
  *out = nullptr;
  if (q->where != BB_DEVICE || res->where != BB_DEVICE)
    return fail(BB_E_ARG, "bb_plan_create: a plan reads device query buffers and writes device results");
  bb_index* root = x->base ? x->base : x;
  bb_index* v = nullptr;
  int rc = bb_create_view(root, &v);
  if (rc) return rc;
  {
    std::lock_guard<std::mutex> lk(x->mu);  // the options of the handle the plan is made from
    v->stream_opt = x->stream_opt;
    v->stream_min_items = x->stream_min_items;
    v->refine_opt = x->refine_opt;
    v->lists_opt = x->lists_opt;
    v->sq_opt = x->sq_opt;
    v->prefilter_opt = x->prefilter_opt;
    v->ws_cap = x->ws_cap;
    v->ws_set = x->ws_set;
  }
  bb_plan* p = new bb_plan();
  p->view = v;
  p->device = v->device;
  {
    DeviceGuard g(v->device);
    p->s = call_stream(v, q);
    bb_result r2 = *res;
    tl_capture = &p->ops;
    rc = search_locked(v, q, &r2, true);
    tl_capture = nullptr;
  }
  if (rc == BB_OK && p->ops.empty()) rc = fail(BB_E_STATE, "bb_plan_create: the search recorded no launches");
  if (rc) {
    const std::string msg = g_err;
    delete p;
    (void)bb_destroy(v);
    g_err = msg;
    return rc == kRetrySlab ? BB_E_HOSTSYNC : rc;
  }
  p->argv.resize(p->ops.size());
  for (size_t i = 0; i < p->ops.size(); ++i)
    for (uint32_t o : p->ops[i].offs) p->argv[i].push_back(p->ops[i].blob.data() + o);
  live_add(p);
  *out = p;
  return BB_OK;
}

int bb_plan_launch(bb_plan* p) {
  if (!p) return fail(BB_E_ARG, "bb_plan_launch: null plan");
  std::unique_lock<std::mutex> pl;
  {
    // the plan's lock is taken while the live set says the plan exists, so a destroy (which
    // removes it from the set first, then takes the plan's lock) waits for this launch
    std::lock_guard<std::mutex> lk(g_live_mu);
    if (!g_live.count(p) || p->magic != kPlanMagic)
      return fail(BB_E_ARG, "bb_plan_launch: stale or foreign plan handle (destroyed, or not from bb_plan_create)");
    pl = std::unique_lock<std::mutex>(p->mu);
  }
  int cur = -1;
  if (hipGetDevice(&cur) != hipSuccess || cur != p->device) BB_HIP(hipSetDevice(p->device));
  for (size_t i = 0; i < p->ops.size(); ++i) {
    const CapturedOp& op = p->ops[i];
    hipError_t e;
    if (op.kind == 0)
      e = hipLaunchKernel(op.func, op.grid, op.block, p->argv[i].data(), op.shmem, p->s);
    else if (op.kind == 1)
      e = hipMemsetAsync(op.dst, op.value, op.bytes, p->s);
    else
      e = hipMemcpyAsync(op.dst, op.src, op.bytes, hipMemcpyDeviceToDevice, p->s);
    if (e != hipSuccess) {
      if (cur >= 0 && cur != p->device) (void)hipSetDevice(cur);
      return fail(BB_E_HIP, std::string("bb_plan_launch: ") + hipGetErrorString(e));
    }
  }
  if (cur >= 0 && cur != p->device) (void)hipSetDevice(cur);
  return BB_OK;
}

int bb_plan_destroy(bb_plan* p) {
  if (!p) return BB_OK;
  if (!live_del(p))
    return fail(BB_E_ARG, "bb_plan_destroy: stale or foreign plan handle (destroyed, or not from bb_plan_create)");
  {
    std::lock_guard<std::mutex> pl(p->mu);  // a launch that passed its check finishes enqueueing
    DeviceGuard g(p->device);
    // the replays ran on the plan's stream (the caller's, valid until now by contract): wait
    // for it, not for the whole device
    (void)hipStreamSynchronize(p->s);
  }
  const int rc = bb_destroy(p->view);
  p->magic = 0;
  delete p;
  return rc;
}

}  // extern "C"
