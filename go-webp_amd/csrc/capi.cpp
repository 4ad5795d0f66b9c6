// extern "C" boundary of libgowebp_amd.so (declared in include/gowebp_amd.h).
//
// Host orchestration of the batch decode: a host thread pool runs the entropy
// stage (one frame per task), inputs are packed into one pinned staging buffer and
// copied to HBM in one transfer, then K1 (reconstruct + deblock) and K2
// (YUV420 -> RGBA) each run as ONE launch over the whole batch.  Mirrors the call
// structure of DecodeInto / WebPDecode (pkg/libwebp/decoder/webp.go:483-556,
// 870-909) with the per-row VP8Io.put chain replaced by whole-frame kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdlib>
#include <condition_variable>
#include <cstring>
#include <memory>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include "../../include/gowebp_amd.h"
#include "device/kernels.h"
#include "device_format.h"
#include "host/batch.h"
#include "host/host.h"

using wg::AlphaDesc;
using wg::AnimFrameDesc;
using wg::EmitDesc;
using wg::FrameDesc;
using wg::FrameParse;
using wg::LLDesc;
using wg::MbRec;
using wg::YuvaDesc;

namespace {

// Device buffers of finished batches, kept for the next batch of the context (the single-frame
// and one-shot batch entry points create and destroy a batch per call).  Best fit among
// buffers at most ~2x the request.  A context keeps at most a quarter of its device's memory
// (and never more than kMaxCached) in idle buffers; when hipMalloc fails, EVERY context's cache
// on that device is emptied before the one retry, so idle buffers of one context never starve
// another's batch.
class DeviceCache;
std::mutex g_caches_mu;
std::vector<DeviceCache*>* g_caches = new std::vector<DeviceCache*>();  // (never destroyed: exit order)
void trim_device_caches(int device);

class DeviceCache {
 public:
  DeviceCache() = default;
  ~DeviceCache() {
    {
      std::lock_guard<std::mutex> lock(g_caches_mu);
      auto& v = *g_caches;
      v.erase(std::remove(v.begin(), v.end(), this), v.end());
    }
    trim(0);
  }
  // bind to a device (hipSetDevice(device) done by the caller): the idle-memory cap
  void init(int device) {
    device_ = device;
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && total_b > 0) cap_ = std::min(kMaxCached, total_b / 4);
    (void)hipGetLastError();
    std::lock_guard<std::mutex> lock(g_caches_mu);
    g_caches->push_back(this);
  }
  int device() const { return device_; }
  void* get(size_t bytes) {
    bytes = std::max<size_t>(bytes, 256);
    {
      std::lock_guard<std::mutex> lock(mu_);
      size_t best = free_.size();
      for (size_t i = 0; i < free_.size(); ++i) {
        const size_t c = free_[i].cap;
        if (c >= bytes && c <= 2 * bytes + (size_t(16) << 20) && (best == free_.size() || c < free_[best].cap)) best = i;
      }
      if (best < free_.size()) {
        void* p = free_[best].p;
        cached_ -= free_[best].cap;
        free_.erase(free_.begin() + (ptrdiff_t)best);
        return p;
      }
    }
    void* p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();
      trim_device_caches(device_);  // make room (every context on this device) and try once more
      if (hipMalloc(&p, bytes) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
      }
    }
    std::lock_guard<std::mutex> lock(mu_);
    caps_.push_back(Entry{p, bytes});
    return p;
  }
  void put(void* p) {
    if (!p) return;
    std::lock_guard<std::mutex> lock(mu_);
    for (size_t i = 0; i < caps_.size(); ++i)
      if (caps_[i].p == p) {
        free_.push_back(caps_[i]);
        cached_ += caps_[i].cap;
        break;
      }
    trim_locked(cap_);
  }
  void trim(size_t keep) {
    std::lock_guard<std::mutex> lock(mu_);
    trim_locked(keep);
  }

 private:
  struct Entry {
    void* p;
    size_t cap;
  };
  void trim_locked(size_t keep) {
    while (cached_ > keep && !free_.empty()) {
      auto it = std::max_element(free_.begin(), free_.end(), [](const Entry& a, const Entry& b) { return a.cap < b.cap; });
      hipFree(it->p);
      cached_ -= it->cap;
      for (size_t i = 0; i < caps_.size(); ++i)
        if (caps_[i].p == it->p) {
          caps_.erase(caps_.begin() + (ptrdiff_t)i);
          break;
        }
      free_.erase(it);
    }
  }
  static constexpr size_t kMaxCached = size_t(64) << 30;
  std::mutex mu_;
  std::vector<Entry> free_, caps_;  // free list; every buffer this cache allocated (and its size)
  size_t cached_ = 0;
  size_t cap_ = size_t(8) << 30;  // until init() reads the device's memory
  int device_ = 0;
};

void trim_device_caches(int device) {
  std::lock_guard<std::mutex> lock(g_caches_mu);
  for (DeviceCache* c : *g_caches)
    if (c->device() == device) c->trim(0);
}

void* pinned_alloc(size_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  return p;
}
void pinned_free(void* p) { hipHostFree(p); }

// the split kernel's launch-tag counter (next_epoch, below)
std::atomic<uint32_t> g_epoch{0};

}  // namespace

struct wg_ctx {
  int device = 0;
  int host_threads = 1;
  hipStream_t stream = nullptr;
  std::mutex mu;  // one batch creation (or pipelined decode) at a time: arenas and pool are shared
  std::unique_ptr<wg::WorkerPool> pool;
  std::unique_ptr<wg::StagingArena> arena;
  DeviceCache cache;
  // the pipelined decode (wg_decode_rgba_batch): a second staging arena, and two work streams
  // (kernels + download of alternate chunks) next to `stream`, which carries every chunk's
  // upload -- so an upload never queues behind an earlier chunk's download
  std::unique_ptr<wg::StagingArena> arena_ring[3];  // with `arena`, a ring of four
  hipStream_t work[2] = {nullptr, nullptr};
  // K7 beside K1 / K2 (wg_batch_run: small batches whose grids fit on the chip together)
  hipStream_t side = nullptr;
  std::mutex side_mu;
  int chunk_frames = 0;  // frames per pipeline chunk, 0 = automatic (wg_ctx_set_chunk_frames)
  wg_pipeline_stats stats{};  // of the last pipelined decode
  // HIP events kept for reuse (batches' stage timings, pipeline chunks): creating ~14 events per
  // call was a fixed cost of every single-frame decode.  [0] default (spin-wait), [1] blocking-sync.
  std::mutex ev_mu;
  std::vector<hipEvent_t> spare_ev[2];
  // pinned words the pipeline's chunks copy their error word into (no synchronous D2H per chunk)
  int32_t* err_words = nullptr;
  int n_err_words = 0;
  hipEvent_t take_event(int blocking) {
    {
      std::lock_guard<std::mutex> lock(ev_mu);
      auto& v = spare_ev[blocking ? 1 : 0];
      if (!v.empty()) {
        hipEvent_t e = v.back();
        v.pop_back();
        return e;
      }
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, blocking ? hipEventBlockingSync : hipEventDefault) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    return e;
  }
  void give_event(hipEvent_t e, int blocking) {
    if (!e) return;
    std::lock_guard<std::mutex> lock(ev_mu);
    spare_ev[blocking ? 1 : 0].push_back(e);
  }
  wg::WorkerPool* workers() {
    if (!pool) pool.reset(new wg::WorkerPool(host_threads));
    return pool.get();
  }
};

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }

// Kernels in launch order (stage) and in the public order of wg_batch_kernel_ms (K1, K2, K3,
// K4, K7, K6, K5): stage s runs between events ev[s] and ev[s + 1].
constexpr int kStages = 7;
constexpr int kStageK1 = 0, kStageK2 = 1, kStageK7 = 2, kStageK3 = 3, kStageK4 = 4, kStageK6 = 5, kStageK5 = 6;
constexpr int kPublicOfStage[kStages] = {0, 1, 4, 2, 3, 5, 6};
struct Timing {
  hipEvent_t ev[kStages + 1] = {};
  bool ran[kStages] = {};
  hipEvent_t side[2] = {};  // K7's start / end when it ran on the context's side stream
  bool forked = false;
  int8_t order[kStages] = {0, 1, 2, 3, 4, 5, 6};  // launch order: ev[i] .. ev[i + 1] bracket stage order[i]
};

// (events from the context's spare list, back to it when the batch goes)
hipError_t timing_create(wg_ctx* c, Timing& t) {
  for (auto& e : t.ev)
    if (!(e = c->take_event(0))) return hipErrorOutOfMemory;
  for (auto& e : t.side)
    if (!(e = c->take_event(0))) return hipErrorOutOfMemory;
  return hipSuccess;
}
void timing_destroy(wg_ctx* c, Timing& t) {
  for (auto& e : t.ev) c->give_event(e, 0), e = nullptr;
  for (auto& e : t.side) c->give_event(e, 0), e = nullptr;
}

}  // namespace

struct wg_batch {
  wg_ctx* ctx = nullptr;
  int n = 0;
  int flags = 0;
  std::vector<FrameParse> fp;
  std::vector<FrameDesc> desc;
  std::vector<LLDesc> lldesc;     // lossless frames and lossless alpha streams (K3)
  std::vector<wg::LLTokDesc> tokdesc;  // the same streams' tokens (K7)
  wg::LLTokDesc* d_tokdesc = nullptr;
  std::vector<AlphaDesc> adesc;   // alpha planes (K4)
  FrameDesc* d_desc = nullptr;
  LLDesc* d_lldesc = nullptr;
  AlphaDesc* d_adesc = nullptr;
  int n_lossy = 0, n_lossless = 0, n_alpha = 0, n_k3 = 0, n_k6 = 0;  // n_k6: frames K6 converts
  int n_alpha_2d = 0;  // alpha planes with filter vertical / gradient (K4's second instantiation)
  bool tail_modes = true, no_tail = false;  // no_tail: frames emitted directly in a mode K1's tail lacks
  int n_tok_w64 = 0;                         // K7 streams on its 64-mask-word instantiation (first in tokdesc)
  int n_tok_alpha = 0;                       // of those, the alpha streams whose bytes K7 writes (first)
  int n_tok_tiled = 0;                       // of those, the ones into band tiles (first)
  bool k2_modes = false;                     // K2 writes some frame in a non-RGBA colorspace (FrameDesc::emit)
  wg_decoder_options opt{};          // output colorspace, cropping, flip (f4)
  bool any_crop = false;             // K2 reads compact cropped planes through desc2
  bool fused = false;                // lossy RGBA emitted by K1's tail (wg::kFrameEmitRgba), no K2 launch
  bool alpha_first = false;          // K4 before the strips, which take A from its planes (set_alpha_first)
  double alpha_px = 0;               // pixels of the alpha planes (algorithmic bytes)
  bool no_side = false;              // K7 always in stream order (the pipelined decode's chunks)
  std::vector<FrameDesc> desc2;
  FrameDesc* d_desc2 = nullptr;
  int max_out_w = 1, max_out_h = 1;
  int ll_groups[wg::kVP8LVariants] = {0, 0, 0, 0, 0};  // K3 frames per kernel variant
  int* d_err = nullptr;
  uint8_t* d_in = nullptr;
  uint8_t* d_planes = nullptr;
  uint8_t* d_rgba = nullptr;
  size_t in_bytes = 0, plane_bytes = 0, rgba_bytes = 0;
  int max_mb_w = 1, max_w = 1, max_h = 1;  // max_mb_w over the frames whose K1 column store is in LDS
  int n_wide = 0;                          // lossy frames wider than that (global column store)
  // K1's split kernel (several workgroups per frame, batches of fewer frames than CUs): parts per
  // frame (1 = the one-workgroup kernels), and the lossy frames' progress flags (one region)
  int split_parts = 1;
  int split_from = 0;  // frames [split_from, n) on the split kernel, [0, split_from) on the others
  size_t off_gprog = 0, gprog_bytes = 0;
  int n_valid = 0;
  int64_t pixels = 0;
  double kbytes[kStages] = {};  // public order: K1, K2, K3, K4, K7, K6, K5
  double k1_fused_bytes = 0;  // K1 with its RGBA tail: inputs + RGBA (planes are an intermediate)
  std::vector<Timing> timings;  // one per run since the last query
  size_t n_runs_pending = 0;
  hipStream_t home = nullptr;   // the batch's own stream: uploads, downloads (the context's by default)
  // one event per stream the batch's work was queued on, recorded after its latest work there:
  // batch_wait waits for all of them, so runs on several user streams are all complete before
  // the buffers go back to the cache
  std::vector<std::pair<hipStream_t, hipEvent_t>> done;
  // K6 (f4): a non-RGBA colorspace or a flipped output is a stage of wg_batch_run, from the
  // frames' RGBA windows into d_out (frame i at off_out[i], rows of bpp * out_w bytes)
  bool k6 = false;
  int out_bpp = 4, k6_maxpx = 1;
  std::vector<EmitDesc> edesc;
  EmitDesc* d_edesc = nullptr;
  uint8_t* d_out = nullptr;
  size_t out_bytes = 0;
  std::vector<size_t> off_out;
  // K8: MODE_YUV / MODE_YUVA (yuv, yuva) -- every frame's output planes in its slot of d_out (Y, U,
  // V, A back to back, yuva_planes), written by K8 in the K6 stage; no RGBA for lossy frames
  bool yuv = false, yuva = false;
  std::vector<YuvaDesc> ydesc;
  YuvaDesc* d_ydesc = nullptr;
  int yuv_max_uw = 1, yuv_max_uh = 1;
  // K5 (f3): an animation batch (wg_anim_batch_create) composites its canvases in wg_batch_run
  bool anim = false;
  int canvas_w = 0, canvas_h = 0;
  std::vector<AnimFrameDesc> fdesc;
  AnimFrameDesc* d_fdesc = nullptr;
  uint8_t* d_canvases = nullptr;
  std::vector<int32_t> timestamps;
};

namespace {
// The single-frame entry points share one lazily created context (device 0 unless
// wg_set_default_device chose another).  Held by shared_ptr for the length of each call, so
// wg_set_default_device can replace it while calls are in flight: the old context is destroyed
// when its last call returns.  (The holder itself is never destroyed: no HIP work at exit.)
std::mutex g_default_mu;
std::shared_ptr<wg_ctx>* g_default_ctx = new std::shared_ptr<wg_ctx>();
int g_default_device = 0;
std::shared_ptr<wg_ctx> default_ctx() {
  std::lock_guard<std::mutex> lock(g_default_mu);
  if (!*g_default_ctx) {
    wg_ctx* c = wg_ctx_create(g_default_device, 0);
    if (c) g_default_ctx->reset(c, wg_ctx_destroy);
  }
  return *g_default_ctx;
}

void fill_vp8l_info(const wg::VP8LFrame& f, wg_vp8l_info* info, uint32_t* tokens, uint32_t* literals,
                    uint32_t* const* transform_data);

// Errors never cross the C ABI as exceptions.
template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return WG_STATUS_OUT_OF_MEMORY;
  } catch (const std::exception&) {
    return WG_STATUS_OUT_OF_MEMORY;
  }
}
}  // namespace

extern "C" {

int wg_version(void) { return 0x000100; }

uint32_t wg_debug_set_epoch(uint32_t value) { return g_epoch.exchange(value, std::memory_order_relaxed); }

int wg_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int wg_get_features(const uint8_t* data, size_t size, wg_features* out) {
  if (out == nullptr) return WG_STATUS_INVALID_PARAM;
  std::memset(out, 0, sizeof(*out));
  wg::Container c;
  return wg::parse_container(data, size, &c, out, /*have_all_data=*/false);
}

int wg_vp8_parse(const uint8_t* data, size_t size, int flags, wg_vp8_info* info, wg_vp8_mb* mbs) {
  if (data == nullptr) return WG_STATUS_INVALID_PARAM;
  return guarded([&] { return wg::vp8_parse(data, size, flags, info, mbs); });
}

int wg_decode_status(const uint8_t* data, size_t size, const wg_decoder_options* opt) {
  if (data == nullptr) return WG_STATUS_INVALID_PARAM;
  wg_decoder_options o{};
  o.colorspace = 1;  // MODE_RGBA
  if (opt) o = *opt;
  return guarded([&] {
    // host stages only; the staged device inputs go to plain heap memory and are dropped
    wg::StagingArena heap([](size_t b) { return std::malloc(b); }, [](void* q) { std::free(q); });
    wg::StagingArena::Cursor cur;
    FrameParse fp;
    return wg::parse_one(data, size, o, &heap, &cur, &fp);
  });
}

int wg_vp8l_parse(const uint8_t* data, size_t size, wg_vp8l_info* info, uint32_t* tokens, uint32_t* literals,
                  uint32_t* const* transform_data) {
  if (data == nullptr || info == nullptr) return WG_STATUS_INVALID_PARAM;
  wg::Container c;
  wg_features feat{};
  int st = wg::parse_container(data, size, &c, &feat);
  if (st != WG_STATUS_OK) return st;
  if (!c.is_lossless) return WG_STATUS_UNSUPPORTED_FEATURE;
  return guarded([&] {
    wg::VP8LFrame f;
    const int st2 = wg::vp8l_parse(data + c.payload_off, c.payload_size, &f);
    if (st2 != WG_STATUS_OK) return st2;
    fill_vp8l_info(f, info, tokens, literals, transform_data);
    return (int)WG_STATUS_OK;
  });
}

int wg_alpha_parse(const uint8_t* data, size_t size, wg_alpha_info* info, uint8_t* filtered,
                   wg_vp8l_info* ll_info, uint32_t* tokens, uint32_t* literals, uint32_t* const* transform_data) {
  if (data == nullptr) return WG_STATUS_INVALID_PARAM;
  wg::Container c;
  wg_features feat{};
  int st = wg::parse_container(data, size, &c, &feat);
  if (st != WG_STATUS_OK) return st;
  if (c.is_lossless || c.alpha_size == 0) return WG_STATUS_UNSUPPORTED_FEATURE;
  const uint8_t* ad = data + c.alpha_off;
  wg::AlphaHeader ah;
  if (info) {
    std::memset(info, 0, sizeof(*info));
    info->width = c.width;
    info->height = c.height;
  }
  if (!wg::parse_alpha_header(ad, c.alpha_size, c.width, c.height, &ah)) return WG_STATUS_OUT_OF_MEMORY;
  if (info) {
    info->method = ah.method;
    info->filter = ah.filter;
    info->pre_processing = ah.pre_processing;
  }
  if (ah.method == 0) {
    if (filtered) std::memcpy(filtered, ad + 1, (size_t)c.width * c.height);
    return WG_STATUS_OK;
  }
  return guarded([&] {
    wg::VP8LFrame f;
    const int st2 = wg::vp8l_parse_alpha(ad + 1, c.alpha_size - 1, c.width, c.height, &f);
    if (st2 != WG_STATUS_OK) return st2;
    if (ll_info) fill_vp8l_info(f, ll_info, tokens, literals, transform_data);
    return (int)WG_STATUS_OK;
  });
}

}  // extern "C"

namespace {
void fill_vp8l_info(const wg::VP8LFrame& f, wg_vp8l_info* info, uint32_t* tokens, uint32_t* literals,
                    uint32_t* const* transform_data) {
  std::memset(info, 0, sizeof(*info));
  info->width = f.width;
  info->height = f.height;
  info->has_alpha = f.has_alpha;
  info->coded_width = f.coded_width;
  info->num_transforms = (int32_t)f.transforms.size();
  info->cache_bits = f.cache_bits;
  info->num_literals = (int32_t)f.lits.size();
  for (size_t i = 0; i < f.transforms.size(); ++i) {
    info->transform_type[i] = f.transforms[i].type;
    info->transform_bits[i] = f.transforms[i].bits;
    info->transform_xsize[i] = f.transforms[i].xsize;
    info->transform_size[i] = (int32_t)f.transforms[i].data.size();
    if (transform_data && transform_data[i] && !f.transforms[i].data.empty())
      std::memcpy(transform_data[i], f.transforms[i].data.data(), f.transforms[i].data.size() * 4);
  }
  if (tokens) std::memcpy(tokens, f.tokens.data(), f.tokens.size() * 4);
  if (literals && !f.lits.empty()) std::memcpy(literals, f.lits.data(), f.lits.size() * 4);
}
}  // namespace

namespace {
wg_batch* batch_create(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                       const wg_decoder_options* opt, int32_t* status);

// Wait for everything the batch has queued (its home stream and its latest work on every stream
// it ran on) -- stream-scoped, so other contexts on the device are not serialised.
hipError_t batch_wait(wg_batch* b) {
  hipError_t e = b->home ? hipStreamSynchronize(b->home) : hipSuccess;
  for (auto& d : b->done)
    if (e == hipSuccess) e = hipEventSynchronize(d.second);
  return e;
}
// Record the batch's latest work on stream s (the event of that stream, created on first use).
hipError_t batch_mark_done(wg_batch* b, hipStream_t s) {
  if (s == b->home) return hipSuccess;  // batch_wait synchronises the home stream itself
  for (auto& d : b->done)
    if (d.first == s) return hipEventRecord(d.second, s);
  hipEvent_t ev = nullptr;
  hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
  if (e != hipSuccess) return e;
  b->done.emplace_back(s, ev);
  return hipEventRecord(ev, s);
}
// hipSetDevice with its failure reported (a wrong device would otherwise surface later as a
// generic launch failure)
bool set_device(int device) {
  if (hipSetDevice(device) == hipSuccess) return true;
  (void)hipGetLastError();
  return false;
}
}  // namespace

extern "C" {

wg_ctx* wg_ctx_create(int device, int host_threads) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
  if (!set_device(device)) return nullptr;
  wg_ctx* c = new (std::nothrow) wg_ctx();
  if (!c) return nullptr;
  c->device = device;
  c->host_threads = host_threads > 0 ? host_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  c->arena.reset(new (std::nothrow) wg::StagingArena(pinned_alloc, pinned_free));
  if (!c->arena) {
    hipStreamDestroy(c->stream);
    delete c;
    return nullptr;
  }
  c->cache.init(device);
  return c;
}

void wg_ctx_destroy(wg_ctx* c) {
  if (!c) return;
  const bool dev_ok = set_device(c->device);
  if (dev_ok && c->stream) hipStreamSynchronize(c->stream);
  for (hipStream_t w : c->work)
    if (dev_ok && w) hipStreamSynchronize(w);
  if (dev_ok && c->side) hipStreamSynchronize(c->side);
  c->pool.reset();
  c->arena.reset();
  for (auto& a : c->arena_ring) a.reset();
  c->cache.trim(0);
  for (auto& v : c->spare_ev)
    for (hipEvent_t e : v) hipEventDestroy(e);
  if (c->err_words) pinned_free(c->err_words);
  if (c->stream) hipStreamDestroy(c->stream);
  for (hipStream_t w : c->work)
    if (w) hipStreamDestroy(w);
  if (c->side) hipStreamDestroy(c->side);
  delete c;
}

int wg_set_default_device(int device) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return WG_STATUS_INVALID_PARAM;
  std::shared_ptr<wg_ctx> old;
  {
    std::lock_guard<std::mutex> lock(g_default_mu);
    if (*g_default_ctx && (*g_default_ctx)->device != device) old.swap(*g_default_ctx);
    g_default_device = device;
  }
  // `old` is destroyed here if no call holds it, else when the last one in flight returns
  return WG_STATUS_OK;
}

void wg_batch_destroy(wg_batch* b) {
  if (!b) return;
  if (set_device(b->ctx->device)) batch_wait(b);  // nothing may still use the buffers handed back to the cache
  for (auto& t : b->timings) timing_destroy(b->ctx, t);
  for (auto& d : b->done) hipEventDestroy(d.second);
  DeviceCache& c = b->ctx->cache;
  c.put(b->d_desc);
  c.put(b->d_lldesc);
  c.put(b->d_tokdesc);
  c.put(b->d_adesc);
  c.put(b->d_desc2);
  c.put(b->d_err);
  c.put(b->d_in);
  c.put(b->d_planes);
  c.put(b->d_rgba);
  c.put(b->d_edesc);
  c.put(b->d_out);
  c.put(b->d_fdesc);
  c.put(b->d_canvases);
  c.put(b->d_ydesc);
  delete b;
}

wg_batch* wg_batch_create(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n, int32_t flags,
                          int32_t* status) {
  wg_decoder_options o{};
  o.colorspace = 1;  // MODE_RGBA
  o.bypass_filtering = !!(flags & WG_FLAG_BYPASS_FILTERING);
  o.no_fancy_upsampling = !!(flags & WG_FLAG_NO_FANCY_UPSAMPLING);
  return wg_batch_create_ex(ctx, data, sizes, n, &o, status);
}

int wg_output_bpp(int colorspace) { return wg::output_bpp(colorspace); }

wg_batch* wg_batch_create_ex(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                             const wg_decoder_options* opt, int32_t* status) {
  if (!ctx || !data || !sizes || n <= 0 || !opt) return nullptr;
  try {
    return batch_create(ctx, data, sizes, n, opt, status);
  } catch (const std::exception&) {  // host-side layout / descriptor vectors (batch_create frees its own)
    if (status)
      for (int i = 0; i < n; ++i)
        if (status[i] == WG_STATUS_OK) status[i] = WG_STATUS_OUT_OF_MEMORY;
    return nullptr;
  }
}

}  // extern "C"

namespace {

struct BatchDeleter {
  void operator()(wg_batch* b) const { wg_batch_destroy(b); }
};

// The LLDesc of one lossless stream (transforms in application order = reverse of read
// order): its coded image is K7's output in the plane buffer; `d_in` + the arena's device
// offsets locate its staged transform data.
LLDesc make_ll(const wg::LLMeta& m, const wg::StagingArena& arena, uint8_t* d_in, uint8_t* d_planes, uint8_t* scratch,
               uint8_t* rgba, int stride) {
  LLDesc l{};
  l.coded = reinterpret_cast<const uint32_t*>(d_planes + m.off_coded);
  l.coded_bytes = (int32_t)(m.n_px() * 4);
  l.scratch = m.two_pass() ? reinterpret_cast<uint32_t*>(scratch) : nullptr;
  l.scratch_bytes = l.scratch ? m.width * m.height * 4 : 0;
  l.rgba = rgba;
  l.rgba_stride = stride;
  l.width = m.width;
  l.height = m.height;
  l.coded_width = m.coded_width;
  l.n_stages = m.n_transforms;
  int types[4], bits[4], tiles[4];
  for (int t = 0; t < l.n_stages; ++t) {
    const int r = l.n_stages - 1 - t;  // read-order index
    wg::LLStage& st = l.stages[t];
    st.type = m.type[r];
    st.bits = m.bits[r];
    st.xsize = m.xsize[r];
    st.tiles_per_row = (st.type == wg::kVP8LPredictor || st.type == wg::kVP8LCrossColor)
                           ? (st.xsize + (1 << st.bits) - 1) >> st.bits
                           : 0;
    st.data = reinterpret_cast<const uint32_t*>(d_in + arena.dev_offset(m.tdata[r]));
    types[t] = st.type;
    bits[t] = st.bits;
    tiles[t] = st.tiles_per_row ? st.tiles_per_row * ((m.height + (1 << st.bits) - 1) >> st.bits) : 0;
  }
  l.valid = 1;
  l.pad1[0] = (uint64_t)wg::vp8l_variant(types, bits, tiles, l.n_stages);  // sort key
  return l;
}

wg::LLTokDesc make_tok(const wg::LLMeta& m, const wg::StagingArena& arena, uint8_t* d_in, uint8_t* d_planes) {
  wg::LLTokDesc t{};
  t.tokens = reinterpret_cast<const uint32_t*>(d_in + arena.dev_offset(m.tokens));
  t.lits = reinterpret_cast<const uint32_t*>(d_in + arena.dev_offset(m.lits));
  t.coded = reinterpret_cast<uint32_t*>(d_planes + m.off_coded);
  t.n_px = (int32_t)m.n_px();
  t.n_lits = (int32_t)(m.lits.bytes / 4);
  t.cache_bits = m.cache_bits;
  t.valid = 1;
  t.trusted = 1;  // vp8l_parse checks every literal index, cache key and distance (host/vp8l_parse.cpp)
  return t;
}

// algorithmic bytes of one lossless stream: K7 reads tokens + literals and writes
// the coded image; K3 reads it and the transform data and writes RGBA (two passes: + scratch)
double k7_bytes(const wg::LLMeta& m) { return (double)m.tokens.bytes + (double)m.lits.bytes + 4.0 * m.n_px(); }
double ll_bytes(const wg::LLMeta& m) {
  const double px = (double)m.width * m.height;
  double bytes = 4.0 * m.n_px() + 4.0 * px;
  for (int t = 0; t < m.n_transforms; ++t) bytes += (double)m.tdata[t].bytes;
  if (m.two_pass()) bytes += 8.0 * px;
  return bytes;
}

using BatchPtr = std::unique_ptr<wg_batch, BatchDeleter>;

// Host half of a batch: every frame's host stages into `arena` (on the context's pool; the
// caller holds ctx->mu), the layout of the planes / RGBA and the algorithmic bytes per kernel.
// status[i] = frame i's status.  Nothing touches the device.
// An empty batch of n frames (their FrameParse records default-initialised).
BatchPtr batch_init(wg_ctx* ctx, hipStream_t home, int n, const wg_decoder_options* opt) {
  BatchPtr bp(new wg_batch());
  wg_batch* b = bp.get();
  b->ctx = ctx;
  b->home = home;
  b->n = n;
  b->opt = *opt;
  b->flags = (opt->bypass_filtering ? WG_FLAG_BYPASS_FILTERING : 0) |
             (opt->no_fancy_upsampling ? WG_FLAG_NO_FANCY_UPSAMPLING : 0);
  b->fp.assign((size_t)n, FrameParse{});
  return bp;
}

void batch_layout(wg_batch* b, wg::StagingArena& arena, int32_t* status);

BatchPtr batch_parse(wg_ctx* ctx, wg::StagingArena& arena, hipStream_t home, const uint8_t* const* data,
                     const size_t* sizes, int n, const wg_decoder_options* opt, int32_t* status) {
  if (status)
    for (int i = 0; i < n; ++i) status[i] = WG_STATUS_OK;
  BatchPtr bp = batch_init(ctx, home, n, opt);
  arena.begin_batch();
  wg::parse_all(data, sizes, n, *opt, ctx->workers(), &arena, bp->fp);
  batch_layout(bp.get(), arena, status);
  return bp;
}

// After every frame of the batch is parsed into `arena`: the arena's chunks laid out back to back
// for the device, the layout of the planes / RGBA and the algorithmic bytes per kernel;
// status[i] = frame i's status.
void batch_layout(wg_batch* b, wg::StagingArena& arena, int32_t* status) {
  const int n = b->n;
  b->in_bytes = std::max<size_t>(arena.layout(), kAlign);
  // layout of the planes / RGBA, and the algorithmic bytes per kernel
  size_t pl_b = 0, rg_b = 0;
  double k1 = 0, k2 = 0, k3 = 0, k4 = 0, k7 = 0;
  // K6: a non-RGBA colorspace or flip.  Lossy frames without alpha or crop window leave the
  // YUV -> RGB strips (K1's tail or K2) in the output colorspace, straight into their output slot:
  // no RGBA copy for them, and K6 converts only the others.
  b->yuv = b->opt.colorspace == 11 || b->opt.colorspace == 12;
  b->yuva = b->opt.colorspace == 12;
  b->k6 = !b->yuv && !(b->opt.colorspace == 1 && !b->opt.flip);
  const int obpp = b->yuv ? 4 : wg::output_bpp(b->opt.colorspace);
  for (int i = 0; i < n; ++i) {
    FrameParse& f = b->fp[(size_t)i];
    if (status) status[i] = f.status;
    if (f.status != WG_STATUS_OK) continue;
    f.emit_direct = b->k6 && !f.lossless && !f.alpha && !f.cropped;
    f.off_rgba = rg_b;
    // (YUV output: a lossy frame's planes are its output, only lossless frames have an RGBA)
    if (!f.emit_direct && !(b->yuv && !f.lossless)) rg_b = align_up(rg_b + (size_t)f.rgba_w * f.rgba_h * 4);
    b->max_w = std::max(b->max_w, f.width);
    b->max_h = std::max(b->max_h, f.height);
    b->max_out_w = std::max(b->max_out_w, f.out_w);
    b->max_out_h = std::max(b->max_out_h, f.out_h);
    b->n_valid++;
    b->pixels += (int64_t)f.out_w * f.out_h;
    const double px = (double)f.width * f.height;
    if (f.lossless) {
      b->n_lossless++;
      b->n_k3++;
      if (f.ll.two_pass()) {
        f.off_scratch = pl_b;
        pl_b = align_up(pl_b + (size_t)f.width * f.height * 4);
      }
      f.ll.off_coded = pl_b;
      pl_b = align_up(pl_b + f.ll.n_px() * 4);
      k3 += ll_bytes(f.ll);
      k7 += k7_bytes(f.ll);
      continue;
    }
    b->n_lossy++;
    const wg_vp8_info& inf = f.info;
    const size_t nmb = (size_t)inf.mb_w * inf.mb_h;
    f.off_y = pl_b;
    pl_b = align_up(pl_b + nmb * 256);
    f.off_u = pl_b;
    pl_b = align_up(pl_b + nmb * 64);
    f.off_v = pl_b;
    pl_b = align_up(pl_b + nmb * 64);
    f.wide = inf.mb_w > wg::vp8_recon_max_mb_w();
    if (f.wide) b->n_wide++;
    else b->max_mb_w = std::max(b->max_mb_w, inf.mb_w);
    // a global column store for every lossy frame: wide frames need it, and the split kernel
    // runs every frame from it (mb_w * 160 B: 38 KB at 4K)
    f.off_cols = pl_b;
    pl_b = align_up(pl_b + (size_t)inf.mb_w * 160);
    f.off_gprog = b->gprog_bytes;
    b->gprog_bytes += wg::kGProgBytes;
    if (f.cropped && !b->yuv) {  // K2 reads the crop window from compact planes (copied after K1)
      b->any_crop = true;
      f.yc_stride = (f.out_w + 15) & ~15;
      f.uvc_stride = ((((f.out_w + 1) >> 1) + 7) & ~7);
      f.off_yc = pl_b;
      pl_b = align_up(pl_b + (size_t)f.yc_stride * f.out_h);
      f.off_uc = pl_b;
      pl_b = align_up(pl_b + (size_t)f.uvc_stride * ((f.out_h + 1) >> 1));
      f.off_vc = pl_b;
      pl_b = align_up(pl_b + (size_t)f.uvc_stride * ((f.out_h + 1) >> 1));
    }
    // algorithmic bytes: K1 reads records + row index + coefficient blocks, writes
    // MB-padded planes (or, with its RGBA tail, the RGBA); K2 reads cropped planes, writes RGBA.
    const double k1_in = (double)nmb * sizeof(MbRec) + inf.mb_h * 4.0 + (double)f.n_blocks * 32.0;
    k1 += k1_in + nmb * 384.0;
    const double obytes = f.emit_direct ? (double)obpp : 4.0;  // output bytes per pixel of the strips
    b->k1_fused_bytes += k1_in + obytes * inf.width * (double)inf.height;
    const double opx = (double)f.out_w * f.out_h;
    k2 += opx + 2.0 * ((f.out_w + 1) / 2) * (double)((f.out_h + 1) / 2) + obytes * opx;
    if (f.alpha) {
      // K4 reads the filtered alpha (raw bytes, or K3's RGBA of the alpha stream) and
      // rewrites the RGBA A bytes (dword read-modify-write)
      b->n_alpha++;
      if (f.ah.filter >= 2) b->n_alpha_2d++;
      if (f.ah.method == 1) {
        b->n_k3++;  // (K7 resolves every lossless stream)
        // libwebp's 8-bit alpha streams (a color map and nothing else, or no transform) under
        // filter none / horizontal: K4 expands the palette itself, straight from K7's output
        // (any filter: K4 reads the coded image itself -- rows in parallel for none / horizontal, a
        // gather into its plane for vertical / gradient)
        f.alpha_direct = (f.al.n_transforms == 0 ||
                                              (f.al.n_transforms == 1 && f.al.type[0] == wg::kVP8LColorIndexing));
        if (f.al.two_pass() && !f.alpha_direct) {
          f.off_ascratch = pl_b;
          pl_b = align_up(pl_b + (size_t)f.width * f.height * 4);
        }
        f.al.off_coded = pl_b;
        pl_b = align_up(pl_b + f.al.n_px() * 4);
        k7 += k7_bytes(f.al);
        // 8-bit streams whose map fits K7's registers (<= 16 entries: bundled indices) or that
        // have none, under filters none / vertical / gradient: K7 writes the filtered bytes itself,
        // into the plane (K4 then works in place: no gather; none: nothing left to do alpha-first).
        // Not horizontal: K4 reads the coded image there as fast as the bytes (c3a, same call:
        // K4 1.40 vs 1.53 ms) and K7's extra stores cost ~1 ms per 256 4K planes
        f.alpha_k7 = f.alpha_direct && f.ah.filter != 1 && (f.al.n_transforms == 0 || f.al.bits[0] >= 1) &&
                     wg::vp8l_resolve_w64(f.al.cache_bits);
        if (f.alpha_k7 && f.ah.filter == 3) {  // (gradient: rows 1.. in K4's band tiles)
          f.off_atile = pl_b;
          pl_b = align_up(pl_b + (size_t)((f.height - 1 + 63) / 64) * ((f.width + 15) / 16) * 1024);
        }
        if (f.alpha_k7) {
          k7 += px;  // (its filtered bytes)
          k4 += px;  // (K4 reads them back)
        } else if (f.alpha_direct) {
          k4 += 4.0 * f.al.n_px() + (f.al.n_transforms ? (double)f.al.tdata[0].bytes : 0.0);
        } else {
          k3 += ll_bytes(f.al);
          f.off_argba = pl_b;
          pl_b = align_up(pl_b + (size_t)f.width * f.height * 4);
          k4 += 4.0 * px;
        }
      } else {
        k4 += px;
      }
      // (a scratch plane for every alpha frame: vertical / gradient unfilter in it, and
      // alpha-first batches leave every unfiltered plane there)
      f.off_aplane = pl_b;
      pl_b = align_up(pl_b + (size_t)f.width * f.height);
      k4 += 8.0 * px;
      b->alpha_px += px;
    }
  }
  // K6 batches: one output window per frame in d_out; K6 reads the RGBA window of the frames not
  // emitted directly and writes bpp bytes per pixel
  double k6 = 0;
  if (b->k6) {
    b->out_bpp = obpp;
    b->off_out.assign((size_t)n, 0);
    size_t ob = 0;
    for (int i = 0; i < n; ++i) {
      const FrameParse& f = b->fp[(size_t)i];
      if (f.status != WG_STATUS_OK) continue;
      b->off_out[(size_t)i] = ob;
      ob = align_up(ob + (size_t)b->out_bpp * f.out_w * f.out_h);
      if (f.emit_direct) continue;
      b->n_k6++;
      b->k6_maxpx = std::max(b->k6_maxpx, f.out_w * f.out_h);
      k6 += (4.0 + b->out_bpp) * f.out_w * (double)f.out_h;
    }
    b->out_bytes = std::max<size_t>(ob, kAlign);
  }
  // K8 batches (MODE_YUV / MODE_YUVA): one slot of planes per frame in d_out; K8 reads the lossless
  // frames' RGBA window / the lossy frames' plane windows (and alpha planes) and writes the planes
  if (b->yuv) {
    b->off_out.assign((size_t)n, 0);
    size_t ob = 0;
    for (int i = 0; i < n; ++i) {
      const FrameParse& f = b->fp[(size_t)i];
      if (f.status != WG_STATUS_OK) continue;
      b->off_out[(size_t)i] = ob;
      const double px = (double)f.out_w * f.out_h, uv = 2.0 * ((f.out_w + 1) / 2) * (double)((f.out_h + 1) / 2);
      const double planes = px + uv + (b->yuva ? px : 0.0);
      ob = align_up(ob + (size_t)planes);
      k6 += planes + (f.lossless ? 4.0 * px : planes);
      b->yuv_max_uw = std::max(b->yuv_max_uw, (f.out_w + 1) / 2);
      b->yuv_max_uh = std::max(b->yuv_max_uh, (f.out_h + 1) / 2);
    }
    b->out_bytes = std::max<size_t>(ob, kAlign);
  }
  b->kbytes[0] = k1;
  b->kbytes[1] = k2;
  b->kbytes[2] = k3;
  b->kbytes[3] = k4;
  b->kbytes[4] = k7;
  b->kbytes[5] = k6;
  // the split kernel's progress flags, one region (zeroed at upload)
  b->off_gprog = pl_b;
  pl_b = align_up(pl_b + b->gprog_bytes);
  b->plane_bytes = std::max<size_t>(pl_b, kAlign);
  b->rgba_bytes = std::max<size_t>(rg_b, kAlign);
}

// Device half: buffers (from the context's cache), descriptors, and the H2D copies of the staged
// inputs, all queued on the batch's home stream; the arena may be reused once they complete.
// OUT_OF_MEMORY if a buffer or a copy could not be had (the batch then holds what it got: its
// deleter hands it back).
// Workgroups per frame for K1 (1 = one per frame, the kernels with the RGBA tail).  A batch of
// fewer frames than CUs leaves CUs idle while each frame's wavefront runs on one of them, so
// with room for two or more workgroups per frame the split kernel spreads each frame's MB-row
// quads over up to three CUs -- if some frame has more quads than one workgroup reconstructs at
// once (a 4K frame: 34 quads, 12 per workgroup).  WG_K1_SPLIT=0 disables it, =N forces N parts
// (measurement).
// A batch of more than CUs frames runs the one-workgroup kernel over whole rounds of 256 frames; a
// short last round (the 257th frame) would cost a full frame's critical path for a few frames, so
// it runs on the split kernel instead, behind the others (*from = its first frame).
int split_k1_parts(const wg_batch* b, int* from = nullptr) {
  static const int forced = [] {
    const char* e = getenv("WG_K1_SPLIT");
    return e ? atoi(e) : -1;
  }();
  if (from) *from = 0;
  if (b->n_lossy == 0 || forced == 0 || forced == 1) return 1;
  constexpr int kCUs = 256, kRecon = 12, kQuadRows = 4;
  if (forced >= 2) return std::min(forced, wg::kMaxSplitParts);
  const int head = b->n > kCUs ? b->n / kCUs * kCUs : 0;  // whole rounds of the one-workgroup kernel
  int max_quads = 0;
  for (int i = head; i < b->n; ++i) {
    const FrameParse& f = b->fp[(size_t)i];
    if (f.status == WG_STATUS_OK && !f.lossless) max_quads = std::max(max_quads, (f.info.mb_h + kQuadRows - 1) / kQuadRows);
  }
  const int cap = kCUs / std::max(1, (b->n - head + 7) / 8 * 8);  // (the grid rounds the frames up to XCD groups)
  const int want = (max_quads + kRecon - 1) / kRecon;              // slabs of at most 12 quads
  // as many parts as fit (up to 3), the quads balanced over them (split_slab): a 1080p frame's 17
  // quads on 3 parts of 6 instead of 2 of 12 + 5 -- anim K1 1.965 -> 1.880 ms (k1_split_slab/)
  const int parts = want >= 2 ? std::min(3, cap) : 1;
  // (fewer parts than slabs would leave the taller frames on part 0 alone, without the RGBA tail:
  // slower than the one-workgroup kernel -- 128 4K frames on 2 parts: 7.8 vs 7.5 ms)
  if (parts < 2 || parts < want) return 1;
  if (from) *from = head;
  return parts;
}

// K7 can run beside K1 / K2 (wg_batch_run) when their grids fit on the chip together: one
// workgroup per CU each -- K1's one-workgroup or split kernel, one K7 workgroup per stream.
// WG_K7_SIDE=0 keeps K7 in stream order, and so does the pipelined decode (its chunks already
// overlap on two work streams; a side stream shared by them measured 7.45-7.59k -> 5.27-5.44k
// MPix/s on c3a end to end, its K7s holding up the uploads and downloads).
bool k7_side_fits(const wg_batch* b) {
  static const bool off = [] {
    const char* e = getenv("WG_K7_SIDE");
    return e && atoi(e) == 0;
  }();
  constexpr int kCUs = 256;
  const int head = b->split_parts >= 2 ? b->split_from : b->n;
  const int k1_wgs = head + (b->split_parts >= 2 ? (b->n - head + 7) / 8 * 8 * b->split_parts : 0);
  return !off && !b->no_side && b->n_lossy > 0 && b->n_k3 > 0 && k1_wgs + (int)b->tokdesc.size() <= kCUs;
}

// Alpha-first: K7 -> K3 -> K4 before the YUV -> RGBA strips, K4 leaving each alpha plane
// unfiltered in its scratch plane and the strips (K1's tail or K2) taking A from it -- instead of
// K4 read-modify-writing the RGBA's A bytes afterwards (8 B/px -> 1 B/px written + 1 B/px read).
// Not with crop windows (K4 would need the window's plane), nor where K7 runs beside K1 and K1's
// tail converts (the overlap is worth more); without the tail only K2 waits for K4, so the split
// kernel's batches keep K7 beside K1 and run alpha-first too.  Decided for the batch's current K1
// configuration (upload, wg_batch_set_emit, wg_batch_set_k1_parts) into the host descriptors;
// returns whether the choice changed (the caller copies desc / adesc to the device).
// WG_ALPHA_FIRST=0 disables it (measurement).
bool set_alpha_first(wg_batch* b) {
  static const bool off = [] {
    const char* e = getenv("WG_ALPHA_FIRST");
    return e && atoi(e) == 0;
  }();
  // (YUV output: always -- K8 takes A from the unfiltered planes)
  const bool af = b->n_alpha > 0 && (b->yuv || (!b->any_crop && !off && (!b->fused || !k7_side_fits(b))));
  const bool changed = af != b->alpha_first;
  b->alpha_first = af;
  size_t j = 0;
  for (int i = 0; i < b->n; ++i) {
    const FrameParse& f = b->fp[(size_t)i];
    if (f.status != WG_STATUS_OK || f.lossless || !f.alpha) continue;
    AlphaDesc& a = b->adesc[j++];
    a.plane = af || !f.alpha_direct || f.ah.filter >= 2 ? b->d_planes + f.off_aplane : nullptr;
    a.to_plane = af ? 1 : 0;
    b->desc[(size_t)i].alpha_off16 = af ? (int32_t)((f.off_aplane - f.off_y) / 16) : 0;
  }
  return changed;
}

// The split kernel's slab (MB-row quads per part): the split frames' quads balanced over the parts,
// at most 12 (one per reconstructing wave); a frame with more quads than parts * slab runs on part 0.
int split_slab(const wg_batch* b, int from) {
  constexpr int kRecon = 12, kQuadRows = 4;
  int max_quads = 0;
  for (int i = from; i < b->n; ++i) {
    const FrameParse& f = b->fp[(size_t)i];
    if (f.status == WG_STATUS_OK && !f.lossless) max_quads = std::max(max_quads, (f.info.mb_h + kQuadRows - 1) / kQuadRows);
  }
  const int p = std::max(2, b->split_parts);
  return std::min(kRecon, std::max(1, (max_quads + p - 1) / p));
}

// Tags of the split kernel's progress flags (epoch << 16 | columns done): a fresh value per launch,
// never 0.  The tag is 16 bits and the counter process-wide, so it repeats every 65,535 split
// launches: correctness does not rest on it.  wg_batch_run zeroes the batch's flags on the launch
// stream before every split launch (hipMemsetAsync, 512 B per frame), so a flag left by an earlier
// launch reads 0 whatever its tag; the tag only keeps a flag from a launch still running on
// another stream (two concurrent runs of one batch, which race on its planes anyway) from being
// taken for this one's.  wg_debug_set_epoch moves the counter (tests: a re-run exactly one tag
// cycle later).
uint32_t next_epoch() {
  uint32_t e;
  do e = (g_epoch.fetch_add(1, std::memory_order_relaxed) + 1) & 0xffffu;
  while (e == 0);
  return e;
}

int batch_upload(wg_batch* b, const wg::StagingArena& arena) {
  wg_ctx* ctx = b->ctx;
  const int n = b->n;
  const int32_t flags = b->flags;
  const hipStream_t home = b->home;
  DeviceCache& cache = ctx->cache;
  b->d_in = static_cast<uint8_t*>(cache.get(b->in_bytes));
  b->d_planes = static_cast<uint8_t*>(cache.get(b->plane_bytes));
  b->d_rgba = static_cast<uint8_t*>(cache.get(b->rgba_bytes));
  b->d_desc = static_cast<FrameDesc*>(cache.get(sizeof(FrameDesc) * (size_t)n));
  b->d_lldesc = static_cast<LLDesc*>(cache.get(sizeof(LLDesc) * (size_t)std::max(b->n_k3, 1)));
  b->d_tokdesc = static_cast<wg::LLTokDesc*>(cache.get(sizeof(wg::LLTokDesc) * (size_t)std::max(b->n_k3, 1)));
  b->d_adesc = static_cast<AlphaDesc*>(cache.get(sizeof(AlphaDesc) * (size_t)std::max(b->n_alpha, 1)));
  b->d_err = static_cast<int*>(cache.get(sizeof(int)));
  if (!b->d_in || !b->d_planes || !b->d_rgba || !b->d_desc || !b->d_lldesc || !b->d_tokdesc || !b->d_adesc || !b->d_err ||
      hipMemsetAsync(b->d_err, 0, sizeof(int), home) != hipSuccess)
    return WG_STATUS_OUT_OF_MEMORY;
  b->desc.assign((size_t)n, FrameDesc{});
  for (int i = 0; i < n; ++i) {
    FrameParse& f = b->fp[(size_t)i];
    FrameDesc& d = b->desc[(size_t)i];
    if (f.status != WG_STATUS_OK) continue;
    d.rgba = b->d_rgba + f.off_rgba;
    d.width = f.width;
    d.height = f.height;
    d.rgba_stride = 4 * f.rgba_w;
    if (f.lossless) {  // K1/K2 skip it (valid = 0); K3 gets an LLDesc
      b->lldesc.push_back(make_ll(f.ll, arena, b->d_in, b->d_planes, b->d_planes + f.off_scratch, d.rgba, d.rgba_stride));
      b->tokdesc.push_back(make_tok(f.ll, arena, b->d_in, b->d_planes));
      continue;
    }
    const wg_vp8_info& inf = f.info;
    uint8_t* in = b->d_in + arena.dev_offset(f.input);
    d.mbs = reinterpret_cast<const MbRec*>(in);
    d.row_block0 = reinterpret_cast<const uint32_t*>(in + f.off_rows);
    d.blocks = reinterpret_cast<const int16_t*>(in + f.off_blocks);
    d.blocks_bytes = (int32_t)(f.n_blocks * 32);
    d.y = b->d_planes + f.off_y;
    d.cols = b->d_planes + f.off_cols;
    d.gprog = reinterpret_cast<uint32_t*>(b->d_planes + b->off_gprog + f.off_gprog);
    d.u = b->d_planes + f.off_u;
    d.v = b->d_planes + f.off_v;
    d.mb_w = inf.mb_w;
    d.mb_h = inf.mb_h;
    d.y_stride = 16 * inf.mb_w;
    d.uv_stride = 8 * inf.mb_w;
    d.filter_type = inf.filter_type;
    d.flags = flags | (f.wide ? wg::kFrameGlobalCols : 0);
    d.valid = 1;
    if (f.alpha) {
      AlphaDesc a{};
      if (f.ah.method == 1) {
        b->tokdesc.push_back(make_tok(f.al, arena, b->d_in, b->d_planes));
        if (f.alpha_k7) {  // (K7 writes the filtered bytes: K4 reads them as it reads a raw plane)
          wg::LLTokDesc& t = b->tokdesc.back();
          uint8_t* dst = b->d_planes + f.off_aplane;
          t.afilt = dst;
          t.a_cw = f.al.coded_width;
          t.a_width = f.width;
          t.a_height = f.height;
          t.a_cbits = f.al.n_transforms ? f.al.bits[0] : 0;
          t.a_pal = f.al.n_transforms ? 1 : 0;
          // p / cw by multiply-shift for p < 2^28 (n_px): l = ceil(log2 cw), m = 2^(28+l) / cw + 1
          int l = 0;
          while ((1 << l) < t.a_cw) ++l;
          t.a_cw_s = l;
          t.a_cw_m = (uint32_t)((uint64_t(1) << (28 + l)) / (uint64_t)t.a_cw + 1);
          if (t.a_pal) {  // ExpandColorMap's padded map: 1 << (8 >> cbits) <= 16 ARGB entries
            const uint32_t* pal = reinterpret_cast<const uint32_t*>(arena.host_ptr(f.al.tdata[0]));
            const int ne = 1 << (8 >> t.a_cbits);
            for (int e = 0; e < ne; ++e) t.a_pg[e >> 2] |= ((pal[e] >> 8) & 0xffu) << (8 * (e & 3));
          }
          if (f.ah.filter == 3) t.atile = b->d_planes + f.off_atile;
          a.raw = dst;
          a.tiles = t.atile;
        } else if (f.alpha_direct) {
          a.coded = reinterpret_cast<const uint32_t*>(b->d_planes + f.al.off_coded);
          a.coded_width = f.al.coded_width;
          a.cbits = f.al.n_transforms ? f.al.bits[0] : 0;
          if (f.al.n_transforms) a.pal = reinterpret_cast<const uint32_t*>(b->d_in + arena.dev_offset(f.al.tdata[0]));
        } else {
          b->lldesc.push_back(make_ll(f.al, arena, b->d_in, b->d_planes, b->d_planes + f.off_ascratch,
                                      b->d_planes + f.off_argba, 4 * f.width));
          a.green = b->d_planes + f.off_argba;
        }
      } else {
        a.raw = b->d_in + arena.dev_offset(f.araw);
      }
      a.plane = f.alpha_direct && f.ah.filter <= 1 ? nullptr : b->d_planes + f.off_aplane;
      a.rgba = d.rgba;
      a.width = f.width;
      a.height = f.height;
      a.rgba_stride = d.rgba_stride;
      a.filter = f.ah.filter;
      a.valid = 1;
      a.win_x = f.cropped ? (b->opt.crop_left & ~1) : 0;
      a.win_y = f.cropped ? (b->opt.crop_top & ~1) : 0;
      a.win_w = f.out_w;
      a.win_h = f.out_h;
      b->adesc.push_back(a);
    }
  }
  // K6 batches: the output slots; frames emitted directly point K1's tail / K2 at theirs
  if (b->k6) {
    b->d_out = static_cast<uint8_t*>(cache.get(b->out_bytes));
    b->d_edesc = static_cast<EmitDesc*>(cache.get(sizeof(EmitDesc) * (size_t)n));
    if (!b->d_out || !b->d_edesc) return WG_STATUS_OUT_OF_MEMORY;
    for (int i = 0; i < n; ++i) {
      const FrameParse& f = b->fp[(size_t)i];
      if (f.status != WG_STATUS_OK || !f.emit_direct) continue;
      FrameDesc& d = b->desc[(size_t)i];
      d.rgba = b->d_out + b->off_out[(size_t)i];
      d.rgba_stride = b->out_bpp * f.out_w;
      d.emit = b->opt.colorspace + 1;
      d.emit_flip = b->opt.flip ? 1 : 0;
      // (RGBA and rgbA of these opaque frames are the plain RGBA stores; K2's RGBA-only kernel
      // does not flip)
      b->k2_modes |= (b->opt.colorspace != 1 && b->opt.colorspace != 7) || b->opt.flip;
    }
  }
  // Fewer frames than CUs: K1's split kernel (split_k1_parts); it has no RGBA tail, K2 converts.
  b->split_parts = split_k1_parts(b, &b->split_from);
  // Full-frame RGBA (no crop window anywhere in the batch): K1 converts each frame in its
  // own tail instead of a separate K2 launch (wg_batch_set_emit() switches back); a split
  // remainder behind whole rounds converts in a K2 over its frames alone.
  if (b->split_parts >= 2 && b->split_from > 0 && b->any_crop) b->split_parts = 1, b->split_from = 0;
  // K1's tail writes RGBA and RGB_565 (rgbA = RGBA for the opaque frames it emits directly); the
  // other output colorspaces of directly emitted frames convert in K2 (yuv_rgba_strip.h store_out)
  const int cs = b->opt.colorspace;
  b->tail_modes = cs == 1 || cs == 7 || cs == 6;
  for (int i = 0; i < n && !b->tail_modes; ++i) b->no_tail |= b->fp[(size_t)i].emit_direct;
  if (b->no_tail && b->split_parts >= 2 && b->split_from > 0) b->split_parts = 1, b->split_from = 0;
  b->fused = !b->any_crop && !b->no_tail && !b->yuv && (b->split_parts < 2 || b->split_from > 0);
  if (b->fused)
    for (int i = 0; i < n; ++i)
      if (b->desc[(size_t)i].valid) b->desc[(size_t)i].flags |= wg::kFrameEmitRgba;
  set_alpha_first(b);
  if (b->any_crop) {  // K2's view: cropped lossy frames read their compact planes
    b->desc2 = b->desc;
    for (int i = 0; i < n; ++i) {
      FrameParse& f = b->fp[(size_t)i];
      FrameDesc& d2 = b->desc2[(size_t)i];
      if (f.status != WG_STATUS_OK || f.lossless || !f.cropped) continue;
      d2.y = b->d_planes + f.off_yc;
      d2.u = b->d_planes + f.off_uc;
      d2.v = b->d_planes + f.off_vc;
      d2.y_stride = f.yc_stride;
      d2.uv_stride = f.uvc_stride;
      d2.width = f.out_w;
      d2.height = f.out_h;
    }
  }
  // K6's descriptors: the RGBA window of every frame not emitted directly -> its slot of d_out
  if (b->k6) {
    b->edesc.assign((size_t)n, EmitDesc{});
    for (int i = 0; i < n; ++i) {
      const FrameParse& f = b->fp[(size_t)i];
      if (f.status != WG_STATUS_OK || f.emit_direct) continue;
      const FrameDesc& d = b->desc[(size_t)i];
      // the output window inside the RGBA (window_ptr: lossless crops are sub-rectangles)
      const uint8_t* src = d.rgba + (size_t)f.win_y * d.rgba_stride + 4 * (size_t)f.win_x;
      b->edesc[(size_t)i] = EmitDesc{src, b->d_out + b->off_out[(size_t)i], d.rgba_stride, b->out_bpp * f.out_w,
                                     f.out_w, f.out_h, b->opt.colorspace, b->opt.flip ? 1 : 0, 1, 0};
    }
  }
  // K8's descriptors: every frame's output window -> its slot of planes in d_out
  if (b->yuv) {
    b->d_out = static_cast<uint8_t*>(cache.get(b->out_bytes));
    b->d_ydesc = static_cast<YuvaDesc*>(cache.get(sizeof(YuvaDesc) * (size_t)n));
    if (!b->d_out || !b->d_ydesc) return WG_STATUS_OUT_OF_MEMORY;
    b->ydesc.assign((size_t)n, YuvaDesc{});
    for (int i = 0; i < n; ++i) {
      const FrameParse& f = b->fp[(size_t)i];
      if (f.status != WG_STATUS_OK) continue;
      const FrameDesc& d = b->desc[(size_t)i];
      YuvaDesc& y = b->ydesc[(size_t)i];
      // the window origin: lossless exact (f.win_x / win_y), lossy snapped to even
      const int wx = f.lossless ? f.win_x : (b->opt.use_cropping ? b->opt.crop_left & ~1 : 0);
      const int wy = f.lossless ? f.win_y : (b->opt.use_cropping ? b->opt.crop_top & ~1 : 0);
      y.width = f.out_w;
      y.height = f.out_h;
      y.flip = b->opt.flip ? 1 : 0;
      y.valid = 1;
      if (f.lossless) {
        y.lossless = 1;
        y.rgba = d.rgba + (size_t)wy * d.rgba_stride + 4 * (size_t)wx;
        y.rgba_stride = d.rgba_stride;
      } else {
        y.y = d.y + (size_t)wy * d.y_stride + wx;
        y.u = d.u + (size_t)(wy >> 1) * d.uv_stride + (wx >> 1);
        y.v = d.v + (size_t)(wy >> 1) * d.uv_stride + (wx >> 1);
        y.y_stride = d.y_stride;
        y.uv_stride = d.uv_stride;
        if (f.alpha && b->yuva) {  // (K4 leaves the unfiltered plane: to_plane, set_alpha_first)
          y.a = b->d_planes + f.off_aplane + (size_t)wy * f.width + wx;
          y.a_stride = f.width;
        }
      }
      const size_t px = (size_t)f.out_w * f.out_h, uv = (size_t)((f.out_w + 1) / 2) * ((f.out_h + 1) / 2);
      y.oy = b->d_out + b->off_out[(size_t)i];
      y.ou = y.oy + px;
      y.ov = y.ou + uv;
      y.oa = b->yuva ? y.ov + uv : nullptr;
    }
  }
  // the staged inputs: one copy per arena chunk, from pinned memory
  hipError_t e = hipSuccess;
  if (b->gprog_bytes) e = hipMemsetAsync(b->d_planes + b->off_gprog, 0, b->gprog_bytes, home);
  for (size_t c = 0; c < arena.n_chunks() && e == hipSuccess; ++c) {
    const wg::StagingArena::Chunk& ch = arena.chunk(c);
    if (ch.used) e = hipMemcpyAsync(b->d_in + ch.dev_base, ch.p, ch.used, hipMemcpyHostToDevice, home);
  }
  if (e == hipSuccess && b->any_crop) {
    b->d_desc2 = static_cast<FrameDesc*>(cache.get(sizeof(FrameDesc) * (size_t)n));
    e = b->d_desc2 ? hipMemcpyAsync(b->d_desc2, b->desc2.data(), sizeof(FrameDesc) * (size_t)n, hipMemcpyHostToDevice,
                                    home)
                   : hipErrorOutOfMemory;
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(b->d_desc, b->desc.data(), sizeof(FrameDesc) * (size_t)n, hipMemcpyHostToDevice,
                       home);
  // K3 launches one kernel per variant over a contiguous group of descriptors
  std::stable_sort(b->lldesc.begin(), b->lldesc.end(),
                   [](const LLDesc& a, const LLDesc& c) { return a.pad1[0] < c.pad1[0]; });
  for (const LLDesc& l : b->lldesc) b->ll_groups[l.pad1[0]]++;
  if (e == hipSuccess && !b->lldesc.empty())
    e = hipMemcpyAsync(b->d_lldesc, b->lldesc.data(), sizeof(LLDesc) * b->lldesc.size(), hipMemcpyHostToDevice,
                       home);
  // K7 launches the streams of its 64-mask-word instantiation first (one kernel each), the alpha
  // streams whose bytes it writes (a 64-word instantiation of their own) before them
  std::stable_partition(b->tokdesc.begin(), b->tokdesc.end(),
                        [](const wg::LLTokDesc& t) { return wg::vp8l_resolve_w64(t.cache_bits); });
  b->n_tok_w64 = (int)std::count_if(b->tokdesc.begin(), b->tokdesc.end(),
                                    [](const wg::LLTokDesc& t) { return wg::vp8l_resolve_w64(t.cache_bits); });
  std::stable_partition(b->tokdesc.begin(), b->tokdesc.begin() + b->n_tok_w64,
                        [](const wg::LLTokDesc& t) { return t.afilt != nullptr; });
  b->n_tok_alpha = (int)std::count_if(b->tokdesc.begin(), b->tokdesc.end(),
                                      [](const wg::LLTokDesc& t) { return t.afilt != nullptr; });
  std::stable_partition(b->tokdesc.begin(), b->tokdesc.begin() + b->n_tok_alpha,
                        [](const wg::LLTokDesc& t) { return t.atile != nullptr; });
  b->n_tok_tiled = (int)std::count_if(b->tokdesc.begin(), b->tokdesc.end(),
                                      [](const wg::LLTokDesc& t) { return t.atile != nullptr; });
  if (e == hipSuccess && !b->tokdesc.empty())
    e = hipMemcpyAsync(b->d_tokdesc, b->tokdesc.data(), sizeof(wg::LLTokDesc) * b->tokdesc.size(),
                       hipMemcpyHostToDevice, home);
  if (e == hipSuccess && !b->adesc.empty())
    e = hipMemcpyAsync(b->d_adesc, b->adesc.data(), sizeof(AlphaDesc) * b->adesc.size(), hipMemcpyHostToDevice,
                       home);
  if (e == hipSuccess && b->k6)
    e = hipMemcpyAsync(b->d_edesc, b->edesc.data(), sizeof(EmitDesc) * (size_t)n, hipMemcpyHostToDevice, home);
  if (e == hipSuccess && b->yuv)
    e = hipMemcpyAsync(b->d_ydesc, b->ydesc.data(), sizeof(YuvaDesc) * (size_t)n, hipMemcpyHostToDevice, home);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    return WG_STATUS_OUT_OF_MEMORY;
  }
  return WG_STATUS_OK;
}

wg_batch* batch_create(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                       const wg_decoder_options* opt, int32_t* status) {
  if (status)
    for (int i = 0; i < n; ++i) status[i] = WG_STATUS_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!set_device(ctx->device)) {
    if (status)
      for (int i = 0; i < n; ++i) status[i] = WG_STATUS_INVALID_PARAM;
    return nullptr;
  }
  BatchPtr bp = batch_parse(ctx, *ctx->arena, ctx->stream, data, sizes, n, opt, status);
  int st = batch_upload(bp.get(), *ctx->arena);
  // the staging memory is reused by the next batch: the copies complete here
  if (st == WG_STATUS_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) {
    (void)hipGetLastError();
    st = WG_STATUS_OUT_OF_MEMORY;
  }
  if (st != WG_STATUS_OK) {
    if (status)
      for (int i = 0; i < n; ++i)
        if (status[i] == WG_STATUS_OK) status[i] = st;
    return nullptr;  // bp's deleter hands every buffer back
  }
  return bp.release();
}
}  // namespace

extern "C" {

namespace {
// The context's side stream for K7 (k7_side_fits; not when K1's tail converts alpha-first frames:
// it waits for K4 and so for K7), else null.  Created on first use.
hipStream_t k7_side_stream(wg_batch* b) {
  if ((b->alpha_first && b->fused) || !k7_side_fits(b)) return nullptr;
  wg_ctx* c = b->ctx;
  std::lock_guard<std::mutex> lock(c->side_mu);
  if (!c->side && hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking) != hipSuccess) c->side = nullptr;
  return c->side;
}
}  // namespace

int wg_batch_run(wg_batch* b, void* stream) {
  if (!b) return WG_STATUS_INVALID_PARAM;
  if (b->n_valid == 0) return WG_STATUS_OK;
  if (!set_device(b->ctx->device)) return WG_STATUS_INVALID_PARAM;
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : b->home;
  if (b->n_runs_pending >= b->timings.size()) {
    Timing t;
    if (timing_create(b->ctx, t) != hipSuccess) {
      timing_destroy(b->ctx, t);
      return WG_STATUS_OUT_OF_MEMORY;
    }
    b->timings.push_back(t);
  }
  Timing& t = b->timings[b->n_runs_pending++];
  t.ran[kStageK1] = b->n_lossy > 0;
  // (a split remainder behind fused rounds: K2 over the remainder)
  const int k2_from = b->fused ? b->split_from : 0;
  t.ran[kStageK2] = b->n_lossy > 0 && !b->yuv && (!b->fused || (b->split_parts >= 2 && b->split_from > 0));
  t.ran[kStageK7] = b->n_k3 > 0;
  t.ran[kStageK3] = !b->lldesc.empty();
  t.ran[kStageK4] = b->n_alpha > 0;
  t.ran[kStageK6] = (b->k6 && b->n_k6 > 0) || b->yuv;  // (YUV output: K8 in K6's place)
  t.ran[kStageK5] = b->anim;
  // launch order (ev[i] .. ev[i + 1] bracket stage order[i]): K1 / K2 first, or, alpha-first,
  // the alpha planes (K7 -> K3 -> K4) before the strips that take A from them: before K1 when its
  // tail converts, else before K2 alone
  static constexpr int8_t kOrderAlphaFirst[kStages] = {kStageK7, kStageK3, kStageK4, kStageK1,
                                                       kStageK2, kStageK6, kStageK5};
  static constexpr int8_t kOrderAlphaK2[kStages] = {kStageK1, kStageK7, kStageK3, kStageK4,
                                                    kStageK2, kStageK6, kStageK5};
  for (int i = 0; i < kStages; ++i)
    t.order[i] = !b->alpha_first ? (int8_t)i : b->fused ? kOrderAlphaFirst[i] : kOrderAlphaK2[i];
  hipEventRecord(t.ev[0], s);
  // K7 only feeds K3 / K4: when its grid fits on the chip beside K1's, it runs on the context's
  // side stream, concurrently with K1 and K2, and K3 waits for it
  hipStream_t side = k7_side_stream(b);
  t.forked = side != nullptr;
  if (side) {
    hipError_t e = hipStreamWaitEvent(side, t.ev[0], 0);
    if (e == hipSuccess) e = hipEventRecord(t.side[0], side);
    if (e == hipSuccess) e = wg::launch_vp8l_resolve(b->d_tokdesc, nullptr, (int)b->tokdesc.size(), b->d_err, side, b->n_tok_w64,
                                                   b->n_tok_alpha, b->n_tok_tiled);
    if (e == hipSuccess) e = hipEventRecord(t.side[1], side);
    if (e != hipSuccess) return WG_STATUS_UNSUPPORTED_FEATURE;
  }
  auto stage = [&](int k) -> int {
    hipError_t e = hipSuccess;
    switch (k) {
      case kStageK1:
        if (b->n_lossy > 0) {
          const int head = b->split_parts >= 2 ? b->split_from : b->n;  // frames on the one-workgroup kernels
          if (head > 0)
            e = wg::launch_vp8_recon_filter(b->d_desc, head, b->max_mb_w, b->n_lossy > b->n_wide, b->n_wide > 0, b->d_err, s);
          // (the split frames' progress flags cleared first, in stream order: see next_epoch)
          if (e == hipSuccess && b->split_parts >= 2)
            e = hipMemsetAsync(b->d_planes + b->off_gprog, 0, b->gprog_bytes, s);
          if (e == hipSuccess && b->split_parts >= 2)
            e = wg::launch_vp8_recon_filter(b->d_desc + head, b->n - head, b->max_mb_w, false, false, b->d_err, s,
                                            b->split_parts, next_epoch(), split_slab(b, head));
        }
        break;
      case kStageK2:
        if (!t.ran[kStageK2]) break;
        if (b->any_crop) {
          // the crop windows of the reconstructed planes (even left/top, so chroma is aligned):
          // upsampled as standalone images, as EmitFancyRGB / EmitSampledRGB see them
          for (int i = 0; i < b->n; ++i) {
            const FrameParse& f = b->fp[i];
            if (f.status != WG_STATUS_OK || f.lossless || !f.cropped) continue;
            const FrameDesc& d = b->desc[i];
            const FrameDesc& d2 = b->desc2[i];
            const int x = b->opt.crop_left & ~1, y = b->opt.crop_top & ~1;
            const int uw = (f.out_w + 1) >> 1, uh = (f.out_h + 1) >> 1;
            e = hipMemcpy2DAsync(d2.y, d2.y_stride, d.y + (size_t)y * d.y_stride + x, d.y_stride, f.out_w, f.out_h,
                                 hipMemcpyDeviceToDevice, s);
            if (e == hipSuccess)
              e = hipMemcpy2DAsync(d2.u, d2.uv_stride, d.u + (size_t)(y >> 1) * d.uv_stride + (x >> 1), d.uv_stride, uw,
                                   uh, hipMemcpyDeviceToDevice, s);
            if (e == hipSuccess)
              e = hipMemcpy2DAsync(d2.v, d2.uv_stride, d.v + (size_t)(y >> 1) * d.uv_stride + (x >> 1), d.uv_stride, uw,
                                   uh, hipMemcpyDeviceToDevice, s);
            if (e != hipSuccess) return WG_STATUS_USER_ABORT;
          }
        }
        e = wg::launch_yuv_to_rgba((b->any_crop ? b->d_desc2 : b->d_desc) + k2_from, nullptr, b->n - k2_from,
                                   b->max_out_w, b->max_out_h, (b->flags & WG_FLAG_NO_FANCY_UPSAMPLING) ? 0 : 1, s,
                                   b->k2_modes);
        break;
      case kStageK7:  // the lossless streams' color cache and back-references
        if (t.forked) e = hipStreamWaitEvent(s, t.side[1], 0);
        else if (b->n_k3 > 0)
          e = wg::launch_vp8l_resolve(b->d_tokdesc, nullptr, (int)b->tokdesc.size(), b->d_err, s, b->n_tok_w64, b->n_tok_alpha,
                                      b->n_tok_tiled);
        break;
      case kStageK3:
        if (!b->lldesc.empty()) e = wg::launch_vp8l_transforms(b->d_lldesc, b->ll_groups, b->d_err, s);
        break;
      case kStageK4:  // after K3 (alpha streams) and K2 / K1's tail (A = 255), or alpha-first before them
        if (b->n_alpha > 0) e = wg::launch_alpha(b->d_adesc, b->n_alpha, s, b->n_alpha_2d);
        break;
      case kStageK6:  // the output colorspace / flip over every frame's final RGBA (YUV output: K8)
        if (b->yuv) e = wg::launch_emit_yuva(b->d_ydesc, b->n, b->yuv_max_uw, b->yuv_max_uh, s);
        else if (t.ran[kStageK6]) e = wg::launch_emit(b->d_edesc, b->n, b->k6_maxpx, s);
        break;
      case kStageK5:  // an animation's canvases from its decoded frames
        if (b->anim) e = wg::launch_anim_compose(b->d_fdesc, b->n, b->d_canvases, b->canvas_w, b->canvas_h, s);
        break;
    }
    return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_UNSUPPORTED_FEATURE;
  };
  for (int i = 0; i < kStages; ++i) {
    if (i > 0) hipEventRecord(t.ev[i], s);
    const int st = stage(t.order[i]);
    if (st != WG_STATUS_OK) {
      // a K7 already forked onto the side stream may still write the batch's planes and error word:
      // the side stream's work joins the batch's completion events, so batch_wait (and
      // wg_batch_destroy, before the buffers go back to the cache) waits for it
      if (t.forked) (void)batch_mark_done(b, side);
      (void)batch_mark_done(b, s);
      return st;
    }
  }
  hipEventRecord(t.ev[kStages], s);
  return batch_mark_done(b, s) == hipSuccess ? WG_STATUS_OK : WG_STATUS_OUT_OF_MEMORY;
}

}  // extern "C"

namespace {
// wg_batch_kernel_ms; the pipeline's chunks read their error word asynchronously (err_word given)
int batch_kernel_ms(wg_batch* b, float* ms, int n_ms, const int32_t* err_word) {
  for (int k = 0; k < n_ms; ++k) ms[k] = 0.f;
  if (b->n_runs_pending == 0) return WG_STATUS_OK;
  double acc[kStages] = {};
  int cnt[kStages] = {};
  for (size_t i = 0; i < b->n_runs_pending; ++i) {
    Timing& t = b->timings[i];
    if (hipEventSynchronize(t.ev[kStages]) != hipSuccess) return WG_STATUS_USER_ABORT;
    for (int i = 0; i < kStages; ++i) {
      const int k = t.order[i];
      if (!t.ran[k]) continue;
      float a = 0;
      if (k == kStageK7 && t.forked)
        hipEventElapsedTime(&a, t.side[0], t.side[1]);
      else
        hipEventElapsedTime(&a, t.ev[i], t.ev[i + 1]);
      acc[k] += a;
      cnt[k]++;
    }
  }
  int err = 0;
  if (err_word) err = *err_word;
  else if (hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess) err = 1;
  if (err) return WG_STATUS_USER_ABORT;
  for (int k = 0; k < kStages; ++k) {
    const int pub = kPublicOfStage[k];
    if (pub < n_ms) ms[pub] = cnt[k] ? (float)(acc[k] / cnt[k]) : 0.f;
  }
  b->n_runs_pending = 0;
  return WG_STATUS_OK;
}
}  // namespace

extern "C" {

int wg_batch_kernel_ms(const wg_batch* bc, float* ms, int n_ms) {
  wg_batch* b = const_cast<wg_batch*>(bc);
  if (!b || !ms || n_ms < 1) return WG_STATUS_INVALID_PARAM;
  return batch_kernel_ms(b, ms, n_ms, nullptr);
}

int wg_batch_kernel_bytes(const wg_batch* b, double* bytes, int n_bytes) {
  if (!b || !bytes || n_bytes < 1) return WG_STATUS_INVALID_PARAM;
  for (int k = 0; k < n_bytes; ++k) bytes[k] = k < kStages ? b->kbytes[k] : 0.0;
  if (b->fused) bytes[0] = b->k1_fused_bytes;
  if (b->alpha_first) {  // K4 writes 1 B/px instead of the 8 B/px read-modify-write; the strips read it
    if (n_bytes > 3) bytes[3] -= 7.0 * b->alpha_px;
    if (b->fused) bytes[0] += b->alpha_px;
    if (n_bytes > 1) bytes[1] += b->alpha_px;
  }
  return WG_STATUS_OK;
}

namespace {
// The frame and alpha descriptors to the device again (after a change of the K1 configuration).
int batch_upload_desc(wg_batch* b) {
  if (!set_device(b->ctx->device)) return WG_STATUS_INVALID_PARAM;
  hipError_t e = hipMemcpyAsync(b->d_desc, b->desc.data(), sizeof(FrameDesc) * (size_t)b->n, hipMemcpyHostToDevice,
                                b->home);
  if (e == hipSuccess && !b->adesc.empty())
    e = hipMemcpyAsync(b->d_adesc, b->adesc.data(), sizeof(AlphaDesc) * b->adesc.size(), hipMemcpyHostToDevice, b->home);
  if (e == hipSuccess) e = hipStreamSynchronize(b->home);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}
// Alpha-first for the current K1 configuration; the descriptors uploaded if the choice changed.
int batch_set_alpha_first(wg_batch* b) { return set_alpha_first(b) ? batch_upload_desc(b) : WG_STATUS_OK; }
}  // namespace

int wg_batch_set_emit(wg_batch* b, int separate) {
  if (!b) return WG_STATUS_INVALID_PARAM;
  // crop windows / modes K2 emits / YUV output (no RGBA for lossy frames): no tail
  if (!separate && (b->any_crop || b->no_tail || b->yuv)) return WG_STATUS_INVALID_PARAM;
  if (!separate) b->split_parts = 1, b->split_from = 0;  // K1's RGBA tail: the one-workgroup kernels
  if (b->fused == !separate) return batch_set_alpha_first(b);
  b->fused = !separate;
  for (FrameDesc& d : b->desc)
    if (d.valid) d.flags = b->fused ? (d.flags | wg::kFrameEmitRgba) : (d.flags & ~wg::kFrameEmitRgba);
  set_alpha_first(b);
  return batch_upload_desc(b);
}

int wg_batch_set_k1_parts(wg_batch* b, int parts) {
  if (!b || parts < 0 || parts > wg::kMaxSplitParts) return WG_STATUS_INVALID_PARAM;
  int from = 0;
  const int p = parts == 0 ? split_k1_parts(b, &from) : parts;
  if (p >= 2 && from == 0 && b->fused) {  // the split kernel has no RGBA tail: K2 converts
    const int st = wg_batch_set_emit(b, 1);
    if (st != WG_STATUS_OK) return st;
  }
  if (p >= 2 && from > 0 && b->any_crop) return WG_STATUS_OK;  // (cropped: whole rounds only)
  // back to one part from a whole-batch split (which had switched the batch to K2): the kernels with
  // the RGBA tail again, where the batch can take them (no crop window, no frame emitted in a mode
  // the tail lacks).  A batch set to K2 by wg_batch_set_emit(b, 1) keeps K2.
  if (p == 1 && b->split_parts >= 2 && b->split_from == 0 && !b->fused && !b->any_crop && !b->no_tail && !b->yuv)
    return wg_batch_set_emit(b, 0);
  b->split_parts = p;
  b->split_from = p >= 2 ? from : 0;
  return batch_set_alpha_first(b);
}

int wg_batch_run_emit(wg_batch* b, void* stream) {
  if (!b) return WG_STATUS_INVALID_PARAM;
  if (b->yuv) return WG_STATUS_UNSUPPORTED_FEATURE;  // (YUV output: no RGBA stage)
  if (b->n_lossy == 0 || b->any_crop) return WG_STATUS_OK;
  if (!set_device(b->ctx->device)) return WG_STATUS_INVALID_PARAM;
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : b->home;
  if (b->n_runs_pending >= b->timings.size()) {
    Timing t;
    if (timing_create(b->ctx, t) != hipSuccess) {
      timing_destroy(b->ctx, t);
      return WG_STATUS_OUT_OF_MEMORY;
    }
    b->timings.push_back(t);
  }
  Timing& t = b->timings[b->n_runs_pending++];
  for (bool& r : t.ran) r = false;
  t.forked = false;
  for (int i = 0; i < kStages; ++i) t.order[i] = (int8_t)i;
  t.ran[kStageK2] = true;
  for (int k = 0; k <= kStageK2; ++k) hipEventRecord(t.ev[k], s);
  hipError_t e = wg::launch_yuv_to_rgba(b->d_desc, nullptr, b->n, b->max_out_w, b->max_out_h,
                                        (b->flags & WG_FLAG_NO_FANCY_UPSAMPLING) ? 0 : 1, s, b->k2_modes);
  for (int k = kStageK2 + 1; k <= kStages; ++k) hipEventRecord(t.ev[k], s);
  if (e != hipSuccess) return WG_STATUS_UNSUPPORTED_FEATURE;
  return batch_mark_done(b, s) == hipSuccess ? WG_STATUS_OK : WG_STATUS_OUT_OF_MEMORY;
}

int wg_batch_size(const wg_batch* b) { return b ? b->n : 0; }

int64_t wg_batch_pixels(const wg_batch* b) { return b ? b->pixels : 0; }

int wg_batch_frame_dims(const wg_batch* b, int i, int32_t* width, int32_t* height) {
  if (!b || i < 0 || i >= b->n) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  if (width) *width = b->fp[i].out_w;
  if (height) *height = b->fp[i].out_h;
  return WG_STATUS_OK;
}

int wg_batch_frame_status(const wg_batch* b, int i) {
  if (!b || i < 0 || i >= b->n) return WG_STATUS_INVALID_PARAM;
  return b->fp[i].status;
}

namespace {
// Wait for the batch's work and check the kernels' error word.
int batch_sync(wg_batch* b) {
  if (!set_device(b->ctx->device)) return WG_STATUS_INVALID_PARAM;
  hipError_t e = batch_wait(b);
  int err = 0;
  if (e == hipSuccess) e = hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost);
  return (e != hipSuccess || err) ? WG_STATUS_USER_ABORT : WG_STATUS_OK;
}
const uint8_t* window_ptr(const wg_batch* b, int i) {
  const FrameParse& f = b->fp[i];
  const FrameDesc& d = b->desc[i];
  return d.rgba + (size_t)f.win_y * d.rgba_stride + 4 * (size_t)f.win_x;
}
// Bytes a row-major output of h rows of `row` bytes at `stride` needs (0 rows: nothing).
size_t out_bytes_needed(int stride, int row, int h) {
  return h > 0 ? (size_t)stride * (size_t)(h - 1) + (size_t)row : 0;
}

// A caller's output buffer i: present, stride >= the row, capacity >= the window.
bool out_ok(uint8_t* const* out, const int32_t* strides, const size_t* caps, int i, int row, int h) {
  return out[i] != nullptr && strides[i] >= row && caps[i] >= out_bytes_needed(strides[i], row, h);
}

// Every OK frame's RGBA window to out[i] (stride strides[i]): one wait for the batch, the
// copies queued on the context stream, one wait for them.
int download_rgba_all(wg_batch* b, uint8_t* const* out, const int32_t* strides, const size_t* caps, int32_t* status) {
  int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  hipError_t e = hipSuccess;
  for (int i = 0; i < b->n && e == hipSuccess; ++i) {
    if (status[i] != WG_STATUS_OK) continue;
    const FrameParse& f = b->fp[(size_t)i];
    if (!out_ok(out, strides, caps, i, 4 * f.out_w, f.out_h)) {
      status[i] = WG_STATUS_INVALID_PARAM;
      continue;
    }
    e = hipMemcpy2DAsync(out[i], strides[i], window_ptr(b, i), b->desc[(size_t)i].rgba_stride, 4 * (size_t)f.out_w,
                         f.out_h, hipMemcpyDefault, b->home);
  }
  const hipError_t se = hipStreamSynchronize(b->home);
  return (e != hipSuccess || se != hipSuccess) ? WG_STATUS_USER_ABORT : WG_STATUS_OK;
}
}  // namespace

}  // extern "C"

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// One chunk of a pipelined decode: frames [a, a + n) of the call, parsed into staging arena
// `arena` and run on stream `s`.  ev: 0/1 around the upload (1 = the arena is free again),
// 2/3 around the download (3 = everything of the chunk is complete).
struct PipeChunk {
  int a = 0, n = 0, arena = 0;
  int32_t* err_word = nullptr;  // pinned: the chunk's error word, copied behind its download
  hipStream_t s = nullptr;
  BatchPtr b;
  hipEvent_t ev[4] = {};
  bool uploaded = false, up_ok = false, ran = false;
  bool layout_ok = true;  // batch_layout ran (false: it threw; the chunk's frames carry the status)
};

// Every frame of [a, a + n) still OK gets `st` (an early exit must not leave frames that were never
// decoded reading OK).
void fail_frames(int32_t* status, int a, int n, int st) {
  for (int i = a; i < a + n; ++i)
    if (status[i] == WG_STATUS_OK) status[i] = st;
}

// Queue the chunk's RGBA windows to the caller's buffers on its stream (asynchronous for pinned
// memory; the runtime stages pageable memory itself).  Frames with bad arguments get
// INVALID_PARAM; the copies' own failure USER_ABORT.
void pipe_download(PipeChunk& c, uint8_t* const* out, const int32_t* strides, const size_t* caps, int32_t* status,
                   double* bytes) {
  wg_batch* b = c.b.get();
  hipEventRecord(c.ev[2], c.s);
  for (int j = 0; j < c.n; ++j) {
    const int i = c.a + j;
    if (status[i] != WG_STATUS_OK) continue;
    const FrameParse& f = b->fp[(size_t)j];
    if (!out_ok(out, strides, caps, i, 4 * f.out_w, f.out_h)) {
      status[i] = WG_STATUS_INVALID_PARAM;
      continue;
    }
    if (hipMemcpy2DAsync(out[i], strides[i], window_ptr(b, j), b->desc[(size_t)j].rgba_stride, 4 * (size_t)f.out_w,
                         f.out_h, hipMemcpyDefault, c.s) != hipSuccess) {
      (void)hipGetLastError();
      status[i] = WG_STATUS_USER_ABORT;
      continue;
    }
    *bytes += 4.0 * f.out_w * f.out_h;
  }
  if (c.err_word && hipMemcpyAsync(c.err_word, b->d_err, sizeof(int32_t), hipMemcpyDeviceToHost, c.s) != hipSuccess) {
    (void)hipGetLastError();
    *c.err_word = 1;  // (reported as the chunk's failure)
  }
  hipEventRecord(c.ev[3], c.s);
}

// Wait for a chunk, fold its timings into the stats, check the kernels' error word, release it.
void pipe_finish(PipeChunk& c, int32_t* status, wg_pipeline_stats* ps) {
  if (c.ran) {
    hipEventSynchronize(c.ev[3]);
    float ms[5] = {};
    const int st = batch_kernel_ms(c.b.get(), ms, 5, c.err_word);  // (checks the error word)
    for (float m : ms) ps->kernel_ms += m;
    float a = 0;
    if (hipEventElapsedTime(&a, c.ev[0], c.ev[1]) == hipSuccess) ps->h2d_ms += a;
    if (hipEventElapsedTime(&a, c.ev[2], c.ev[3]) == hipSuccess) ps->d2h_ms += a;
    (void)hipGetLastError();
    if (st != WG_STATUS_OK)
      for (int j = 0; j < c.n; ++j)
        if (status[c.a + j] == WG_STATUS_OK) status[c.a + j] = st;
  } else if (c.uploaded && c.b) {
    hipStreamSynchronize(c.s);  // (an error path: whatever of the chunk was queued has finished)
    if (c.b->home) hipStreamSynchronize(c.b->home);
  }
  if (c.b) c.b->home = nullptr;  // complete: destroying it must not wait for later chunks on the stream
  c.b.reset();
  // (the events outlive the chunk: a pool thread readying arena k mod 3 for chunk k + 3 may still be
  // waiting on ev[1]; decode_pipelined destroys them once every thread is done)
}

// wg_decode_rgba_batch: chunked, two staging arenas and two streams.  The calling thread and the
// context's pool run the entropy stage over all frames; a device thread uploads chunk k as soon
// as its last frame is parsed, launches its kernels, then queues chunk k - 1's download and
// retires chunk k - 2, so the host stage of one chunk, the kernels of the next and the transfers
// of a third overlap.
int decode_pipelined(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n, uint8_t* const* out,
                     const int32_t* strides, const size_t* caps, int32_t* status, int32_t flags) {
  const double t_start = now_s();
  wg_decoder_options o{};
  o.colorspace = 1;  // MODE_RGBA
  o.bypass_filtering = !!(flags & WG_FLAG_BYPASS_FILTERING);
  o.no_fancy_upsampling = !!(flags & WG_FLAG_NO_FANCY_UPSAMPLING);
  for (int i = 0; i < n; ++i) status[i] = WG_STATUS_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (!set_device(ctx->device)) {
    fail_frames(status, 0, n, WG_STATUS_INVALID_PARAM);
    return WG_STATUS_INVALID_PARAM;
  }
  // chunks: a fixed frame count, or about a sixteenth of the batch's pixels (>= 32 MPix each)
  std::vector<int> bounds{0};
  if (ctx->chunk_frames > 0) {
    for (int a = ctx->chunk_frames; a < n; a += ctx->chunk_frames) bounds.push_back(a);
  } else {
    std::vector<double> px((size_t)n, 0.0);
    double total = 0;
    for (int i = 0; i < n; ++i) {
      wg_features f{};
      if (data[i] && wg_get_features(data[i], sizes[i], &f) == WG_STATUS_OK) px[(size_t)i] = (double)f.width * f.height;
      total += px[(size_t)i];
    }
    // Only the last chunk's device work (upload, kernels, download) is exposed after the host
    // stage ends, so the batch's last 2T of pixels go in halving chunks: R/2, R/4, R/8, R/8.
    const double T = std::max(32e6, total / 16);
    double target = T, acc = 0, consumed = 0, tail_r = 0;
    int tail = 0;
    for (int i = 0; i < n; ++i) {
      acc += px[(size_t)i];
      if (acc >= target && i + 1 < n) {
        bounds.push_back(i + 1);
        consumed += acc;
        acc = 0;
        if (tail == 0 && total - consumed <= 2 * T) tail_r = total - consumed;
        if (tail_r > 0 && tail < 3) target = tail_r / (double)(2 << tail++);
      }
    }
  }
  bounds.push_back(n);
  const int K = (int)bounds.size() - 1;
  wg_pipeline_stats ps{};
  ps.frames = n;
  ps.chunks = K;
  ps.host_threads = ctx->workers()->threads();
  if (K > 1) {
    for (auto& a : ctx->arena_ring)
      if (!a) a.reset(new wg::StagingArena(pinned_alloc, pinned_free));
    for (hipStream_t& w : ctx->work)
      if (!w && hipStreamCreateWithFlags(&w, hipStreamNonBlocking) != hipSuccess) {
        (void)hipGetLastError();
        w = nullptr;
        fail_frames(status, 0, n, WG_STATUS_OUT_OF_MEMORY);
        return WG_STATUS_OUT_OF_MEMORY;
      }
  }
  // staging arenas in a ring of four: chunk k parses into arena k % 4 once chunk k - 4's upload
  // from it has completed (three left the host stage waiting 5-11 ms per 256-frame c3 call for the
  // device thread, which queues a chunk's upload only after retiring the chunk two before it; with
  // four the waits are gone and the drain grows by less: 7.97k -> 8.10k MPix/s, same call; a fourth
  // halving of the last chunks measured no better)
  constexpr int kRing = 4;
  wg::StagingArena* arenas[kRing] = {ctx->arena.get(), K > 1 ? ctx->arena_ring[0].get() : nullptr,
                                     K > 1 ? ctx->arena_ring[1].get() : nullptr,
                                     K > 1 ? ctx->arena_ring[2].get() : nullptr};
  // one chunk: everything on the context stream; else uploads on it, the rest on a work stream
  hipStream_t streams[2] = {K > 1 ? ctx->work[0] : ctx->stream, K > 1 ? ctx->work[1] : ctx->stream};
  std::vector<PipeChunk> ch((size_t)K);
  // the chunks' events go on every exit path, once no thread can still wait on them
  // (blocking-sync events when a device thread waits on them beside the entropy stage's 16 threads:
  // it sleeps instead of spinning on their CPUs; one chunk: the calling thread waits, spinning --
  // no wake-up latency on the single-frame path)
  const int blocking = K > 1 ? 1 : 0;
  struct EventsGuard {
    std::vector<PipeChunk>& ch;
    wg_ctx* ctx;
    int blocking;
    ~EventsGuard() {
      for (PipeChunk& c : ch)
        for (hipEvent_t& e : c.ev) ctx->give_event(e, blocking), e = nullptr;
    }
  } events_guard{ch, ctx, blocking};
  // one pinned error word per chunk
  if (ctx->n_err_words < K) {
    if (ctx->err_words) pinned_free(ctx->err_words);
    ctx->n_err_words = 0;
    ctx->err_words = static_cast<int32_t*>(pinned_alloc(sizeof(int32_t) * (size_t)std::max(K, 64)));
    if (!ctx->err_words) {
      fail_frames(status, 0, n, WG_STATUS_OUT_OF_MEMORY);
      return WG_STATUS_OUT_OF_MEMORY;
    }
    ctx->n_err_words = std::max(K, 64);
  }
  for (int k = 0; k < K; ++k) {
    PipeChunk& c = ch[(size_t)k];
    c.a = bounds[(size_t)k];
    c.n = bounds[(size_t)k + 1] - c.a;
    c.arena = k % kRing;
    c.s = streams[k & 1];
    c.err_word = ctx->err_words + k;
    *c.err_word = 0;
    for (hipEvent_t& e : c.ev)
      if (!(e = ctx->take_event(blocking))) {
        fail_frames(status, 0, n, WG_STATUS_OUT_OF_MEMORY);
        return WG_STATUS_OUT_OF_MEMORY;
      }
  }
  // every chunk's batch up front (an allocation failure fails the call before any thread starts)
  std::vector<int> chunk_of((size_t)n);
  for (int k = 0; k < K; ++k) {
    ch[(size_t)k].b = batch_init(ctx, ctx->stream, ch[(size_t)k].n, &o);  // home: the upload stream
    if (ch[(size_t)k].b) ch[(size_t)k].b->no_side = true;
    for (int j = 0; j < ch[(size_t)k].n; ++j) chunk_of[(size_t)(ch[(size_t)k].a + j)] = k;
  }
  std::mutex qmu;
  std::condition_variable qcv;
  // per chunk, under qmu: its arena is being readied / is ready; its frames are all parsed; its
  // upload has been queued (the arena is reusable once ev[1] completes)
  std::vector<char> started((size_t)K, 0), ready((size_t)K, 0), parsed((size_t)K, 0), uploaded((size_t)K, 0);
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[(size_t)K]);
  for (int k = 0; k < K; ++k) left[k].store(ch[(size_t)k].n);
  auto device_side = [&] {
    set_device(ctx->device);
    for (int k = 0; k < K; ++k) {
      {
        std::unique_lock<std::mutex> ql(qmu);
        qcv.wait(ql, [&] { return parsed[(size_t)k] != 0; });
      }
      PipeChunk& c = ch[(size_t)k];
      hipEventRecord(c.ev[0], ctx->stream);
      int st = c.layout_ok ? guarded([&] { return batch_upload(c.b.get(), *arenas[c.arena]); })
                           : (int)WG_STATUS_OUT_OF_MEMORY;
      hipEventRecord(c.ev[1], ctx->stream);
      c.up_ok = st == WG_STATUS_OK;
      if (st == WG_STATUS_OK && c.s != ctx->stream && hipStreamWaitEvent(c.s, c.ev[1], 0) != hipSuccess) {
        (void)hipGetLastError();
        st = WG_STATUS_USER_ABORT;
      }
      {
        std::lock_guard<std::mutex> ql(qmu);
        c.uploaded = true;
        uploaded[(size_t)k] = 1;
      }
      qcv.notify_all();
      if (st == WG_STATUS_OK) st = wg_batch_run(c.b.get(), c.s);
      c.ran = st == WG_STATUS_OK;
      if (st != WG_STATUS_OK)
        for (int j = 0; j < c.n; ++j)
          if (status[c.a + j] == WG_STATUS_OK) status[c.a + j] = st;
      if (k >= 1 && ch[(size_t)k - 1].ran) pipe_download(ch[(size_t)k - 1], out, strides, caps, status, &ps.d2h_bytes);
      if (k >= 2) pipe_finish(ch[(size_t)k - 2], status, &ps);
    }
    if (ch[(size_t)K - 1].ran) pipe_download(ch[(size_t)K - 1], out, strides, caps, status, &ps.d2h_bytes);
    for (int k = std::max(0, K - 2); k < K; ++k) pipe_finish(ch[(size_t)k], status, &ps);
  };
  // the device thread is joined on every exit path (a joinable std::thread destroyed would
  // terminate the process)
  struct Joiner {
    std::thread t;
    ~Joiner() {
      if (t.joinable()) t.join();
    }
  } dev;
  if (K > 1) {
    try {
      dev.t = std::thread(device_side);
    } catch (const std::system_error&) {  // nothing started yet: fail the call cleanly
      fail_frames(status, 0, n, WG_STATUS_OUT_OF_MEMORY);
      return WG_STATUS_OUT_OF_MEMORY;
    }
  }
  // The entropy stage as ONE pool run over all frames, claimed in order: a chunk's stragglers
  // overlap the next chunk's frames (no barrier per chunk).  A chunk's first frame readies its
  // arena (chunk k - 3, on the same arena, uploaded); its last frame lays it out and hands it to
  // the device thread.
  wg::WorkerPool* pool = ctx->workers();
  std::vector<wg::StagingArena::Cursor> cursors[kRing];
  for (auto& cv : cursors) cv.resize((size_t)pool->threads() + 1);
  const double t_parse0 = now_s();
  pool->run(n, [&](int i, int worker) {
    const int k = chunk_of[(size_t)i];
    PipeChunk& c = ch[(size_t)k];
    {
      std::unique_lock<std::mutex> ql(qmu);
      if (!started[(size_t)k]) {
        started[(size_t)k] = 1;
        const double t0 = now_s();
        if (k >= kRing) {
          qcv.wait(ql, [&] { return uploaded[(size_t)(k - kRing)] != 0; });
          ql.unlock();
          // (ev[1] is recorded after every upload attempt: a failed upload may still have queued
          // copies out of the arena, which must finish before it is reused)
          hipEventSynchronize(ch[(size_t)(k - kRing)].ev[1]);
          ql.lock();
        }
        arenas[c.arena]->begin_batch();
        ready[(size_t)k] = 1;
        ps.parse_wait_s += now_s() - t0;
        qcv.notify_all();
      } else {
        qcv.wait(ql, [&] { return ready[(size_t)k] != 0; });
      }
    }
    wg::parse_frame(data[i], sizes[i], o, arenas[c.arena], &cursors[c.arena][(size_t)worker],
                    &c.b->fp[(size_t)(i - c.a)]);
    if (left[k].fetch_sub(1) == 1) {
      // (on a worker thread, outside guarded(): an allocation failure marks the chunk's frames and
      // still hands the chunk over, so the device thread never waits for it forever)
      try {
        for (auto& cu : cursors[c.arena]) arenas[c.arena]->release(&cu);
        batch_layout(c.b.get(), *arenas[c.arena], status + c.a);
      } catch (...) {
        c.layout_ok = false;
        for (int j = 0; j < c.n; ++j) status[c.a + j] = WG_STATUS_OUT_OF_MEMORY;
      }
      std::lock_guard<std::mutex> ql(qmu);
      ps.h2d_bytes += (double)c.b->in_bytes;
      parsed[(size_t)k] = 1;
      qcv.notify_all();
    }
  });
  const double t_parsed = now_s();
  ps.parse_s = t_parsed - t_parse0;
  if (K > 1) dev.t.join();
  else device_side();
  const double t_end = now_s();
  ps.drain_s = t_end - t_parsed;
  ps.wall_s = t_end - t_start;
  ctx->stats = ps;
  return WG_STATUS_OK;
}

}  // namespace

extern "C" {

int wg_batch_download_rgba(wg_batch* b, int i, uint8_t* rgba, int stride) {
  if (!b || i < 0 || i >= b->n || !rgba) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  const FrameParse& f = b->fp[i];
  if (f.emit_direct) return WG_STATUS_UNSUPPORTED_FEATURE;  // emitted in the batch's colorspace only
  if (b->yuv && !f.lossless) return WG_STATUS_UNSUPPORTED_FEATURE;  // (YUV output: planes only)
  if (stride < 4 * f.out_w) return WG_STATUS_INVALID_PARAM;
  int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  const hipError_t e = hipMemcpy2D(rgba, stride, window_ptr(b, i), b->desc[i].rgba_stride, 4 * (size_t)f.out_w,
                                   f.out_h, hipMemcpyDefault);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_batch_download(wg_batch* b, int i, uint8_t* out, int stride) {
  if (!b || i < 0 || i >= b->n || !out) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  if (b->yuv) return WG_STATUS_UNSUPPORTED_FEATURE;  // planes: wg_batch_download_yuva
  const FrameParse& f = b->fp[i];
  const int bpp = wg::output_bpp(b->opt.colorspace);
  if (stride < bpp * f.out_w) return WG_STATUS_INVALID_PARAM;
  if (!b->k6) return wg_batch_download_rgba(b, i, out, stride);
  int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  // K6 ran in wg_batch_run: one 2D copy of the frame's slot of d_out
  const size_t row = (size_t)bpp * f.out_w;
  const hipError_t e =
      hipMemcpy2D(out, stride, b->d_out + b->off_out[(size_t)i], row, row, f.out_h, hipMemcpyDefault);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_batch_download_yuv(wg_batch* b, int i, uint8_t* y, uint8_t* u, uint8_t* v) {
  if (!b || i < 0 || i >= b->n) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  if (b->fp[i].lossless) return WG_STATUS_UNSUPPORTED_FEATURE;  // VP8L has no YUV planes
  const FrameDesc& d = b->desc[i];
  if (!set_device(b->ctx->device)) return WG_STATUS_INVALID_PARAM;
  hipError_t e = batch_wait(b);
  const int uw = (d.width + 1) / 2, uh = (d.height + 1) / 2;
  if (e == hipSuccess && y) e = hipMemcpy2D(y, d.width, d.y, d.y_stride, d.width, d.height, hipMemcpyDeviceToHost);
  if (e == hipSuccess && u) e = hipMemcpy2D(u, uw, d.u, d.uv_stride, uw, uh, hipMemcpyDeviceToHost);
  if (e == hipSuccess && v) e = hipMemcpy2D(v, uw, d.v, d.uv_stride, uw, uh, hipMemcpyDeviceToHost);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

}  // extern "C"

namespace {
// CheckDecBuffer's test of external YUV(A) memory (buffer_dec.c.go): every plane present, strides at
// least the plane widths, sizes at least stride * (h - 1) + width; the A plane only for MODE_YUVA.
bool yuva_out_ok(const wg_yuva_buffer* o, int w, int h, bool yuva) {
  if (!o || !o->y || !o->u || !o->v || (yuva && !o->a)) return false;
  const int uw = (w + 1) / 2, uh = (h + 1) / 2;
  auto fits = [](int stride, size_t size, int pw, int ph) {
    return stride >= pw && size >= (size_t)stride * (size_t)(ph - 1) + (size_t)pw;
  };
  return fits(o->y_stride, o->y_size, w, h) && fits(o->u_stride, o->u_size, uw, uh) &&
         fits(o->v_stride, o->v_size, uw, uh) && (!yuva || fits(o->a_stride, o->a_size, w, h));
}

// Queue frame i's planes (its slot of d_out, K8's output) to the caller's buffers on `s`.
hipError_t queue_yuva_download(wg_batch* b, int i, const wg_yuva_buffer* o, hipStream_t s) {
  const FrameParse& f = b->fp[(size_t)i];
  const int w = f.out_w, h = f.out_h, uw = (w + 1) / 2, uh = (h + 1) / 2;
  const uint8_t* base = b->d_out + b->off_out[(size_t)i];
  const uint8_t* py = base;
  const uint8_t* pu = py + (size_t)w * h;
  const uint8_t* pv = pu + (size_t)uw * uh;
  hipError_t e = hipMemcpy2DAsync(o->y, o->y_stride, py, w, w, h, hipMemcpyDefault, s);
  if (e == hipSuccess) e = hipMemcpy2DAsync(o->u, o->u_stride, pu, uw, uw, uh, hipMemcpyDefault, s);
  if (e == hipSuccess) e = hipMemcpy2DAsync(o->v, o->v_stride, pv, uw, uw, uh, hipMemcpyDefault, s);
  if (e == hipSuccess && b->yuva) e = hipMemcpy2DAsync(o->a, o->a_stride, pv + (size_t)uw * uh, w, w, h, hipMemcpyDefault, s);
  return e;
}
}  // namespace

extern "C" {

int wg_batch_download_yuva(wg_batch* b, int i, const wg_yuva_buffer* out) {
  if (!b || i < 0 || i >= b->n) return WG_STATUS_INVALID_PARAM;
  if (b->fp[(size_t)i].status != WG_STATUS_OK) return b->fp[(size_t)i].status;
  if (!b->yuv) return WG_STATUS_UNSUPPORTED_FEATURE;  // an RGB-family batch: wg_batch_download
  const FrameParse& f = b->fp[(size_t)i];
  if (!yuva_out_ok(out, f.out_w, f.out_h, b->yuva)) return WG_STATUS_INVALID_PARAM;
  int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  hipError_t e = queue_yuva_download(b, i, out, b->home);
  if (e == hipSuccess) e = hipStreamSynchronize(b->home);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_decode_yuv_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                        const wg_decoder_options* opt, const wg_yuva_buffer* outs, int32_t* status) {
  if (!ctx || !data || !sizes || !outs || !status || !opt || n <= 0 || (opt->colorspace != 11 && opt->colorspace != 12))
    return WG_STATUS_INVALID_PARAM;
  wg_batch* b = wg_batch_create_ex(ctx, data, sizes, n, opt, status);
  if (!b) return WG_STATUS_OUT_OF_MEMORY;
  int st = wg_batch_run(b, nullptr);
  if (st == WG_STATUS_OK) st = batch_sync(b);
  hipError_t e = hipSuccess;
  for (int i = 0; st == WG_STATUS_OK && i < n && e == hipSuccess; ++i) {
    if (status[i] != WG_STATUS_OK) continue;
    const FrameParse& f = b->fp[(size_t)i];
    if (!yuva_out_ok(&outs[i], f.out_w, f.out_h, b->yuva)) {
      status[i] = WG_STATUS_INVALID_PARAM;
      continue;
    }
    e = queue_yuva_download(b, i, &outs[i], b->home);
  }
  if (st == WG_STATUS_OK && (e != hipSuccess || hipStreamSynchronize(b->home) != hipSuccess)) st = WG_STATUS_USER_ABORT;
  wg_batch_destroy(b);
  return st;
}

int wg_decode_yuv_into(const uint8_t* data, size_t size, const wg_decoder_options* opt, const wg_yuva_buffer* out) {
  if (!data || !opt || !out || (opt->colorspace != 11 && opt->colorspace != 12)) return WG_STATUS_INVALID_PARAM;
  const std::shared_ptr<wg_ctx> ctx = default_ctx();  // held until this call returns
  if (!ctx) return WG_STATUS_UNSUPPORTED_FEATURE;    // no GPU: no CPU fallback by design
  const uint8_t* d[1] = {data};
  const size_t s[1] = {size};
  int32_t fs[1] = {0};
  const int st = wg_decode_yuv_batch(ctx.get(), d, s, 1, opt, out, fs);
  return st != WG_STATUS_OK ? st : fs[0];
}

int wg_decode_rgba_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                         uint8_t* const* rgba, const int32_t* strides, const size_t* caps, int32_t* status,
                         int32_t flags) {
  if (!ctx || !data || !sizes || !rgba || !strides || !caps || !status || n <= 0) return WG_STATUS_INVALID_PARAM;
  return guarded([&] { return decode_pipelined(ctx, data, sizes, n, rgba, strides, caps, status, flags); });
}

int wg_ctx_set_chunk_frames(wg_ctx* ctx, int frames) {
  if (!ctx || frames < 0) return WG_STATUS_INVALID_PARAM;
  std::lock_guard<std::mutex> lock(ctx->mu);
  ctx->chunk_frames = frames;
  return WG_STATUS_OK;
}

int wg_ctx_pipeline_stats(const wg_ctx* ctx, wg_pipeline_stats* out) {
  if (!ctx || !out) return WG_STATUS_INVALID_PARAM;
  std::lock_guard<std::mutex> lock(const_cast<wg_ctx*>(ctx)->mu);
  *out = ctx->stats;
  return WG_STATUS_OK;
}

void* wg_host_alloc(size_t bytes) { return bytes ? pinned_alloc(bytes) : nullptr; }
void wg_host_free(void* p) {
  if (p) pinned_free(p);
}

int wg_decode_rgba_batch_multi(wg_ctx* const* ctxs, int n_ctx, const uint8_t* const* data, const size_t* sizes,
                               int n, uint8_t* const* rgba, const int32_t* strides, const size_t* caps,
                               int32_t* status, int32_t flags) {
  if (!ctxs || n_ctx <= 0 || !data || !sizes || !rgba || !strides || !caps || !status || n <= 0)
    return WG_STATUS_INVALID_PARAM;
  for (int k = 0; k < n_ctx; ++k)
    if (!ctxs[k]) return WG_STATUS_INVALID_PARAM;
  const int shards = std::min(n_ctx, n);
  std::vector<int> rc((size_t)shards, WG_STATUS_OK);
  // contiguous shards, frames [k * n / shards, (k + 1) * n / shards) on context k
  auto run = [&](int k) {
    const int a = (int)((int64_t)k * n / shards), e = (int)((int64_t)(k + 1) * n / shards);
    rc[(size_t)k] = guarded([&] {
      return wg_decode_rgba_batch(ctxs[k], data + a, sizes + a, e - a, rgba + a, strides + a, caps + a, status + a,
                                  flags);
    });
  };
  std::vector<std::thread> th;
  for (int k = 1; k < shards; ++k) {
    try {
      th.emplace_back(run, k);
    } catch (const std::system_error&) {
      run(k);  // no thread: this shard on the calling thread
    }
  }
  run(0);
  for (auto& t : th) t.join();
  for (int r : rc)
    if (r != WG_STATUS_OK) return r;
  return WG_STATUS_OK;
}

int wg_decode_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n, const wg_decoder_options* opt,
                    uint8_t* const* out, const int32_t* strides, const size_t* caps, int32_t* status) {
  if (!ctx || !data || !sizes || !out || !strides || !caps || !status || !opt || n <= 0)
    return WG_STATUS_INVALID_PARAM;
  if (opt->colorspace == 11 || opt->colorspace == 12) return WG_STATUS_INVALID_PARAM;  // wg_decode_yuv_batch
  wg_batch* b = wg_batch_create_ex(ctx, data, sizes, n, opt, status);
  if (!b) return WG_STATUS_OUT_OF_MEMORY;
  int st = wg_batch_run(b, nullptr);
  const int bpp = wg::output_bpp(opt->colorspace);
  if (st == WG_STATUS_OK && b->k6) {  // K6 ran as the batch's last stage: copy each frame's slot out
    st = batch_sync(b);
    for (int i = 0; st == WG_STATUS_OK && i < n; ++i) {
      const FrameParse& f = b->fp[i];
      if (status[i] != WG_STATUS_OK) continue;
      if (!out_ok(out, strides, caps, i, bpp * f.out_w, f.out_h)) {
        status[i] = WG_STATUS_INVALID_PARAM;
        continue;
      }
      const size_t row = (size_t)bpp * f.out_w;
      if (hipMemcpy2D(out[i], strides[i], b->d_out + b->off_out[(size_t)i], row, row, f.out_h, hipMemcpyDefault) !=
          hipSuccess)
        status[i] = WG_STATUS_USER_ABORT;
    }
  } else if (st == WG_STATUS_OK) {
    st = download_rgba_all(b, out, strides, caps, status);
  }
  wg_batch_destroy(b);
  return st;
}

int wg_decode_into(const uint8_t* data, size_t size, const wg_decoder_options* opt, uint8_t* out, size_t cap,
                   int stride) {
  if (!data || !out || !opt) return WG_STATUS_INVALID_PARAM;
  if (opt->colorspace == 11 || opt->colorspace == 12) return WG_STATUS_INVALID_PARAM;  // wg_decode_yuv_into
  wg_features f{};
  int st = wg_get_features(data, size, &f);
  if (st != WG_STATUS_OK) return st;
  const int bpp = wg::output_bpp(opt->colorspace);
  int w = f.width, h = f.height;
  if (opt->use_cropping) {
    w = opt->crop_width;
    h = opt->crop_height;
  }
  if (bpp && w > 0 && h > 0 && (stride < bpp * w || (size_t)stride * (h - 1) + (size_t)bpp * w > cap))
    return WG_STATUS_INVALID_PARAM;
  const std::shared_ptr<wg_ctx> ctx = default_ctx();  // held until this call returns
  if (!ctx) return WG_STATUS_UNSUPPORTED_FEATURE;  // no GPU: no CPU fallback by design
  const uint8_t* d[1] = {data};
  const size_t s[1] = {size};
  uint8_t* o[1] = {out};
  const int32_t str[1] = {stride};
  const size_t caps[1] = {cap};
  int32_t fs[1] = {0};
  st = wg_decode_batch(ctx.get(), d, s, 1, opt, o, str, caps, fs);
  return st != WG_STATUS_OK ? st : fs[0];
}

int wg_decode_rgba_into(const uint8_t* data, size_t size, uint8_t* rgba, size_t cap, int stride, int flags) {
  if (!data || !rgba) return WG_STATUS_INVALID_PARAM;
  wg_features f{};
  int st = wg_get_features(data, size, &f);
  if (st != WG_STATUS_OK) return st;
  if (stride < 4 * f.width || (size_t)stride * (f.height - 1) + 4 * (size_t)f.width > cap)
    return WG_STATUS_INVALID_PARAM;
  const std::shared_ptr<wg_ctx> ctx = default_ctx();  // held until this call returns
  if (!ctx) return WG_STATUS_UNSUPPORTED_FEATURE;  // no GPU: no CPU fallback by design
  const uint8_t* d[1] = {data};
  const size_t s[1] = {size};
  uint8_t* o[1] = {rgba};
  const int32_t str[1] = {stride};
  const size_t caps[1] = {cap};
  int32_t fs[1] = {0};
  st = wg_decode_rgba_batch(ctx.get(), d, s, 1, o, str, caps, fs, flags);
  return st != WG_STATUS_OK ? st : fs[0];
}

int wg_anim_demux(const uint8_t* data, size_t size, wg_anim_info* info, wg_anim_frame* frames, int max_frames) {
  if (data == nullptr || info == nullptr) return WG_STATUS_INVALID_PARAM;
  wg::AnimInfo ai;
  std::vector<wg::AnimFrame> fr;
  std::memset(info, 0, sizeof(*info));
  const int st = wg::anim_demux(data, size, &ai, &fr);
  if (st != WG_STATUS_OK) return st;
  info->canvas_width = (uint32_t)ai.canvas_width;
  info->canvas_height = (uint32_t)ai.canvas_height;
  info->loop_count = (uint32_t)ai.loop_count;
  info->bgcolor = ai.bgcolor;
  info->frame_count = (uint32_t)ai.frame_count;
  for (int i = 0; frames && i < std::min(max_frames, ai.frame_count); ++i) {
    const wg::AnimFrame& f = fr[(size_t)i];
    wg_anim_frame& o = frames[i];
    o.x_offset = f.x_offset;
    o.y_offset = f.y_offset;
    o.width = f.width;
    o.height = f.height;
    o.duration = f.duration;
    o.dispose_background = f.dispose_bg;
    o.no_blend = f.no_blend;
    o.has_alpha = f.has_alpha;
    o.fragment_offset = f.off;
    o.fragment_size = f.size;
  }
  return WG_STATUS_OK;
}

wg_batch* wg_anim_batch_create(wg_ctx* ctx, const uint8_t* data, size_t size, int32_t flags, int32_t* status) {
  int32_t st_local = WG_STATUS_OK;
  int32_t& st_out = status ? *status : st_local;
  st_out = WG_STATUS_OK;
  if (!ctx || !data) {
    st_out = WG_STATUS_INVALID_PARAM;
    return nullptr;
  }
  wg::AnimInfo ai;
  std::vector<wg::AnimFrame> fr;
  int st = guarded([&] { return wg::anim_demux(data, size, &ai, &fr); });
  if (st == WG_STATUS_OK && ai.frame_count <= 0) st = WG_STATUS_BITSTREAM_ERROR;
  if (st != WG_STATUS_OK) {
    st_out = st;
    return nullptr;
  }
  const int n = ai.frame_count;
  // every frame's fragment decodes as one batch (K1..K4)
  std::vector<const uint8_t*> ptrs((size_t)n);
  std::vector<size_t> sizes((size_t)n);
  std::vector<int32_t> fst((size_t)n, 0);
  for (int i = 0; i < n; ++i) {
    ptrs[(size_t)i] = data + fr[(size_t)i].off;
    sizes[(size_t)i] = fr[(size_t)i].size;
  }
  wg_batch* b = wg_batch_create(ctx, ptrs.data(), sizes.data(), n, flags, fst.data());
  if (!b) {
    st_out = WG_STATUS_OUT_OF_MEMORY;
    for (int i = n - 1; i >= 0; --i)
      if (fst[(size_t)i] != WG_STATUS_OK) st_out = fst[(size_t)i];
    return nullptr;
  }
  for (int i = 0; i < n; ++i) {
    st = fst[(size_t)i];
    if (st == WG_STATUS_OK &&
        (b->desc[(size_t)i].width != fr[(size_t)i].width || b->desc[(size_t)i].height != fr[(size_t)i].height))
      st = WG_STATUS_BITSTREAM_ERROR;
    if (st != WG_STATUS_OK) {  // WebPAnimDecoder stops at the first frame that fails
      wg_batch_destroy(b);
      st_out = st;
      return nullptr;
    }
  }
  // frame descriptors: IsKeyFrame (anim_decode.go:183-197) and the blend / dispose flags
  b->fdesc.assign((size_t)n, AnimFrameDesc{});
  b->timestamps.assign((size_t)n, 0);
  int32_t t = 0;
  bool prev_key = false;
  double k5 = 0;
  auto full = [&](const wg::AnimFrame& f) { return f.width == ai.canvas_width && f.height == ai.canvas_height; };
  for (int i = 0; i < n; ++i) {
    const wg::AnimFrame& f = fr[(size_t)i];
    bool key;
    if (i == 0) key = true;
    else if ((!f.has_alpha || f.no_blend) && full(f)) key = true;
    else key = fr[(size_t)i - 1].dispose_bg && (full(fr[(size_t)i - 1]) || prev_key);
    AnimFrameDesc& d = b->fdesc[(size_t)i];
    d.rgba = b->desc[(size_t)i].rgba;
    d.x = f.x_offset;
    d.y = f.y_offset;
    d.width = f.width;
    d.height = f.height;
    d.key = key;
    d.blend = i > 0 && !f.no_blend && !key;
    d.dispose_bg = f.dispose_bg;
    if (i > 0) {
      const wg::AnimFrame& p = fr[(size_t)i - 1];
      d.prev_dispose_bg = p.dispose_bg;
      d.px = p.x_offset;
      d.py = p.y_offset;
      d.pw = p.width;
      d.ph = p.height;
    }
    prev_key = key;
    t += f.duration;
    b->timestamps[(size_t)i] = t;
    // K5's algorithmic bytes: the canvas written + the frame's rectangle read
    k5 += 4.0 * ai.canvas_width * (double)ai.canvas_height + 4.0 * f.width * (double)f.height;
  }
  b->canvas_w = ai.canvas_width;
  b->canvas_h = ai.canvas_height;
  b->kbytes[6] = k5;
  const size_t canvas_bytes = (size_t)ai.canvas_width * ai.canvas_height * 4;
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    hipError_t e = set_device(ctx->device) ? hipSuccess : hipErrorInvalidDevice;
    if (e == hipSuccess) {
      b->d_fdesc = static_cast<AnimFrameDesc*>(ctx->cache.get(sizeof(AnimFrameDesc) * (size_t)n));
      b->d_canvases = static_cast<uint8_t*>(ctx->cache.get(canvas_bytes * (size_t)n));
      if (!b->d_fdesc || !b->d_canvases) e = hipErrorOutOfMemory;
    }
    if (e == hipSuccess)
      e = hipMemcpyAsync(b->d_fdesc, b->fdesc.data(), sizeof(AnimFrameDesc) * (size_t)n, hipMemcpyHostToDevice,
                         b->home);
    if (e == hipSuccess) e = hipStreamSynchronize(b->home);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      wg_batch_destroy(b);
      st_out = e == hipErrorInvalidDevice ? WG_STATUS_INVALID_PARAM : WG_STATUS_OUT_OF_MEMORY;
      return nullptr;
    }
  }
  b->anim = true;
  return b;
}

int wg_anim_batch_info(const wg_batch* b, int32_t* canvas_width, int32_t* canvas_height, int32_t* frames) {
  if (!b || !b->anim) return WG_STATUS_INVALID_PARAM;
  if (canvas_width) *canvas_width = b->canvas_w;
  if (canvas_height) *canvas_height = b->canvas_h;
  if (frames) *frames = b->n;
  return WG_STATUS_OK;
}

int wg_anim_batch_download(wg_batch* b, uint8_t* canvases, size_t cap, int32_t* timestamps) {
  if (!b || !b->anim || !canvases) return WG_STATUS_INVALID_PARAM;
  const size_t bytes = (size_t)b->canvas_w * b->canvas_h * 4 * (size_t)b->n;
  if (cap < bytes) return WG_STATUS_INVALID_PARAM;
  const int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  if (hipMemcpy(canvases, b->d_canvases, bytes, hipMemcpyDefault) != hipSuccess) {
    (void)hipGetLastError();
    return WG_STATUS_USER_ABORT;
  }
  if (timestamps) std::memcpy(timestamps, b->timestamps.data(), sizeof(int32_t) * (size_t)b->n);
  return WG_STATUS_OK;
}

int wg_anim_decode(wg_ctx* ctx, const uint8_t* data, size_t size, uint8_t* canvases, int32_t* timestamps,
                   int32_t flags) {
  if (!ctx || !data || !canvases || !timestamps) return WG_STATUS_INVALID_PARAM;
  int32_t st = WG_STATUS_OK;
  wg_batch* b = wg_anim_batch_create(ctx, data, size, flags, &st);
  if (!b) return st;
  st = wg_batch_run(b, nullptr);
  if (st == WG_STATUS_OK)
    st = wg_anim_batch_download(b, canvases, (size_t)b->canvas_w * b->canvas_h * 4 * (size_t)b->n, timestamps);
  wg_batch_destroy(b);
  return st;
}

int wg_yuv420_to_rgba_device(const uint8_t* y, const uint8_t* u, const uint8_t* v, int y_stride, int uv_stride,
                             uint8_t* rgba, int rgba_stride, int width, int height, int fancy, void* stream) {
  if (!y || !u || !v || !rgba || width <= 0 || height <= 0 || rgba_stride < 4 * width ||
      y_stride < ((width + 15) & ~15) || uv_stride < ((((width + 1) >> 1) + 7) & ~7) || (y_stride & 15) ||
      (uv_stride & 3) || (reinterpret_cast<uintptr_t>(y) & 15) || (reinterpret_cast<uintptr_t>(u) & 3) ||
      (reinterpret_cast<uintptr_t>(v) & 3) ||
      (int64_t)rgba_stride * height > INT32_MAX)  // the emitter addresses the RGBA with 32-bit offsets
    return WG_STATUS_INVALID_PARAM;
  FrameDesc d{};
  d.y = const_cast<uint8_t*>(y);
  d.u = const_cast<uint8_t*>(u);
  d.v = const_cast<uint8_t*>(v);
  d.rgba = rgba;
  d.width = width;
  d.height = height;
  d.y_stride = y_stride;
  d.uv_stride = uv_stride;
  d.rgba_stride = rgba_stride;
  d.valid = 1;
  const hipError_t e = wg::launch_yuv_to_rgba(nullptr, &d, 1, width, height, fancy,
                                              reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_INVALID_PARAM;
}

int wg_vp8l_resolve_device(const uint32_t* tokens, const uint32_t* lits, int n_lits, int n_px, int cache_bits,
                           uint32_t* argb, void* stream) {
  if (!tokens || !argb || n_px < 0 || n_lits < 0 || (n_lits > 0 && !lits) || cache_bits < 0 || cache_bits > 11 ||
      (reinterpret_cast<uintptr_t>(tokens) & 15) || (reinterpret_cast<uintptr_t>(argb) & 15) ||
      n_px > (INT32_MAX >> 2) || n_lits > (INT32_MAX >> 2))  // (byte offsets are 32-bit)
    return WG_STATUS_INVALID_PARAM;
  if (n_px == 0) return WG_STATUS_OK;  // an empty stream: nothing to resolve
  wg::LLTokDesc t{};
  t.tokens = tokens;
  t.lits = lits;
  t.coded = argb;
  t.n_px = n_px;
  t.n_lits = n_lits;
  t.cache_bits = cache_bits;
  t.valid = 1;
  const hipError_t e = wg::launch_vp8l_resolve(nullptr, &t, 1, nullptr, reinterpret_cast<hipStream_t>(stream));
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_INVALID_PARAM;
}

}  // extern "C"

