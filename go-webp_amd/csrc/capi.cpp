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
#include <climits>
#include <new>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/gowebp_amd.h"
#include "device/kernels.h"
#include "device_format.h"
#include "host/host.h"

using wg::FrameDesc;
using wg::LLDesc;
using wg::AlphaDesc;
using wg::AnimFrameDesc;
using wg::MbRec;

struct wg_ctx {
  int device = 0;
  int host_threads = 1;
  hipStream_t stream = nullptr;
  std::mutex mu;
};

namespace {

constexpr size_t kAlign = 256;
inline size_t align_up(size_t v) { return (v + kAlign - 1) & ~(kAlign - 1); }

struct FrameParse {
  int status = WG_STATUS_OK;
  bool lossless = false;
  wg::SparseFrame sf;  // lossy
  wg::VP8LFrame lf;    // lossless
  size_t off_recs = 0, off_rows = 0, off_blocks = 0;  // within the input buffer (lossy)
  size_t off_coded = 0, off_tdata[4] = {0, 0, 0, 0};  // within the input buffer (lossless)
  size_t off_y = 0, off_u = 0, off_v = 0;            // within the plane buffer
  size_t off_cols = 0;                                // K1 global column store (wide frames)
  bool wide = false;                                  // mb_w > vp8_recon_max_mb_w()
  size_t off_scratch = 0;                             // lossless two-pass scratch (plane buffer)
  size_t off_rgba = 0;                                // within the RGBA buffer
  int width = 0, height = 0;
  // ALPH plane of a lossy frame (f2): raw bytes, or a lossless stream K3 decodes
  bool alpha = false;
  wg::AlphaHeader ah;
  wg::VP8LFrame af;
  const uint8_t* alpha_raw = nullptr;  // into the caller's input (valid during batch creation)
  size_t off_araw = 0, off_acoded = 0, off_atdata[4] = {0, 0, 0, 0};  // input buffer
  size_t off_ascratch = 0, off_argba = 0, off_aplane = 0;            // plane buffer
  // output (cropping, f4): out_w x out_h, taken at (win_x, win_y) of the frame's RGBA buffer
  // (rgba_w x rgba_h: the window itself for lossy frames, the whole frame for lossless)
  int out_w = 0, out_h = 0, win_x = 0, win_y = 0, rgba_w = 0, rgba_h = 0;
  bool cropped = false;
  size_t off_yc = 0, off_uc = 0, off_vc = 0;  // cropped lossy planes (plane buffer)
  int yc_stride = 0, uvc_stride = 0;
};

struct Timing {
  hipEvent_t ev[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  bool ran[4] = {false, false, false, false};  // K1, K2, K3, K4 launched in this run
};

// Does the lossless frame need a second pass (predictor and color indexing both present)?
bool ll_two_pass(const wg::VP8LFrame& f) {
  int cores = 0;
  for (const auto& t : f.transforms) cores += (t.type == wg::kVP8LPredictor || t.type == wg::kVP8LColorIndexing);
  return cores > 1;
}

// Allocation failure anywhere in the host stages (vectors sized by the bitstream) is
// reported as WebPDecode does, never thrown across the C ABI or out of a parse thread.
template <class F>
int guarded(F&& f) {
  try {
    return f();
  } catch (const std::bad_alloc&) {
    return WG_STATUS_OUT_OF_MEMORY;
  }
}

constexpr int kFilterExtraRows[3] = {0, 2, 8};  // frame_dec.c.go (VP8EnterCritical)

// Output options (WebPIoInitFromOptions / WebPAllocateDecBuffer, webp.go): colorspace,
// scaling (disabled in the reference, io_dec.c.go:540-541), cropping (WebPCheckCropDimensions
// -> INVALID_PARAM).  Sets the frame's output window.
int apply_output_options(const wg_decoder_options& opt, FrameParse* f) {
  if (!wg::output_bpp(opt.colorspace))
    return (opt.colorspace == 11 || opt.colorspace == 12) ? WG_STATUS_UNSUPPORTED_FEATURE : WG_STATUS_INVALID_PARAM;
  if (opt.use_scaling) return WG_STATUS_UNSUPPORTED_FEATURE;
  f->out_w = f->width;
  f->out_h = f->height;
  if (opt.use_cropping) {
    // WebPAllocateDecBuffer checks the window with its origin snapped to even
    // (buffer_dec.c.go:201-209); the decoder's window (WebPIoInitFromOptions, webp.go:922-945)
    // snaps only for YUV sources: lossy frames use the snapped origin, lossless the exact one
    const int cw = opt.crop_width, ch = opt.crop_height;
    auto inside = [&](int x, int y) {
      return x >= 0 && y >= 0 && cw > 0 && ch > 0 && x < f->width && y < f->height && cw <= f->width - x &&
             ch <= f->height - y;
    };
    const int x = f->lossless ? opt.crop_left : (opt.crop_left & ~1);
    const int y = f->lossless ? opt.crop_top : (opt.crop_top & ~1);
    if (!inside(opt.crop_left & ~1, opt.crop_top & ~1) || !inside(x, y)) return WG_STATUS_INVALID_PARAM;
    f->cropped = x != 0 || y != 0 || cw != f->width || ch != f->height;
    f->out_w = cw;
    f->out_h = ch;
    f->win_x = f->lossless ? x : 0;  // lossy: K2 writes the window itself
    f->win_y = f->lossless ? y : 0;
  }
  f->rgba_w = f->lossless ? f->width : f->out_w;
  f->rgba_h = f->lossless ? f->height : f->out_h;
  return WG_STATUS_OK;
}

// The MB row at whose FinishRow libwebp's lazy alpha decode fails, INT_MAX if never.
// FinishRow(m) (frame_dec.c.go) requests alpha rows [y_start, y_end): 16m minus the filter
// delay, the last parsed row (m = rows - 1) through its bottom, clamped to the crop bottom;
// the first request runs ALPHInit (header + lossless stream header), pre-processed
// (quantized) alpha is decoded whole at that first request (VP8DecompressAlphaRows).  A
// lossless pixel failure is hit once the requested rows reach it.
int alpha_fail_row(int rows, int extra, int bottom, bool init_fails, size_t fail_pixel, int coded_width,
                   bool whole_plane) {
  for (int m = 0; m < rows; ++m) {
    const int y_start = m ? 16 * m - extra : 0;
    const int y_end = std::min(m == rows - 1 ? 16 * (m + 1) : 16 * (m + 1) - extra, bottom);
    if (y_start >= y_end) continue;
    if (init_fails) return m;
    const uint64_t last = (uint64_t)(whole_plane ? bottom : y_end);
    if (last * (uint64_t)coded_width > (uint64_t)fail_pixel) return m;
    if (whole_plane) break;
  }
  return INT_MAX;
}

// One frame's host stages and its WebPDecode status, in DecodeInto's order (webp.go:483-556):
// container, bitstream headers, output options, then the image data -- bounded, like
// libwebp's, to the rows a crop window needs, with a lossy frame's ALPH data decoded
// lazily per MB row (its failure wins over a token failure further down).
int parse_one(const uint8_t* data, size_t size, const wg_decoder_options& opt, FrameParse* fp) {
  wg::Container c;
  wg_features feat{};
  // WebPDecode first runs GetFeatures; its NOT_ENOUGH_DATA is "treated as error"
  int st = wg::parse_container(data, size, &c, &feat, /*have_all_data=*/false);
  if (st != WG_STATUS_OK) return st == WG_STATUS_NOT_ENOUGH_DATA ? WG_STATUS_BITSTREAM_ERROR : st;
  st = wg::parse_container(data, size, &c, &feat);  // DecodeInto's WebPParseHeaders
  if (st != WG_STATUS_OK) return st;
  if (c.is_lossless) {  // VP8L: host entropy stage, K3 on device
    fp->lossless = true;
    st = wg::vp8l_parse(data + c.payload_off, c.payload_size, &fp->lf);
    if (st != WG_STATUS_OK && fp->lf.fail_pixel == SIZE_MAX) return st;  // VP8LDecodeHeader
    fp->width = fp->lf.width;
    fp->height = fp->lf.height;
    const int ost = apply_output_options(opt, fp);
    if (ost != WG_STATUS_OK) return ost;
    if (st != WG_STATUS_OK) {  // DecodeImageData stops at the crop bottom (io->crop_bottom)
      const int bottom = opt.use_cropping ? opt.crop_top + opt.crop_height : fp->height;
      if ((uint64_t)bottom * (uint64_t)fp->lf.coded_width > (uint64_t)fp->lf.fail_pixel) return st;
    }
    return WG_STATUS_OK;
  }
  const int flags = opt.bypass_filtering ? WG_FLAG_BYPASS_FILTERING : 0;
  const int crop_bottom = opt.use_cropping ? (opt.crop_top & ~1) + opt.crop_height : -1;
  st = wg::vp8_parse(data, size, flags, nullptr, nullptr, &fp->sf, crop_bottom);
  if (st != WG_STATUS_OK && fp->sf.fail_row < 0) return st;  // VP8GetHeaders
  fp->width = fp->sf.info.width;
  fp->height = fp->sf.info.height;
  const int ost = apply_output_options(opt, fp);
  if (ost != WG_STATUS_OK) return ost;
  if (c.alpha_size > 0) {  // ALPH (VP8DecompressAlphaRows, alpha_dec.go:164-213)
    const uint8_t* ad = data + c.alpha_off;
    fp->alpha = true;
    int ast = WG_STATUS_OK;
    bool init_fails = false;
    if (!wg::parse_alpha_header(ad, c.alpha_size, fp->width, fp->height, &fp->ah)) {
      ast = WG_STATUS_OUT_OF_MEMORY;  // ALPHInit failure without a VP8L decoder
      init_fails = true;
    } else if (fp->ah.method == 1) {
      ast = wg::vp8l_parse_alpha(ad + 1, c.alpha_size - 1, fp->width, fp->height, &fp->af);
      init_fails = ast == WG_STATUS_OUT_OF_MEMORY;
    } else {
      fp->alpha_raw = ad + 1;
    }
    if (ast != WG_STATUS_OK) {
      const int bottom = crop_bottom >= 0 ? crop_bottom : fp->height;
      const int arow = alpha_fail_row(fp->sf.br_mb_y, kFilterExtraRows[fp->sf.info.filter_type], bottom, init_fails,
                                      fp->af.fail_pixel, fp->af.coded_width, fp->ah.pre_processing == 1);
      if (arow < (st != WG_STATUS_OK ? fp->sf.fail_row : INT_MAX)) return ast;
    }
  }
  return st;
}

void parse_all(const uint8_t* const* data, const size_t* sizes, int n, const wg_decoder_options& opt, int threads,
               std::vector<FrameParse>& out) {
  out.resize(n);
  std::atomic<int> next{0};
  auto work = [&]() {
    for (;;) {
      const int i = next.fetch_add(1);
      if (i >= n) break;
      if (data[i] == nullptr) {
        out[i].status = WG_STATUS_INVALID_PARAM;
        continue;
      }
      out[i].status = guarded([&] { return parse_one(data[i], sizes[i], opt, &out[i]); });
      if (out[i].status != WG_STATUS_OK) out[i] = FrameParse{out[i].status};  // drop partial host data
    }
  };
  const int t = std::max(1, std::min(threads, n));
  if (t == 1) {
    work();
  } else {
    std::vector<std::thread> pool;
    for (int k = 0; k < t; ++k) pool.emplace_back(work);
    for (auto& th : pool) th.join();
  }
}

}  // namespace

struct wg_batch {
  wg_ctx* ctx = nullptr;
  int n = 0;
  int flags = 0;
  std::vector<FrameParse> fp;
  std::vector<FrameDesc> desc;
  std::vector<LLDesc> lldesc;     // lossless frames and lossless alpha streams (K3)
  std::vector<AlphaDesc> adesc;   // alpha planes (K4)
  FrameDesc* d_desc = nullptr;
  LLDesc* d_lldesc = nullptr;
  AlphaDesc* d_adesc = nullptr;
  int n_lossy = 0, n_lossless = 0, n_alpha = 0, n_k3 = 0;
  wg_decoder_options opt{};          // output colorspace, cropping, flip (f4)
  bool any_crop = false;             // K2 reads compact cropped planes through desc2
  bool fused = false;                // lossy RGBA emitted by K1's tail (wg::kFrameEmitRgba), no K2 launch
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
  int n_valid = 0;
  int64_t pixels = 0;
  double kbytes[4] = {0, 0, 0, 0};
  double k1_fused_bytes = 0;  // K1 with its RGBA tail: inputs + RGBA (planes are an intermediate)
  std::vector<Timing> timings;  // one per run since the last query
  size_t n_runs_pending = 0;
};

namespace {
void fill_vp8l_info(const wg::VP8LFrame& f, wg_vp8l_info* info, uint32_t* argb, uint32_t* const* transform_data);
// The single-frame entry points share one lazily created context on device 0.
wg_ctx* default_ctx() {
  static std::mutex mu;
  static wg_ctx* ctx = nullptr;
  std::lock_guard<std::mutex> lock(mu);
  if (!ctx) ctx = wg_ctx_create(0, 1);
  return ctx;
}
}  // namespace

extern "C" {

int wg_version(void) { return 0x000100; }

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
  return guarded([&] { return wg::vp8_parse(data, size, flags, info, mbs, nullptr); });
}

int wg_decode_status(const uint8_t* data, size_t size, const wg_decoder_options* opt) {
  if (data == nullptr) return WG_STATUS_INVALID_PARAM;
  wg_decoder_options o{};
  o.colorspace = 1;  // MODE_RGBA
  if (opt) o = *opt;
  return guarded([&] {
    FrameParse fp;
    return parse_one(data, size, o, &fp);
  });
}

int wg_vp8l_parse(const uint8_t* data, size_t size, wg_vp8l_info* info, uint32_t* argb,
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
    fill_vp8l_info(f, info, argb, transform_data);
    return (int)WG_STATUS_OK;
  });
}

int wg_alpha_parse(const uint8_t* data, size_t size, wg_alpha_info* info, uint8_t* filtered,
                   wg_vp8l_info* ll_info, uint32_t* argb, uint32_t* const* transform_data) {
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
    if (ll_info) fill_vp8l_info(f, ll_info, argb, transform_data);
    return (int)WG_STATUS_OK;
  });
}

}  // extern "C"

namespace {
void fill_vp8l_info(const wg::VP8LFrame& f, wg_vp8l_info* info, uint32_t* argb, uint32_t* const* transform_data) {
  std::memset(info, 0, sizeof(*info));
  info->width = f.width;
  info->height = f.height;
  info->has_alpha = f.has_alpha;
  info->coded_width = f.coded_width;
  info->num_transforms = (int32_t)f.transforms.size();
  for (size_t i = 0; i < f.transforms.size(); ++i) {
    info->transform_type[i] = f.transforms[i].type;
    info->transform_bits[i] = f.transforms[i].bits;
    info->transform_xsize[i] = f.transforms[i].xsize;
    info->transform_size[i] = (int32_t)f.transforms[i].data.size();
    if (transform_data && transform_data[i] && !f.transforms[i].data.empty())
      std::memcpy(transform_data[i], f.transforms[i].data.data(), f.transforms[i].data.size() * 4);
  }
  if (argb) std::memcpy(argb, f.argb.data(), f.argb.size() * 4);
}
}  // namespace

namespace {
wg_batch* batch_create(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                       const wg_decoder_options* opt, int32_t* status);
}

extern "C" {

wg_ctx* wg_ctx_create(int device, int host_threads) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
  if (hipSetDevice(device) != hipSuccess) return nullptr;
  wg_ctx* c = new wg_ctx();
  c->device = device;
  c->host_threads = host_threads > 0 ? host_threads : (int)std::max(1u, std::thread::hardware_concurrency());
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return nullptr;
  }
  return c;
}

void wg_ctx_destroy(wg_ctx* c) {
  if (!c) return;
  hipSetDevice(c->device);
  if (c->stream) hipStreamDestroy(c->stream);
  delete c;
}

void wg_batch_destroy(wg_batch* b) {
  if (!b) return;
  hipSetDevice(b->ctx->device);
  hipStreamSynchronize(b->ctx->stream);
  for (auto& t : b->timings)
    for (auto& e : t.ev)
      if (e) hipEventDestroy(e);
  if (b->d_desc) hipFree(b->d_desc);
  if (b->d_lldesc) hipFree(b->d_lldesc);
  if (b->d_adesc) hipFree(b->d_adesc);
  if (b->d_desc2) hipFree(b->d_desc2);
  if (b->d_err) hipFree(b->d_err);
  if (b->d_in) hipFree(b->d_in);
  if (b->d_planes) hipFree(b->d_planes);
  if (b->d_rgba) hipFree(b->d_rgba);
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
  } catch (const std::bad_alloc&) {  // host-side layout / descriptor vectors
    if (status)
      for (int i = 0; i < n; ++i)
        if (status[i] == WG_STATUS_OK) status[i] = WG_STATUS_OUT_OF_MEMORY;
    return nullptr;
  }
}

}  // extern "C"

namespace {
wg_batch* batch_create(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                       const wg_decoder_options* opt, int32_t* status) {
  if (status)
    for (int i = 0; i < n; ++i) status[i] = WG_STATUS_OK;
  std::lock_guard<std::mutex> lock(ctx->mu);
  if (hipSetDevice(ctx->device) != hipSuccess) return nullptr;
  wg_batch* b = new wg_batch();
  b->ctx = ctx;
  b->n = n;
  b->opt = *opt;
  const int32_t flags = (opt->bypass_filtering ? WG_FLAG_BYPASS_FILTERING : 0) |
                        (opt->no_fancy_upsampling ? WG_FLAG_NO_FANCY_UPSAMPLING : 0);
  b->flags = flags;
  parse_all(data, sizes, n, *opt, ctx->host_threads, b->fp);
  // layout
  size_t in_b = 0, pl_b = 0, rg_b = 0;
  double k1 = 0, k2 = 0, k3 = 0, k4 = 0;
  // K3 input (coded image + transform data) and two-pass scratch of one lossless stream;
  // returns its algorithmic bytes (reads + RGBA write)
  auto layout_ll = [&](const wg::VP8LFrame& lf, int w, int h, size_t* off_coded, size_t* off_tdata,
                       size_t* off_scratch) {
    const double px = (double)w * h;
    *off_coded = in_b;
    in_b = align_up(in_b + lf.argb.size() * 4);
    double bytes = lf.argb.size() * 4.0 + 4.0 * px;
    for (size_t t = 0; t < lf.transforms.size(); ++t) {
      off_tdata[t] = in_b;
      in_b = align_up(in_b + std::max<size_t>(lf.transforms[t].data.size(), 1) * 4);
      bytes += lf.transforms[t].data.size() * 4.0;
    }
    if (ll_two_pass(lf)) {
      *off_scratch = pl_b;
      pl_b = align_up(pl_b + (size_t)w * h * 4);
      bytes += 8.0 * px;
    }
    return bytes;
  };
  for (int i = 0; i < n; ++i) {
    FrameParse& f = b->fp[i];
    if (status) status[i] = f.status;
    if (f.status != WG_STATUS_OK) continue;
    f.off_rgba = rg_b;
    rg_b = align_up(rg_b + (size_t)f.rgba_w * f.rgba_h * 4);
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
      k3 += layout_ll(f.lf, f.width, f.height, &f.off_coded, f.off_tdata, &f.off_scratch);
      continue;
    }
    b->n_lossy++;
    const wg_vp8_info& inf = f.sf.info;
    const size_t nmb = (size_t)inf.mb_w * inf.mb_h;
    f.off_recs = in_b;
    in_b = align_up(in_b + nmb * sizeof(MbRec));
    f.off_rows = in_b;
    in_b = align_up(in_b + (size_t)inf.mb_h * 4);
    f.off_blocks = in_b;
    in_b = align_up(in_b + f.sf.blocks.size() * 2);
    f.off_y = pl_b;
    pl_b = align_up(pl_b + nmb * 256);
    f.off_u = pl_b;
    pl_b = align_up(pl_b + nmb * 64);
    f.off_v = pl_b;
    pl_b = align_up(pl_b + nmb * 64);
    f.wide = inf.mb_w > wg::vp8_recon_max_mb_w();
    if (f.wide) {
      b->n_wide++;
      f.off_cols = pl_b;
      pl_b = align_up(pl_b + (size_t)inf.mb_w * 160);
    } else {
      b->max_mb_w = std::max(b->max_mb_w, inf.mb_w);
    }
    if (f.cropped) {  // K2 reads the crop window from compact planes (copied after K1)
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
    // algorithmic bytes: K1 reads records + coefficients, writes MB-padded
    // planes; K2 reads cropped planes, writes RGBA.
    const double uvpx = 2.0 * ((inf.width + 1) / 2) * (double)((inf.height + 1) / 2);
    k1 += (double)nmb * sizeof(MbRec) + inf.mb_h * 4.0 + f.sf.blocks.size() * 2.0 + nmb * 384.0;
    b->k1_fused_bytes += (double)nmb * sizeof(MbRec) + inf.mb_h * 4.0 + f.sf.blocks.size() * 2.0 +
                         4.0 * inf.width * (double)inf.height;
    const double opx = (double)f.out_w * f.out_h;
    k2 += opx + 2.0 * ((f.out_w + 1) / 2) * (double)((f.out_h + 1) / 2) + 4.0 * opx;
    (void)uvpx;
    if (f.alpha) {
      // K4 reads the filtered alpha (raw bytes, or K3's RGBA of the alpha stream) and
      // rewrites the RGBA A bytes (dword read-modify-write)
      b->n_alpha++;
      if (f.ah.method == 1) {
        b->n_k3++;
        k3 += layout_ll(f.af, f.width, f.height, &f.off_acoded, f.off_atdata, &f.off_ascratch);
        f.off_argba = pl_b;
        pl_b = align_up(pl_b + (size_t)f.width * f.height * 4);
        k4 += 4.0 * px;
      } else {
        f.off_araw = in_b;
        in_b = align_up(in_b + (size_t)f.width * f.height);
        k4 += px;
      }
      f.off_aplane = pl_b;
      pl_b = align_up(pl_b + (size_t)f.width * f.height);
      k4 += 8.0 * px;
    }
  }
  b->kbytes[3] = k4;
  b->kbytes[2] = k3;
  b->kbytes[0] = k1;
  b->kbytes[1] = k2;
  b->in_bytes = std::max<size_t>(in_b, kAlign);
  b->plane_bytes = std::max<size_t>(pl_b, kAlign);
  b->rgba_bytes = std::max<size_t>(rg_b, kAlign);
  auto fail = [&](int st) {
    if (status)
      for (int i = 0; i < n; ++i)
        if (status[i] == WG_STATUS_OK) status[i] = st;
    wg_batch_destroy(b);
    return (wg_batch*)nullptr;
  };
  if (hipMalloc(&b->d_in, b->in_bytes) != hipSuccess || hipMalloc(&b->d_planes, b->plane_bytes) != hipSuccess ||
      hipMalloc(&b->d_rgba, b->rgba_bytes) != hipSuccess ||
      hipMalloc(&b->d_desc, sizeof(FrameDesc) * (size_t)n) != hipSuccess ||
      hipMalloc(&b->d_lldesc, sizeof(LLDesc) * (size_t)std::max(b->n_k3, 1)) != hipSuccess ||
      hipMalloc(&b->d_adesc, sizeof(AlphaDesc) * (size_t)std::max(b->n_alpha, 1)) != hipSuccess ||
      hipMalloc(&b->d_err, sizeof(int)) != hipSuccess || hipMemset(b->d_err, 0, sizeof(int)) != hipSuccess)
    return fail(WG_STATUS_OUT_OF_MEMORY);
  // stage inputs in pinned memory, one H2D copy
  uint8_t* h_in = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&h_in), b->in_bytes, hipHostMallocDefault) != hipSuccess)
    return fail(WG_STATUS_OUT_OF_MEMORY);
  // Staging copies are collected first and run on the host threads afterwards (the
  // parsed data they read is released only after that).
  struct CopyJob {
    uint8_t* dst;
    const void* src;
    size_t n;
  };
  std::vector<CopyJob> jobs;
  auto stage = [&](size_t off, const void* src, size_t nbytes) {
    if (nbytes) jobs.push_back(CopyJob{h_in + off, src, nbytes});
  };
  // the LLDesc of one lossless stream (transforms in application order = reverse of read
  // order); its coded image and transform data go to the staging buffer
  auto make_ll = [&](wg::VP8LFrame& lf, int w, int h, size_t off_coded, const size_t* off_tdata,
                     size_t off_scratch, uint8_t* rgba, int stride) {
    LLDesc l{};
    stage(off_coded, lf.argb.data(), lf.argb.size() * 4);
    l.coded = reinterpret_cast<const uint32_t*>(b->d_in + off_coded);
    l.coded_bytes = (int32_t)(lf.argb.size() * 4);
    l.scratch = ll_two_pass(lf) ? reinterpret_cast<uint32_t*>(b->d_planes + off_scratch) : nullptr;
    l.scratch_bytes = l.scratch ? w * h * 4 : 0;
    l.rgba = rgba;
    l.rgba_stride = stride;
    l.width = w;
    l.height = h;
    l.coded_width = lf.coded_width;
    l.n_stages = (int32_t)lf.transforms.size();
    int types[4], bits[4], tiles[4];
    for (int t = 0; t < l.n_stages; ++t) {
      const wg::VP8LTransform& tr = lf.transforms[(size_t)(l.n_stages - 1 - t)];
      const size_t off = off_tdata[l.n_stages - 1 - t];
      stage(off, tr.data.data(), tr.data.size() * 4);
      wg::LLStage& st = l.stages[t];
      st.type = tr.type;
      st.bits = tr.bits;
      st.xsize = tr.xsize;
      st.tiles_per_row = (tr.type == wg::kVP8LPredictor || tr.type == wg::kVP8LCrossColor)
                             ? (tr.xsize + (1 << tr.bits) - 1) >> tr.bits
                             : 0;
      st.data = reinterpret_cast<const uint32_t*>(b->d_in + off);
      types[t] = st.type;
      bits[t] = st.bits;
      tiles[t] = st.tiles_per_row ? st.tiles_per_row * ((h + (1 << st.bits) - 1) >> st.bits) : 0;
    }
    l.valid = 1;
    l.pad1[0] = (uint64_t)wg::vp8l_variant(types, bits, tiles, l.n_stages);  // sort key
    return l;
  };
  b->desc.assign(n, FrameDesc{});
  for (int i = 0; i < n; ++i) {
    FrameParse& f = b->fp[i];
    FrameDesc& d = b->desc[i];
    if (f.status != WG_STATUS_OK) continue;
    d.rgba = b->d_rgba + f.off_rgba;
    d.width = f.width;
    d.height = f.height;
    d.rgba_stride = 4 * f.rgba_w;
    if (f.lossless) {  // K1/K2 skip it (valid = 0); K3 gets an LLDesc
      b->lldesc.push_back(make_ll(f.lf, f.width, f.height, f.off_coded, f.off_tdata, f.off_scratch, d.rgba,
                                  d.rgba_stride));
      continue;
    }
    const wg_vp8_info& inf = f.sf.info;
    stage(f.off_recs, f.sf.mbs.data(), f.sf.mbs.size() * sizeof(MbRec));
    stage(f.off_rows, f.sf.row_block0.data(), f.sf.row_block0.size() * 4);
    stage(f.off_blocks, f.sf.blocks.data(), f.sf.blocks.size() * 2);
    d.mbs = reinterpret_cast<const MbRec*>(b->d_in + f.off_recs);
    d.row_block0 = reinterpret_cast<const uint32_t*>(b->d_in + f.off_rows);
    d.blocks = reinterpret_cast<const int16_t*>(b->d_in + f.off_blocks);
    d.blocks_bytes = (int32_t)(f.sf.blocks.size() * 2);
    d.y = b->d_planes + f.off_y;
    d.cols = f.wide ? b->d_planes + f.off_cols : nullptr;
    d.u = b->d_planes + f.off_u;
    d.v = b->d_planes + f.off_v;
    d.mb_w = inf.mb_w;
    d.mb_h = inf.mb_h;
    d.y_stride = 16 * inf.mb_w;
    d.uv_stride = 8 * inf.mb_w;
    d.filter_type = inf.filter_type;
    d.flags = flags;
    d.valid = 1;
    if (f.alpha) {
      AlphaDesc a{};
      if (f.ah.method == 1) {
        b->lldesc.push_back(make_ll(f.af, f.width, f.height, f.off_acoded, f.off_atdata, f.off_ascratch,
                                    b->d_planes + f.off_argba, 4 * f.width));
        a.green = b->d_planes + f.off_argba;
      } else {
        stage(f.off_araw, f.alpha_raw, (size_t)f.width * f.height);
        a.raw = b->d_in + f.off_araw;
      }
      a.plane = b->d_planes + f.off_aplane;
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
  // run the staging copies on the host threads (large ones split into 4 MB pieces)
  {
    constexpr size_t kPiece = size_t(4) << 20;
    std::vector<CopyJob> pieces;
    for (const CopyJob& j : jobs)
      for (size_t o = 0; o < j.n; o += kPiece)
        pieces.push_back(CopyJob{j.dst + o, static_cast<const uint8_t*>(j.src) + o, std::min(kPiece, j.n - o)});
    std::atomic<size_t> next{0};
    auto work = [&]() {
      for (size_t k; (k = next.fetch_add(1)) < pieces.size();) std::memcpy(pieces[k].dst, pieces[k].src, pieces[k].n);
    };
    const int t = (int)std::max<size_t>(1, std::min<size_t>((size_t)ctx->host_threads, pieces.size()));
    std::vector<std::thread> pool;
    for (int k = 1; k < t; ++k) pool.emplace_back(work);
    work();
    for (auto& th : pool) th.join();
  }
  // release host-side copies of the parsed data: the device owns them now
  for (int i = 0; i < n; ++i) {
    FrameParse& f = b->fp[i];
    std::vector<MbRec>().swap(f.sf.mbs);
    f.sf.blocks.release();
    std::vector<uint32_t>().swap(f.sf.row_block0);
    wg::VP8LFrame().transforms.swap(f.lf.transforms);
    std::vector<uint32_t>().swap(f.lf.argb);
    wg::VP8LFrame().transforms.swap(f.af.transforms);
    std::vector<uint32_t>().swap(f.af.argb);
    f.alpha_raw = nullptr;
  }
  // Full-frame RGBA (no crop window anywhere in the batch): K1 converts each frame in its
  // own tail instead of a separate K2 launch (wg_batch_set_emit() switches back).
  b->fused = !b->any_crop;
  if (b->fused)
    for (int i = 0; i < n; ++i)
      if (b->desc[i].valid) b->desc[i].flags |= wg::kFrameEmitRgba;
  if (b->any_crop) {  // K2's view: cropped lossy frames read their compact planes
    b->desc2 = b->desc;
    for (int i = 0; i < n; ++i) {
      FrameParse& f = b->fp[i];
      FrameDesc& d2 = b->desc2[i];
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
  hipError_t e = hipMemcpyAsync(b->d_in, h_in, b->in_bytes, hipMemcpyHostToDevice, ctx->stream);
  if (e == hipSuccess && b->any_crop) {
    e = hipMalloc(&b->d_desc2, sizeof(FrameDesc) * (size_t)n);
    if (e == hipSuccess)
      e = hipMemcpyAsync(b->d_desc2, b->desc2.data(), sizeof(FrameDesc) * (size_t)n, hipMemcpyHostToDevice,
                         ctx->stream);
  }
  if (e == hipSuccess)
    e = hipMemcpyAsync(b->d_desc, b->desc.data(), sizeof(FrameDesc) * (size_t)n, hipMemcpyHostToDevice,
                       ctx->stream);
  // K3 launches one kernel per variant over a contiguous group of descriptors
  std::stable_sort(b->lldesc.begin(), b->lldesc.end(),
                   [](const LLDesc& a, const LLDesc& c) { return a.pad1[0] < c.pad1[0]; });
  for (const LLDesc& l : b->lldesc) b->ll_groups[l.pad1[0]]++;
  if (e == hipSuccess && !b->lldesc.empty())
    e = hipMemcpyAsync(b->d_lldesc, b->lldesc.data(), sizeof(LLDesc) * b->lldesc.size(), hipMemcpyHostToDevice,
                       ctx->stream);
  if (e == hipSuccess && !b->adesc.empty())
    e = hipMemcpyAsync(b->d_adesc, b->adesc.data(), sizeof(AlphaDesc) * b->adesc.size(), hipMemcpyHostToDevice,
                       ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
  hipHostFree(h_in);
  if (e != hipSuccess) return fail(WG_STATUS_OUT_OF_MEMORY);
  return b;
}
}  // namespace

extern "C" {

int wg_batch_run(wg_batch* b, void* stream) {
  if (!b) return WG_STATUS_INVALID_PARAM;
  if (b->n_valid == 0) return WG_STATUS_OK;
  hipSetDevice(b->ctx->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : b->ctx->stream;
  if (b->n_runs_pending >= b->timings.size()) {
    Timing t;
    for (auto& e : t.ev)
      if (hipEventCreate(&e) != hipSuccess) return WG_STATUS_OUT_OF_MEMORY;
    b->timings.push_back(t);
  }
  Timing& t = b->timings[b->n_runs_pending++];
  t.ran[0] = b->n_lossy > 0;
  t.ran[1] = b->n_lossy > 0 && !b->fused;
  t.ran[2] = b->n_k3 > 0;
  t.ran[3] = b->n_alpha > 0;
  hipEventRecord(t.ev[0], s);
  if (b->n_lossy > 0) {
    hipError_t e = wg::launch_vp8_recon_filter(b->d_desc, b->n, b->max_mb_w, b->n_lossy > b->n_wide,
                                               b->n_wide > 0, b->d_err, s);
    if (e != hipSuccess) return WG_STATUS_UNSUPPORTED_FEATURE;
  }
  hipEventRecord(t.ev[1], s);
  if (t.ran[1]) {
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
        hipError_t e = hipMemcpy2DAsync(d2.y, d2.y_stride, d.y + (size_t)y * d.y_stride + x, d.y_stride, f.out_w,
                                        f.out_h, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
          e = hipMemcpy2DAsync(d2.u, d2.uv_stride, d.u + (size_t)(y >> 1) * d.uv_stride + (x >> 1), d.uv_stride, uw,
                               uh, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
          e = hipMemcpy2DAsync(d2.v, d2.uv_stride, d.v + (size_t)(y >> 1) * d.uv_stride + (x >> 1), d.uv_stride, uw,
                               uh, hipMemcpyDeviceToDevice, s);
        if (e != hipSuccess) return WG_STATUS_USER_ABORT;
      }
    }
    hipError_t e = wg::launch_yuv_to_rgba(b->any_crop ? b->d_desc2 : b->d_desc, nullptr, b->n, b->max_out_w,
                                          b->max_out_h, (b->flags & WG_FLAG_NO_FANCY_UPSAMPLING) ? 0 : 1, s);
    if (e != hipSuccess) return WG_STATUS_UNSUPPORTED_FEATURE;
  }
  hipEventRecord(t.ev[2], s);
  if (b->n_k3 > 0) {
    hipError_t e = wg::launch_vp8l_transforms(b->d_lldesc, b->ll_groups, b->d_err, s);
    if (e != hipSuccess) return WG_STATUS_UNSUPPORTED_FEATURE;
  }
  hipEventRecord(t.ev[3], s);
  if (b->n_alpha > 0) {  // after K2 (A = 255) and K3 (alpha streams)
    hipError_t e = wg::launch_alpha(b->d_adesc, b->n_alpha, s);
    if (e != hipSuccess) return WG_STATUS_UNSUPPORTED_FEATURE;
  }
  hipEventRecord(t.ev[4], s);
  return WG_STATUS_OK;
}

int wg_batch_kernel_ms(const wg_batch* bc, float* ms, int n_ms) {
  wg_batch* b = const_cast<wg_batch*>(bc);
  if (!b || !ms || n_ms < 1) return WG_STATUS_INVALID_PARAM;
  for (int k = 0; k < n_ms; ++k) ms[k] = 0.f;
  if (b->n_runs_pending == 0) return WG_STATUS_OK;
  double acc[4] = {0, 0, 0, 0};
  int cnt[4] = {0, 0, 0, 0};
  for (size_t i = 0; i < b->n_runs_pending; ++i) {
    Timing& t = b->timings[i];
    if (hipEventSynchronize(t.ev[4]) != hipSuccess) return WG_STATUS_USER_ABORT;
    for (int k = 0; k < 4; ++k) {
      if (!t.ran[k]) continue;
      float a = 0;
      hipEventElapsedTime(&a, t.ev[k], t.ev[k + 1]);
      acc[k] += a;
      cnt[k]++;
    }
  }
  int err = 0;
  if (hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost) != hipSuccess || err) return WG_STATUS_USER_ABORT;
  for (int k = 0; k < std::min(n_ms, 4); ++k) ms[k] = cnt[k] ? (float)(acc[k] / cnt[k]) : 0.f;
  b->n_runs_pending = 0;
  return WG_STATUS_OK;
}

int wg_batch_kernel_bytes(const wg_batch* b, double* bytes, int n_bytes) {
  if (!b || !bytes || n_bytes < 1) return WG_STATUS_INVALID_PARAM;
  for (int k = 0; k < n_bytes; ++k) bytes[k] = k < 4 ? b->kbytes[k] : 0.0;
  if (b->fused) bytes[0] = b->k1_fused_bytes;
  return WG_STATUS_OK;
}

int wg_batch_set_emit(wg_batch* b, int separate) {
  if (!b) return WG_STATUS_INVALID_PARAM;
  if (!separate && b->any_crop) return WG_STATUS_INVALID_PARAM;  // crop windows need K2
  if (b->fused == !separate) return WG_STATUS_OK;
  b->fused = !separate;
  for (FrameDesc& d : b->desc)
    if (d.valid) d.flags = b->fused ? (d.flags | wg::kFrameEmitRgba) : (d.flags & ~wg::kFrameEmitRgba);
  hipSetDevice(b->ctx->device);
  hipError_t e = hipMemcpyAsync(b->d_desc, b->desc.data(), sizeof(FrameDesc) * (size_t)b->n, hipMemcpyHostToDevice,
                                b->ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(b->ctx->stream);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_batch_run_emit(wg_batch* b, void* stream) {
  if (!b) return WG_STATUS_INVALID_PARAM;
  if (b->n_lossy == 0 || b->any_crop) return WG_STATUS_OK;
  hipSetDevice(b->ctx->device);
  hipStream_t s = stream ? reinterpret_cast<hipStream_t>(stream) : b->ctx->stream;
  if (b->n_runs_pending >= b->timings.size()) {
    Timing t;
    for (auto& e : t.ev)
      if (hipEventCreate(&e) != hipSuccess) return WG_STATUS_OUT_OF_MEMORY;
    b->timings.push_back(t);
  }
  Timing& t = b->timings[b->n_runs_pending++];
  t.ran[0] = t.ran[2] = t.ran[3] = false;
  t.ran[1] = true;
  for (int k = 0; k < 2; ++k) hipEventRecord(t.ev[k], s);
  hipError_t e = wg::launch_yuv_to_rgba(b->d_desc, nullptr, b->n, b->max_out_w, b->max_out_h,
                                        (b->flags & WG_FLAG_NO_FANCY_UPSAMPLING) ? 0 : 1, s);
  for (int k = 2; k < 5; ++k) hipEventRecord(t.ev[k], s);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_UNSUPPORTED_FEATURE;
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
  hipSetDevice(b->ctx->device);
  hipError_t e = hipStreamSynchronize(b->ctx->stream);
  if (e == hipSuccess) e = hipDeviceSynchronize();
  int err = 0;
  if (e == hipSuccess) e = hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost);
  return (e != hipSuccess || err) ? WG_STATUS_USER_ABORT : WG_STATUS_OK;
}
const uint8_t* window_ptr(const wg_batch* b, int i) {
  const FrameParse& f = b->fp[i];
  const FrameDesc& d = b->desc[i];
  return d.rgba + (size_t)f.win_y * d.rgba_stride + 4 * (size_t)f.win_x;
}
}  // namespace

int wg_batch_download_rgba(wg_batch* b, int i, uint8_t* rgba, int stride) {
  if (!b || i < 0 || i >= b->n || !rgba) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  const FrameParse& f = b->fp[i];
  if (stride < 4 * f.out_w) return WG_STATUS_INVALID_PARAM;
  int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  const hipError_t e = hipMemcpy2D(rgba, stride, window_ptr(b, i), b->desc[i].rgba_stride, 4 * (size_t)f.out_w,
                                   f.out_h, hipMemcpyDeviceToHost);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_batch_download(wg_batch* b, int i, uint8_t* out, int stride) {
  if (!b || i < 0 || i >= b->n || !out) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  const FrameParse& f = b->fp[i];
  const int bpp = wg::output_bpp(b->opt.colorspace);
  if (stride < bpp * f.out_w) return WG_STATUS_INVALID_PARAM;
  if (b->opt.colorspace == 1 && !b->opt.flip) return wg_batch_download_rgba(b, i, out, stride);
  int st = batch_sync(b);
  if (st != WG_STATUS_OK) return st;
  // K6 into a device staging buffer, then one 2D copy
  const size_t row = (size_t)bpp * f.out_w;
  uint8_t* d_out = nullptr;
  wg::EmitDesc* d_ed = nullptr;
  wg::EmitDesc ed{window_ptr(b, i), nullptr, b->desc[i].rgba_stride, (int32_t)row, f.out_w, f.out_h,
                  b->opt.colorspace, b->opt.flip ? 1 : 0, 1, 0};
  hipError_t e = hipMalloc(&d_out, row * f.out_h);
  if (e == hipSuccess) e = hipMalloc(&d_ed, sizeof(ed));
  if (e == hipSuccess) {
    ed.dst = d_out;
    e = hipMemcpyAsync(d_ed, &ed, sizeof(ed), hipMemcpyHostToDevice, b->ctx->stream);
  }
  if (e == hipSuccess) e = wg::launch_emit(d_ed, 1, f.out_w * f.out_h, b->ctx->stream);
  if (e == hipSuccess) e = hipMemcpy2DAsync(out, stride, d_out, row, row, f.out_h, hipMemcpyDeviceToHost, b->ctx->stream);
  if (e == hipSuccess) e = hipStreamSynchronize(b->ctx->stream);
  if (d_out) hipFree(d_out);
  if (d_ed) hipFree(d_ed);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_batch_download_yuv(wg_batch* b, int i, uint8_t* y, uint8_t* u, uint8_t* v) {
  if (!b || i < 0 || i >= b->n) return WG_STATUS_INVALID_PARAM;
  if (b->fp[i].status != WG_STATUS_OK) return b->fp[i].status;
  if (b->fp[i].lossless) return WG_STATUS_UNSUPPORTED_FEATURE;  // VP8L has no YUV planes
  const FrameDesc& d = b->desc[i];
  hipSetDevice(b->ctx->device);
  hipError_t e = hipDeviceSynchronize();
  const int uw = (d.width + 1) / 2, uh = (d.height + 1) / 2;
  if (e == hipSuccess && y) e = hipMemcpy2D(y, d.width, d.y, d.y_stride, d.width, d.height, hipMemcpyDeviceToHost);
  if (e == hipSuccess && u) e = hipMemcpy2D(u, uw, d.u, d.uv_stride, uw, uh, hipMemcpyDeviceToHost);
  if (e == hipSuccess && v) e = hipMemcpy2D(v, uw, d.v, d.uv_stride, uw, uh, hipMemcpyDeviceToHost);
  return e == hipSuccess ? WG_STATUS_OK : WG_STATUS_USER_ABORT;
}

int wg_decode_rgba_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                         uint8_t* const* rgba, const int32_t* strides, int32_t* status, int32_t flags) {
  if (!ctx || !data || !sizes || !rgba || !strides || !status || n <= 0) return WG_STATUS_INVALID_PARAM;
  wg_batch* b = wg_batch_create(ctx, data, sizes, n, flags, status);
  if (!b) return WG_STATUS_OUT_OF_MEMORY;
  int st = wg_batch_run(b, nullptr);
  if (st == WG_STATUS_OK && hipStreamSynchronize(ctx->stream) != hipSuccess) st = WG_STATUS_USER_ABORT;
  if (st == WG_STATUS_OK) {
    for (int i = 0; i < n; ++i) {
      if (status[i] != WG_STATUS_OK) continue;
      if (rgba[i] == nullptr || strides[i] < 4 * b->desc[i].width) {
        status[i] = WG_STATUS_INVALID_PARAM;
        continue;
      }
      status[i] = wg_batch_download_rgba(b, i, rgba[i], strides[i]);
    }
  }
  wg_batch_destroy(b);
  return st;
}

int wg_decode_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n, const wg_decoder_options* opt,
                    uint8_t* const* out, const int32_t* strides, int32_t* status) {
  if (!ctx || !data || !sizes || !out || !strides || !status || !opt || n <= 0) return WG_STATUS_INVALID_PARAM;
  wg_batch* b = wg_batch_create_ex(ctx, data, sizes, n, opt, status);
  if (!b) return WG_STATUS_OUT_OF_MEMORY;
  int st = wg_batch_run(b, nullptr);
  const int bpp = wg::output_bpp(opt->colorspace);
  if (st == WG_STATUS_OK && !(opt->colorspace == 1 && !opt->flip)) {
    // K6 over every frame in one launch into one staging buffer
    std::vector<wg::EmitDesc> ed((size_t)n, wg::EmitDesc{});
    std::vector<size_t> offs((size_t)n, 0);
    size_t total = 0;
    int maxpx = 1;
    for (int i = 0; i < n; ++i) {
      const FrameParse& f = b->fp[i];
      if (f.status != WG_STATUS_OK) continue;
      offs[(size_t)i] = total;
      total = align_up(total + (size_t)bpp * f.out_w * f.out_h);
      maxpx = std::max(maxpx, f.out_w * f.out_h);
    }
    uint8_t* d_out = nullptr;
    wg::EmitDesc* d_ed = nullptr;
    hipError_t e = hipMalloc(&d_out, std::max<size_t>(total, kAlign));
    if (e == hipSuccess) e = hipMalloc(&d_ed, sizeof(wg::EmitDesc) * (size_t)n);
    for (int i = 0; e == hipSuccess && i < n; ++i) {
      const FrameParse& f = b->fp[i];
      if (f.status != WG_STATUS_OK) continue;
      ed[(size_t)i] = wg::EmitDesc{window_ptr(b, i), d_out + offs[(size_t)i], b->desc[i].rgba_stride,
                                   bpp * f.out_w, f.out_w, f.out_h, opt->colorspace, opt->flip ? 1 : 0, 1, 0};
    }
    if (e == hipSuccess)
      e = hipMemcpyAsync(d_ed, ed.data(), sizeof(wg::EmitDesc) * (size_t)n, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess) e = wg::launch_emit(d_ed, n, maxpx, ctx->stream);
    if (e == hipSuccess) st = batch_sync(b);
    else st = WG_STATUS_USER_ABORT;
    for (int i = 0; st == WG_STATUS_OK && i < n; ++i) {
      const FrameParse& f = b->fp[i];
      if (status[i] != WG_STATUS_OK) continue;
      if (out[i] == nullptr || strides[i] < bpp * f.out_w) {
        status[i] = WG_STATUS_INVALID_PARAM;
        continue;
      }
      const size_t row = (size_t)bpp * f.out_w;
      if (hipMemcpy2D(out[i], strides[i], d_out + offs[(size_t)i], row, row, f.out_h, hipMemcpyDeviceToHost) !=
          hipSuccess)
        status[i] = WG_STATUS_USER_ABORT;
    }
    if (d_out) hipFree(d_out);
    if (d_ed) hipFree(d_ed);
  } else if (st == WG_STATUS_OK) {
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) st = WG_STATUS_USER_ABORT;
    for (int i = 0; st == WG_STATUS_OK && i < n; ++i) {
      if (status[i] != WG_STATUS_OK) continue;
      if (out[i] == nullptr || strides[i] < 4 * b->fp[i].out_w) {
        status[i] = WG_STATUS_INVALID_PARAM;
        continue;
      }
      status[i] = wg_batch_download_rgba(b, i, out[i], strides[i]);
    }
  }
  wg_batch_destroy(b);
  return st;
}

int wg_decode_into(const uint8_t* data, size_t size, const wg_decoder_options* opt, uint8_t* out, size_t cap,
                   int stride) {
  if (!data || !out || !opt) return WG_STATUS_INVALID_PARAM;
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
  wg_ctx* ctx = default_ctx();
  if (!ctx) return WG_STATUS_UNSUPPORTED_FEATURE;  // no GPU: no CPU fallback by design
  const uint8_t* d[1] = {data};
  const size_t s[1] = {size};
  uint8_t* o[1] = {out};
  const int32_t str[1] = {stride};
  int32_t fs[1] = {0};
  st = wg_decode_batch(ctx, d, s, 1, opt, o, str, fs);
  return st != WG_STATUS_OK ? st : fs[0];
}

int wg_decode_rgba_into(const uint8_t* data, size_t size, uint8_t* rgba, size_t cap, int stride, int flags) {
  if (!data || !rgba) return WG_STATUS_INVALID_PARAM;
  wg_features f{};
  int st = wg_get_features(data, size, &f);
  if (st != WG_STATUS_OK) return st;
  if (stride < 4 * f.width || (size_t)stride * (f.height - 1) + 4 * (size_t)f.width > cap)
    return WG_STATUS_INVALID_PARAM;
  wg_ctx* ctx = default_ctx();
  if (!ctx) return WG_STATUS_UNSUPPORTED_FEATURE;  // no GPU: no CPU fallback by design
  const uint8_t* d[1] = {data};
  const size_t s[1] = {size};
  uint8_t* o[1] = {rgba};
  const int32_t str[1] = {stride};
  int32_t fs[1] = {0};
  st = wg_decode_rgba_batch(ctx, d, s, 1, o, str, fs, flags);
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

int wg_anim_decode(wg_ctx* ctx, const uint8_t* data, size_t size, uint8_t* canvases, int32_t* timestamps,
                   int32_t flags) {
  if (!ctx || !data || !canvases || !timestamps) return WG_STATUS_INVALID_PARAM;
  wg::AnimInfo ai;
  std::vector<wg::AnimFrame> fr;
  int st = wg::anim_demux(data, size, &ai, &fr);
  if (st != WG_STATUS_OK) return st;
  const int n = ai.frame_count;
  // every frame's fragment decodes as one batch (K1..K4)
  std::vector<const uint8_t*> ptrs((size_t)n);
  std::vector<size_t> sizes((size_t)n);
  std::vector<int32_t> status((size_t)n, 0);
  for (int i = 0; i < n; ++i) {
    ptrs[(size_t)i] = data + fr[(size_t)i].off;
    sizes[(size_t)i] = fr[(size_t)i].size;
  }
  wg_batch* b = wg_batch_create(ctx, ptrs.data(), sizes.data(), n, flags, status.data());
  if (!b) {
    for (int i = 0; i < n; ++i)
      if (status[(size_t)i] != WG_STATUS_OK) return status[(size_t)i];
    return WG_STATUS_OUT_OF_MEMORY;
  }
  for (int i = 0; i < n; ++i) {
    if (status[(size_t)i] != WG_STATUS_OK) {
      wg_batch_destroy(b);
      return status[(size_t)i];
    }
    if (b->desc[(size_t)i].width != fr[(size_t)i].width || b->desc[(size_t)i].height != fr[(size_t)i].height) {
      wg_batch_destroy(b);
      return WG_STATUS_BITSTREAM_ERROR;
    }
  }
  st = wg_batch_run(b, nullptr);
  // frame descriptors: IsKeyFrame (anim_decode.go:183-197) and the blend / dispose flags
  std::vector<AnimFrameDesc> fd((size_t)n);
  int32_t t = 0;
  bool prev_key = false;
  auto full = [&](const wg::AnimFrame& f) { return f.width == ai.canvas_width && f.height == ai.canvas_height; };
  for (int i = 0; i < n; ++i) {
    const wg::AnimFrame& f = fr[(size_t)i];
    bool key;
    if (i == 0) key = true;
    else if ((!f.has_alpha || f.no_blend) && full(f)) key = true;
    else key = fr[(size_t)i - 1].dispose_bg && (full(fr[(size_t)i - 1]) || prev_key);
    AnimFrameDesc& d = fd[(size_t)i];
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
    timestamps[i] = t;
  }
  const size_t canvas_bytes = (size_t)ai.canvas_width * ai.canvas_height * 4;
  AnimFrameDesc* d_fd = nullptr;
  uint8_t* d_canvases = nullptr;
  {
    std::lock_guard<std::mutex> lock(ctx->mu);
    hipSetDevice(ctx->device);
    hipError_t e = st == WG_STATUS_OK ? hipSuccess : hipErrorUnknown;
    if (e == hipSuccess) e = hipMalloc(&d_fd, sizeof(AnimFrameDesc) * (size_t)n);
    if (e == hipSuccess) e = hipMalloc(&d_canvases, canvas_bytes * (size_t)n);
    if (e == hipSuccess)
      e = hipMemcpyAsync(d_fd, fd.data(), sizeof(AnimFrameDesc) * (size_t)n, hipMemcpyHostToDevice, ctx->stream);
    if (e == hipSuccess)
      e = wg::launch_anim_compose(d_fd, n, d_canvases, ai.canvas_width, ai.canvas_height, ctx->stream);
    if (e == hipSuccess)
      e = hipMemcpyAsync(canvases, d_canvases, canvas_bytes * (size_t)n, hipMemcpyDeviceToHost, ctx->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
    int err = 0;
    if (e == hipSuccess) e = hipMemcpy(&err, b->d_err, sizeof(int), hipMemcpyDeviceToHost);
    if (st == WG_STATUS_OK && (e != hipSuccess || err)) st = WG_STATUS_USER_ABORT;
    if (d_fd) hipFree(d_fd);
    if (d_canvases) hipFree(d_canvases);
  }
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

}  // extern "C"
