// Host stages of a decode batch: parse_one / parse_all (declared in batch.h).
//
// Mirrors the status logic of WebPDecode -> DecodeInto (pkg/libwebp/decoder/webp.go:483-556,
// 870-909): GetFeatures, the header pass, the output options, then the image data -- bounded,
// like libwebp's, to the rows a crop window needs, with a lossy frame's ALPH data decoded
// lazily per MB row (its failure wins over a token failure further down).
#include <algorithm>
#include <climits>
#include <cstring>
#include <new>

#include "batch.h"

namespace wg {
namespace {

constexpr int kFilterExtraRows[3] = {0, 2, 8};  // frame_dec.c.go (VP8EnterCritical)

// Allocation failure anywhere in the host stages (vectors sized by the bitstream) is
// reported as WebPDecode does, never thrown across the C ABI or out of a worker thread.
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

// The lossy frame's sink: one staging region, MbRec | row_block0 | blocks (device_format.h).
struct LossySink {
  StagingArena* arena;
  StagingArena::Cursor* cur;
  FrameParse* fp;
  bool reserved;
};

bool lossy_alloc(void* p, const wg_vp8_info& inf, int rows, SparseSink* sink) {
  LossySink* a = static_cast<LossySink*>(p);
  const size_t nmb = (size_t)inf.mb_w * inf.mb_h;
  const size_t off_rows = StagingArena::align(nmb * sizeof(MbRec));
  const size_t off_blocks = StagingArena::align(off_rows + (size_t)inf.mb_h * 4);
  uint8_t* base = a->arena->reserve(a->cur, off_blocks + sparse_max_blocks(inf.mb_w, rows) * 32);
  if (!base) return false;
  // alignment gaps zeroed: the staged bytes are a function of the bitstream alone
  std::memset(base + nmb * sizeof(MbRec), 0, off_rows - nmb * sizeof(MbRec));
  std::memset(base + off_rows + (size_t)inf.mb_h * 4, 0, off_blocks - off_rows - (size_t)inf.mb_h * 4);
  sink->mbs = reinterpret_cast<MbRec*>(base);
  sink->row_block0 = reinterpret_cast<uint32_t*>(base + off_rows);
  sink->blocks = reinterpret_cast<int16_t*>(base + off_blocks);
  a->fp->off_rows = off_rows;
  a->fp->off_blocks = off_blocks;
  a->reserved = true;
  return true;
}

// A lossless stream into staging: its coded-image tokens, literals and transform data.
bool stage_ll(const VP8LFrame& f, StagingArena* arena, StagingArena::Cursor* cur, LLMeta* m) {
  m->width = f.width;
  m->height = f.height;
  m->coded_width = f.coded_width;
  m->fail_pixel = f.fail_pixel;
  m->n_transforms = (int)f.transforms.size();
  for (int t = 0; t < m->n_transforms; ++t) {
    const VP8LTransform& tr = f.transforms[(size_t)t];
    m->type[t] = tr.type;
    m->bits[t] = tr.bits;
    m->xsize[t] = tr.xsize;
    if (!arena->put(cur, tr.data.data(), tr.data.size() * 4, &m->tdata[t])) return false;
  }
  m->cache_bits = f.cache_bits;
  return arena->put(cur, f.lits.data(), f.lits.size() * 4, &m->lits) &&
         arena->put(cur, f.tokens.data(), f.tokens.size() * 4, &m->tokens);
}

// Per worker thread: the lossless entropy stage's output, reused frame after frame (its
// vectors keep their capacity, so a batch does not page-fault fresh heap memory per frame).
// Capacity beyond kKeepLLBytes (a 16k x 16k frame's tokens are 1 GB) is released once the
// frame is staged, so pool threads and callers' threads do not hold it for good.
thread_local VP8LFrame tl_lf;
constexpr size_t kKeepLLBytes = size_t(64) << 20;
void trim_ll(VP8LFrame& f) {
  if ((f.tokens.capacity() + f.lits.capacity()) * 4 > kKeepLLBytes) f = VP8LFrame();
}

}  // namespace

int apply_output_options(const wg_decoder_options& opt, FrameParse* f) {
  // the RGB family (0..10), or MODE_YUV / MODE_YUVA (11, 12: K8 writes the planes)
  if (!output_bpp(opt.colorspace) && opt.colorspace != 11 && opt.colorspace != 12) return WG_STATUS_INVALID_PARAM;
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

int parse_one(const uint8_t* data, size_t size, const wg_decoder_options& opt, StagingArena* arena,
              StagingArena::Cursor* cur, FrameParse* fp) {
  Container c;
  wg_features feat{};
  // WebPDecode first runs GetFeatures; its NOT_ENOUGH_DATA is "treated as error"
  int st = parse_container(data, size, &c, &feat, /*have_all_data=*/false);
  if (st != WG_STATUS_OK) return st == WG_STATUS_NOT_ENOUGH_DATA ? WG_STATUS_BITSTREAM_ERROR : st;
  st = parse_container(data, size, &c, &feat);  // DecodeInto's WebPParseHeaders
  if (st != WG_STATUS_OK) return st;
  if (c.is_lossless) {  // VP8L: host entropy stage, K3 on device
    fp->lossless = true;
    VP8LFrame& lf = tl_lf;
    // the output options between the header/transforms/codes and the pixels, as DecodeInto
    // orders VP8LDecodeHeader, WebPIoInitFromOptions and VP8LDecodeImage (webp.go:528-544)
    struct Opt {
      const wg_decoder_options* opt;
      FrameParse* fp;
      const VP8LFrame* lf;
    } oc{&opt, fp, &lf};
    auto check = [](void* p) {
      Opt* o = static_cast<Opt*>(p);
      o->fp->width = o->lf->width;
      o->fp->height = o->lf->height;
      return apply_output_options(*o->opt, o->fp);
    };
    st = vp8l_parse(data + c.payload_off, c.payload_size, &lf, check, &oc);
    if (st != WG_STATUS_OK && lf.fail_pixel == SIZE_MAX) return st;  // VP8LDecodeHeader or the options
    if (st != WG_STATUS_OK) {  // DecodeImageData stops at the crop bottom (io->crop_bottom)
      // int64: crop_top + crop_height of a validated window fits, but keep it overflow-free
      const int64_t bottom = opt.use_cropping ? (int64_t)opt.crop_top + opt.crop_height : fp->height;
      if ((uint64_t)bottom * (uint64_t)lf.coded_width > (uint64_t)lf.fail_pixel) return st;
    }
    const bool staged = stage_ll(lf, arena, cur, &fp->ll);
    trim_ll(lf);
    return staged ? WG_STATUS_OK : WG_STATUS_OUT_OF_MEMORY;
  }
  const int flags = opt.bypass_filtering ? WG_FLAG_BYPASS_FILTERING : 0;
  // crop bottom in int64, clamped to the frame: an adversarial crop_top + crop_height must
  // not overflow (the window itself is validated by apply_output_options below)
  int crop_bottom = -1;
  if (opt.use_cropping) {
    const int64_t b = (int64_t)(opt.crop_top & ~1) + (int64_t)opt.crop_height;
    crop_bottom = (int)std::min<int64_t>(std::max<int64_t>(b, 0), 1 << 14);
  }
  LossySink sink{arena, cur, fp, false};
  SparseResult res;
  st = vp8_parse_sparse(data, size, flags, crop_bottom, lossy_alloc, &sink, &res);
  fp->info = res.info;
  fp->n_blocks = res.n_blocks;
  fp->n_y2 = res.n_y2;
  fp->br_mb_y = res.br_mb_y;
  fp->fail_row = res.fail_row;
  if (sink.reserved) fp->input = arena->commit(cur, fp->off_blocks + res.n_blocks * 32);
  if (st != WG_STATUS_OK && res.fail_row < 0) return st;  // VP8GetHeaders
  fp->width = res.info.width;
  fp->height = res.info.height;
  const int ost = apply_output_options(opt, fp);
  if (ost != WG_STATUS_OK) return ost;
  if (c.alpha_size > 0) {  // ALPH (VP8DecompressAlphaRows, alpha_dec.go:164-213)
    const uint8_t* ad = data + c.alpha_off;
    fp->alpha = true;
    int ast = WG_STATUS_OK;
    bool init_fails = false;
    size_t afail = SIZE_MAX;
    int acw = fp->width;
    if (!parse_alpha_header(ad, c.alpha_size, fp->width, fp->height, &fp->ah)) {
      ast = WG_STATUS_OUT_OF_MEMORY;  // ALPHInit failure without a VP8L decoder
      init_fails = true;
    } else if (fp->ah.method == 1) {
      VP8LFrame& af = tl_lf;
      ast = vp8l_parse_alpha(ad + 1, c.alpha_size - 1, fp->width, fp->height, &af);
      init_fails = ast == WG_STATUS_OUT_OF_MEMORY;
      afail = af.fail_pixel;
      acw = af.coded_width;
      const bool staged = init_fails || stage_ll(af, arena, cur, &fp->al);
      trim_ll(af);
      if (!staged) return WG_STATUS_OUT_OF_MEMORY;
    } else if (!arena->put(cur, ad + 1, (size_t)fp->width * fp->height, &fp->araw)) {
      return WG_STATUS_OUT_OF_MEMORY;
    }
    if (ast != WG_STATUS_OK) {
      const int bottom = crop_bottom >= 0 ? std::min(crop_bottom, fp->height) : fp->height;
      const int arow = alpha_fail_row(fp->br_mb_y, kFilterExtraRows[fp->info.filter_type], bottom, init_fails,
                                      afail, acw, fp->ah.pre_processing == 1);
      if (arow < (st != WG_STATUS_OK ? fp->fail_row : INT_MAX)) return ast;
    }
  }
  return st;
}

void parse_frame(const uint8_t* data, size_t size, const wg_decoder_options& opt, StagingArena* arena,
                 StagingArena::Cursor* cur, FrameParse* f) {
  if (data == nullptr) {
    f->status = WG_STATUS_INVALID_PARAM;
    return;
  }
  f->status = guarded([&] { return parse_one(data, size, opt, arena, cur, f); });
  if (f->status != WG_STATUS_OK) {  // drop partial host data
    const int st = f->status;
    *f = FrameParse();
    f->status = st;
  }
}

void parse_all(const uint8_t* const* data, const size_t* sizes, int n, const wg_decoder_options& opt,
               WorkerPool* pool, StagingArena* arena, std::vector<FrameParse>& out) {
  out.assign((size_t)n, FrameParse{});
  std::vector<StagingArena::Cursor> cursors((size_t)pool->threads() + 1);
  pool->run(n, [&](int i, int worker) {
    parse_frame(data[i], sizes[i], opt, arena, &cursors[(size_t)worker], &out[(size_t)i]);
  });
  for (auto& c : cursors) arena->release(&c);
}

}  // namespace wg
