/*
 * gowebp_amd.h -- C ABI of the MI355X-native WebP decode path.
 *
 * This is the drop-in boundary that replaces everything below libwebp's
 * DecodeInto() in the reference (pkg/libwebp/decoder/webp.go:483-556): the VP8
 * per-macroblock DSP loop (frame_dec.c.go ReconstructRow/DoFilter,
 * dsp/dec.c.go) and the YUV420->RGBA emitters (io_dec.c.go EmitFancyRGB /
 * EmitSampledRGB, dsp/upsampling.c.go, pkg/color/yuv/conversion.go).  The
 * RIFF/VP8 bool-decoder entropy stage runs on host cores; reconstruction,
 * in-loop deblocking and colour conversion run as HIP kernels on gfx950.
 *
 * Conventions (mirroring libwebp / the reference):
 *   - every int-returning call returns a wg_status (== VP8StatusCode values,
 *     pkg/vp8/enums.go:20-31); "first error wins" per frame;
 *   - no caller pointer is retained after a call returns (cgo pointer rule);
 *   - plain pointers and sizes only; no HIP or torch types in signatures
 *     (streams are passed as opaque `void*`, NULL = the context's stream);
 *   - output RGBA is byte order R,G,B,A, alpha 0xff for opaque lossy input
 *     (VP8YuvToRgba semantics, dsp/yuv.go).
 */
#ifndef GOWEBP_AMD_H_
#define GOWEBP_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes: VP8StatusCode (pkg/vp8/enums.go:20-31) ------------------------------ */
typedef enum {
  WG_STATUS_OK = 0,
  WG_STATUS_OUT_OF_MEMORY = 1,
  WG_STATUS_INVALID_PARAM = 2,
  WG_STATUS_BITSTREAM_ERROR = 3,
  WG_STATUS_UNSUPPORTED_FEATURE = 4,
  WG_STATUS_SUSPENDED = 5,
  WG_STATUS_USER_ABORT = 6,
  WG_STATUS_NOT_ENOUGH_DATA = 7
} wg_status;

/* ---- decode flags: subset of WebPDecoderOptions (pkg/libwebp/webp/decode.go:59-76) ------ */
#define WG_FLAG_BYPASS_FILTERING    1 /* options.bypass_filtering    */
#define WG_FLAG_NO_FANCY_UPSAMPLING 2 /* options.no_fancy_upsampling */

/* ---- bitstream features: WebPBitstreamFeatures (pkg/libwebp/webp/decode.go:33-41) ------- */
typedef struct {
  int32_t width;
  int32_t height;
  int32_t has_alpha;
  int32_t has_animation;
  int32_t format; /* 0 = undefined/mixed, 1 = lossy (VP8), 2 = lossless (VP8L) */
} wg_features;

/* Library version, libwebp-style packed 0xMMmmrr. */
int wg_version(void);

/* Number of HIP devices visible (0 when no GPU). */
int wg_device_count(void);

/* Test hook (no libwebp counterpart): sets the process-wide counter behind the split K1 kernel's
 * 16-bit launch tags and returns its previous value, so a test can re-run a batch exactly one tag
 * cycle (65,535 split launches) later.  Correctness does not depend on the tags: every split launch
 * clears its batch's progress flags first. */
uint32_t wg_debug_set_epoch(uint32_t value);

/* Replaces WebPGetFeatures (pkg/libwebp/webp/decode.go:54-56 -> webp.go:764-779,
 * ParseHeadersInternal webp.go:300-440).  Host only, no GPU needed.
 * Backs Go's webp.DecodeConfig (decode.go:12-14). */
int wg_get_features(const uint8_t* data, size_t size, wg_features* out);

/* Replaces WebPDecodeRGBAInto (webp.go:592-594): decode one frame on the GPU
 * (device 0 context, created lazily) into caller memory of `cap` bytes with
 * row `stride` (>= 4*width).  flags = WG_FLAG_*.  Backs Go's webp.Decode
 * (decode.go:8-10).  Fails with UNSUPPORTED_FEATURE when no GPU is present:
 * there is no CPU fallback for the DSP path. */
int wg_decode_rgba_into(const uint8_t* data, size_t size, uint8_t* rgba, size_t cap,
                        int stride, int flags);

/* The HIP device of the context behind the single-frame entry points (wg_decode_rgba_into,
 * wg_decode_into): 0 by default.  Replaces that context if it exists on another device; calls
 * in flight finish on the context they started with, which is destroyed when the last of them
 * returns.  INVALID_PARAM for a device that does not exist.  No libwebp counterpart (libwebp
 * has no devices). */
int wg_set_default_device(int device);

/* ---- output options (WebPDecoderConfig subset, pkg/libwebp/webp/decode.go:59-83) --------- */
/* colorspace = WEBP_CSP_MODE: the RGB family 0 RGB, 1 RGBA, 2 BGR, 3 BGRA, 4 ARGB, 5 RGBA_4444,
 * 6 RGB_565, 7 rgbA, 8 bgrA, 9 Argb, 10 rgbA_4444 (lower case = premultiplied), or the YUV modes
 * 11 MODE_YUV / 12 MODE_YUVA (planes: wg_decode_yuv_into / wg_decode_yuv_batch /
 * wg_batch_download_yuva; the single-buffer entry points wg_decode_into / wg_decode_batch refuse
 * them with INVALID_PARAM).
 * Cropping as WebPIoInitFromOptions: left/top snapped to even, the window must lie inside the
 * frame (else INVALID_PARAM).  Scaling is disabled in the reference (io_dec.c.go:540-541):
 * use_scaling -> UNSUPPORTED_FEATURE.  flip emits rows bottom-up. */
typedef struct {
  int32_t colorspace;
  int32_t bypass_filtering, no_fancy_upsampling;
  int32_t use_cropping, crop_left, crop_top, crop_width, crop_height;
  int32_t use_scaling, scaled_width, scaled_height;
  int32_t flip;
  int32_t reserved[4];
} wg_decoder_options;

/* Bytes per pixel of a colorspace (3, 4 or 2); 0 if not an RGB-family mode. */
int wg_output_bpp(int colorspace);

/* ---- YUV output (MODE_YUV / MODE_YUVA) ---------------------------------------------------- */
/* WebPYUVABuffer (pkg/libwebp/webp/buffer.go:17-25): caller memory for the Y plane (width x
 * height), U and V ((width + 1) / 2 x (height + 1) / 2) and, MODE_YUVA, A (width x height) of the
 * output window, rows of the given strides.  Checked as CheckDecBuffer checks external memory
 * (buffer_dec.c.go): stride >= the plane's width, size >= stride * (rows - 1) + width, A present
 * for MODE_YUVA (else INVALID_PARAM, nothing written). */
typedef struct {
  uint8_t *y, *u, *v, *a;
  int32_t y_stride, u_stride, v_stride, a_stride;
  size_t y_size, u_size, v_size, a_size;
} wg_yuva_buffer;

/* Replaces WebPDecodeYUVInto (webp.go:615-650) and WebPDecode with a MODE_YUV / MODE_YUVA
 * config.output in external memory (webp.go:870-909): one frame on the GPU (default context) in
 * opt->colorspace 11 or 12 with the options' crop window (lossy origins snapped to even) and flip.
 * Lossy frames: the reconstructed planes' window (EmitYUV, io_dec.c.go:36-50) and the alpha plane
 * or 0xff (EmitAlphaYUV :128-150); lossless frames: libwebp 1.6.0's per-row ConvertToYUVA
 * (vp8l_dec.c.go:544-563).  Kernel K8 (device/emit_yuva.hip) writes the planes. */
int wg_decode_yuv_into(const uint8_t* data, size_t size, const wg_decoder_options* opt,
                       const wg_yuva_buffer* out);

/* The status WebPDecode (webp.go:870-909) returns for this input and options (NULL = RGBA,
 * no crop), from the host stages alone: container, headers, options, then the entropy-coded
 * data in libwebp's order (crop-bounded rows, lazily decoded alpha).  Host only, no GPU
 * needed; the batch entry points report the same per-frame status. */
int wg_decode_status(const uint8_t* data, size_t size, const wg_decoder_options* opt);

/* Replaces WebPDecode with config.output in external memory (webp.go:870-909): one frame on
 * the GPU (device 0 context) in the options' colorspace / crop window / orientation, rows of
 * `stride` bytes. */
int wg_decode_into(const uint8_t* data, size_t size, const wg_decoder_options* opt, uint8_t* out,
                   size_t cap, int stride);

/* ---- batched decode: one context per device ------------------------------------------ */
typedef struct wg_ctx wg_ctx;

/* Create a decode context bound to HIP device `device` (host threads for the entropy
 * stage = `host_threads`, 0 = hardware concurrency).  NULL on failure.  The context keeps a
 * worker pool, pinned staging memory and device buffers of finished batches for reuse by
 * later batches; all are released by wg_ctx_destroy.  Batches of one context are created one
 * at a time (internal lock); contexts are independent (synchronisation is per stream). */
wg_ctx* wg_ctx_create(int device, int host_threads);
void wg_ctx_destroy(wg_ctx* ctx);

/* Decode n independent frames: entropy stage on host threads, the DSP kernels on the device,
 * RGBA back to rgba[i].  Per-frame status in status[i]; a bad frame does not abort the batch.
 * Returns OK if the batch ran (check status[]).  Pipelined: the frames go in chunks (see
 * wg_ctx_set_chunk_frames), and chunk k + 1's entropy stage (host threads) and upload overlap
 * chunk k's kernels and download (two staging arenas, two streams) -- the parse / finish
 * overlap of libwebp's threaded decode (frame_dec.c.go:505-534, 611-667) at batch scale.  Each
 * frame's result is that of a one-batch decode.  Output memory from wg_host_alloc (pinned) is
 * written by DMA; any other memory through the HIP runtime's staged copies.  caps[i] is the
 * size in bytes of the buffer at rgba[i]: a frame whose output (strides[i] * (h - 1) + 4 * w
 * bytes) does not fit, or whose rgba[i] is NULL or strides[i] < 4 * w, is INVALID_PARAM and
 * nothing is written to it (WebPDecodeRGBAInto's output_buffer_size check, webp.go:592-594). */
int wg_decode_rgba_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                         uint8_t* const* rgba, const int32_t* strides, const size_t* caps,
                         int32_t* status, int32_t flags);

/* Frames per pipeline chunk of wg_decode_rgba_batch (0 = automatic: about a sixteenth of the
 * batch's pixels, at least 32 MPix per chunk, the last chunks halving; n >= the batch = no
 * pipelining).  INVALID_PARAM for a negative count.  No libwebp counterpart. */
int wg_ctx_set_chunk_frames(wg_ctx* ctx, int frames);

/* Where the time of the context's last wg_decode_rgba_batch went.  Host times are wall clock
 * on the calling thread; device times are HIP events summed over the chunks (the stages of
 * different chunks overlap, so they need not add up to wall_s). */
typedef struct {
  int32_t frames, chunks, host_threads, reserved;
  double wall_s;         /* the whole call                                                    */
  double parse_s;        /* entropy stage of every chunk (caller thread + pool)             */
  double parse_wait_s;   /* of wall_s: the caller waiting for a staging arena to come free  */
  double h2d_ms, kernel_ms, d2h_ms;  /* device side, summed over chunks                    */
  double h2d_bytes, d2h_bytes;
  double drain_s;        /* after the last chunk's entropy stage: waiting for the device  */
} wg_pipeline_stats;
int wg_ctx_pipeline_stats(const wg_ctx* ctx, wg_pipeline_stats* out);

/* Page-locked host memory for output buffers (hipHostMalloc): the device writes it by DMA.
 * NULL on failure.  Free with wg_host_free.  (The Go shim backs image.RGBA.Pix with it in
 * DecodeBatchInto.) */
void* wg_host_alloc(size_t bytes);
void wg_host_free(void* p);

/* Multi-GPU batch: the n frames are split into n_ctx contiguous shards, shard k
 * decoded by wg_decode_rgba_batch on ctxs[k] (normally one context per device), all shards
 * concurrently from their own host threads.  Frames are independent: nothing is exchanged
 * between devices, and every frame's output and status are those of a single-context decode.
 * Returns OK if every shard ran (check status[]), else the first failing shard's code. */
int wg_decode_rgba_batch_multi(wg_ctx* const* ctxs, int n_ctx, const uint8_t* const* data,
                               const size_t* sizes, int n, uint8_t* const* rgba,
                               const int32_t* strides, const size_t* caps, int32_t* status,
                               int32_t flags);

/* As wg_decode_rgba_batch with full output options (colorspace, cropping, flip); caps[i] is
 * checked against strides[i] * (h - 1) + bpp * w of the output window. */
int wg_decode_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                    const wg_decoder_options* opt, uint8_t* const* out, const int32_t* strides,
                    const size_t* caps, int32_t* status);

/* wg_decode_yuv_into over n frames of one batch (opt->colorspace 11 or 12): outs[i] receives frame
 * i's planes; per-frame status[i] (a frame whose buffer fails the check is INVALID_PARAM). */
int wg_decode_yuv_batch(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                        const wg_decoder_options* opt, const wg_yuva_buffer* outs, int32_t* status);

/* ---- device-resident batch (benchmarks, tests) -------------------------------------- */
typedef struct wg_batch wg_batch;

/* Parse n frames on host and upload their coefficient/mode buffers to HBM; allocates the
 * device YUV planes and RGBA outputs.  Subsequent wg_batch_run() calls execute only the
 * device path (inputs resident in HBM).  NULL on failure (status[] says why per frame). */
wg_batch* wg_batch_create(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                          int32_t flags, int32_t* status);
/* As wg_batch_create with output options; flags-only creation = colorspace RGBA, no crop. */
wg_batch* wg_batch_create_ex(wg_ctx* ctx, const uint8_t* const* data, const size_t* sizes, int n,
                             const wg_decoder_options* opt, int32_t* status);
void wg_batch_destroy(wg_batch* b);

/* Run the device DSP path for the whole batch on `stream` (NULL = ctx stream):
 * lossy frames: K1 reconstruct+deblock wavefront (+ YUV420->RGBA in its tail, or K2), K4 ALPH plane -> A;
 * lossless frames (and lossless ALPH streams): K3 inverse transforms + RGBA; then K6 (non-RGBA
 * colorspace or flip) and K5 (animation batches).  Kernel durations of the last run
 * (HIP events on that stream) are available from wg_batch_kernel_ms(). */
int wg_batch_run(wg_batch* b, void* stream);

/* Where a batch's lossy RGBA is produced.  Default (no crop window in the batch): by K1
 * itself, in the tail of each frame's workgroup (waves done with reconstruction convert
 * finished row bands while the last rows decode) -- no separate K2 launch.  separate = 1:
 * K1 writes only the planes and K2 converts them (the path cropped batches always take).
 * Both are bit-identical; replaces nothing in the reference (its EmitFancyRGB runs per row
 * inside the decode loop, io_dec.c.go:65-115). */
int wg_batch_set_emit(wg_batch* b, int separate);

/* Workgroups per frame for K1 (tests, measurement): 1 = one per frame -- coming from a split of
 * the whole batch, the kernels with the RGBA tail again when the batch can take them (no crop
 * window, no frame emitted in a mode the tail lacks); a batch set to K2 by wg_batch_set_emit(b, 1)
 * keeps K2; 2..4 = the split kernel, each frame's MB-row quads spread over that many CUs (K2
 * converts); 0 = the automatic choice, which a batch makes at creation: split when it holds
 * fewer frames than CUs and a frame has more quads than one workgroup runs at once. */
int wg_batch_set_k1_parts(wg_batch* b, int parts);

/* The YUV420->RGBA stage alone (K2: EmitFancyRGB / EmitSampledRGB, io_dec.c.go:53-115) over the batch's
 * reconstructed planes (after a wg_batch_run): the stage-roofline measurement of the
 * metric.  Its duration is reported as ms[1] by wg_batch_kernel_ms().  (Frames with alpha take A
 * from the planes the run's K4 left when the batch runs alpha-first, else A = 255.) */
int wg_batch_run_emit(wg_batch* b, void* stream);

/* Per-launch kernel durations averaged over the runs since the last query:
 * ms[0] = VP8 reconstruct+filter (K1, with its RGBA tail by default), ms[1] = YUV->RGBA (K2), ms[2] = VP8L inverse
 * transforms (K3, lossless frames and lossless ALPH streams), ms[3] = ALPH unfilter + A
 * channel (K4), ms[4] = VP8L color cache + back-references (K7, before K3), ms[5] = output
 * colorspace / flip (K6, batches created with a non-RGBA colorspace or flip), ms[6] = animation
 * canvases (K5, wg_anim_batch_create); a kernel with no frames in the batch reports 0.
 * n_ms >= 1 (entries beyond n_ms are not written). */
int wg_batch_kernel_ms(const wg_batch* b, float* ms, int n_ms);

/* Algorithmic HBM bytes per launch of K1, K2, K3, K4, K7, K6, K5;
 * K1 with its RGBA tail: records + coefficients in, RGBA out (the planes are an intermediate). */
int wg_batch_kernel_bytes(const wg_batch* b, double* bytes, int n_bytes);

int wg_batch_size(const wg_batch* b);
int wg_batch_frame_dims(const wg_batch* b, int i, int32_t* width, int32_t* height); /* output size */
int wg_batch_frame_status(const wg_batch* b, int i);
int64_t wg_batch_pixels(const wg_batch* b);

/* Copy results of frame i back to host: RGBA of the output window (stride >= 4*width; no flip,
 * whatever the batch's colorspace -- except a lossy frame without alpha or crop window in a
 * non-RGBA / flipped batch, which is written straight in the batch's colorspace and has no RGBA
 * copy: UNSUPPORTED_FEATURE; such a batch is read with wg_batch_download, and a caller that needs
 * RGBA creates the batch in MODE_RGBA), the batch's colorspace / flip (wg_batch_download, stride >=
 * bpp*width), and/or the full frame's Y/U/V planes (strides width, (width+1)/2).
 * wg_batch_download_rgba's destination may also be device memory (e.g. a torch tensor on the
 * batch's device): the copy is then device to device and the frame never crosses PCIe. */
int wg_batch_download_rgba(wg_batch* b, int i, uint8_t* rgba, int stride);
int wg_batch_download(wg_batch* b, int i, uint8_t* out, int stride);
int wg_batch_download_yuv(wg_batch* b, int i, uint8_t* y, uint8_t* u, uint8_t* v); /* lossy only */
/* Frame i's MODE_YUV / MODE_YUVA planes of a batch created with colorspace 11 / 12 (K8's output of
 * the last wg_batch_run; UNSUPPORTED_FEATURE for another batch; such a batch's wg_batch_download is
 * UNSUPPORTED_FEATURE, its lossy frames have no RGBA). */
int wg_batch_download_yuva(wg_batch* b, int i, const wg_yuva_buffer* out);

/* ---- stage entry point: YUV420 -> RGBA on device pointers ---------------------------- */
/* Fancy (fancy!=0, UpsampleRgbaLinePair, upsampling.c.go:43-107) or point-sampled
 * (EmitSampledRGB, io_dec.c.go:53-59) conversion of one frame; all pointers are device
 * pointers.  Asynchronous on `stream`.  The kernel reads planes in 16-byte (luma) and
 * 8-byte (chroma) groups, so: y and y_stride 16-byte aligned with
 * y_stride >= round_up(width, 16); u, v and uv_stride 4-byte aligned with
 * uv_stride >= round_up((width+1)/2, 8) (the batch's MB-padded planes satisfy this).
 * Anything else -> WG_STATUS_INVALID_PARAM. */
int wg_yuv420_to_rgba_device(const uint8_t* y, const uint8_t* u, const uint8_t* v,
                             int y_stride, int uv_stride, uint8_t* rgba, int rgba_stride,
                             int width, int height, int fancy, void* stream);

/* ---- stage entry point: VP8L color cache + back-references on device pointers -------- */
/* The value half of DecodeImageData's pixel loop (pkg/vp8/vp8l_dec.c.go:1038-1189; cache
 * pkg/vp8/color_cache.go:46-63) on one token stream, the form the host entropy stage hands K7
 * (one uint32 per pixel: kind in bits 31:30 -- 0 literal index into `lits`, 1 color-cache key,
 * 2 backward distance, 3 unset = 0 without a cache insert -- payload in bits 29:0).  Writes
 * the n_px coded ARGB pixels to `argb`.  Device pointers; tokens and argb 16-byte aligned;
 * cache_bits 0..11.  A token outside the stream's bounds (literal index >= n_lits, key >=
 * 1 << cache_bits, distance 0 or before the start) resolves to 0.  Asynchronous on `stream`.
 * n_px = 0 is a no-op (WG_STATUS_OK).  Null / misaligned pointers, negative counts, n_px or
 * n_lits above 2^29 - 1 (32-bit byte offsets) or cache_bits outside 0..11 ->
 * WG_STATUS_INVALID_PARAM, checked before any device call. */
int wg_vp8l_resolve_device(const uint32_t* tokens, const uint32_t* lits, int n_lits, int n_px,
                           int cache_bits, uint32_t* argb, void* stream);

/* ---- host entropy stage in the libwebp data model (tests / CPU checker) --------------- */
/* One macroblock as libwebp keeps it after parsing: VP8MBData (pkg/vp8/models.go:89-107)
 * plus the VP8FInfo filter strengths (models.go:66-71). */
typedef struct {
  int16_t coeffs[384];  /* dequantized, de-zigzagged, int16-wrapped; Y 0..15, U 16..19, V 20..23 */
  uint32_t non_zero_y;  /* 2-bit transform codes, block 0 in bits 31:30 (NzCodeBits)           */
  uint32_t non_zero_uv; /* U codes bits 7:0, V codes bits 15:8                                  */
  uint8_t is_i4x4;
  uint8_t uvmode;       /* DC=0 TM=1 V=2 H=3                                                    */
  uint8_t segment;
  uint8_t skip;
  uint8_t imodes[16];   /* i4x4: B_* modes 0..9 raster order; i16: imodes[0] = ymode           */
  uint8_t f_limit, f_ilevel, f_inner, hev_thresh;
} wg_vp8_mb;

typedef struct {
  int32_t width, height;     /* picture size                                             */
  int32_t mb_w, mb_h;        /* macroblocks                                              */
  int32_t filter_type;       /* 0 none, 1 simple, 2 complex (after bypass_filtering)    */
  int32_t num_parts;         /* token partitions                                         */
  int32_t use_segment;
  int32_t frame_offset;      /* byte offset of the VP8 frame inside `data`               */
} wg_vp8_info;

/* Parse container + VP8 headers + modes + residual tokens of a lossy frame on the host.
 * `mbs` (mb_w*mb_h entries, raster order) may be NULL to only fill `info`. */
int wg_vp8_parse(const uint8_t* data, size_t size, int flags, wg_vp8_info* info, wg_vp8_mb* mbs);

/* ---- host entropy stage of VP8L (lossless) --------------------------------------------- */
/* A lossless frame after the prefix-code walk (libwebp DecodeImageStream, reference
 * pkg/vp8/vp8l_dec.c.go), before its color cache, back-references and inverse transforms: one
 * token per coded pixel -- bits 31..30: 0 literal (bits 29..0 = index into the literal array),
 * 1 color-cache reference (key), 2 backward reference (distance in pixels), 3 unset (pixels
 * after a failing symbol, value 0) -- plus the literals.  The device resolves the tokens
 * (color cache: VP8LColorCache, color_cache.go:16-80; copies: CopyBlock32b) and applies the
 * transforms.  Transforms are listed in bitstream (read) order; they are undone in reverse.
 * Types: 0 predictor, 1 cross-color, 2 subtract-green, 3 color indexing. */
typedef struct {
  int32_t width, height, has_alpha;
  int32_t coded_width;          /* width of the entropy-coded image (< width with pixel packing) */
  int32_t num_transforms;
  int32_t transform_type[4];
  int32_t transform_bits[4];    /* tile bits, or packing bits for color indexing              */
  int32_t transform_xsize[4];   /* output width of the transform                              */
  int32_t transform_size[4];    /* uint32 words of its data (tile image / expanded palette)    */
  int32_t cache_bits;           /* color cache size 1 << cache_bits (0 = no cache)             */
  int32_t num_literals;         /* uint32 words of the literal array                           */
} wg_vp8l_info;

/* `tokens` (coded_width*height words), `literals` (num_literals words) and
 * `transform_data[i]` (transform_size[i] words) may be NULL to only fill `info`. */
int wg_vp8l_parse(const uint8_t* data, size_t size, wg_vp8l_info* info, uint32_t* tokens,
                  uint32_t* literals, uint32_t* const* transform_data);

/* ---- host stage of an ALPH plane (VP8 + alpha) ----------------------------------------- */
/* The ALPH chunk of a lossy frame (reference ALPHInit / VP8LDecodeAlphaHeader,
 * pkg/libwebp/decoder/alpha_dec.go:47-105, pkg/vp8/vp8l_dec.c.go:1493-1556). */
typedef struct {
  int32_t width, height;        /* the frame's size = the plane's size                       */
  int32_t method;               /* 0 raw bytes, 1 lossless (VP8L stream, alpha = green)      */
  int32_t filter;               /* 0 none, 1 horizontal, 2 vertical, 3 gradient             */
  int32_t pre_processing;       /* 1: level-quantized (dequantized only with dithering > 0) */
  int32_t reserved;
} wg_alpha_info;

/* Parse the ALPH chunk of `data` (a whole WebP file).  method 0: the width*height filtered
 * bytes go to `filtered`; method 1: the alpha stream's entropy stage goes to ll_info / tokens /
 * literals / transform_data exactly as wg_vp8l_parse fills them.  Any output pointer may be NULL.
 * Status as WebPDecode would report the plane: an invalid header or stream header is
 * OUT_OF_MEMORY (libwebp's ALPHInit failure path), a bad pixel stream BITSTREAM_ERROR; a frame
 * without ALPH is UNSUPPORTED_FEATURE. */
int wg_alpha_parse(const uint8_t* data, size_t size, wg_alpha_info* info, uint8_t* filtered,
                   wg_vp8l_info* ll_info, uint32_t* tokens, uint32_t* literals,
                   uint32_t* const* transform_data);

/* ---- animation (ANIM / ANMF) --------------------------------------------------------- */
/* WebPAnimInfo (reference pkg/libwebp/webp/demux.go:124-131). */
typedef struct {
  uint32_t canvas_width, canvas_height, loop_count, bgcolor, frame_count;
  uint32_t pad[4];
} wg_anim_info;

/* One frame as WebPDemuxGetFrame's iterator describes it (demux.go SynthesizeFrame): its
 * rectangle on the canvas (size from the frame's bitstream), duration, disposal / blending and
 * its fragment -- the bytes from its ALPH chunk (if any) to the end of its image chunk, which
 * decode as a standalone input. */
typedef struct {
  int32_t x_offset, y_offset, width, height, duration;
  int32_t dispose_background;   /* WEBP_MUX_DISPOSE_BACKGROUND                              */
  int32_t no_blend;             /* WEBP_MUX_NO_BLEND                                        */
  int32_t has_alpha;
  uint64_t fragment_offset, fragment_size;
} wg_anim_frame;

/* Host-only demux (WebPDemux + WebPDemuxGetFrame): a still image is a one-frame animation.
 * Fills info and up to max_frames frames (frames may be NULL).  BITSTREAM_ERROR for an invalid
 * container, NOT_ENOUGH_DATA for truncated data. */
int wg_anim_demux(const uint8_t* data, size_t size, wg_anim_info* info, wg_anim_frame* frames, int max_frames);

/* Decode every frame of an animation and composite the canvases on the device (replaces the
 * WebPAnimDecoderNew + WebPAnimDecoderGetNext loop, anim_decode.go:66-433; MODE_RGBA).
 * canvases: frame_count * canvas_height * canvas_width * 4 bytes (stride 4 * canvas_width);
 * timestamps: frame_count ints (ms, end of each frame, as GetNext reports).  The frames decode
 * as one batch (K1..K4), then K5 composites.  Returns the first failing frame's status. */
int wg_anim_decode(wg_ctx* ctx, const uint8_t* data, size_t size, uint8_t* canvases, int32_t* timestamps,
                   int32_t flags);

/* The same animation decode kept resident in HBM (benchmarks, tests): the frames' inputs
 * parsed and uploaded once, then every wg_batch_run() runs K1..K4 over the frames and K5 over
 * the canvases (its time is wg_batch_kernel_ms' seventh entry).  NULL on failure, *status says
 * why (the first failing frame's status, as WebPAnimDecoderGetNext stops there). */
wg_batch* wg_anim_batch_create(wg_ctx* ctx, const uint8_t* data, size_t size, int32_t flags, int32_t* status);
/* canvas size and frame count of an animation batch */
int wg_anim_batch_info(const wg_batch* b, int32_t* canvas_width, int32_t* canvas_height, int32_t* frames);
/* every canvas of the last run (frames * canvas_height * canvas_width * 4 bytes; cap checked)
 * and the frames' end timestamps (ms) */
int wg_anim_batch_download(wg_batch* b, uint8_t* canvases, size_t cap, int32_t* timestamps);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif /* GOWEBP_AMD_H_ */
