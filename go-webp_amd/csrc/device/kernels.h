// Launchers of the device kernels (host-callable).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

#include "../device_format.h"

namespace wg {

// K1: fused reconstruction + loop filter, one 1024-thread workgroup per frame.
size_t vp8_recon_lds_bytes(int mb_w);
int vp8_recon_max_mb_w();
// d_err: device int, OR-ed with 1 if a wave gave up waiting (bounded spin).
// split_parts >= 2: the split kernel (split_parts workgroups per frame, every frame, no RGBA
// tail; `epoch` tags its part-boundary flags and must differ from the previous launch's on the
// same descriptors); `slab`: MB-row quads per part (one per reconstructing wave, at most 12; 0 = 12).
hipError_t launch_vp8_recon_filter(const FrameDesc* d_frames, int n_frames, int max_mb_w, bool lds_frames,
                                   bool wide_frames, int* d_err, hipStream_t stream, int split_parts = 1,
                                   uint32_t epoch = 0, int slab = 0);

// K2: YUV420 -> RGBA (fancy 9-3-3-1 upsampling or point sampling) over a batch.
// `single` (when non-null, n_frames == 1) is passed by value instead of d_frames.
hipError_t launch_yuv_to_rgba(const FrameDesc* d_frames, const FrameDesc* single, int n_frames,
                              int max_w, int max_h, int fancy, hipStream_t stream, bool modes = false);

// K3: VP8L inverse transforms + BGRA->RGBA, one 1024-thread workgroup per lossless frame.
size_t vp8l_lds_bytes();
// Frames are grouped by variant (vp8l_variant(): 0 generic, 1..4 compile-time predictor
// passes); d_frames holds group 0 first, then 1..4; group_count[v] frames each.
// d_err: OR-ed with 2 if a wave gave up waiting (bounded spin).
constexpr int kVP8LVariants = 5;
int vp8l_variant(const int* types, const int* bits, const int* tiles, int n_stages);  // stages in application order
hipError_t launch_vp8l_transforms(const LLDesc* d_frames, const int* group_count, int* d_err, hipStream_t stream);

// K7: VP8L color cache + back-references (tokens -> coded ARGB), one 1024-thread workgroup per
// lossless stream; runs before K3.  d_err: OR-ed with 4 on an invalid token.
// d_descs null: the single stream `single` (stage entry).  The first n_w64 of d_descs take the
// 64-mask-word instantiation (vp8l_resolve_w64(cache_bits): one window per block), the rest the
// 32-word one.
bool vp8l_resolve_w64(int cache_bits);
// The first n_alpha of the 64-word streams write their alpha bytes too (LLTokDesc::afilt), the
// first n_tiled of those into band tiles (LLTokDesc::atile).
hipError_t launch_vp8l_resolve(const LLTokDesc* d_descs, const LLTokDesc* single, int n, int* d_err,
                               hipStream_t stream, int n_w64 = 0, int n_alpha = 0, int n_tiled = 0);

// K4: ALPH planes (unfilter) -> A bytes of the RGBA output, one 1024-thread workgroup per
// plane; runs after K2 and K3.
// n_wave: planes with filter vertical / gradient (a second kernel instantiation, one workgroup each).
hipError_t launch_alpha(const AlphaDesc* d_frames, int n_frames, hipStream_t stream, int n_wave);

// K6: output colorspace / cropping window / flip, RGBA -> WEBP_CSP_MODE (0..10) bytes.
hipError_t launch_emit(const EmitDesc* d_frames, int n_frames, int max_pixels, hipStream_t stream);

// K8: MODE_YUV / MODE_YUVA output planes of every frame (YuvaDesc): lossy windows copied from the
// reconstructed planes, lossless RGBA converted (ConvertToYUVA), A from the alpha plane / RGBA.
// max_uw / max_uh: the largest chroma window.
hipError_t launch_emit_yuva(const YuvaDesc* d_frames, int n_frames, int max_uw, int max_uh, hipStream_t stream);

// K5: animation canvases (frames in display order, already decoded) -> n_frames canvases of
// canvas_w x canvas_h RGBA.
hipError_t launch_anim_compose(const AnimFrameDesc* d_frames, int n_frames, uint8_t* d_canvases, int canvas_w,
                               int canvas_h, hipStream_t stream);

}  // namespace wg
