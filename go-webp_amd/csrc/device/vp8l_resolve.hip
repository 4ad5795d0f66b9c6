// K7: VP8L color cache + LZ77 back-references on the device (config C5's "ColorCache on
// device").  Replaces the value half of the reference's symbol loop:
//   DecodeImageData        pkg/vp8/vp8l_dec.c.go:1038-1189 (copies :1124, cache :1105-1109,
//                          :1141-1153)
//   VP8LColorCache         pkg/vp8/color_cache.go:16-80 (hash 0x1e35a7bd :46-48, insert
//                          :50-55, lookup :57-63)
// The host walks the prefix codes and leaves one token per pixel (device_format.h kTok*):
// a literal's index, a cache key, or a backward distance.  This kernel turns the tokens into
// the coded ARGB image that K3 (vp8l_transforms.hip) inverts.
//
// What a cache lookup returns.  libwebp inserts EVERY pixel in scan order and a lookup of key
// k returns the last pixel inserted with hash k.  A pixel that came from the cache re-inserts
// the value it read from slot k into slot k (its hash is k), so only literals and copied
// pixels ("updaters") ever change a slot: lookup(k) at pixel i = the value of the last
// updater before i whose hash is k, or 0 if there is none (the cache is calloc'd).  A lookup
// of a never-written slot k returns 0 and inserts it into slot hash(0) = 0: harmless for
// k = 0 (encoders emit exactly that for black pixels: the empty slot 0 already matches), not
// for k != 0 (a stream no encoder writes) -- that case takes the exact serial path below.
//
// Geometry.  One 1024-thread workgroup per stream, walking the image in blocks of 4096 pixels
// (4 consecutive per thread) in scan order; the cache (up to 2048 slots) lives in LDS.  Two ways to
// resolve a block: dense blocks (cache_bits <= 7, below: kW64) need no ranks; the others do.  The
// updaters of a block get RANKS (their order in the block, a block-wide prefix count: known
// before any value is, since whether a pixel is an updater depends on its token only).  Per
// key, a bitmask over ranks marks the block's updaters with that hash, so a lookup at pixel i
// with key k finds "the last updater before i with hash k" as the highest set bit below i's
// rank count -- one or two LDS words, however many updaters the key has.  (C5's blocks hold
// ~143 updaters, and ~400 of their ~3,950 lookups have updaters of their key on both sides.)
// The masks hold 64 x W ranks per key, W = min(32, 8192 >> cache_bits) (64 KB of LDS); a block
// with more updaters than that runs as 2..16 consecutive windows of whole waves, each with its
// own masks, the slot table carried from window to window.
//
// Per window: (1) updaters with known values -- literals, copies from before the block (the
// previous block from LDS, older ones from the already-final image) -- register: value by
// rank, mask bit, per-key summary of non-empty mask words, per-key last rank.  (2) rounds
// until nothing is pending (one without in-block copies, C5's case): (a) every lookup before
// the first pending copy resolves (all updaters before it have known hashes); (b) every pending
// copy whose source is known takes its value and registers, the others jump their source
// pointer one link further back along a chain of pending copies (pointer jumping: log-depth
// chains); the earliest pending pixel always resolves, so the rounds end, and a cap sends the
// window to the serial path.  (3) each key's last updater writes the slot and clears the key's
// masks.  A window with a bad token, a lookup of a never-written slot k != 0, or too many
// rounds is redone, with the rest of its block, exactly in scan order by one lane (the
// reference loop over the same LDS table): always correct, slow, never taken by encoder
// output so far.  (Bad tokens -- out-of-range literal index, key or distance -- are only
// checked for caller streams of the stage entry; the host entropy stage's streams are in
// bounds by construction, LLTokDesc::trusted.)
//
// Latency: tokens are loaded two blocks ahead and literal values one block ahead, so a block
// waits on HBM only for copies that reach back more than one block.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 1024;
constexpr int kWaves = kThreads / 64;
constexpr int kPer = 4;                   // consecutive pixels per thread
constexpr int kBlock = kThreads * kPer;   // 4096 pixels per block
constexpr int kWavePx = 64 * kPer;        // pixels per wave in a block
constexpr int kSlots = 2048;              // 1 << MAX_CACHE_BITS (format_constants.go)
constexpr int kMaskWords = 8192;          // 64 KB of 64-bit rank masks, split over the keys
constexpr int kMaxW = 32;                 // mask words per key (the summary is 32 bits)
constexpr int kW64Bits = 7;               // kW64: cache_bits <= 7 (<= 128 keys x 64 words)
constexpr int kKeysW64 = 1 << kW64Bits;
constexpr int kMaxRounds = 32;
constexpr int kWalk = 8;                  // dense blocks: links a pending copy walks per round
constexpr uint8_t kKnown = 1, kPendCopy = 2, kPendLookup = 3;
constexpr uint32_t kDropOff = 0xffffffc0u;  // buffer offset past any stream: loads return 0

__device__ __forceinline__ uint32_t hash_px(uint32_t v, int shift) { return (v * 0x1e35a7bdu) >> shift; }

// number of set bits of `m` in lanes below this one
__device__ __forceinline__ int count_below(uint64_t m) {
  return (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

}  // namespace

// Measurement build only (make VARIANT=timing): block / window / round counts and wave 0's
// cycles per phase.
#ifdef WG_K7_STATS
// counts: 0 blocks, 1 serial windows, 2 rounds, 3 windows, 9 empty-slot lookups, 10 round caps;
// each wave's cycles: 8 token classification (waits for the prefetched literal values), 15
// previous-block copies + the previous block's store, 14 the next blocks' loads, 4 ranks +
// barrier, 11 registration, 12 lookups, 5 copies (rounds b), 13 slot table, 6 serial path,
// 7 end of block
__device__ unsigned long long g_k7_stats[16];
__device__ unsigned long long g_k7_wave[kWaves][16];  // per wave (lane 0): the same phase cycles
// The accumulators live in LDS (k7_lds[wave][i], counts in wave 0's row) and the clock in a
// scalar pair: per-lane register accumulators spilled 29 VGPRs in the 128-VGPR kernel, and the
// scratch traffic skewed the phase split (the timing build ran 65 % slower than the product).
#define K7_T(i)                                                      \
  do {                                                               \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                \
    if (lane == 0) atomicAdd(&k7_lds[wave][i], (unsigned long long)(t_ - k7_t)); \
    k7_t = t_;                                                       \
  } while (0)
#define K7_COUNT(i, v)                                               \
  do {                                                               \
    if (tid == 0) atomicAdd(&k7_lds[0][i], (unsigned long long)(v)); \
  } while (0)
#else
#define K7_T(i) (void)0
#define K7_COUNT(i, v) (void)0
#endif

// kW64 (streams with cache_bits <= 7, none included, chosen by the host): the instantiation for
// dense blocks -- alpha planes and flat content, nearly every pixel a copy, a few lookups -- which
// resolve without ranks or masks (round 6; the block body's dense branch, steps R H L J T there):
// copies pointer-jump with the lookups as roots (a slot only holds values of its own hash, so a
// lookup and its copies insert under its key before the value is known), a per-wave last pixel
// per key gives each lookup its source, and the chains are walked several links per round.
// C5-like streams (cache_bits 10, ~143 updaters per block among ~3,950 lookups) keep the 32-word
// instantiation: rank masks suit sparse updaters (its machine code is unchanged by the dense path).
// kSingle: the one stream `single` passed by value (the stage entry wg_vp8l_resolve_device; err may
// be null there: bad tokens then only resolve to 0, the serial path's rule); else stream
// blockIdx.x of `descs`.  (Two instantiations: a descriptor chosen at run time between the two
// loses its uniformity and the pointers' address space -- flat loads and spills.)
// kAlpha: the 8-bit alpha streams whose filtered bytes K7 writes too (LLTokDesc::afilt): 1 in
// width-byte rows, 2 rows 1.. in band tiles (LLTokDesc::atile).  Instantiations of their own, so the
// other streams' code is unchanged (measured: the alpha code's mere presence cost c3a's K7 1.7 %,
// the tiles' c3av's 3 %).
template <bool kSingle, bool kW64, int kAlpha>
__global__ void __launch_bounds__(1024) vp8l_resolve_kernel(const LLTokDesc* __restrict__ descs, LLTokDesc single,
                                                            int* err) {
  __shared__ uint64_t mask[kMaskWords];          // per key k: words k*W .. k*W+W-1, bit = rank in window
  __shared__ uint32_t summ[kSlots];              // per key: mask words holding a bit
  // per key: x = 1 + the window's last updater rank (0 none), y = the slot (VP8LColorCache.colors_):
  // one 8-byte read gives a lookup both
  __shared__ uint2 slotrec[kSlots];
  __shared__ uint32_t slot_set[kSlots / 32];     // slot written at least once
  __shared__ __attribute__((aligned(16))) uint32_t uval[kBlock];    // window updater values by rank
                                                                     // (serial path: the block's tokens)
  // this / the previous block's values (two objects, not one array: the literal values of block b + 1
  // are loaded straight into the previous block's array, and the waitcnt pass must see that this
  // block's array is not the loads' target)
  __shared__ __attribute__((aligned(16))) uint32_t val0[kBlock];
  __shared__ __attribute__((aligned(16))) uint32_t val1[kBlock];
  __shared__ __attribute__((aligned(16))) int16_t ref[kBlock];  // pending copy: source pointer (pointer jumping)
  __shared__ __attribute__((aligned(16))) uint8_t st[kBlock];  // kKnown / kPendCopy / kPendLookup
  __shared__ __attribute__((aligned(16))) uint32_t wsum[kWaves];  // updaters per wave of the block
  __shared__ int first_pend[2];                  // per round parity: first pending copy (local)
  // this window goes serial; one flag per block parity: with no barrier at a block's end, a
  // wave already in block b+1 may raise its flag while a slower one has yet to read block b's
  __shared__ int slow[2];
  __shared__ int orflag[4];                      // sync_or: a ring of flag words
  __shared__ uint2 sscr[kWaves * 64];            // a wave's straddling lookups, compacted (key, rank)
  __shared__ int rscan[kWaves];                  // in-block copies: each wave's last run root (max-scan)
  const LLTokDesc D = kSingle ? single : descs[blockIdx.x];
  if (!D.valid) return;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = D.n_px, cache_bits = D.cache_bits;
  const int nkeys = cache_bits > 0 ? 1 << cache_bits : 0;
  const int shift = 32 - cache_bits;
  const int W = cache_bits > 0 ? min(kMaxW, kMaskWords >> cache_bits) : 1;  // mask words per key (32-word path)
  const int cap = 64 * W;                                                              // ranks per window
  // Buffer descriptors: out-of-range loads return 0 with no branch, so the prefetches below are
  // straight-line code and the waitcnt pass can count them precisely (a load under a lane
  // branch makes it wait for every outstanding load at the join).
  const __amdgpu_buffer_rsrc_t tok_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(D.tokens), 0, 4 * n, 0x00020000);
  const __amdgpu_buffer_rsrc_t lit_rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(D.lits), 0, 4 * D.n_lits, 0x00020000);
  const __amdgpu_buffer_rsrc_t out_rs = __builtin_amdgcn_make_buffer_rsrc(D.coded, 0, 4 * n, 0x00020000);
  for (int i = tid; i < kMaskWords; i += kThreads) mask[i] = 0;
  for (int i = tid; i < kSlots; i += kThreads) {
    slotrec[i] = make_uint2(0u, 0u);
    summ[i] = 0;
  }
  if (tid < kSlots / 32) slot_set[tid] = 0;
  if (tid == 0) {
    slow[0] = slow[1] = 0;
    first_pend[0] = first_pend[1] = kBlock;
  }
  if (tid < 4) orflag[tid] = 0;
  // A barrier that also returns whether any thread's p was set: one s_barrier (HIP's
  // __syncthreads_or costs three).  Flag word k & 3 is set before barrier k and read after it;
  // word (k + 2) & 3, last read before barrier k - 1, is cleared after barrier k for call k + 2.
  // A workgroup barrier for LDS hand-offs only: __syncthreads() also waits vmcnt(0) while an
  // LDS-destination load is in flight, which would drain the literal prefetch at every barrier.
  // (Global memory needs no fence here: a block's stores are complete before the wait for the
  // next block's staged literals, ahead of that block's rank barrier; see store_block.)
  auto bar = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
  int orseq = 0;
  auto sync_or = [&](bool p) -> bool {
    const int slot = orseq & 3;
    if (p) orflag[slot] = 1;
    bar();
    const bool r = orflag[slot] != 0;
    if (tid == 0) orflag[(slot + 2) & 3] = 0;
    ++orseq;
    return r;
  };

  const int nblocks = (n + kBlock - 1) / kBlock;
  const int li0 = kPer * tid;
  // (tokens past the stream read as 0 and are treated as unset by position in step 1)
  auto load_tokens = [&](int b, uint32_t* tk) {
    const uint32_t p = (uint32_t)(b * kBlock + li0);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(tok_rs, b < nblocks ? 4u * p : kDropOff, 0, 0);
    tk[0] = q.x, tk[1] = q.y, tk[2] = q.z, tk[3] = q.w;
  };
  // literal values straight into LDS: slot j of the wave's 64 threads at stage[wave * 256 + 64 j +
  // lane] of the block's value array (lane-linear, as an LDS-destination load writes); each
  // thread reads its four back in step 1 before its own values overwrite the wave's range
  auto load_lits = [&](const uint32_t* tk, uint32_t* stage) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const bool is_lit = (tk[j] & ~kTokPayload) == kTokLiteral;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(lit_rs, stage + wave * kWavePx + 64 * j,
                                               4, is_lit ? 4u * (tk[j] & kTokPayload) : kDropOff, 0, 0, 0);
    }
  };
  // Software pipeline: tokens two blocks ahead, literal values one block ahead.  Two register
  // sets (A for even blocks, B for odd), the block body inlined once per set: rotating one set
  // through copies at the loop latch would make every copy wait for its load (a register with
  // a load in flight cannot be read), collapsing the prefetch distance to nothing.
  uint32_t tkA[kPer], tkB[kPer];
  load_tokens(0, tkA);
  load_tokens(1, tkB);
  load_lits(tkA, val0);
  __syncthreads();
#ifdef WG_K7_STATS
  __shared__ unsigned long long k7_lds[kWaves][16];
  if ((tid & 63) < 16) k7_lds[wave][tid & 63] = 0;
  __syncthreads();
  uint64_t k7_t = __builtin_amdgcn_s_memtime();
#endif

  // Per-pixel state of a thread's four pixels, packed in one register: bits 2j..2j+1 the
  // pixel's pending kind, bit 8+j updater.
  constexpr uint32_t kPK = 0, kPC = 1, kPL = 2, kPF = 3;  // known / copy / lookup / far copy
  auto pk = [](uint32_t ps, int j) { return (ps >> (2 * j)) & 3u; };
  auto is_upd = [](uint32_t ps, int j) { return (ps >> (8 + j)) & 1u; };
  auto set_known = [](uint32_t& ps, int j) { ps &= ~(3u << (2 * j)); };
  // a slot beyond any rank for stores that are not registrations (ranks < cap <= 2048): one per
  // thread, so the dropped stores of one instruction do not collide on one address (kW64: ranks
  // reach 4095, the dummies go to the straddle scratch, rewritten before every read of it)
  const int uval_dummy = 2048 + tid;  // (kW64: not used; its ranks reach 4095)
  // A block's values go to the coded image (K3's input) from LDS during the NEXT block, ahead of
  // that block's prefetches: in the in-order vmcnt, a store issued at the end of its own block
  // would sit between the next block's loads and their first use.  Copies reaching back past
  // the previous block read this image; they come two blocks later, after a barrier that every
  // wave reaches only once its prefetch loads -- issued after its stores -- have completed.
  // 8-bit alpha streams (LLTokDesc::afilt): the four pixels' filtered alpha bytes too -- each
  // coded pixel's green holds 1 << a_cbits bundled map indices (low bits first), or is the byte
  // itself without a map (ColorIndexInverseTransform, lossless.go:428-459; ExtractAlphaRows,
  // vp8l_dec.c.go:1462-1489 keeps the green).  The map's <= 16 green bytes sit in a_pg: v_perm
  // on four indices at once.  Rows of the coded image map to rows of the plane, so the bytes of
  // four coded pixels within a row are contiguous: one 4-byte (no map) or 8-byte (5..16 colours:
  // two indices per coded pixel, libwebp's usual alpha map) store when aligned; maps of 2..4
  // colours, row ends and unaligned rows byte by byte (kept small: the kernel's code size shows
  // in its time).
  const __amdgpu_buffer_rsrc_t af_rs =
      __builtin_amdgcn_make_buffer_rsrc(D.afilt, 0, D.afilt ? D.a_width * D.a_height : 0, 0x00020000);
  auto palq = [&](uint32_t i4) {  // four map indices (bytes of i4) -> their green bytes
    const uint32_t sel = i4 & 0x07070707u;
    const uint32_t lo = __builtin_amdgcn_perm(D.a_pg[1], D.a_pg[0], sel), hi = __builtin_amdgcn_perm(D.a_pg[3], D.a_pg[2], sel);
    const uint32_t m = ((i4 >> 3) & 0x01010101u) * 0xffu;
    return (hi & m) | (lo & ~m);
  };
  const int a_ncb = (D.a_width + 15) >> 4;
  const __amdgpu_buffer_rsrc_t at_rs = __builtin_amdgcn_make_buffer_rsrc(
      D.atile, 0, kAlpha == 2 ? ((D.a_height - 1 + 63) >> 6) * a_ncb * 1024 : 0, 0x00020000);
  auto div_cw = [&](int p) {  // (a multiply-shift: the host's magic number, p < 2^28)
    return (int)(((uint64_t)(uint32_t)p * D.a_cw_m) >> (28 + D.a_cw_s));
  };
  // (kAlpha) row and column of this thread's first pixel of the block store_block writes next:
  // stepped by a block's rows and columns per store instead of a division per block
  int a_y = 0, a_x = 0, a_q = 0, a_r = 0;
  if constexpr (kAlpha != 0) {
    a_q = div_cw(kBlock), a_r = kBlock - a_q * D.a_cw;
    a_y = div_cw(li0), a_x = li0 - a_y * D.a_cw;
  }
  auto store_alpha = [&](int pos0, const int yc, const int xc, const uint32_t* ov) {
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const int cw = D.a_cw, W = D.a_width, cb = D.a_cbits;
    // byte (y, x): row-major in afilt, or (atile, rows >= 1) in its band tile
    auto tile_off = [&](int y, int x) {
      const int r = y - 1;
      return (uint32_t)((((r >> 6) * a_ncb + (x >> 4)) << 10) + ((r & 63) << 4) + (x & 15));
    };
    const uint32_t g0 = (ov[0] >> 8) & 0xffu, g1 = (ov[1] >> 8) & 0xffu, g2 = (ov[2] >> 8) & 0xffu, g3 = (ov[3] >> 8) & 0xffu;
    const int x0 = xc << cb, nbytes = kPer << cb;
    const bool tiled = kAlpha == 2 && yc >= 1;
    const __amdgpu_buffer_rsrc_t rs = tiled ? at_rs : af_rs;
    // (tiles: the bytes of four coded pixels lie in one tile row, 16 for cbits 3 in each of two)
    const uint32_t base = tiled ? tile_off(yc, x0) : (uint32_t)(yc * W + x0);
    const bool whole = xc + kPer <= cw && pos0 + kPer <= n && x0 + nbytes <= W;
    if (whole && cb == 0 && !D.a_pal && (base & 3) == 0) {
      __builtin_amdgcn_raw_buffer_store_b32(g0 | g1 << 8 | g2 << 16 | g3 << 24, rs, base, 0, 0);
    } else if (whole && cb == 1 && (base & 7) == 0) {
      const uint32_t a = palq((g0 & 15) | (g0 >> 4) << 8 | (g1 & 15) << 16 | (g1 >> 4) << 24);
      const uint32_t b = palq((g2 & 15) | (g2 >> 4) << 8 | (g3 & 15) << 16 | (g3 >> 4) << 24);
      __builtin_amdgcn_raw_buffer_store_b64(u32x2{a, b}, rs, base, 0, 0);
    } else {  // row ends, the stream's end, unaligned rows: byte by byte (one flat loop: small code)
      const int per = 1 << cb, bpp = 8 >> cb;
#pragma unroll 1
      for (int i = 0; i < nbytes; ++i) {
        const int j = i >> cb, k = i & (per - 1), p = pos0 + j;
        const int y = div_cw(p), x = ((p - y * cw) << cb) + k;
        const uint32_t w = j == 0 ? ov[0] : j == 1 ? ov[1] : j == 2 ? ov[2] : ov[3];
        const uint32_t g = (w >> 8) & 0xffu;
        const uint32_t idx = (g >> (k * bpp)) & ((1u << bpp) - 1u);
        const uint32_t v = D.a_pal ? palq(idx) & 0xffu : g;
        const bool t = kAlpha == 2 && y >= 1;
        // (past the stream or the row: an offset past the buffer, dropped)
        const uint32_t off = p >= n || x >= W ? 0x80000000u : t ? tile_off(y, x) : (uint32_t)(y * W + x);
        __builtin_amdgcn_raw_buffer_store_b8(v, t ? at_rs : af_rs, off, 0, 0);
      }
    }
  };
  auto store_block = [&](int b, const uint32_t* vals) {
    const int pos0 = b * kBlock + li0;
    const uint4 o = *reinterpret_cast<const uint4*>(&vals[li0]);
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    if (pos0 + kPer <= n) {
      __builtin_amdgcn_raw_buffer_store_b128(u32x4{o.x, o.y, o.z, o.w}, out_rs, 4u * (uint32_t)pos0, 0, 0);
    } else {  // the stream's last pixels (the buffer range drops what lies past it)
      const uint32_t ov[kPer] = {o.x, o.y, o.z, o.w};
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        __builtin_amdgcn_raw_buffer_store_b32(ov[j], out_rs, pos0 + j < n ? 4u * (uint32_t)(pos0 + j) : kDropOff, 0, 0);
    }
    if constexpr (kAlpha != 0) {
      if (pos0 < n) {
        const uint32_t ov[kPer] = {o.x, o.y, o.z, o.w};
        store_alpha(pos0, a_y, a_x, ov);
      }
      a_x += a_r, a_y += a_q;
      if (a_x >= D.a_cw) a_x -= D.a_cw, ++a_y;
    }
  };
  // LDS atomics without return as inline asm: the waitcnt pass makes every LDS atomic wait
  // vmcnt(0) while an LDS-destination load is in flight (it cannot tell the target apart), which
  // would drain the literal prefetch in every registration.  No result, so nothing waits on them;
  // bar() orders them (lgkmcnt(0)), and a wave's LDS operations execute in order.
  auto lds_addr = [](const void* p) { return (uint32_t)(size_t)p; };
  auto ds_or_b64 = [&](uint64_t* p, uint64_t v) { asm volatile("ds_or_b64 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory"); };
  auto ds_or_b32 = [&](uint32_t* p, uint32_t v) { asm volatile("ds_or_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory"); };
  auto ds_max_u32 = [&](uint32_t* p, uint32_t v) { asm volatile("ds_max_u32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory"); };
  auto ds_min_i32 = [&](int* p, int v) { asm volatile("ds_min_i32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory"); };
  auto ds_write_u32 = [&](uint32_t* p, uint32_t v) { asm volatile("ds_write_b32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory"); };
  // mask bit, summary, last rank of an updater whose value is in uval[r]
  auto reg_hash = [&](int r, uint32_t x) {
    const uint32_t h = hash_px(x, shift);
    ds_or_b64(&mask[h * W + (r >> 6)], 1ull << (r & 63));
    ds_or_b32(&summ[h], 1u << (r >> 6));
    ds_max_u32(&slotrec[h].x, (uint32_t)r + 1u);
  };
  // step 3 for one registered updater: if it is its key's last in the window, write the slot
  // (unless the window goes serial) and clear the key's masks.  The other updaters of the key
  // only read its last rank, which the last one may already have reset (then they read 0: not
  // theirs either).
  auto table_update = [&](int r, uint32_t x, bool go_serial) {
    const uint32_t h = hash_px(x, shift);
    if (slotrec[h].x == (uint32_t)r + 1u) {
      for (uint32_t sm = summ[h]; sm; sm &= sm - 1) mask[h * W + __builtin_ctz(sm)] = 0;
      summ[h] = 0;
      if (!go_serial) {
        slotrec[h] = make_uint2(0u, x);
        ds_or_b32(&slot_set[h >> 5], 1u << (h & 31));
      } else {
        slotrec[h].x = 0u;
      }
    }
  };
  const int lane = tid & 63;
  static_assert(kBlock >= 2048 + kThreads, "uval: ranks below 2048, one dummy slot per thread above");
  auto wave_sync = [] {  // intra-wave LDS hand-off: a wave's DS ops execute in order
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };

  // A lookup whose key has window updaters on both sides of it: the highest bit of the key's
  // rank mask below rr (the window updaters before the pixel), from the summary's top one or
  // two words; ~0 if none.
  auto straddle_idx = [&](uint32_t k, int rr) -> uint32_t {
    const int wt = (rr - 1) >> 6;
    int w1, w2;
    bool h1, h2;  // the top / second non-empty words below the pixel exist
    {
      const uint32_t sm = rr <= 0 ? 0u : summ[k] & (wt >= 31 ? ~0u : (2u << wt) - 1u);
      w1 = sm ? 31 - __builtin_clz(sm) : 0;
      const uint32_t sm2 = sm & ~(1u << w1);
      w2 = sm2 ? 31 - __builtin_clz(sm2) : 0;
      h1 = sm != 0, h2 = sm2 != 0;
    }
    const uint64_t m1 = h1 ? mask[k * W + w1] : 0ull;
    const uint64_t m2 = h2 ? mask[k * W + w2] : 0ull;
    // the top word is the pixel's own word: keep only the ranks below it (lb = 1..64)
    const int lb = rr - 64 * w1;
    const uint64_t top = lb < 64 ? m1 & ((1ull << lb) - 1ull) : m1;
    const uint64_t m = top ? top : m2;
    const int w = top ? w1 : w2;
    return m ? (uint32_t)(64 * w + 63 - __builtin_clzll(m)) : ~0u;
  };

  // one block: tk_in / lv_in its tokens and literal values; tk_nxt the next block's tokens
  // (arrived), whose literal loads go out into lv_nxt, and tk_in is reloaded with the tokens two
  // blocks on, once step 1 has consumed it.
  //
  // Instruction economy: K7 is bound by VALU issue (a wave64 VALU op holds its SIMD for four
  // cycles and the four waves of a SIMD take turns; per-wave phase timings show the youngest
  // wave of each SIMD setting every barrier's pace).  So the per-pixel work is branch-free
  // (selects; a wave walks every side of a lane branch), the rare cases sit behind wave-uniform
  // branches, and the per-updater work (3.5 % of C5's pixels) runs one updater per lane over
  // the wave's compacted updaters instead of once per pixel slot.
  auto block = [&](const int b, uint32_t* tk_in, uint32_t* tk_nxt, uint32_t* vcur,
                   uint32_t* vprv) __attribute__((always_inline)) {
    const int base = b * kBlock;

    // ---- 1. tokens: literals, copies from before the block, unset pixels are known; in-block
    //         copies and lookups are pending.  Literals and copies are updaters (ranked).  A
    //         lookup's key / a copy's distance stays in `aux`.  (Literal values come from buffer
    //         loads that read 0 out of range.)
    uint32_t ps = 0, nearm = 0;
    uint32_t v[kPer], aux[kPer];
    bool bad = false;
    if (base + kBlock > n) {  // the stream's last block: pixels past its end are unset
#pragma unroll
      for (int j = 0; j < kPer; ++j) tk_in[j] = base + li0 + j < n ? tk_in[j] : kTokUnset;
    }
    // The staged literal values (buffer_load ... lds, issued last in the previous block) have
    // landed before step 1 reads them, and so have this wave's stores of block b - 2 before the
    // rank barrier below (far copies of other waves read them).  The waitcnt pass would place the
    // same wait only because it tells val0 from val1; this one does not depend on that analysis
    // (tests/test_k7_isa.py checks that no path reaches these reads from an LDS-DMA load without
    // a vmcnt(0)).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int li = li0 + j;
      const uint32_t t = tk_in[j], kind = t >> 30, pl = t & kTokPayload;
      const bool is_copy = kind == 2, is_cache = kind == 1;
      // out of the stream's bounds: literal index >= n_lits, key >= 1 << cache_bits, distance 0
      // or before the start ((pl - 1) >= pos, unsigned) -- one compare against a per-kind limit
      // (tokens of the host entropy stage are in bounds by construction: D.trusted skips this)
      if (!D.trusted) {
        const uint32_t lim = kind == 0 ? (uint32_t)D.n_lits : is_cache ? (uint32_t)nkeys : is_copy ? (uint32_t)(base + li) : ~0u;
        bad |= (is_copy ? pl - 1u : pl) >= lim;
      }
      // copies: in-block source (pl <= li), previous block (li < pl <= li + 4096), older
      const bool inb = is_copy & (pl - 1u < (uint32_t)li);  // (pl = 0 wraps: not in-block)
      const bool farc = is_copy & (pl > (uint32_t)(li + kBlock));
      const uint32_t code = inb ? kPC : farc ? kPF : is_cache ? kPL : kPK;
      ps |= code << (2 * j) | (~kind & 1u) << (8 + j);  // updaters: kinds 0 (literal) and 2 (copy)
      nearm |= (uint32_t)(is_copy & !inb & !farc) << j;
      v[j] = vcur[wave * kWavePx + 64 * j + lane];
      // (kW64: a lookup's value register and vcur entry hold its key until it resolves)
      if (kW64 && is_cache) v[j] = pl & (uint32_t)(nkeys - 1) & (kKeysW64 - 1);
      aux[j] = is_cache ? pl & (kSlots - 1) : pl;
    }
    K7_T(8);
    if (__any(nearm != 0)) {  // copies from the previous block, in LDS
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const bool nc = (nearm >> j) & 1u;
        const uint32_t x = vprv[nc ? (int)(li0 + j + kBlock) - (int)aux[j] : 0];
        v[j] = nc ? x : v[j];
      }
    }
    *reinterpret_cast<uint4*>(&vcur[li0]) = make_uint4(v[0], v[1], v[2], v[3]);
    if (b > 0) store_block(b - 1, vprv);
    K7_T(15);
    // the tokens two blocks on go out now (tk_in is consumed)
    load_tokens(b + 2, tk_in);
    K7_T(14);
    if (bad) {
      if (err) atomicOr(err, 4);
      slow[b & 1] = 1;
    }
    // ranks: updaters before each pixel, a block-wide prefix count (per-thread count 0..4 in
    // three ballots).  wsum: the wave's updaters, bit 16 a copy reaching back past the last
    // block, bit 17 an in-block copy (pending), bit 18 (kW64) a cache lookup.
    const uint32_t cm = ps & (ps >> 1) & 0x55u, pm = ps & ~(ps >> 1) & 0x55u;  // codes kPF / kPC
    const bool my_pc = pm != 0u;
    const bool wave_pc = __any(my_pc);
    const int cnt = __builtin_popcount((ps >> 8) & 0xfu);
    const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2), b2 = __ballot(cnt & 4);
    const int excl = count_below(b0) + 2 * count_below(b1) + 4 * count_below(b2);
    const bool wave_far = __any(cm != 0u);
    const bool wave_pl = kW64 && __any((~ps & (ps >> 1) & 0x55u) != 0u);  // (kW64) a cache lookup, code kPL
    // Runs of distance-1 copies (run-length coding, CopyBlock32b with dist 1: every pixel of the run
    // equals the one before it) point straight at their root -- the last pixel before them that is
    // not such a copy -- from a block-wide max-scan of root positions, so the pointer jumping below
    // meets no chain of a run's length (alpha planes and flat lossless content are mostly runs) but
    // only the short chains of the other distances.  Pixel 0 of a block is never an in-block copy,
    // so a root always exists.  The wave's part depends on the tokens alone: kW64 sends its last root
    // out before the rank barrier, which orders it for the setup (a wave without in-block copies ends
    // on a root); the 32-word instantiation scans in the setup behind a barrier of its own (measured:
    // the early scan cost C5's K7 2 %, its values live across the rank barrier in a 128-VGPR kernel).
    auto run_scan = [&](uint32_t& runm, int& root) {  // root: the last root before my first pixel
#pragma unroll
      for (int j = 0; j < kPer; ++j) runm |= (uint32_t)(pk(ps, j) == kPC && aux[j] == 1u) << j;
      const uint32_t nonrun = ~runm & 0xfu;
      int sc = nonrun ? li0 + 31 - __builtin_clz(nonrun) : -1;  // my last root
      sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x111, 0xf, 0xf, false));  // row_shr:1
      sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x112, 0xf, 0xf, false));  // row_shr:2
      sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x114, 0xf, 0xf, false));  // row_shr:4
      sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x118, 0xf, 0xf, false));  // row_shr:8
      sc = lane >= 16 ? max(sc, __builtin_amdgcn_readlane(sc, 15)) : sc;
      sc = lane >= 32 ? max(sc, __builtin_amdgcn_readlane(sc, 31)) : sc;
      sc = lane >= 48 ? max(sc, __builtin_amdgcn_readlane(sc, 47)) : sc;
      if (lane == 63) rscan[wave] = sc;
      root = __builtin_amdgcn_update_dpp(-1, sc, 0x138, 0xf, 0xf, false);  // wave_shr:1: lanes before me
    };
    uint32_t runm_w = 0;
    int root_w = -1;
    if constexpr (kW64) {
      if (wave_pc) run_scan(runm_w, root_w);
      else if (lane == 63) rscan[wave] = li0 + kPer - 1;
    }
    if (lane == 0)
      wsum[wave] = (uint32_t)(__builtin_popcountll(b0) + 2 * __builtin_popcountll(b1) + 4 * __builtin_popcountll(b2)) |
                   (wave_far ? 0x10000u : 0u) | (wave_pc ? 0x20000u : 0u) | (wave_pl ? 0x40000u : 0u);
    bar();
    K7_T(4);
    // the sixteen wave counts in lanes 0..15 (one DPP row): inclusive scan, then read lanes
    const uint32_t wraw = wsum[lane & 15];
    const int wc = (int)(wraw & 0xffffu);
    int scan = wc;
    scan += __builtin_amdgcn_update_dpp(0, scan, 0x111, 0xf, 0xf, false);  // row_shr:1
    scan += __builtin_amdgcn_update_dpp(0, scan, 0x112, 0xf, 0xf, false);  // row_shr:2
    scan += __builtin_amdgcn_update_dpp(0, scan, 0x114, 0xf, 0xf, false);  // row_shr:4
    scan += __builtin_amdgcn_update_dpp(0, scan, 0x118, 0xf, 0xf, false);  // row_shr:8
    const int total = __builtin_amdgcn_readlane(scan, 15);
    const int my_wc = __builtin_amdgcn_readlane(wc, wave);
    const int woff = __builtin_amdgcn_readlane(scan, wave) - my_wc;
    const uint64_t fl = __ballot(lane < 16 && (wraw & 0x10000u)), plm = __ballot(lane < 16 && (wraw & 0x20000u));
    const bool blk_pc = plm != 0;
    // kW64: a block with no cache lookup needs no rank masks -- only each key's last updater for
    // the slot table (one max pass after the rounds); most ALPH blocks have none
    const bool blk_pl = !kW64 || __ballot(lane < 16 && (wraw & 0x40000u)) != 0;
    // windows: the fewest (1, 2, 4, 8 or 16 runs of whole waves) with at most `cap` updaters
    // each (a one-wave window has at most 256 <= cap); almost always one
    auto prefix = [&](int w) { return w <= 0 ? 0 : __builtin_amdgcn_readlane(scan, w - 1); };  // waves < w
    int wpw = kWaves;  // waves per window
    if (!kW64 && nkeys && total > cap) {
      int l = 4;
      for (int lv = 3; lv >= 1; --lv) {
        const int span = kWaves >> lv;
        int mx = 0;
        for (int w0 = 0; w0 < kWaves; w0 += span) mx = max(mx, prefix(w0 + span) - prefix(w0));
        if (mx <= cap) l = lv;  // ends at the smallest level that fits
      }
      wpw = kWaves >> l;
    }
    // copies reaching back more than one block read the final image (stored during the
    // previous block, complete before the barrier above); rare, so the whole workgroup takes
    // this branch or none does (a load under a lane branch would make every later use wait for
    // all outstanding loads)
    if (fl != 0) {
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const bool f = pk(ps, j) == kPF;
        const uint32_t s_off = f ? 4u * (uint32_t)(base + li0 + j - (int)aux[j]) : kDropOff;
        const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(out_rs, s_off, 0, 0);
        if (f) {
          set_known(ps, j);
          v[j] = x;
          vcur[li0 + j] = x;  // (read by in-block copies in the rounds, after a barrier)
        }
      }
    }
    // the next block's literal values, into the previous block's array (every wave is past its
    // step 1, the last reader of vprv, since the rank barrier)
    load_lits(tk_nxt, vprv);
    // in-block copies: sources and every pixel's state for the pointer jumping (rare in C5)
    if (blk_pc || (kW64 && blk_pl)) {
      uint32_t runm = runm_w;
      int root = root_w;
      if constexpr (!kW64) {  // (written out as before the kW64 change: the same machine code)
        runm = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) runm |= (uint32_t)(pk(ps, j) == kPC && aux[j] == 1u) << j;
        const uint32_t nonrun = ~runm & 0xfu;
        int sc = nonrun ? li0 + 31 - __builtin_clz(nonrun) : -1;  // my last root
        sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x111, 0xf, 0xf, false));  // row_shr:1
        sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x112, 0xf, 0xf, false));  // row_shr:2
        sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x114, 0xf, 0xf, false));  // row_shr:4
        sc = max(sc, __builtin_amdgcn_update_dpp(-1, sc, 0x118, 0xf, 0xf, false));  // row_shr:8
        sc = lane >= 16 ? max(sc, __builtin_amdgcn_readlane(sc, 15)) : sc;
        sc = lane >= 32 ? max(sc, __builtin_amdgcn_readlane(sc, 31)) : sc;
        sc = lane >= 48 ? max(sc, __builtin_amdgcn_readlane(sc, 47)) : sc;
        if (lane == 63) rscan[wave] = sc;
        root = __builtin_amdgcn_update_dpp(-1, sc, 0x138, 0xf, 0xf, false);  // wave_shr:1: lanes before me
        bar();
      }
      {  // the earlier waves' last roots: lane w < wave reads wave w's, a max over row 0's lanes
        int x = lane < wave ? rscan[lane & 15] : -1;
        x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x111, 0xf, 0xf, false));  // row_shr:1
        x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x112, 0xf, 0xf, false));  // row_shr:2
        x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x114, 0xf, 0xf, false));  // row_shr:4
        x = max(x, __builtin_amdgcn_update_dpp(-1, x, 0x118, 0xf, 0xf, false));  // row_shr:8
        root = max(root, __builtin_amdgcn_readlane(x, 15));
      }
      uint32_t stw = 0, rfw[2] = {0u, 0u};
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t c = pk(ps, j);
        stw |= (uint32_t)(c == kPC ? kPendCopy : c == kPL ? kPendLookup : kKnown) << (8 * j);
        const uint32_t src = (runm >> j) & 1u ? (uint32_t)root : (uint32_t)(li0 + j) - aux[j];
        rfw[j >> 1] |= (c == kPC ? src : 0u) << (16 * (j & 1));
        if (!((runm >> j) & 1u)) root = li0 + j;
      }
      *reinterpret_cast<uint2*>(&ref[li0]) = make_uint2(rfw[0], rfw[1]);
      *reinterpret_cast<uint32_t*>(&st[li0]) = stw;
    }
    int serial_from = kBlock;  // local pixel where the serial path takes over
    if constexpr (kW64) {
      K7_T(6);
      // ---- Dense blocks (the small-cache instantiation: alpha planes and flat content, nearly
      //      every pixel a copy and a few lookups).  No ranks and no masks:
      //  R  pointer jumping over the in-block copies with the lookups as roots: every copy ends
      //     known or pointing at a lookup -- whose value is not known yet, but whose hash is: a
      //     slot only ever holds values of its own hash (the one exception, a never-written slot
      //     k != 0, sends the block to the serial path), so the lookup and the copies of it insert
      //     under its key.
      //  H  every inserting pixel's hash is now known: per wave and key, the last such pixel.
      //  L  a lookup's source is the last pixel before it that inserts under its key (its own
      //     wave's lanes, else the earlier waves' H entries) -- or, with none in the block, the
      //     slot as the blocks before left it.
      //  J  pointer jumping again until every pixel is known (lookups and copies of lookups).
      //  T  each key's last pixel in the block writes its slot.
      uint32_t* const lastp = reinterpret_cast<uint32_t*>(mask);  // [wave][key]: 1 + local pixel, 0 none
      static_assert(sizeof(mask) >= kWaves * kKeysW64 * 4, "lastp");
      // One pointer-jumping step over my pending copies (their sources gathered first, as
      // independent LDS reads; the hand-off protocol of the rounds below): a known source gives
      // its value, a pending copy its link, a pending lookup stops the copy.  The four slots'
      // values, states and links go back as one store each (the values before the states).
      // Returns whether a copy of mine took a link.
      auto jump_round = [&]() -> bool {
        uint32_t pcm = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) pcm |= (uint32_t)(pk(ps, j) == kPC) << j;
        if (!__any(pcm != 0)) return false;
        bool still = false;
        if (pcm) {
          const uint2 rw = *reinterpret_cast<const uint2*>(&ref[li0]);
          int rv[kPer] = {(int16_t)(rw.x & 0xffffu), (int16_t)(rw.x >> 16), (int16_t)(rw.y & 0xffffu),
                          (int16_t)(rw.y >> 16)};
          int src[kPer];
          uint32_t ss[kPer], xs[kPer];
          int nref[kPer];
          // four consecutive sources from an aligned pixel (copies at a distance of a multiple of
          // four: the row above in the alpha planes): one vector read per array -- the strided
          // scalar reads of the lanes conflict in the LDS banks
          const bool vec = pcm == 0xfu && (rv[0] & 3) == 0 && rv[1] == rv[0] + 1 && rv[2] == rv[0] + 2 && rv[3] == rv[0] + 3;
          if (vec) {
            // (one asm block, states first: as plain reads the compiler merged them with the scalar
            // path's into reads of a merged address, whose lost alias information made the waitcnt
            // pass wait vmcnt(0) for the next block's staged literals at every round)
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
            uint32_t s4;
            u32x4 x4;
            u32x2 r4;
            asm volatile("ds_read_b32 %0, %3\n\tds_read_b128 %1, %4\n\tds_read_b64 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                         : "=&v"(s4), "=&v"(x4), "=&v"(r4)
                         : "v"(lds_addr(&st[rv[0]])), "v"(lds_addr(&vcur[rv[0]])), "v"(lds_addr(&ref[rv[0]]))
                         : "memory");
            ss[0] = s4 & 0xffu, ss[1] = (s4 >> 8) & 0xffu, ss[2] = (s4 >> 16) & 0xffu, ss[3] = s4 >> 24;
            xs[0] = x4.x, xs[1] = x4.y, xs[2] = x4.z, xs[3] = x4.w;
            nref[0] = (int16_t)(r4.x & 0xffffu), nref[1] = (int16_t)(r4.x >> 16), nref[2] = (int16_t)(r4.y & 0xffffu),
            nref[3] = (int16_t)(r4.y >> 16);
          } else {
#pragma unroll
            for (int j = 0; j < kPer; ++j) src[j] = (pcm >> j) & 1u ? rv[j] : li0 + j;
#pragma unroll
            for (int j = 0; j < kPer; ++j) ss[j] = st[src[j]];
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int j = 0; j < kPer; ++j) xs[j] = vcur[src[j]];
#pragma unroll
            for (int j = 0; j < kPer; ++j) nref[j] = ref[src[j]];
          }
          uint32_t walk = 0;  // slots whose source was a pending copy: walking on along the chain
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            if ((pcm >> j) & 1u) {
              if (ss[j] == kKnown) {
                set_known(ps, j);
                v[j] = xs[j];
              } else if (ss[j] == kPendCopy) {
                rv[j] = nref[j];  // (a stale or fresh link: both lie on the chain)
                walk |= 1u << j;
              }
            }
          }
          // the chain further, link by link within the round (the links are static, or shortcuts
          // other lanes have since taken): most chains end within the first round, which leaves
          // one barrier per phase instead of one per link doubling
          for (int h = 0; h < kWalk && walk; ++h) {
#pragma unroll
            for (int j = 0; j < kPer; ++j) ss[j] = (walk >> j) & 1u ? st[rv[j]] : 0u;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int j = 0; j < kPer; ++j) xs[j] = (walk >> j) & 1u ? vcur[rv[j]] : 0u;
#pragma unroll
            for (int j = 0; j < kPer; ++j) nref[j] = (walk >> j) & 1u ? ref[rv[j]] : 0;
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
              if (!((walk >> j) & 1u)) continue;
              if (ss[j] == kKnown) {
                set_known(ps, j);
                v[j] = xs[j];
                walk &= ~(1u << j);
              } else if (ss[j] == kPendCopy) {
                rv[j] = nref[j];
              } else {  // a lookup: the copy points at it
                walk &= ~(1u << j);
              }
            }
          }
          still = walk != 0;
          uint32_t stw = 0;
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const uint32_t c = pk(ps, j);
            stw |= (uint32_t)(c == kPC ? kPendCopy : c == kPL ? kPendLookup : kKnown) << (8 * j);
          }
          *reinterpret_cast<uint4*>(&vcur[li0]) = make_uint4(v[0], v[1], v[2], v[3]);
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
          *reinterpret_cast<uint32_t*>(&st[li0]) = stw;
          *reinterpret_cast<uint2*>(&ref[li0]) =
              make_uint2((uint32_t)(uint16_t)rv[0] | (uint32_t)rv[1] << 16, (uint32_t)(uint16_t)rv[2] | (uint32_t)rv[3] << 16);
        }
        return still;
      };
      auto jump_rounds = [&]() {
        for (int r = 0;; ++r) {
          if (r == kMaxRounds) {  // (uniform)
            K7_COUNT(10, 1);
            slow[b & 1] = 1;
            break;
          }
          K7_COUNT(2, 1);
          if (!sync_or(jump_round())) break;
        }
      };
      // R (the setup's ref / st stores are complete first)
      if (blk_pc) {
        bar();
        jump_rounds();
      }
      K7_T(5);
      // H: the hash each pixel inserts under (known updaters: of the value; lookups and copies
      // of one: the key), and per wave and key the last pixel -- the lanes of one key combined
      // while a key still gathers four lanes (a dense wave is mostly one key), the rest by ds_max
      uint32_t hk[kPer] = {0u, 0u, 0u, 0u}, hm = 0;
      // a flat wave (every pixel a known updater of one value: most of an alpha plane's waves) has
      // one hash, computed once, and its last pixel as the key's (no lookup of its own reads hk)
      const uint32_t v0u = (uint32_t)__builtin_amdgcn_readfirstlane((int)v[0]);
      const bool flat = nkeys && __all((ps & 0xfffu) == 0xf00u && v[0] == v0u && v[1] == v0u && v[2] == v0u && v[3] == v0u);
      if (flat) {
        if (lane == 63) ds_write_u32(&lastp[wave * kKeysW64 + hash_px(v0u, shift)], (uint32_t)(li0 + kPer));
      } else if (nkeys) {
        uint32_t pcm = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) pcm |= (uint32_t)(pk(ps, j) == kPC) << j;
        uint32_t lk[kPer] = {0u, 0u, 0u, 0u};
        if (__any(pcm != 0)) {  // a copy of a lookup: the key in the lookup's vcur entry
          const uint2 rw = *reinterpret_cast<const uint2*>(&ref[li0]);
          const int rv[kPer] = {(int16_t)(rw.x & 0xffffu), (int16_t)(rw.x >> 16), (int16_t)(rw.y & 0xffffu),
                                (int16_t)(rw.y >> 16)};
#pragma unroll
          for (int j = 0; j < kPer; ++j) lk[j] = vcur[(pcm >> j) & 1u ? rv[j] : li0 + j];
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const uint32_t c = pk(ps, j);
          hk[j] = c == kPK ? hash_px(v[j], shift) : c == kPL ? v[j] : lk[j] & (kKeysW64 - 1);
          hm |= (uint32_t)(c != kPK || is_upd(ps, j)) << j;
        }
        uint32_t pend = hm;
        for (int it = 0; it < 8; ++it) {
          const uint64_t bm = __ballot(pend != 0);
          if (bm == 0) break;
          const int lead = __builtin_ctzll(bm);
          const int jf = __builtin_ctz(pend | 0x10u);
          const uint32_t kf = jf == 0 ? hk[0] : jf == 1 ? hk[1] : jf == 2 ? hk[2] : hk[3];
          const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)kf, lead);
          uint32_t mm = 0;
#pragma unroll
          for (int j = 0; j < kPer; ++j) mm |= (uint32_t)(((pend >> j) & 1u) && hk[j] == kl) << j;
          const uint64_t mb = __ballot(mm != 0);
          if (lane == 63 - __builtin_clzll(mb))
            ds_write_u32(&lastp[wave * kKeysW64 + kl], (uint32_t)(li0 + 31 - __builtin_clz(mm)) + 1u);
          pend &= ~mm;
          if (__builtin_popcountll(mb) < 4) break;
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if ((pend >> j) & 1u) ds_max_u32(&lastp[wave * kKeysW64 + hk[j]], (uint32_t)(li0 + j) + 1u);
      }
      bar();  // (also orders step 1's far-copy values before the next block's reads)
      K7_T(11);
      // L: the wave's lookups one at a time (wave-uniform loop; most waves hold none)
      if (blk_pl && nkeys) {
        uint32_t lm = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) lm |= (uint32_t)(pk(ps, j) == kPL) << j;
        while (true) {
          const uint64_t bm = __ballot(lm != 0);
          if (bm == 0) break;
          const int lead = __builtin_ctzll(bm);
          const int jf = __builtin_ctz(lm | 0x10u);
          const uint32_t kf = jf == 0 ? v[0] : jf == 1 ? v[1] : jf == 2 ? v[2] : v[3];  // (a lookup's key)
          const int j0 = __builtin_amdgcn_readlane(jf, lead);
          const uint32_t kl = (uint32_t)__builtin_amdgcn_readlane((int)kf, lead);
          const int pos = wave * kWavePx + kPer * lead + j0;
          uint32_t mm = 0;  // my pixels before it that insert under its key
#pragma unroll
          for (int j = 0; j < kPer; ++j) mm |= (uint32_t)(((hm >> j) & 1u) && hk[j] == kl && li0 + j < pos) << j;
          const uint64_t mb = __ballot(mm != 0);
          int p;
          if (mb) {
            p = __builtin_amdgcn_readlane(li0 + 31 - __builtin_clz(mm | 1u), 63 - __builtin_clzll(mb));
          } else {  // the earlier waves' last pixels of the key: lane w < wave reads wave w's
            const uint32_t x = lane < wave ? lastp[lane * kKeysW64 + kl] : 0u;
            const uint64_t wb = __ballot(x != 0u);
            p = wb ? (int)__builtin_amdgcn_readlane((int)x, 63 - __builtin_clzll(wb)) - 1 : -1;
          }
          if (lane == lead) {
            // pixel p: known (its value), a lookup (a copy of it now), or a copy of a lookup (a
            // copy of that lookup) -- its state as R left it or as L has since made it, either
            // way a pointer along the chain
            const uint32_t sp = p >= 0 ? st[p] : kKnown;
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t xp = vcur[p >= 0 ? p : 0];
            const int rp = ref[p >= 0 ? p : 0];
            if (p >= 0 && sp != kKnown) {
              ps ^= (kPL ^ kPC) << (2 * j0);
              ref[pos] = (int16_t)(sp == kPendLookup ? p : rp);
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              st[pos] = kPendCopy;
            } else if (p >= 0) {
#pragma unroll
              for (int j = 0; j < kPer; ++j) v[j] = j == j0 ? xp : v[j];
              set_known(ps, j0);
              vcur[pos] = xp;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              st[pos] = kKnown;
            } else {  // the slot as the blocks before left it
              const uint2 rec = slotrec[kl];
              if (kl != 0u && !((slot_set[kl >> 5] >> (kl & 31)) & 1u)) {
                K7_COUNT(9, 1);
                slow[b & 1] = 1;
              }
#pragma unroll
              for (int j = 0; j < kPer; ++j) v[j] = j == j0 ? rec.y : v[j];
              set_known(ps, j0);
              vcur[pos] = rec.y;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              st[pos] = kKnown;
            }
            lm &= ~(1u << j0);
          }
        }
        K7_T(12);
        // J
        uint32_t pcm = 0;
#pragma unroll
        for (int j = 0; j < kPer; ++j) pcm |= (uint32_t)(pk(ps, j) == kPC) << j;
        if (sync_or(pcm != 0)) jump_rounds();
      }
      K7_T(13);
      // T (after a barrier: every pixel known, every lookup done with the table)
      const bool go_serial = slow[b & 1] != 0;
      // (one lane per key and wave, a key's sixteen in one DPP row: spread over the waves, not a
      // chain of reads in one, which the other waves waited for at the next block's rank barrier)
      if (nkeys) {
        const int tot = nkeys * kWaves;
        for (int e0 = 0; e0 < tot; e0 += kThreads) {
          if (e0 + wave * 64 >= tot) break;  // (wave-uniform: whole rows of sixteen lanes)
          const int e = e0 + tid, k = e >> 4, w = e & 15;
          const bool ok = e < tot;
          uint32_t x = ok ? lastp[w * kKeysW64 + k] : 0u;
          if (ok) lastp[w * kKeysW64 + k] = 0u;
          x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false));  // row_shr:1
          x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false));  // row_shr:2
          x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false));  // row_shr:4
          x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false));  // row_shr:8
          if (ok && (lane & 15) == 15 && x != 0u && !go_serial) {
            slotrec[k].y = vcur[x - 1u];
            ds_or_b32(&slot_set[k >> 5], 1u << (k & 31));
          }
        }
      }
      if (go_serial) serial_from = 0;
    } else {
    // updaters of the block before pixel j (recomputed at each use: four live ranks cost registers)
    const int r0 = woff + excl;
    auto R = [&](int j) { return r0 + __builtin_popcount((ps >> 8) & ((1u << j) - 1u)); };
    const int nwin = kWaves / wpw;
    const int myq = wave / wpw;
    for (int q = 0; q < nwin; ++q) {
      const bool in_win = myq == q;
      const int rb = prefix(q * wpw);  // updaters before the window
      K7_COUNT(3, 1);
      // ---- 2. register the known updaters of the window: values by rank (one store per pixel
      //         slot, to a dummy slot when it is not one), then one updater per lane over the
      //         wave's ranks [woff - rb, woff - rb + my_wc) -- or per pixel slot when the wave
      //         has in-block copies, whose ranks lie in the same range unregistered
      const bool pc = in_win && my_pc;
      {
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          uval[in_win && is_upd(ps, j) && pk(ps, j) == kPK ? R(j) - rb : uval_dummy] = v[j];
        if (in_win && nkeys) {
          if (!wave_pc) {
            wave_sync();
            for (int i = lane; i < my_wc; i += 64) {
              const int r = woff - rb + i;
              reg_hash(r, uval[r]);
            }
          } else {
#pragma unroll
            for (int j = 0; j < kPer; ++j)
              if (is_upd(ps, j) && pk(ps, j) == kPK) reg_hash(R(j) - rb, v[j]);
          }
        }
        if (pc) {
          int fp = kBlock;
#pragma unroll
          for (int j = kPer - 1; j >= 0; --j)
            if (pk(ps, j) == kPC) fp = li0 + j;
          ds_min_i32(&first_pend[0], fp);
        }
      }
      // (a) of a round: lookups of the window before the first pending copy fp.  kRounds: the
      // window has in-block copies (fp varies, and copies read the lookups' states); instantiated
      // twice so that the common case (no in-block copy: one pass, every lookup resolves)
      // carries none of it.
      auto lookups = [&](const int fp, auto kRoundsC) __attribute__((always_inline)) {
        constexpr bool kRounds = decltype(kRoundsC)::value;
        // (a) lookups before the first pending copy: the key's last updater in the window if it
        //     precedes the pixel, none (the slot as the previous window left it), or -- it
        //     straddles the pixel -- the highest mask bit below the pixel's rank count
          uint32_t act = 0, strad = 0;
          uint2 rec[kPer];
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const bool a = pk(ps, j) == kPL && (!kRounds || li0 + j < fp);
            act |= (uint32_t)a << j;
            rec[j] = slotrec[a ? aux[j] : 0u];
          }
          uint32_t idx[kPer];  // uval index of the last updater below the pixel, or ~0
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const uint32_t rr = (uint32_t)(R(j) - rb), d = rec[j].x - 1u;  // (lr = 0: d = ~0)
            idx[j] = d < rr ? d : ~0u;
            strad |= (uint32_t)(d != ~0u && d >= rr) << j;
          }
          strad &= act;
          if (__any(strad != 0)) {
            // (10 % of C5's lookups, in 96 % of its waves): compacted, one straddling lookup per
            // lane, instead of each pixel slot's branch walked by the whole wave
            const int sc = __builtin_popcount(strad);
            const uint64_t s0 = __ballot(sc & 1), s1 = __ballot(sc & 2), s2 = __ballot(sc & 4);
            const int sx = count_below(s0) + 2 * count_below(s1) + 4 * count_below(s2);
            const int stot = __builtin_popcountll(s0) + 2 * __builtin_popcountll(s1) + 4 * __builtin_popcountll(s2);
            uint2* const scr = sscr + wave * 64;
            if (stot <= 64) {
              int slot = sx;
#pragma unroll
              for (int j = 0; j < kPer; ++j)
                if ((strad >> j) & 1u) scr[slot++] = make_uint2(aux[j], (uint32_t)(R(j) - rb));
              wave_sync();
              if (lane < stot) {
                const uint2 e = scr[lane];
                scr[lane].x = straddle_idx(e.x, (int)e.y);
              }
              wave_sync();
              slot = sx;
#pragma unroll
              for (int j = 0; j < kPer; ++j)
                if ((strad >> j) & 1u) idx[j] = scr[slot++].x;
            } else {
#pragma unroll
              for (int j = 0; j < kPer; ++j)
                if ((strad >> j) & 1u) idx[j] = straddle_idx(aux[j], R(j) - rb);
            }
          }
          uint32_t empty = 0;  // lookups of a slot that may never have been written
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const uint32_t xin = uval[idx[j] & (kBlock - 1)];
            const bool a = (act >> j) & 1u;
            const uint32_t x = idx[j] != ~0u ? xin : rec[j].y;
            empty |= (uint32_t)(a & (idx[j] == ~0u) & (aux[j] != 0u) & (x == 0u)) << j;
            v[j] = a ? x : v[j];
          }
          ps &= ~((act & 1u) * 0x3u | (act & 2u) * 0x6u | (act & 4u) * 0xcu | (act & 8u) * 0x18u);  // codes -> known
          if (__any(empty != 0)) {
#pragma unroll
            for (int j = 0; j < kPer; ++j) {
              const uint32_t k = aux[j];
              if ((empty >> j) & 1u && !((slot_set[k >> 5] >> (k & 31)) & 1u)) {
                K7_COUNT(9, 1);
                slow[b & 1] = 1;
              }
            }
          }
          if (act) *reinterpret_cast<uint4*>(&vcur[li0]) = make_uint4(v[0], v[1], v[2], v[3]);
          // copies in (b) read these states, after the barrier -- also those of a LATER window
          // of the block: a window without pending copies of its own resolves its lookups on
          // the no-rounds path, and an in-block copy further on may have one as its source
          // (blk_pc is block-uniform; without it such a copy could never resolve)
          if ((kRounds || blk_pc) && act) {
#pragma unroll
            for (int j = 0; j < kPer; ++j)
              if ((act >> j) & 1u) st[li0 + j] = kKnown;
          }
      };
      // ---- rounds (one when the window has no pending copy: every lookup resolves in (a))
      // (one window: every thread is in it, so "any pending copy" is the block's flag from the
      // rank barrier, and a plain barrier orders the registrations before the lookups)
      int any_pc;
      if (nwin == 1) {
        bar();
        any_pc = blk_pc;
      } else {
        any_pc = sync_or(pc);
      }
      K7_T(11);
      if (!any_pc) {
        K7_COUNT(2, 1);
        if (in_win) lookups(kBlock, std::false_type{});
        K7_T(12);
      }
      for (int r = 0; any_pc || r > 0; ++r) {  // (entered only with copies; ends after the (a) that follows the last)
        K7_COUNT(2, 1);
        if (r == kMaxRounds) {
          K7_COUNT(10, 1);
          slow[b & 1] = 1;
          break;  // uniform: any_pc and r are the same in every thread
        }
        const int fp = any_pc ? first_pend[r & 1] : kBlock;
        // first_pend[(r + 1) & 1] was last read in round r - 1; it is next written in (b), after
        // the barrier below
        if (tid == 0) first_pend[(r + 1) & 1] = kBlock;
        if (in_win) lookups(fp, std::true_type{});
        K7_T(12);
        if (!any_pc) break;
        bar();
        // (b) pending copies: take a known source's value and register, else jump one link back
        bool still = false;  // a copy of mine still pending
        if (in_win) {
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const int li = li0 + j;
            if (pk(ps, j) != kPC) continue;
            const int src = ref[li];
            const uint8_t ss = st[src];
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (ss == kKnown) {
              const uint32_t x = vcur[src];
              set_known(ps, j);
              v[j] = x;
              vcur[li] = x;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              st[li] = kKnown;
              uval[R(j) - rb] = x;
              if (nkeys) reg_hash(R(j) - rb, x);
            } else {
              if (ss == kPendCopy) ref[li] = ref[src];  // (a stale or fresh link: both lie on the chain)
              ds_min_i32(&first_pend[(r + 1) & 1], li);
              still = true;
            }
          }
        }
        any_pc = sync_or(still);
        K7_T(5);
      }
      bar();  // every lookup has read the slot table; the masks are complete
      const bool go_serial = slow[b & 1] != 0;
      // ---- 3. each key's last updater writes its slot and clears the key's masks
      // the window's updaters packed 64 to a wave by rank (uval is complete after the barrier):
      // C5's ~143 per block take three waves' single pass instead of a sparse pass in each of
      // sixteen.  A pending copy that never resolved (the window goes serial) never registered,
      // so its rank is no key's last: its stale uval entry changes nothing.
      if (in_win && nkeys) {
        const int wtot = prefix(q * wpw + wpw) - rb, wi = wave - q * wpw;
        for (int i = wi * 64 + lane; i < wtot; i += wpw * 64) table_update(i, uval[i], go_serial);
      }
      if (tid == 0) first_pend[0] = first_pend[1] = kBlock;
      if (go_serial) {
        // (pending copies of the window never registered: nothing of theirs to clear; a
        // window whose rounds hit the cap leaves their registered bits, cleared above)
        serial_from = q * wpw * kWavePx;
        bar();
        break;
      }
      // between windows: the next window's registration follows this one's slot table.  After
      // the last window no barrier: the next block's rank barrier orders this slot table before
      // its registration, and nothing before that barrier touches the table, the masks or uval
      if (q + 1 < nwin) bar();
      K7_T(13);
    }
    K7_T(5);
    }
    // ---- the exact serial path: DecodeImageData's order, one pixel at a time, from the start
    //      of the window that could not be resolved, on the table as the windows before it left
    //      it.  Literal and older-copy values are in vcur from step 1; everything else is
    //      recomputed here.  The block's tokens are read again (rare path).
    if (serial_from < kBlock) {
      K7_COUNT(1, 1);
      {
        typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
        const u32x4 q = __builtin_amdgcn_raw_buffer_load_b128(tok_rs, 4u * (uint32_t)(base + li0), 0, 0);
        *reinterpret_cast<uint4*>(&uval[li0]) = make_uint4(q.x, q.y, q.z, q.w);
      }
      bar();
      if (tid == 0) {
        const int cnt_px = min(kBlock, n - base);
        for (int li = serial_from; li < cnt_px; ++li) {
          const int pos = base + li;
          const uint32_t t = uval[li], kind = t & ~kTokPayload, pl = t & kTokPayload;
          uint32_t x = 0;
          if (kind == kTokLiteral) {
            x = vcur[li];
          } else if (kind == kTokCopy) {
            const int s = pos - (int)pl;
            x = (pl == 0 || s < 0) ? 0 : s < base ? vcur[li] : vcur[s - base];
          } else if (kind == kTokCache) {
            x = pl < (uint32_t)nkeys ? slotrec[pl].y : 0;
          }
          if (kind != kTokUnset && nkeys) {
            const uint32_t h = hash_px(x, shift);
            slotrec[h].y = x;
            slot_set[h >> 5] |= 1u << (h & 31);
          }
          vcur[li] = x;
        }
        slow[b & 1] = 0;
      }
      bar();
    }
    K7_T(7);
  };

  for (int b = 0; b < nblocks; b += 2) {
    block(b, tkA, tkB, val0, val1);
    if (b + 1 < nblocks) block(b + 1, tkB, tkA, val1, val0);
  }
  if (nblocks > 0) store_block(nblocks - 1, (nblocks - 1) & 1 ? val1 : val0);
  // the last block's literal load (past the stream) must land before the workgroup's LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#ifdef WG_K7_STATS
  if (tid == 0) {
    k7_lds[0][0] = (unsigned long long)nblocks;
    for (int i : {0, 1, 2, 3, 9, 10}) atomicAdd(&g_k7_stats[i], k7_lds[0][i]);
    for (int i : {4, 5, 6, 7, 8, 11, 12, 13, 14, 15}) atomicAdd(&g_k7_stats[i], k7_lds[0][i]);
  }
  if (lane == 0)
    for (int i : {4, 5, 6, 7, 8, 11, 12, 13, 14, 15}) atomicAdd(&g_k7_wave[wave][i], k7_lds[wave][i]);
#endif
}

#ifdef WG_K7_STATS
extern "C" int wg_debug_k7_stats(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k7_stats), sizeof(g_k7_stats)) != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(out + 16, HIP_SYMBOL(g_k7_wave), sizeof(g_k7_wave)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[16 * (1 + kWaves)] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_k7_stats), z, sizeof(g_k7_stats)) != hipSuccess) return -1;
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_k7_wave), z, sizeof(g_k7_wave)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

bool vp8l_resolve_w64(int cache_bits) { return cache_bits <= kW64Bits; }

hipError_t launch_vp8l_resolve(const LLTokDesc* d_descs, const LLTokDesc* single, int n, int* d_err,
                               hipStream_t stream, int n_w64, int n_alpha, int n_tiled) {
  if (n <= 0) return hipSuccess;
  if (single) {
    if (vp8l_resolve_w64(single->cache_bits))
      hipLaunchKernelGGL((vp8l_resolve_kernel<true, true, 0>), dim3(1), dim3(kThreads), 0, stream, nullptr, *single, d_err);
    else
      hipLaunchKernelGGL((vp8l_resolve_kernel<true, false, 0>), dim3(1), dim3(kThreads), 0, stream, nullptr, *single,
                         d_err);
    return hipGetLastError();
  }
  // the first n_alpha streams (64-word, with their alpha bytes: the first n_tiled of them into band
  // tiles), then the other n_w64 - n_alpha on the 64-word instantiation, the rest on the 32-word one
  if (n_tiled > 0)
    hipLaunchKernelGGL((vp8l_resolve_kernel<false, true, 2>), dim3(n_tiled), dim3(kThreads), 0, stream, d_descs,
                       LLTokDesc{}, d_err);
  if (n_alpha > n_tiled)
    hipLaunchKernelGGL((vp8l_resolve_kernel<false, true, 1>), dim3(n_alpha - n_tiled), dim3(kThreads), 0, stream,
                       d_descs + n_tiled, LLTokDesc{}, d_err);
  if (n_w64 > n_alpha)
    hipLaunchKernelGGL((vp8l_resolve_kernel<false, true, 0>), dim3(n_w64 - n_alpha), dim3(kThreads), 0, stream,
                       d_descs + n_alpha, LLTokDesc{}, d_err);
  if (n > n_w64)
    hipLaunchKernelGGL((vp8l_resolve_kernel<false, false, 0>), dim3(n - n_w64), dim3(kThreads), 0, stream,
                       d_descs + n_w64, LLTokDesc{}, d_err);
  return hipGetLastError();
}

}  // namespace wg
