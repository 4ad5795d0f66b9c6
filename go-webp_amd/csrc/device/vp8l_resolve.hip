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
// (4 consecutive per thread) in scan order; the cache (up to 2048 slots) lives in LDS.  The
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
// output so far.
//
// Latency: tokens are loaded two blocks ahead and literal values one block ahead, so a block
// waits on HBM only for copies that reach back more than one block.
#include <hip/hip_runtime.h>
#include <stdint.h>

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
constexpr int kMaxRounds = 32;
constexpr uint8_t kKnown = 1, kPendCopy = 2, kPendLookup = 3, kPendFar = 4;
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
// blocks, serial windows, rounds, windows, t_phase1, t_windows, t_serial, t_store,
// serial because: bad token, empty slot, round cap; lookups
__device__ unsigned long long g_k7_stats[12];
#define K7_T(i)                                                      \
  do {                                                               \
    if (tid == 0) {                                                  \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();              \
      k7_acc[i] += t_ - k7_t;                                        \
      k7_t = t_;                                                     \
    }                                                                \
  } while (0)
#define K7_COUNT(i, v)                                               \
  do {                                                               \
    if (tid == 0) k7_cnt[i] += (v);                                  \
  } while (0)
#else
#define K7_T(i) (void)0
#define K7_COUNT(i, v) (void)0
#endif

// kSingle: the one stream `single` passed by value (the stage entry wg_vp8l_resolve_device; err may
// be null there: bad tokens then only resolve to 0, the serial path's rule); else stream
// blockIdx.x of `descs`.  (Two instantiations: a descriptor chosen at run time between the two
// loses its uniformity and the pointers' address space -- flat loads and spills.)
template <bool kSingle>
__global__ void __launch_bounds__(1024) vp8l_resolve_kernel(const LLTokDesc* __restrict__ descs, LLTokDesc single,
                                                            int* err) {
  __shared__ uint64_t mask[kMaskWords];          // per key k: words k*W .. k*W+W-1, bit = rank in window
  __shared__ uint32_t summ[kSlots];              // per key: mask words holding a bit
  __shared__ uint32_t last_rank[kSlots];         // per key: 1 + the window's last updater rank (0 none)
  __shared__ uint32_t slot_val[kSlots];          // the color cache (VP8LColorCache.colors_)
  __shared__ uint32_t slot_set[kSlots / 32];     // slot written at least once
  __shared__ __attribute__((aligned(16))) uint32_t uval[kBlock];    // window updater values by rank
                                                                     // (serial path: the block's tokens)
  __shared__ __attribute__((aligned(16))) uint32_t val[2][kBlock];  // this / the previous block's values
  __shared__ int16_t ref[kBlock];                // pending copy: source pointer (pointer jumping)
  __shared__ uint8_t st[kBlock];                 // kKnown / kPendCopy / kPendLookup
  __shared__ __attribute__((aligned(16))) uint32_t wsum[kWaves];  // updaters per wave of the block
  __shared__ int first_pend[2];                  // per round parity: first pending copy (local)
  __shared__ int slow;                           // this window goes serial
  __shared__ int orflag[4];                      // sync_or: a ring of flag words
  const LLTokDesc D = kSingle ? single : descs[blockIdx.x];
  if (!D.valid) return;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int n = D.n_px, cache_bits = D.cache_bits;
  const int nkeys = cache_bits > 0 ? 1 << cache_bits : 0;
  const int shift = 32 - cache_bits;
  const int W = cache_bits > 0 ? min(kMaxW, kMaskWords >> cache_bits) : 1;  // mask words per key
  const int cap = 64 * W;                                                    // ranks per window
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
    slot_val[i] = 0;
    summ[i] = 0;
    last_rank[i] = 0;
  }
  if (tid < kSlots / 32) slot_set[tid] = 0;
  if (tid == 0) {
    slow = 0;
    first_pend[0] = first_pend[1] = kBlock;
  }
  if (tid < 4) orflag[tid] = 0;
  // A barrier that also returns whether any thread's p was set: one s_barrier (HIP's
  // __syncthreads_or costs three).  Flag word k & 3 is set before barrier k and read after it;
  // word (k + 2) & 3, last read before barrier k - 1, is cleared after barrier k for call k + 2.
  int orseq = 0;
  auto sync_or = [&](bool p) -> bool {
    const int slot = orseq & 3;
    if (p) orflag[slot] = 1;
    __syncthreads();
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
  auto load_lits = [&](const uint32_t* tk, uint32_t* lv) {
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const bool is_lit = (tk[j] & ~kTokPayload) == kTokLiteral;
      lv[j] = __builtin_amdgcn_raw_buffer_load_b32(lit_rs, is_lit ? 4u * (tk[j] & kTokPayload) : kDropOff, 0, 0);
    }
  };
  // software pipeline: tokens two blocks ahead, literal values one block ahead
  uint32_t tk[kPer], lv[kPer], tk1[kPer], lv1[kPer], tk2[kPer];
  load_tokens(0, tk);
  load_tokens(1, tk1);
  load_lits(tk, lv);
  __syncthreads();
#ifdef WG_K7_STATS
  uint64_t k7_acc[8] = {}, k7_t = __builtin_amdgcn_s_memtime();
  unsigned long long k7_cnt[12] = {};
#endif

  for (int b = 0; b < nblocks; ++b) {
    const int base = b * kBlock;
    const int cur = b & 1, prv = cur ^ 1;
    uint32_t* vcur = val[cur];
    const uint32_t* vprv = val[prv];
    // next blocks' inputs in flight while this block resolves
    load_tokens(b + 2, tk2);
    load_lits(tk1, lv1);

    // ---- 1. tokens: literals, copies from before the block, unset pixels are known; in-block
    //         copies and lookups are pending.  Literals and copies are updaters (ranked).
    uint8_t pend[kPer];  // 0 known, else kPendCopy / kPendLookup / kPendFar
    bool upd[kPer];
    uint32_t v[kPer];
    bool bad = false, far = false;
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int li = li0 + j, pos = base + li;
      const uint32_t t = pos < n ? tk[j] : kTokUnset, kind = t & ~kTokPayload, pl = t & kTokPayload;
      v[j] = 0;
      pend[j] = 0;
      upd[j] = false;
      if (kind == kTokLiteral) {
        if (pl >= (uint32_t)D.n_lits) bad = true;
        v[j] = pl < (uint32_t)D.n_lits ? lv[j] : 0u;
        upd[j] = true;
      } else if (kind == kTokCopy) {
        const int s = pos - (int)pl;
        upd[j] = true;
        if (pl == 0 || s < 0) {
          bad = true;
        } else if (s >= base) {
          pend[j] = kPendCopy;
          ref[li] = (int16_t)(s - base);
        } else if (s >= base - kBlock) {
          v[j] = vprv[s - base + kBlock];
        } else {
          pend[j] = kPendFar;  // loaded below, off the common path
          far = true;
        }
      } else if (kind == kTokCache) {
        if (pl >= (uint32_t)nkeys) bad = true;
        else pend[j] = kPendLookup;
      }
      st[li] = pend[j] == kPendCopy || pend[j] == kPendLookup ? pend[j] : kKnown;
    }
    *reinterpret_cast<uint4*>(&vcur[li0]) = make_uint4(v[0], v[1], v[2], v[3]);
    if (bad) {
      if (err) atomicOr(err, 4);
      slow = 1;
    }
    // ranks: updaters before each pixel, a block-wide prefix count (per-thread count 0..4 in
    // three ballots)
    const int cnt = (int)upd[0] + (int)upd[1] + (int)upd[2] + (int)upd[3];
    const uint64_t b0 = __ballot(cnt & 1), b1 = __ballot(cnt & 2), b2 = __ballot(cnt & 4);
    const int excl = count_below(b0) + 2 * count_below(b1) + 4 * count_below(b2);
    const bool wave_far = __any(far);
    if ((tid & 63) == 0)  // the wave's updaters, bit 16: it has a copy reaching back past the last block
      wsum[wave] = (uint32_t)(__builtin_popcountll(b0) + 2 * __builtin_popcountll(b1) + 4 * __builtin_popcountll(b2)) |
                   (wave_far ? 0x10000u : 0u);
    __syncthreads();
    K7_T(4);
    int ws[kWaves];  // (static indices only: a dynamic index would put the array in scratch)
    uint32_t any_far = 0;
#pragma unroll
    for (int w = 0; w < kWaves; w += 4) {
      const uint4 q = *reinterpret_cast<const uint4*>(&wsum[w]);
      any_far |= q.x | q.y | q.z | q.w;
      ws[w] = (int)(q.x & 0xffff), ws[w + 1] = (int)(q.y & 0xffff), ws[w + 2] = (int)(q.z & 0xffff),
      ws[w + 3] = (int)(q.w & 0xffff);
    }
    // copies reaching back more than one block read the final image (stored at the end of their
    // block, before a barrier); rare, so the whole workgroup takes this branch or none does (a
    // load under a lane branch would make every later use wait for all outstanding loads)
    if (any_far >> 16) {
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const uint32_t s_off =
            pend[j] == kPendFar ? 4u * (uint32_t)(base + li0 + j - (int)(tk[j] & kTokPayload)) : kDropOff;
        const uint32_t x = __builtin_amdgcn_raw_buffer_load_b32(out_rs, s_off, 0, 0);
        if (pend[j] == kPendFar) {
          v[j] = x;
          pend[j] = 0;
          vcur[li0 + j] = x;  // (read by in-block copies in the rounds, after a barrier)
        }
      }
    }
    int woff = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) woff += w < wave ? ws[w] : 0;
    // windows: the fewest (1, 2, 4, 8 or 16 runs of whole waves) with at most `cap` updaters
    // each (a one-wave window has at most 256 <= cap)
    int wpw = kWaves;  // waves per window
    if (nkeys) {
      int mx[5] = {0, 0, 0, 0, 0};  // largest window for 16, 8, 4, 2, 1 waves per window
#pragma unroll
      for (int l = 0; l < 5; ++l) {
        const int span = kWaves >> l;
#pragma unroll
        for (int w0 = 0; w0 < kWaves; w0 += span) {
          int s = 0;
#pragma unroll
          for (int w = w0; w < w0 + span; ++w) s += ws[w];
          mx[l] = max(mx[l], s);
        }
      }
      int l = 0;
#pragma unroll
      for (int i = 4; i >= 0; --i)
        if (mx[i] <= cap) l = i;  // ends at the smallest level that fits (level 4 always does)
      wpw = __builtin_amdgcn_readfirstlane(kWaves >> l);
    }
    const int nwin = kWaves / wpw;
    const int myq = wave / wpw;
    int R[kPer];  // updaters of the block before each pixel
    {
      int r = woff + excl;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        R[j] = r;
        r += (int)upd[j];
      }
    }
    int serial_from = kBlock;  // local pixel where the serial path takes over
    int rb = 0;                // updaters before the window
    for (int q = 0; q < nwin; ++q) {
      const bool in_win = myq == q;
      K7_COUNT(3, 1);
      // ---- register the known updaters of the window
      bool pc = false;  // a pending copy of mine in the window
      if (in_win) {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          if (!upd[j]) continue;
          if (pend[j]) {
            pc = true;
            continue;
          }
          const int r = R[j] - rb;
          uval[r] = v[j];
          if (nkeys) {
            const uint32_t h = hash_px(v[j], shift);
            atomicOr(reinterpret_cast<unsigned long long*>(&mask[h * W + (r >> 6)]), 1ull << (r & 63));
            atomicOr(&summ[h], 1u << (r >> 6));
            atomicMax(&last_rank[h], (uint32_t)r + 1u);
          }
        }
        if (pc) {
          int fp = kBlock;
#pragma unroll
          for (int j = kPer - 1; j >= 0; --j)
            if (pend[j] == kPendCopy) fp = li0 + j;
          atomicMin(&first_pend[0], fp);
        }
      }
      // ---- rounds (one when the window has no pending copy: every lookup resolves in (a))
      int any_pc = sync_or(pc);
      for (int r = 0;; ++r) {
        K7_COUNT(2, 1);
        if (r == kMaxRounds) {
          K7_COUNT(10, 1);
          slow = 1;
          break;  // uniform: any_pc and r are the same in every thread
        }
        const int fp = any_pc ? first_pend[r & 1] : kBlock;
        // first_pend[(r + 1) & 1] was last read in round r - 1; it is next written in (b), after
        // the barrier below
        if (tid == 0) first_pend[(r + 1) & 1] = kBlock;
        // (a) lookups before the first pending copy: the key's mask below the pixel's rank
        //     count, else the slot as the previous window left it
        if (in_win) {
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            if (pend[j] != kPendLookup || li0 + j >= fp) continue;
            const uint32_t k = tk[j] & kTokPayload;
            const int rr = R[j] - rb;  // window updaters before the pixel
            uint32_t x;
            bool found = false;
            if (rr > 0) {
              const int wt = (rr - 1) >> 6;
              uint32_t sm = summ[k] & (wt >= 31 ? ~0u : (2u << wt) - 1u);
              if (sm) {
                int w = 31 - __builtin_clz(sm);
                uint64_t m = mask[k * W + w];
                if (w == wt) {
                  const int lb = rr - 64 * wt;  // 1..64 bits below the pixel
                  m &= lb >= 64 ? ~0ull : (1ull << lb) - 1ull;
                  if (!m) {
                    sm &= (1u << wt) - 1u;
                    if (sm) {
                      w = 31 - __builtin_clz(sm);
                      m = mask[k * W + w];
                    }
                  }
                }
                if (m) {
                  x = uval[64 * w + 63 - __builtin_clzll(m)];
                  found = true;
                }
              }
            }
            if (!found) {
              x = slot_val[k];
              if (k != 0 && !((slot_set[k >> 5] >> (k & 31)) & 1)) {
                K7_COUNT(9, 1);
                slow = 1;
              }
            }
            v[j] = x;
            pend[j] = 0;
            vcur[li0 + j] = x;  // (read by copies in (b), after the barrier)
            st[li0 + j] = kKnown;
          }
        }
        if (!any_pc) break;
        __syncthreads();
        // (b) pending copies: take a known source's value and register, else jump one link back
        bool still = false;  // a copy of mine still pending
        if (in_win) {
#pragma unroll
          for (int j = 0; j < kPer; ++j) {
            const int li = li0 + j;
            if (pend[j] != kPendCopy) continue;
            const int src = ref[li];
            const uint8_t ss = st[src];
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            if (ss == kKnown) {
              const uint32_t x = vcur[src];
              v[j] = x;
              pend[j] = 0;
              vcur[li] = x;
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              st[li] = kKnown;
              const int rk = R[j] - rb;
              uval[rk] = x;
              if (nkeys) {
                const uint32_t h = hash_px(x, shift);
                atomicOr(reinterpret_cast<unsigned long long*>(&mask[h * W + (rk >> 6)]), 1ull << (rk & 63));
                atomicOr(&summ[h], 1u << (rk >> 6));
                atomicMax(&last_rank[h], (uint32_t)rk + 1u);
              }
            } else {
              if (ss == kPendCopy) ref[li] = ref[src];  // (a stale or fresh link: both lie on the chain)
              atomicMin(&first_pend[(r + 1) & 1], li);
              still = true;
            }
          }
        }
        any_pc = sync_or(still);
      }
      __syncthreads();  // every lookup has read the slot table; the masks are complete
      const bool go_serial = slow != 0;
      // ---- 3. each key's last updater writes its slot (unless the window goes serial) and
      //         clears the key's masks; the other updaters of the key only read last_rank, which
      //         the last one may already have reset (then they read 0: not theirs either)
      if (in_win && nkeys) {
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          if (!upd[j] || pend[j]) continue;
          const uint32_t h = hash_px(v[j], shift);
          const int rk = R[j] - rb;
          if (last_rank[h] == (uint32_t)rk + 1u) {
            if (!go_serial) {
              slot_val[h] = v[j];
              atomicOr(&slot_set[h >> 5], 1u << (h & 31));
            }
            for (uint32_t sm = summ[h]; sm; sm &= sm - 1) mask[h * W + __builtin_ctz(sm)] = 0;
            summ[h] = 0;
            last_rank[h] = 0;
          }
        }
      }
      if (tid == 0) first_pend[0] = first_pend[1] = kBlock;
      if (go_serial) {
        // (pending copies of the window never registered: nothing of theirs to clear; a
        // window whose rounds hit the cap leaves their registered bits, cleared above)
        serial_from = q * wpw * kWavePx;
        __syncthreads();
        break;
      }
      for (int w = q * wpw; w < (q + 1) * wpw; ++w) rb += (int)(wsum[w] & 0xffffu);  // (LDS: a dynamic index)
      __syncthreads();
    }
    K7_T(5);
    // ---- the exact serial path: DecodeImageData's order, one pixel at a time, from the start
    //      of the window that could not be resolved, on the table as the windows before it left
    //      it.  Literal and older-copy values are in vcur from step 1; everything else is
    //      recomputed here.
    if (serial_from < kBlock) {
      K7_COUNT(1, 1);
      *reinterpret_cast<uint4*>(&uval[li0]) = make_uint4(tk[0], tk[1], tk[2], tk[3]);
      __syncthreads();
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
            x = pl < (uint32_t)nkeys ? slot_val[pl] : 0;
          }
          if (kind != kTokUnset && nkeys) {
            const uint32_t h = hash_px(x, shift);
            slot_val[h] = x;
            slot_set[h >> 5] |= 1u << (h & 31);
          }
          vcur[li] = x;
        }
        slow = 0;
      }
      __syncthreads();
    }
    K7_T(6);
    // ---- the block's values to the coded image (K3's input; older copies read them back)
    {
      const int pos0 = base + li0;
      const uint4 o = *reinterpret_cast<const uint4*>(&vcur[li0]);
      typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
      if (pos0 + kPer <= n) {
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{o.x, o.y, o.z, o.w}, out_rs, 4u * (uint32_t)pos0, 0, 0);
      } else {  // the stream's last pixels (the buffer range drops what lies past it)
        const uint32_t ov[kPer] = {o.x, o.y, o.z, o.w};
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          __builtin_amdgcn_raw_buffer_store_b32(ov[j], out_rs, pos0 + j < n ? 4u * (uint32_t)(pos0 + j) : kDropOff, 0, 0);
      }
    }
    // rotate the pipeline
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      tk[j] = tk1[j];
      lv[j] = lv1[j];
      tk1[j] = tk2[j];
    }
    // vcur becomes the next block's vprv, and the stores above must be visible to copies that
    // reach back further than one block
    __syncthreads();
    K7_T(7);
  }
#ifdef WG_K7_STATS
  if (tid == 0) {
    k7_cnt[0] = (unsigned long long)nblocks;
    for (int i = 0; i < 4; ++i) atomicAdd(&g_k7_stats[i], k7_cnt[i]);
    for (int i = 4; i < 8; ++i) atomicAdd(&g_k7_stats[i], k7_acc[i]);
    for (int i = 8; i < 12; ++i) atomicAdd(&g_k7_stats[i], k7_cnt[i]);
  }
#endif
}

#ifdef WG_K7_STATS
extern "C" int wg_debug_k7_stats(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_k7_stats), sizeof(g_k7_stats)) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[12] = {};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_k7_stats), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

hipError_t launch_vp8l_resolve(const LLTokDesc* d_descs, const LLTokDesc* single, int n, int* d_err,
                               hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  if (single) hipLaunchKernelGGL(vp8l_resolve_kernel<true>, dim3(1), dim3(kThreads), 0, stream, nullptr, *single, d_err);
  else hipLaunchKernelGGL(vp8l_resolve_kernel<false>, dim3(n), dim3(kThreads), 0, stream, d_descs, LLTokDesc{}, d_err);
  return hipGetLastError();
}

}  // namespace wg
