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
// (4 consecutive per thread) in scan order; the cache (2048 slots, cache bits <= 11) lives in
// LDS.  Per block:
//   1. every thread decodes its pixels' tokens: literals from the literal array, copies whose
//      source precedes the block from the already-final image.  Each updater registers its
//      hash in LDS: the last and the first in-block updater per hash (atomic max) and a
//      per-hash list of all of them (atomic exchange: unordered).  Copies with an in-block
//      source and cache lookups stay pending.
//   2. rounds until nothing is pending (one in C5's blocks; a few where a back-reference
//      lands inside the block): (a) every pending lookup before the first pending copy (so
//      every updater before it has a known hash) resolves: no in-block updater of its key
//      before it -> the slot table as the previous block left it; else the last such updater
//      (the last overall if it precedes the lookup; else, when every in-block updater of the
//      key has one value -- runs of one color copied over and over -- that value; else a walk
//      of the key's list for the largest index below it); (b) every pending copy whose source is known takes its value
//      and registers as an updater, the others jump their source pointer one link further
//      back along a chain of pending copies (pointer jumping: log-depth chains).  The earliest
//      pending pixel always resolves, so the rounds end; a cap sends the block to the serial
//      path.  Values leave as 16-byte stores.
//   3. the slot table takes each hash's last in-block updater, which also resets the hash's
//      value range for the next block.
// A block with a lookup of a never-written slot k != 0, a list walk over 64 entries, or more
// than kMaxRounds rounds is redone exactly in scan order by one lane (the reference loop over
// the same LDS table, literal and far-copy values already in LDS): always correct, slow, and
// never taken by encoder output so far (C5: 3.5 % literals, 96.5 % cache lookups).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../device_format.h"
#include "kernels.h"

namespace wg {
namespace {

constexpr int kThreads = 1024;
constexpr int kPer = 4;                   // consecutive pixels per thread
constexpr int kBlock = kThreads * kPer;   // 4096 pixels per step
constexpr int kLocalBits = 12;            // log2(kBlock)
constexpr int kSlots = 2048;              // 1 << MAX_CACHE_BITS (format_constants.go)
constexpr int kMaxWalk = 64;
constexpr int kMaxRounds = 32;

__device__ __forceinline__ uint32_t hash_px(uint32_t v, int shift) { return (v * 0x1e35a7bdu) >> shift; }

}  // namespace

// Measurement build only (make VARIANT=timing): per-phase cycles of wave 0 and block counts.
#ifdef WG_K7_STATS
__device__ unsigned long long g_k7_stats[12];  // blocks, slow, rounds, t_phase1, t_rounds, t_store, t_table,
                                              // slow because: bad token, empty slot, long walk, round cap
#define K7_T(i)                                                      \
  do {                                                               \
    if (tid == 0) {                                                  \
      const uint64_t t_ = __builtin_amdgcn_s_memtime();              \
      k7_acc[i] += t_ - k7_t;                                        \
      k7_t = t_;                                                     \
    }                                                                \
  } while (0)
#else
#define K7_T(i) (void)0
#endif

__global__ void __launch_bounds__(1024) vp8l_resolve_kernel(const LLTokDesc* __restrict__ descs, int* err) {
  __shared__ uint32_t slot_val[kSlots];        // the color cache (VP8LColorCache.colors_)
  __shared__ uint32_t slot_set[kSlots / 32];   // slot written at least once
  __shared__ int32_t head[kSlots];             // position of the last in-block updater of a hash
  __shared__ uint32_t first_tag[kSlots];       // tag | (kBlock - 1 - local) of the first one (max)
  __shared__ uint32_t list_tag[kSlots];        // tag | local of the most recently linked one
  __shared__ uint32_t umin[kSlots], umax[kSlots];  // value range of the block's updaters per hash
  __shared__ int16_t nxt[kBlock];              // per updater: the previously linked one, -1 none
  __shared__ int16_t ref[kBlock];              // pending copy: source pointer (pointer jumping)
  __shared__ uint8_t st[kBlock];               // kKnown / kPendCopy / kPendLookup
  __shared__ __attribute__((aligned(16))) uint32_t val[kBlock];   // the block's values
  __shared__ __attribute__((aligned(16))) uint32_t toks[kBlock];  // the block's tokens (serial path)
  __shared__ int slow[2];                      // per block parity: redo this block serially
  __shared__ int first_pend[2];                // per round parity: first pending copy (local)
  constexpr uint8_t kKnown = 1, kPendCopy = 2, kPendLookup = 3;
  const LLTokDesc D = descs[blockIdx.x];
  if (!D.valid) return;
  const int tid = threadIdx.x;
  const int n = D.n_px, cache_bits = D.cache_bits;
  const int shift = 32 - cache_bits;
  const uint32_t* __restrict__ tokens = D.tokens;
  const uint32_t* __restrict__ lits = D.lits;
  uint32_t* coded = D.coded;
  for (int i = tid; i < kSlots; i += kThreads) {
    slot_val[i] = 0;
    head[i] = -1;
    first_tag[i] = 0;
    list_tag[i] = 0;
    umin[i] = 0xffffffffu;
    umax[i] = 0;
  }
  if (tid < kSlots / 32) slot_set[tid] = 0;
  if (tid < 2) slow[tid] = 0;
  __syncthreads();

  const int nblocks = (n + kBlock - 1) / kBlock;
#ifdef WG_K7_STATS
  uint64_t k7_acc[8] = {}, k7_t = __builtin_amdgcn_s_memtime();
  unsigned long long k7_slow = 0, k7_rounds = 0;
#endif
  for (int b = 0; b < nblocks; ++b) {
    const int base = b * kBlock;
    const uint32_t tag = (uint32_t)(b + 1) << kLocalBits;  // 0 never matches: fresh arrays
    const int li0 = kPer * tid;
    const int pos0 = base + li0;
    int* slow_b = &slow[b & 1];
    if (tid == 0) {
      slow[(b + 1) & 1] = 0;  // last read in block b - 1, next written in block b + 1
      first_pend[0] = kBlock;
    }
    // register an updater (value known) in the block's per-hash structures
    auto reg = [&](int li, uint32_t v) {
      const uint32_t h = hash_px(v, shift);
      atomicMax(&head[h], base + li);
      atomicMax(&first_tag[h], tag | (uint32_t)(kBlock - 1 - li));
      atomicMin(&umin[h], v);
      atomicMax(&umax[h], v);
      const uint32_t prev = atomicExch(&list_tag[h], tag | (uint32_t)li);
      nxt[li] = (prev & ~(uint32_t)(kBlock - 1)) == tag ? (int16_t)(prev & (kBlock - 1)) : (int16_t)-1;
    };
    // ---- 1. tokens, literals, far copies; register those updaters
    uint32_t tk[kPer];
    if (pos0 + kPer <= n) {
      const uint4 q = *reinterpret_cast<const uint4*>(tokens + pos0);
      tk[0] = q.x, tk[1] = q.y, tk[2] = q.z, tk[3] = q.w;
    } else {
#pragma unroll
      for (int j = 0; j < kPer; ++j) tk[j] = pos0 + j < n ? tokens[pos0 + j] : kTokUnset;
    }
    *reinterpret_cast<uint4*>(&toks[li0]) = make_uint4(tk[0], tk[1], tk[2], tk[3]);
    uint32_t v[kPer];
    uint8_t pend[kPer];  // 0 done, else kPendCopy / kPendLookup
    bool upd[kPer];
    bool bad = false, local_slow = false;
    __syncthreads();  // (first_pend reset before the atomics below)
#pragma unroll
    for (int j = 0; j < kPer; ++j) {
      const int li = li0 + j, pos = base + li;
      const uint32_t t = tk[j], kind = t & ~kTokPayload, pl = t & kTokPayload;
      v[j] = 0;
      pend[j] = 0;
      upd[j] = false;
      if (kind == kTokLiteral) {
        if (pl < (uint32_t)D.n_lits) v[j] = lits[pl];
        else bad = true;
        upd[j] = true;
      } else if (kind == kTokCopy) {
        const int s = pos - (int)pl;
        if (pl == 0 || s < 0) {
          bad = true;
        } else if (s < base) {
          v[j] = coded[s];
          upd[j] = true;
        } else {
          pend[j] = kPendCopy;
          ref[li] = (int16_t)(s - base);
          atomicMin(&first_pend[0], li);
        }
      } else if (kind == kTokCache) {
        if (pl >= (uint32_t)kSlots) bad = true;
        else pend[j] = kPendLookup;
      }
      st[li] = pend[j] ? pend[j] : kKnown;
      if (upd[j] && cache_bits) reg(li, v[j]);
    }
    *reinterpret_cast<uint4*>(&val[li0]) = make_uint4(v[0], v[1], v[2], v[3]);
    if (bad) atomicOr(err, 4);
#ifdef WG_K7_STATS
    if (bad) atomicAdd(&g_k7_stats[7], 1ull);
#endif
    local_slow = bad;
    int any_pend = __syncthreads_or(pend[0] | pend[1] | pend[2] | pend[3]);
    K7_T(3);
    // ---- 2. rounds
    for (int r = 0; any_pend; ++r) {
#ifdef WG_K7_STATS
      ++k7_rounds;
#endif
      if (r == kMaxRounds) {
#ifdef WG_K7_STATS
        if (tid == 0) atomicAdd(&g_k7_stats[10], 1ull);
#endif
        local_slow = true;
        break;  // uniform: any_pend and r are the same in every thread
      }
      const int fp = first_pend[r & 1];
      if (tid == 0) first_pend[(r + 1) & 1] = kBlock;  // read in round r - 1, written below after a barrier
      // (a) lookups before the first pending copy.  Everything a lookup needs is indexed by its
      //     key alone: the four table reads of the lane's four pixels issue together.
      uint32_t ft[kPer], sv[kPer], sw[kPer];
      int hd[kPer];
      bool act[kPer];
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        act[j] = pend[j] == kPendLookup && li0 + j < fp;
        const uint32_t k = act[j] ? tk[j] & kTokPayload : 0u;
        ft[j] = first_tag[k];
        hd[j] = head[k];
        sv[j] = slot_val[k];
        sw[j] = slot_set[k >> 5];
      }
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if (!act[j]) continue;
        const int li = li0 + j;
        const uint32_t k = tk[j] & kTokPayload;
        const bool in_block = (ft[j] & ~(uint32_t)(kBlock - 1)) == tag;
        const int first = in_block ? kBlock - 1 - (int)(ft[j] & (kBlock - 1)) : kBlock;
        uint32_t x;
        if (first >= li) {  // (an updater is never a lookup: first != li)
          if (k != 0 && !((sw[j] >> (k & 31)) & 1)) {
            local_slow = true;
#ifdef WG_K7_STATS
            atomicAdd(&g_k7_stats[8], 1ull);
#endif
          }
          x = sv[j];
        } else {
          const int last = hd[j] - base;
          const uint32_t lo = umin[k];
          if (last < li) {
            x = val[last];
          } else if (lo == umax[k]) {
            x = lo;
          } else {
            int best = -1, cur = (int)(list_tag[k] & (kBlock - 1)), steps = 0;
            while (cur >= 0 && steps < kMaxWalk) {
              if (cur < li && cur > best) best = cur;
              cur = nxt[cur];
              ++steps;
            }
            if (cur >= 0) {
              local_slow = true;
#ifdef WG_K7_STATS
              atomicAdd(&g_k7_stats[9], 1ull);
#endif
            }
            x = best >= 0 ? val[best] : 0;
          }
        }
        v[j] = x;
        pend[j] = 0;
        val[li] = x;  // (read by copies in (b), after the barrier)
        st[li] = kKnown;
      }
      __syncthreads();
      // (b) pending copies: take a known source's value, else jump one link back
      bool still = false;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        const int li = li0 + j;
        if (pend[j] != kPendCopy) {
          still |= pend[j] != 0;
          continue;
        }
        const int src = ref[li];
        const uint8_t ss = st[src];
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        if (ss == kKnown) {
          const uint32_t x = val[src];
          v[j] = x;
          pend[j] = 0;
          upd[j] = true;
          val[li] = x;
          __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
          st[li] = kKnown;
          if (cache_bits) reg(li, x);
        } else {
          if (ss == kPendCopy) ref[li] = ref[src];  // (a stale or fresh link: both lie on the chain)
          atomicMin(&first_pend[(r + 1) & 1], li);
          still = true;
        }
      }
      any_pend = __syncthreads_or(still);
    }
    if (local_slow) *slow_b = 1;
    K7_T(4);
    if (pos0 + kPer <= n) {
      *reinterpret_cast<uint4*>(coded + pos0) = make_uint4(v[0], v[1], v[2], v[3]);
    } else {
#pragma unroll
      for (int j = 0; j < kPer; ++j)
        if (pos0 + j < n) coded[pos0 + j] = v[j];
    }
    __syncthreads();
    K7_T(5);
    // ---- 3. the slot table after the block
    if (*slow_b) {
#ifdef WG_K7_STATS
      ++k7_slow;
#endif
      // DecodeImageData's order, one pixel at a time, on the table as the previous block
      // left it (step 2 only read it).  Literal and far-copy values are final in val[] from
      // step 1; everything else is recomputed here.
      if (tid == 0) {
        const int cnt = min(kBlock, n - base);
        for (int li = 0; li < cnt; ++li) {
          const int pos = base + li;
          const uint32_t t = toks[li], kind = t & ~kTokPayload, pl = t & kTokPayload;
          uint32_t x = 0;
          if (kind == kTokLiteral) {
            x = val[li];
          } else if (kind == kTokCopy) {
            const int s = pos - (int)pl;
            x = (pl == 0 || s < 0) ? 0 : s < base ? val[li] : val[s - base];
          } else if (kind == kTokCache) {
            x = pl < (uint32_t)kSlots ? slot_val[pl] : 0;
          }
          if (kind != kTokUnset && cache_bits) {
            const uint32_t h = hash_px(x, shift);
            slot_val[h] = x;
            slot_set[h >> 5] |= 1u << (h & 31);
          }
          val[li] = x;
          coded[pos] = x;
        }
      }
      __syncthreads();
    }
    if (cache_bits) {
      // each hash's last registered updater (every hash with one has one) resets its value
      // range; on the fast path it also writes the slot
      const bool fast = !*slow_b;
#pragma unroll
      for (int j = 0; j < kPer; ++j) {
        if (!upd[j]) continue;
        const uint32_t h = hash_px(v[j], shift);
        if (head[h] == base + li0 + j) {
          umin[h] = 0xffffffffu;
          umax[h] = 0;
          if (fast) {
            slot_val[h] = v[j];
            atomicOr(&slot_set[h >> 5], 1u << (h & 31));
          }
        }
      }
    }
    __syncthreads();
    K7_T(6);
  }
#ifdef WG_K7_STATS
  if (tid == 0) {
    atomicAdd(&g_k7_stats[0], (unsigned long long)nblocks);
    atomicAdd(&g_k7_stats[1], k7_slow);
    atomicAdd(&g_k7_stats[2], k7_rounds);
    for (int i = 3; i < 7; ++i) atomicAdd(&g_k7_stats[i], k7_acc[i]);
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

hipError_t launch_vp8l_resolve(const LLTokDesc* d_descs, int n, int* d_err, hipStream_t stream) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(vp8l_resolve_kernel, dim3(n), dim3(kThreads), 0, stream, d_descs, d_err);
  return hipGetLastError();
}

}  // namespace wg
