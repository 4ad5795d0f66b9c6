/*
 * vp8_dsp_oracle.c -- CPU restatement of the reference's VP8 decode DSP path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker for the HIP kernels
 * (tests/, __graft_entry__.smoke()) and the timed CPU baseline (bench.py
 * cpu_baseline leg).  Nothing in the product library links or calls it.
 *
 * Pinning: the reference (DaanV2/go-webp) cannot be built (no Go toolchain, and
 * the tree does not compile: SURVEY.md §2.3, §8(c)); its own tests pin nothing on
 * this path.  This restatement is pinned instead against libwebp 1.6.0 -- the
 * exact C library the reference translates (pkg/vp8/constants.go:18-20) -- run
 * with its plain-C kernels in the build container (tests/golden/make_golden.py):
 * post-filter YUV, bypass-filter YUV, fancy RGBA and point-sampled RGBA of 22
 * lossy fixtures must match byte for byte (tests/test_oracle.py).
 *
 * Input is the libwebp macroblock model produced by the host entropy stage
 * (wg_vp8_mb == VP8MBData + VP8FInfo, pkg/vp8/models.go:66-107).  Semantics
 * follow, function by function (file:line in /root/reference):
 *   clip tables                 pkg/libwebp/dsp/dec_clip_tables.go:13-28 (signed
 *                               sclip1/sclip2 per dsp.h.go:115-116, clip1 restored)
 *   TransformOne/AC3/DC/UV/DCUV pkg/libwebp/dsp/dec.c.go:29-134, MUL1/MUL2 dsp.h.go
 *   DoTransform/DoUVTransform   pkg/libwebp/decoder/frame_dec.c.go:43-67
 *   intra predictors            pkg/libwebp/dsp/dec.c.go:178-474, indexed by the
 *                               mode enum (decoder/enums.go:14-25), NOT by the
 *                               mis-ordered table at dec.c.go:727
 *   CheckMode, ReconstructRow   pkg/libwebp/decoder/frame_dec.c.go:28-37, 69-197
 *   loop filters                pkg/libwebp/dsp/dec.c.go:484-682
 *   DoFilter / FilterRow        pkg/libwebp/decoder/frame_dec.c.go:204-261
 *   fancy upsampler             pkg/libwebp/dsp/upsampling.c.go:43-107 + the
 *                               EmitFancyRGB row loop, decoder/io_dec.c.go:65-115
 *   point sampler               io_dec.c.go:53-59, dsp/yuv.go:19-58
 *   YUV->RGB                    pkg/color/yuv/conversion.go:28-49
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/gowebp_amd.h"

#define BPS 32
#define YUV_SIZE (BPS * 17 + BPS * 9)
#define Y_OFF (BPS * 1 + 8)
#define U_OFF (Y_OFF + BPS * 16 + BPS)
#define V_OFF (U_OFF + 16)

/* ------------------------------------------------------------------ clip helpers */
static int clip_8b(int v) { return (!(v & ~0xff)) ? v : (v < 0) ? 0 : 255; } /* dec.c.go:29-31 */
static int abs0(int v) { return v < 0 ? -v : v; }                              /* VP8kabs0 */
static int sclip1(int v) { return v < -128 ? -128 : v > 127 ? 127 : v; }       /* [-1020,1020]->[-128,127] */
static int sclip2(int v) { return v < -16 ? -16 : v > 15 ? 15 : v; }           /* [-112,112]->[-16,15] */
static int clip1(int v) { return v < 0 ? 0 : v > 255 ? 255 : v; }              /* [-255,511]->[0,255] */

/* 32-bit wrapping multiply-high helpers (C int arithmetic as compiled by gcc) */
static int mul1(int a) { return (int)(((int32_t)((uint32_t)a * 20091u)) >> 16) + a; }
static int mul2(int a) { return (int)(((int32_t)((uint32_t)a * 35468u)) >> 16); }

/* ------------------------------------------------------------------ transforms */
#define STORE(x, y, v) dst[(x) + (y) * BPS] = (uint8_t)clip_8b(dst[(x) + (y) * BPS] + ((v) >> 3))

static void TransformOne(const int16_t* in, uint8_t* dst) {
  int C[4 * 4], *tmp = C;
  for (int i = 0; i < 4; ++i) { /* vertical pass */
    const int a = in[0] + in[8];
    const int b = in[0] - in[8];
    const int c = mul2(in[4]) - mul1(in[12]);
    const int d = mul1(in[4]) + mul2(in[12]);
    tmp[0] = a + d;
    tmp[1] = b + c;
    tmp[2] = b - c;
    tmp[3] = a - d;
    tmp += 4;
    in++;
  }
  tmp = C;
  for (int i = 0; i < 4; ++i) { /* horizontal pass */
    const int dc = tmp[0] + 4;
    const int a = dc + tmp[8];
    const int b = dc - tmp[8];
    const int c = mul2(tmp[4]) - mul1(tmp[12]);
    const int d = mul1(tmp[4]) + mul2(tmp[12]);
    STORE(0, 0, a + d);
    STORE(1, 0, b + c);
    STORE(2, 0, b - c);
    STORE(3, 0, a - d);
    tmp++;
    dst += BPS;
  }
}

static void TransformAC3(const int16_t* in, uint8_t* dst) {
  const int a = in[0] + 4;
  const int c4 = mul2(in[4]);
  const int d4 = mul1(in[4]);
  const int c1 = mul2(in[1]);
  const int d1 = mul1(in[1]);
  const int dcs[4] = {a + d4, a + c4, a - c4, a - d4};
  for (int y = 0; y < 4; ++y) {
    const int DC = dcs[y];
    STORE(0, y, DC + d1);
    STORE(1, y, DC + c1);
    STORE(2, y, DC - c1);
    STORE(3, y, DC - d1);
  }
}

static void TransformDC(const int16_t* in, uint8_t* dst) {
  const int DC = in[0] + 4;
  for (int j = 0; j < 4; ++j)
    for (int i = 0; i < 4; ++i) STORE(i, j, DC);
}
#undef STORE

static void TransformUV(const int16_t* in, uint8_t* dst) {
  TransformOne(in + 0 * 16, dst);
  TransformOne(in + 1 * 16, dst + 4);
  TransformOne(in + 2 * 16, dst + 4 * BPS);
  TransformOne(in + 3 * 16, dst + 4 * BPS + 4);
}

static void TransformDCUV(const int16_t* in, uint8_t* dst) {
  if (in[0 * 16]) TransformDC(in + 0 * 16, dst);
  if (in[1 * 16]) TransformDC(in + 1 * 16, dst + 4);
  if (in[2 * 16]) TransformDC(in + 2 * 16, dst + 4 * BPS);
  if (in[3 * 16]) TransformDC(in + 3 * 16, dst + 4 * BPS + 4);
}

static void DoTransform(uint32_t bits, const int16_t* src, uint8_t* dst) {
  switch (bits >> 30) {
    case 3: TransformOne(src, dst); break;
    case 2: TransformAC3(src, dst); break;
    case 1: TransformDC(src, dst); break;
    default: break;
  }
}

static void DoUVTransform(uint32_t bits, const int16_t* src, uint8_t* dst) {
  if (bits & 0xff) {
    if (bits & 0xaa) TransformUV(src, dst);
    else TransformDCUV(src, dst);
  }
}

/* ------------------------------------------------------------------ predictors */
#define DST(x, y) dst[(x) + (y) * BPS]
#define AVG3(a, b, c) ((uint8_t)(((a) + 2 * (b) + (c) + 2) >> 2))
#define AVG2(a, b) (((a) + (b) + 1) >> 1)

static void TrueMotion(uint8_t* dst, int size) {
  const uint8_t* top = dst - BPS;
  const int tl = top[-1];
  for (int y = 0; y < size; ++y) {
    const int l = dst[-1];
    for (int x = 0; x < size; ++x) dst[x] = (uint8_t)clip1(top[x] + l - tl);
    dst += BPS;
  }
}

static void Fill(uint8_t* dst, int v, int size) {
  for (int j = 0; j < size; ++j) memset(dst + j * BPS, v, size);
}

/* 16x16 */
static void VE16(uint8_t* dst) { for (int j = 0; j < 16; ++j) memcpy(dst + j * BPS, dst - BPS, 16); }
static void HE16(uint8_t* dst) { for (int j = 0; j < 16; ++j) memset(dst + j * BPS, dst[j * BPS - 1], 16); }
static void DC16(uint8_t* dst) {
  int DC = 16;
  for (int j = 0; j < 16; ++j) DC += dst[-1 + j * BPS] + dst[j - BPS];
  Fill(dst, DC >> 5, 16);
}
static void DC16NoTop(uint8_t* dst) {
  int DC = 8;
  for (int j = 0; j < 16; ++j) DC += dst[-1 + j * BPS];
  Fill(dst, DC >> 4, 16);
}
static void DC16NoLeft(uint8_t* dst) {
  int DC = 8;
  for (int i = 0; i < 16; ++i) DC += dst[i - BPS];
  Fill(dst, DC >> 4, 16);
}
static void DC16NoTopLeft(uint8_t* dst) { Fill(dst, 0x80, 16); }
static void TM16(uint8_t* dst) { TrueMotion(dst, 16); }

/* chroma 8x8 */
static void VE8uv(uint8_t* dst) { for (int j = 0; j < 8; ++j) memcpy(dst + j * BPS, dst - BPS, 8); }
static void HE8uv(uint8_t* dst) { for (int j = 0; j < 8; ++j) memset(dst + j * BPS, dst[j * BPS - 1], 8); }
static void DC8uv(uint8_t* dst) {
  int dc0 = 8;
  for (int i = 0; i < 8; ++i) dc0 += dst[i - BPS] + dst[-1 + i * BPS];
  Fill(dst, dc0 >> 4, 8);
}
static void DC8uvNoLeft(uint8_t* dst) {
  int dc0 = 4;
  for (int i = 0; i < 8; ++i) dc0 += dst[i - BPS];
  Fill(dst, dc0 >> 3, 8);
}
static void DC8uvNoTop(uint8_t* dst) {
  int dc0 = 4;
  for (int i = 0; i < 8; ++i) dc0 += dst[-1 + i * BPS];
  Fill(dst, dc0 >> 3, 8);
}
static void DC8uvNoTopLeft(uint8_t* dst) { Fill(dst, 0x80, 8); }
static void TM8uv(uint8_t* dst) { TrueMotion(dst, 8); }

/* 4x4 */
static void DC4(uint8_t* dst) {
  int dc = 4;
  for (int i = 0; i < 4; ++i) dc += dst[i - BPS] + dst[-1 + i * BPS];
  dc >>= 3;
  for (int i = 0; i < 4; ++i) memset(dst + i * BPS, dc, 4);
}
static void TM4(uint8_t* dst) { TrueMotion(dst, 4); }
static void VE4(uint8_t* dst) {
  const uint8_t* top = dst - BPS;
  const uint8_t vals[4] = {AVG3(top[-1], top[0], top[1]), AVG3(top[0], top[1], top[2]),
                           AVG3(top[1], top[2], top[3]), AVG3(top[2], top[3], top[4])};
  for (int i = 0; i < 4; ++i) memcpy(dst + i * BPS, vals, 4);
}
static void HE4(uint8_t* dst) {
  const int A = dst[-1 - BPS], B = dst[-1], C = dst[-1 + BPS], D = dst[-1 + 2 * BPS], E = dst[-1 + 3 * BPS];
  memset(dst + 0 * BPS, AVG3(A, B, C), 4);
  memset(dst + 1 * BPS, AVG3(B, C, D), 4);
  memset(dst + 2 * BPS, AVG3(C, D, E), 4);
  memset(dst + 3 * BPS, AVG3(D, E, E), 4);
}
static void RD4(uint8_t* dst) {
  const int I = dst[-1 + 0 * BPS], J = dst[-1 + 1 * BPS], K = dst[-1 + 2 * BPS], L = dst[-1 + 3 * BPS];
  const int X = dst[-1 - BPS], A = dst[0 - BPS], B = dst[1 - BPS], C = dst[2 - BPS], D = dst[3 - BPS];
  DST(0, 3) = AVG3(J, K, L);
  DST(1, 3) = DST(0, 2) = AVG3(I, J, K);
  DST(2, 3) = DST(1, 2) = DST(0, 1) = AVG3(X, I, J);
  DST(3, 3) = DST(2, 2) = DST(1, 1) = DST(0, 0) = AVG3(A, X, I);
  DST(3, 2) = DST(2, 1) = DST(1, 0) = AVG3(B, A, X);
  DST(3, 1) = DST(2, 0) = AVG3(C, B, A);
  DST(3, 0) = AVG3(D, C, B);
}
static void LD4(uint8_t* dst) {
  const int A = dst[0 - BPS], B = dst[1 - BPS], C = dst[2 - BPS], D = dst[3 - BPS];
  const int E = dst[4 - BPS], F = dst[5 - BPS], G = dst[6 - BPS], H = dst[7 - BPS];
  DST(0, 0) = AVG3(A, B, C);
  DST(1, 0) = DST(0, 1) = AVG3(B, C, D);
  DST(2, 0) = DST(1, 1) = DST(0, 2) = AVG3(C, D, E);
  DST(3, 0) = DST(2, 1) = DST(1, 2) = DST(0, 3) = AVG3(D, E, F);
  DST(3, 1) = DST(2, 2) = DST(1, 3) = AVG3(E, F, G);
  DST(3, 2) = DST(2, 3) = AVG3(F, G, H);
  DST(3, 3) = AVG3(G, H, H);
}
static void VR4(uint8_t* dst) {
  const int I = dst[-1 + 0 * BPS], J = dst[-1 + 1 * BPS], K = dst[-1 + 2 * BPS];
  const int X = dst[-1 - BPS], A = dst[0 - BPS], B = dst[1 - BPS], C = dst[2 - BPS], D = dst[3 - BPS];
  DST(0, 0) = DST(1, 2) = AVG2(X, A);
  DST(1, 0) = DST(2, 2) = AVG2(A, B);
  DST(2, 0) = DST(3, 2) = AVG2(B, C);
  DST(3, 0) = AVG2(C, D);
  DST(0, 3) = AVG3(K, J, I);
  DST(0, 2) = AVG3(J, I, X);
  DST(0, 1) = DST(1, 3) = AVG3(I, X, A);
  DST(1, 1) = DST(2, 3) = AVG3(X, A, B);
  DST(2, 1) = DST(3, 3) = AVG3(A, B, C);
  DST(3, 1) = AVG3(B, C, D);
}
static void VL4(uint8_t* dst) {
  const int A = dst[0 - BPS], B = dst[1 - BPS], C = dst[2 - BPS], D = dst[3 - BPS];
  const int E = dst[4 - BPS], F = dst[5 - BPS], G = dst[6 - BPS], H = dst[7 - BPS];
  DST(0, 0) = AVG2(A, B);
  DST(1, 0) = DST(0, 2) = AVG2(B, C);
  DST(2, 0) = DST(1, 2) = AVG2(C, D);
  DST(3, 0) = DST(2, 2) = AVG2(D, E);
  DST(0, 1) = AVG3(A, B, C);
  DST(1, 1) = DST(0, 3) = AVG3(B, C, D);
  DST(2, 1) = DST(1, 3) = AVG3(C, D, E);
  DST(3, 1) = DST(2, 3) = AVG3(D, E, F);
  DST(3, 2) = AVG3(E, F, G);
  DST(3, 3) = AVG3(F, G, H);
}
static void HU4(uint8_t* dst) {
  const int I = dst[-1 + 0 * BPS], J = dst[-1 + 1 * BPS], K = dst[-1 + 2 * BPS], L = dst[-1 + 3 * BPS];
  DST(0, 0) = AVG2(I, J);
  DST(2, 0) = DST(0, 1) = AVG2(J, K);
  DST(2, 1) = DST(0, 2) = AVG2(K, L);
  DST(1, 0) = AVG3(I, J, K);
  DST(3, 0) = DST(1, 1) = AVG3(J, K, L);
  DST(3, 1) = DST(1, 2) = AVG3(K, L, L);
  DST(3, 2) = DST(2, 2) = DST(0, 3) = DST(1, 3) = DST(2, 3) = DST(3, 3) = L;
}
static void HD4(uint8_t* dst) {
  const int I = dst[-1 + 0 * BPS], J = dst[-1 + 1 * BPS], K = dst[-1 + 2 * BPS], L = dst[-1 + 3 * BPS];
  const int X = dst[-1 - BPS], A = dst[0 - BPS], B = dst[1 - BPS], C = dst[2 - BPS];
  DST(0, 0) = DST(2, 1) = AVG2(I, X);
  DST(0, 1) = DST(2, 2) = AVG2(J, I);
  DST(0, 2) = DST(2, 3) = AVG2(K, J);
  DST(0, 3) = AVG2(L, K);
  DST(3, 0) = AVG3(A, B, C);
  DST(2, 0) = AVG3(X, A, B);
  DST(1, 0) = DST(3, 1) = AVG3(I, X, A);
  DST(1, 1) = DST(3, 2) = AVG3(J, I, X);
  DST(1, 2) = DST(3, 3) = AVG3(K, J, I);
  DST(1, 3) = AVG3(L, K, J);
}
#undef DST
#undef AVG3
#undef AVG2

typedef void (*PredFunc)(uint8_t* dst);
/* index = B_* mode enum: DC TM VE HE RD VR LD VL HD HU (decoder/enums.go:14-25) */
static const PredFunc kPredLuma4[10] = {DC4, TM4, VE4, HE4, RD4, VR4, LD4, VL4, HD4, HU4};
/* DC TM VE HE DC_NOTOP DC_NOLEFT DC_NOTOPLEFT (dec.c.go:728-729) */
static const PredFunc kPredLuma16[7] = {DC16, TM16, VE16, HE16, DC16NoTop, DC16NoLeft, DC16NoTopLeft};
static const PredFunc kPredChroma8[7] = {DC8uv, TM8uv, VE8uv, HE8uv, DC8uvNoTop, DC8uvNoLeft, DC8uvNoTopLeft};

static int CheckMode(int mb_x, int mb_y, int mode) { /* frame_dec.c.go:28-37 */
  if (mode == 0) {
    if (mb_x == 0) return (mb_y == 0) ? 6 : 5;
    return (mb_y == 0) ? 4 : 0;
  }
  return mode;
}

static const int kScan[16] = {0 + 0 * BPS,  4 + 0 * BPS,  8 + 0 * BPS,  12 + 0 * BPS,
                              0 + 4 * BPS,  4 + 4 * BPS,  8 + 4 * BPS,  12 + 4 * BPS,
                              0 + 8 * BPS,  4 + 8 * BPS,  8 + 8 * BPS,  12 + 8 * BPS,
                              0 + 12 * BPS, 4 + 12 * BPS, 8 + 12 * BPS, 12 + 12 * BPS};

/* ReconstructRow (frame_dec.c.go:69-197): one MB row into full padded planes. */
static void ReconstructRow(const wg_vp8_info* info, const wg_vp8_mb* row, int mb_y, uint8_t* yuv_b,
                           uint8_t* yuv_t /* [mb_w][32]: y16 u8 v8 */, uint8_t* Y, uint8_t* U, uint8_t* V) {
  const int mb_w = info->mb_w, mb_h = info->mb_h;
  const int ys = 16 * mb_w, uvs = 8 * mb_w;
  uint8_t* const y_dst = yuv_b + Y_OFF;
  uint8_t* const u_dst = yuv_b + U_OFF;
  uint8_t* const v_dst = yuv_b + V_OFF;
  for (int j = 0; j < 16; ++j) y_dst[j * BPS - 1] = 129;
  for (int j = 0; j < 8; ++j) {
    u_dst[j * BPS - 1] = 129;
    v_dst[j * BPS - 1] = 129;
  }
  if (mb_y > 0) {
    y_dst[-1 - BPS] = u_dst[-1 - BPS] = v_dst[-1 - BPS] = 129;
  } else {
    memset(y_dst - BPS - 1, 127, 16 + 4 + 1);
    memset(u_dst - BPS - 1, 127, 8 + 1);
    memset(v_dst - BPS - 1, 127, 8 + 1);
  }
  for (int mb_x = 0; mb_x < mb_w; ++mb_x) {
    const wg_vp8_mb* block = row + mb_x;
    if (mb_x > 0) {
      for (int j = -1; j < 16; ++j) memcpy(&y_dst[j * BPS - 4], &y_dst[j * BPS + 12], 4);
      for (int j = -1; j < 8; ++j) {
        memcpy(&u_dst[j * BPS - 4], &u_dst[j * BPS + 4], 4);
        memcpy(&v_dst[j * BPS - 4], &v_dst[j * BPS + 4], 4);
      }
    }
    {
      uint8_t* const top = yuv_t + 32 * mb_x;
      const int16_t* const coeffs = block->coeffs;
      uint32_t bits = block->non_zero_y;
      if (mb_y > 0) {
        memcpy(y_dst - BPS, top, 16);
        memcpy(u_dst - BPS, top + 16, 8);
        memcpy(v_dst - BPS, top + 24, 8);
      }
      if (block->is_i4x4) {
        uint8_t* const top_right = y_dst - BPS + 16;
        if (mb_y > 0) {
          if (mb_x >= mb_w - 1) memset(top_right, top[15], 4);
          else memcpy(top_right, top + 32, 4);
        }
        memcpy(top_right + BPS * 4, top_right, 4);
        memcpy(top_right + BPS * 8, top_right, 4);
        memcpy(top_right + BPS * 12, top_right, 4);
        for (int n = 0; n < 16; ++n, bits <<= 2) {
          uint8_t* const dst = y_dst + kScan[n];
          kPredLuma4[block->imodes[n]](dst);
          DoTransform(bits, coeffs + n * 16, dst);
        }
      } else {
        kPredLuma16[CheckMode(mb_x, mb_y, block->imodes[0])](y_dst);
        if (bits != 0) {
          for (int n = 0; n < 16; ++n, bits <<= 2) DoTransform(bits, coeffs + n * 16, y_dst + kScan[n]);
        }
      }
      {
        const uint32_t bits_uv = block->non_zero_uv;
        const int pred_func = CheckMode(mb_x, mb_y, block->uvmode);
        kPredChroma8[pred_func](u_dst);
        kPredChroma8[pred_func](v_dst);
        DoUVTransform(bits_uv >> 0, coeffs + 16 * 16, u_dst);
        DoUVTransform(bits_uv >> 8, coeffs + 20 * 16, v_dst);
      }
      if (mb_y < mb_h - 1) {
        memcpy(top, y_dst + 15 * BPS, 16);
        memcpy(top + 16, u_dst + 7 * BPS, 8);
        memcpy(top + 24, v_dst + 7 * BPS, 8);
      }
    }
    for (int j = 0; j < 16; ++j) memcpy(Y + (size_t)(mb_y * 16 + j) * ys + mb_x * 16, y_dst + j * BPS, 16);
    for (int j = 0; j < 8; ++j) {
      memcpy(U + (size_t)(mb_y * 8 + j) * uvs + mb_x * 8, u_dst + j * BPS, 8);
      memcpy(V + (size_t)(mb_y * 8 + j) * uvs + mb_x * 8, v_dst + j * BPS, 8);
    }
  }
}

/* ------------------------------------------------------------------ loop filter */
static void DoFilter2(uint8_t* p, int step) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  const int a = 3 * (q0 - p0) + sclip1(p1 - q1);
  const int a1 = sclip2((a + 4) >> 3);
  const int a2 = sclip2((a + 3) >> 3);
  p[-step] = (uint8_t)clip1(p0 + a2);
  p[0] = (uint8_t)clip1(q0 - a1);
}
static void DoFilter4(uint8_t* p, int step) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  const int a = 3 * (q0 - p0);
  const int a1 = sclip2((a + 4) >> 3);
  const int a2 = sclip2((a + 3) >> 3);
  const int a3 = (a1 + 1) >> 1;
  p[-2 * step] = (uint8_t)clip1(p1 + a3);
  p[-step] = (uint8_t)clip1(p0 + a2);
  p[0] = (uint8_t)clip1(q0 - a1);
  p[step] = (uint8_t)clip1(q1 - a3);
}
static void DoFilter6(uint8_t* p, int step) {
  const int p2 = p[-3 * step], p1 = p[-2 * step], p0 = p[-step];
  const int q0 = p[0], q1 = p[step], q2 = p[2 * step];
  const int a = sclip1(3 * (q0 - p0) + sclip1(p1 - q1));
  const int a1 = (27 * a + 63) >> 7;
  const int a2 = (18 * a + 63) >> 7;
  const int a3 = (9 * a + 63) >> 7;
  p[-3 * step] = (uint8_t)clip1(p2 + a3);
  p[-2 * step] = (uint8_t)clip1(p1 + a2);
  p[-step] = (uint8_t)clip1(p0 + a1);
  p[0] = (uint8_t)clip1(q0 - a1);
  p[step] = (uint8_t)clip1(q1 - a2);
  p[2 * step] = (uint8_t)clip1(q2 - a3);
}
static int Hev(const uint8_t* p, int step, int thresh) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  return (abs0(p1 - p0) > thresh) || (abs0(q1 - q0) > thresh);
}
static int NeedsFilter(const uint8_t* p, int step, int t) {
  const int p1 = p[-2 * step], p0 = p[-step], q0 = p[0], q1 = p[step];
  return ((4 * abs0(p0 - q0) + abs0(p1 - q1)) <= t);
}
static int NeedsFilter2(const uint8_t* p, int step, int t, int it) {
  const int p3 = p[-4 * step], p2 = p[-3 * step], p1 = p[-2 * step];
  const int p0 = p[-step], q0 = p[0];
  const int q1 = p[step], q2 = p[2 * step], q3 = p[3 * step];
  if ((4 * abs0(p0 - q0) + abs0(p1 - q1)) > t) return 0;
  return abs0(p3 - p2) <= it && abs0(p2 - p1) <= it && abs0(p1 - p0) <= it && abs0(q3 - q2) <= it &&
         abs0(q2 - q1) <= it && abs0(q1 - q0) <= it;
}
static void SimpleVFilter16(uint8_t* p, int stride, int thresh) {
  const int thresh2 = 2 * thresh + 1;
  for (int i = 0; i < 16; ++i)
    if (NeedsFilter(p + i, stride, thresh2)) DoFilter2(p + i, stride);
}
static void SimpleHFilter16(uint8_t* p, int stride, int thresh) {
  const int thresh2 = 2 * thresh + 1;
  for (int i = 0; i < 16; ++i)
    if (NeedsFilter(p + i * stride, 1, thresh2)) DoFilter2(p + i * stride, 1);
}
static void SimpleVFilter16i(uint8_t* p, int stride, int thresh) {
  for (int k = 3; k > 0; --k) {
    p += 4 * stride;
    SimpleVFilter16(p, stride, thresh);
  }
}
static void SimpleHFilter16i(uint8_t* p, int stride, int thresh) {
  for (int k = 3; k > 0; --k) {
    p += 4;
    SimpleHFilter16(p, stride, thresh);
  }
}
static void FilterLoop26(uint8_t* p, int hstride, int vstride, int size, int thresh, int ithresh, int hev_thresh) {
  const int thresh2 = 2 * thresh + 1;
  while (size-- > 0) {
    if (NeedsFilter2(p, hstride, thresh2, ithresh)) {
      if (Hev(p, hstride, hev_thresh)) DoFilter2(p, hstride);
      else DoFilter6(p, hstride);
    }
    p += vstride;
  }
}
static void FilterLoop24(uint8_t* p, int hstride, int vstride, int size, int thresh, int ithresh, int hev_thresh) {
  const int thresh2 = 2 * thresh + 1;
  while (size-- > 0) {
    if (NeedsFilter2(p, hstride, thresh2, ithresh)) {
      if (Hev(p, hstride, hev_thresh)) DoFilter2(p, hstride);
      else DoFilter4(p, hstride);
    }
    p += vstride;
  }
}
static void VFilter16(uint8_t* p, int s, int t, int it, int h) { FilterLoop26(p, s, 1, 16, t, it, h); }
static void HFilter16(uint8_t* p, int s, int t, int it, int h) { FilterLoop26(p, 1, s, 16, t, it, h); }
static void VFilter16i(uint8_t* p, int s, int t, int it, int h) {
  for (int k = 3; k > 0; --k) {
    p += 4 * s;
    FilterLoop24(p, s, 1, 16, t, it, h);
  }
}
static void HFilter16i(uint8_t* p, int s, int t, int it, int h) {
  for (int k = 3; k > 0; --k) {
    p += 4;
    FilterLoop24(p, 1, s, 16, t, it, h);
  }
}
static void VFilter8(uint8_t* u, uint8_t* v, int s, int t, int it, int h) {
  FilterLoop26(u, s, 1, 8, t, it, h);
  FilterLoop26(v, s, 1, 8, t, it, h);
}
static void HFilter8(uint8_t* u, uint8_t* v, int s, int t, int it, int h) {
  FilterLoop26(u, 1, s, 8, t, it, h);
  FilterLoop26(v, 1, s, 8, t, it, h);
}
static void VFilter8i(uint8_t* u, uint8_t* v, int s, int t, int it, int h) {
  FilterLoop24(u + 4 * s, s, 1, 8, t, it, h);
  FilterLoop24(v + 4 * s, s, 1, 8, t, it, h);
}
static void HFilter8i(uint8_t* u, uint8_t* v, int s, int t, int it, int h) {
  FilterLoop24(u + 4, 1, s, 8, t, it, h);
  FilterLoop24(v + 4, 1, s, 8, t, it, h);
}

/* DoFilter (frame_dec.c.go:204-251) on the full planes */
static void DoFilter(const wg_vp8_info* info, const wg_vp8_mb* mb, int mb_x, int mb_y, uint8_t* Y, uint8_t* U,
                     uint8_t* V) {
  const int y_bps = 16 * info->mb_w, uv_bps = 8 * info->mb_w;
  uint8_t* const y_dst = Y + (size_t)mb_y * 16 * y_bps + mb_x * 16;
  const int ilevel = mb->f_ilevel;
  const int limit = mb->f_limit;
  if (limit == 0) return;
  if (info->filter_type == 1) {
    if (mb_x > 0) SimpleHFilter16(y_dst, y_bps, limit + 4);
    if (mb->f_inner) SimpleHFilter16i(y_dst, y_bps, limit);
    if (mb_y > 0) SimpleVFilter16(y_dst, y_bps, limit + 4);
    if (mb->f_inner) SimpleVFilter16i(y_dst, y_bps, limit);
  } else {
    uint8_t* const u_dst = U + (size_t)mb_y * 8 * uv_bps + mb_x * 8;
    uint8_t* const v_dst = V + (size_t)mb_y * 8 * uv_bps + mb_x * 8;
    const int hev_thresh = mb->hev_thresh;
    if (mb_x > 0) {
      HFilter16(y_dst, y_bps, limit + 4, ilevel, hev_thresh);
      HFilter8(u_dst, v_dst, uv_bps, limit + 4, ilevel, hev_thresh);
    }
    if (mb->f_inner) {
      HFilter16i(y_dst, y_bps, limit, ilevel, hev_thresh);
      HFilter8i(u_dst, v_dst, uv_bps, limit, ilevel, hev_thresh);
    }
    if (mb_y > 0) {
      VFilter16(y_dst, y_bps, limit + 4, ilevel, hev_thresh);
      VFilter8(u_dst, v_dst, uv_bps, limit + 4, ilevel, hev_thresh);
    }
    if (mb->f_inner) {
      VFilter16i(y_dst, y_bps, limit, ilevel, hev_thresh);
      VFilter8i(u_dst, v_dst, uv_bps, limit, ilevel, hev_thresh);
    }
  }
}

/* ------------------------------------------------------------------ YUV -> RGBA */
static int MultHi(int v, int coeff) { return (v * coeff) >> 8; }
static int Clip8(int v) { return ((v & ~16383) == 0) ? (v >> 6) : (v < 0) ? 0 : 255; } /* YUV_FIX2=6 */
static void YuvToRgba(int y, int u, int v, uint8_t* rgba) {
  rgba[0] = (uint8_t)Clip8(MultHi(y, 19077) + MultHi(v, 26149) - 14234);
  rgba[1] = (uint8_t)Clip8(MultHi(y, 19077) - MultHi(u, 6419) - MultHi(v, 13320) + 8708);
  rgba[2] = (uint8_t)Clip8(MultHi(y, 19077) + MultHi(u, 33050) - 17685);
  rgba[3] = 0xff;
}

#define LOAD_UV(u, v) ((uint32_t)(u) | ((uint32_t)(v) << 16))
/* UpsampleRgbaLinePair_C (upsampling.c.go:43-107) */
static void UpsampleRgbaLinePair(const uint8_t* top_y, const uint8_t* bottom_y, const uint8_t* top_u,
                                 const uint8_t* top_v, const uint8_t* cur_u, const uint8_t* cur_v,
                                 uint8_t* top_dst, uint8_t* bottom_dst, int len) {
  const int last_pixel_pair = (len - 1) >> 1;
  uint32_t tl_uv = LOAD_UV(top_u[0], top_v[0]);
  uint32_t l_uv = LOAD_UV(cur_u[0], cur_v[0]);
  {
    const uint32_t uv0 = (3 * tl_uv + l_uv + 0x00020002u) >> 2;
    YuvToRgba(top_y[0], uv0 & 0xff, (uv0 >> 16), top_dst);
  }
  if (bottom_y != NULL) {
    const uint32_t uv0 = (3 * l_uv + tl_uv + 0x00020002u) >> 2;
    YuvToRgba(bottom_y[0], uv0 & 0xff, (uv0 >> 16), bottom_dst);
  }
  for (int x = 1; x <= last_pixel_pair; ++x) {
    const uint32_t t_uv = LOAD_UV(top_u[x], top_v[x]);
    const uint32_t uv = LOAD_UV(cur_u[x], cur_v[x]);
    const uint32_t avg = tl_uv + t_uv + l_uv + uv + 0x00080008u;
    const uint32_t diag_12 = (avg + 2 * (t_uv + l_uv)) >> 3;
    const uint32_t diag_03 = (avg + 2 * (tl_uv + uv)) >> 3;
    {
      const uint32_t uv0 = (diag_12 + tl_uv) >> 1;
      const uint32_t uv1 = (diag_03 + t_uv) >> 1;
      YuvToRgba(top_y[2 * x - 1], uv0 & 0xff, (uv0 >> 16), top_dst + (2 * x - 1) * 4);
      YuvToRgba(top_y[2 * x - 0], uv1 & 0xff, (uv1 >> 16), top_dst + (2 * x - 0) * 4);
    }
    if (bottom_y != NULL) {
      const uint32_t uv0 = (diag_03 + l_uv) >> 1;
      const uint32_t uv1 = (diag_12 + uv) >> 1;
      YuvToRgba(bottom_y[2 * x - 1], uv0 & 0xff, (uv0 >> 16), bottom_dst + (2 * x - 1) * 4);
      YuvToRgba(bottom_y[2 * x + 0], uv1 & 0xff, (uv1 >> 16), bottom_dst + (2 * x + 0) * 4);
    }
    tl_uv = t_uv;
    l_uv = uv;
  }
  if (!(len & 1)) {
    {
      const uint32_t uv0 = (3 * tl_uv + l_uv + 0x00020002u) >> 2;
      YuvToRgba(top_y[len - 1], uv0 & 0xff, (uv0 >> 16), top_dst + (len - 1) * 4);
    }
    if (bottom_y != NULL) {
      const uint32_t uv0 = (3 * l_uv + tl_uv + 0x00020002u) >> 2;
      YuvToRgba(bottom_y[len - 1], uv0 & 0xff, (uv0 >> 16), bottom_dst + (len - 1) * 4);
    }
  }
}
#undef LOAD_UV

/* EmitFancyRGB (io_dec.c.go:65-115) over the whole picture in one call. */
int oracle_yuv_to_rgba_fancy(const uint8_t* Y, int y_stride, const uint8_t* U, const uint8_t* V, int uv_stride,
                             uint8_t* rgba, int rgba_stride, int width, int height) {
  const uint8_t *cur_y = Y, *cur_u = U, *cur_v = V;
  uint8_t* dst = rgba;
  int y = 0;
  UpsampleRgbaLinePair(cur_y, NULL, cur_u, cur_v, cur_u, cur_v, dst, NULL, width);
  for (; y + 2 < height; y += 2) {
    const uint8_t* top_u = cur_u;
    const uint8_t* top_v = cur_v;
    cur_u += uv_stride;
    cur_v += uv_stride;
    dst += 2 * rgba_stride;
    cur_y += 2 * y_stride;
    UpsampleRgbaLinePair(cur_y - y_stride, cur_y, top_u, top_v, cur_u, cur_v, dst - rgba_stride, dst, width);
  }
  cur_y += y_stride;
  if (!(height & 1)) UpsampleRgbaLinePair(cur_y, NULL, cur_u, cur_v, cur_u, cur_v, dst + rgba_stride, NULL, width);
  return 0;
}

/* EmitSampledRGB -> WebPSamplerProcessPlane (yuv.go:19-58) */
int oracle_yuv_to_rgba_point(const uint8_t* Y, int y_stride, const uint8_t* U, const uint8_t* V, int uv_stride,
                             uint8_t* rgba, int rgba_stride, int width, int height) {
  for (int j = 0; j < height; ++j) {
    const uint8_t* y = Y + (size_t)j * y_stride;
    const uint8_t* u = U + (size_t)(j >> 1) * uv_stride;
    const uint8_t* v = V + (size_t)(j >> 1) * uv_stride;
    uint8_t* d = rgba + (size_t)j * rgba_stride;
    for (int i = 0; i < width; ++i) YuvToRgba(y[i], u[i >> 1], v[i >> 1], d + 4 * i);
  }
  return 0;
}

/* ------------------------------------------------------------------ frame driver */
/* Reconstruct (+ filter when info->filter_type > 0) a parsed frame into padded
 * planes: Y (16*mb_w x 16*mb_h), U/V (8*mb_w x 8*mb_h). */
int oracle_vp8_reconstruct(const wg_vp8_info* info, const wg_vp8_mb* mbs, uint8_t* Y, uint8_t* U, uint8_t* V) {
  const int mb_w = info->mb_w, mb_h = info->mb_h;
  uint8_t yuv_b[YUV_SIZE];
  uint8_t* yuv_t = (uint8_t*)calloc((size_t)mb_w + 1, 32);
  if (!yuv_t) return WG_STATUS_OUT_OF_MEMORY;
  memset(yuv_b, 0, sizeof(yuv_b));
  for (int mb_y = 0; mb_y < mb_h; ++mb_y) {
    const wg_vp8_mb* row = mbs + (size_t)mb_y * mb_w;
    ReconstructRow(info, row, mb_y, yuv_b, yuv_t, Y, U, V);
    if (info->filter_type > 0)
      for (int mb_x = 0; mb_x < mb_w; ++mb_x) DoFilter(info, row + mb_x, mb_x, mb_y, Y, U, V);
  }
  free(yuv_t);
  return WG_STATUS_OK;
}

/* Full CPU decode of a parsed frame: cropped planes (strides width, (width+1)/2)
 * and/or RGBA (stride 4*width).  Any output pointer may be NULL. */
int oracle_vp8_decode(const wg_vp8_info* info, const wg_vp8_mb* mbs, uint8_t* y_out, uint8_t* u_out,
                      uint8_t* v_out, uint8_t* rgba, int fancy) {
  const int mb_w = info->mb_w, mb_h = info->mb_h;
  const int ys = 16 * mb_w, uvs = 8 * mb_w;
  const int w = info->width, h = info->height, uw = (w + 1) / 2, uh = (h + 1) / 2;
  uint8_t* Y = (uint8_t*)malloc((size_t)ys * 16 * mb_h);
  uint8_t* U = (uint8_t*)malloc((size_t)uvs * 8 * mb_h);
  uint8_t* V = (uint8_t*)malloc((size_t)uvs * 8 * mb_h);
  if (!Y || !U || !V) {
    free(Y); free(U); free(V);
    return WG_STATUS_OUT_OF_MEMORY;
  }
  int st = oracle_vp8_reconstruct(info, mbs, Y, U, V);
  if (st == WG_STATUS_OK) {
    if (y_out)
      for (int j = 0; j < h; ++j) memcpy(y_out + (size_t)j * w, Y + (size_t)j * ys, w);
    if (u_out)
      for (int j = 0; j < uh; ++j) memcpy(u_out + (size_t)j * uw, U + (size_t)j * uvs, uw);
    if (v_out)
      for (int j = 0; j < uh; ++j) memcpy(v_out + (size_t)j * uw, V + (size_t)j * uvs, uw);
    if (rgba) {
      if (fancy) oracle_yuv_to_rgba_fancy(Y, ys, U, V, uvs, rgba, 4 * w, w, h);
      else oracle_yuv_to_rgba_point(Y, ys, U, V, uvs, rgba, 4 * w, w, h);
    }
  }
  free(Y); free(U); free(V);
  return st;
}

/* Isolated transform for known-answer tests: 0 = dispatch by code (libwebp), 1 = TransformOne. */
void oracle_transform_block(const int16_t* in, uint8_t* dst4x4_bps32, int code) {
  if (code < 0) TransformOne(in, dst4x4_bps32);
  else DoTransform((uint32_t)code << 30, in, dst4x4_bps32);
}

/* Isolated 4x4 luma predictor (mode = B_* enum) on a BPS=32 workspace whose block origin
 * is `dst` (known-answer tests of the device's per-pixel predictor table). */
void oracle_pred_luma4(int mode, uint8_t* dst) { kPredLuma4[mode](dst); }
