// ba3c_split.h — conv0 on bf16 MFMA with exact operand splitting (gfx950).
//
// conv0 (train.py:167-185) multiplies uint8 frame values by fp32 weights.  Every value 0..255
// is exact in bf16 (8 significant bits), and every fp32 weight w is exactly the sum of three
// bf16 numbers hi + mid + lo (8 + 8 + 8 significant bits, round-to-nearest at each stage,
// each residual exact in fp32).  So
//
//     sum_k u8_k * w_k  =  sum_k u8_k * hi_k + sum_k u8_k * mid_k + sum_k u8_k * lo_k
//
// where every product is exact (16 significant bits) and the sums accumulate in fp32 inside
// v_mfma_f32_16x16x32_bf16: three bf16 MFMAs give the fp32 convolution at fp32 accumulation
// accuracy, at 16/3 the fp32 MFMA rate.  The result is scaled by 1/255 once (TF scales each
// frame value first, train.py:167; both are within fp32 rounding of the exact sum).
//
// Operand layout of v_mfma_f32_16x16x32_bf16: lane l supplies row/column (l & 15) and eight
// K values of lane group q = l >> 4.  Only A and B agreeing on the K order matters, so
// K-step s, lane group q, element e is tap 8s + 2q + (e >> 2), frame channel e & 3: a lane's
// A fragment is two 8-byte LDS reads (two taps x 4 channels of one bf16 pixel).
#pragma once
#include "ba3c_conv.h"

namespace ba3c {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ bf16x8 as_bf16x8(uint2 a, uint2 b) {
  u32x4 u = {a.x, a.y, b.x, b.y};
  return __builtin_bit_cast(bf16x8, u);
}

// bf16 bits of a small non-negative integer (exact: <= 8 significant bits)
__device__ __forceinline__ uint32_t u8_bf16(uint32_t v) { return __float_as_uint((float)v) >> 16; }

// round-to-nearest-even fp32 -> bf16 bits (finite inputs) and back
__device__ __forceinline__ uint32_t f32_bf16_rne(float f) {
  const uint32_t u = __float_as_uint(f);
  return (u + 0x7FFFu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ float bf16_f32(uint32_t b) { return __uint_as_float(b << 16); }

// w = hi + mid + lo exactly (bf16 bits)
__device__ __forceinline__ void split3(float w, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  hi = f32_bf16_rne(w);
  const float r1 = w - bf16_f32(hi);
  mid = f32_bf16_rne(r1);
  const float r2 = r1 - bf16_f32(mid);
  lo = f32_bf16_rne(r2);
}

typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

// RNE fp32 pair -> packed bf16 pair (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, bf16x2v));
}
// (a, b) = hi + mid + lo exactly, each a packed bf16 pair (RNE at every stage)
__device__ __forceinline__ void split3x2(float a, float b, uint32_t& hi, uint32_t& mid, uint32_t& lo) {
  hi = pack_bf16x2(a, b);
  const float ra = a - __uint_as_float(hi << 16), rb = b - __uint_as_float(hi & 0xFFFF0000u);
  mid = pack_bf16x2(ra, rb);
  const float sa = ra - __uint_as_float(mid << 16), sb = rb - __uint_as_float(mid & 0xFFFF0000u);
  lo = pack_bf16x2(sa, sb);
}

// ---------------------------------------------------------------------------------------
// The second split family (default): fp16 hi + lo of a power-of-two-scaled value.
//
// x * 2^k = hi + lo + r with hi = RN_f16(x 2^k), lo = RN_f16(x 2^k - hi) (the difference is
// exact in fp32: Sterbenz), |r| <= 2^-22 |x 2^k|: 22 significant bits in two fp16 numbers.
// a*b = a1b1 + a1b2 + a2b1 + O(3 * 2^-22 |a||b|), every product exact in fp32, accumulated in
// fp32 by v_mfma_f32_16x16x32_f16: THREE MFMAs per fp32 product (vs six for bf16 hi/mid/lo).
// fp16's exponent range is narrow, so every operand tensor is scaled by 2^k chosen from its
// max |x| (amax_exp: max * 2^k in [2^14, 2^15)); the scale is exact and the accumulator is
// multiplied by 2^-(ka + kb) in the epilogue.  The activation / gradient maps are scaled PER
// IMAGE (the results of an image do not depend on the batch it runs in), weights per tensor,
// and the weight-gradient kernels use the whole tensor's max.  Producers publish the maxima
// (amax_publish) into per-image slots [1 + img]; the weight-gradient kernels reduce them.
// ---------------------------------------------------------------------------------------
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2v __attribute__((ext_vector_type(2)));

// RNE fp32 pair -> packed fp16 pair (v_cvt_pk_f16_f32)
__device__ __forceinline__ uint32_t pack_f16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2v){a, b}, f16x2v));
}
// (a, b) = hi + lo (+ 2^-22 relative), each a packed fp16 pair.  lo = RN_f16(a - hi) with
// a - hi exact in fp32: v_fma_mixlo_f16 / v_fma_mixhi_f16 take hi's halves as fp16 operands
// and write the rounded fp16 results into lo's halves, 2 instructions for the pair instead of
// 2 conversions to fp32 and a packed fma + pack (BA3C_SPLIT_MIX=1).  Bit-identical, but slower:
// conv1 forward 0.2856 -> 0.2913 ms, conv1 dgrad +3 us (r06q), so the plain form is the default
#ifndef BA3C_SPLIT_MIX
#define BA3C_SPLIT_MIX 0
#endif
__device__ __forceinline__ void split2x2(float a, float b, uint32_t& hi, uint32_t& lo) {
  hi = pack_f16x2(a, b);
#if BA3C_SPLIT_MIX
  asm("v_fma_mixlo_f16 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(lo) : "v"(hi), "v"(a));
  asm("v_fma_mixhi_f16 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "+v"(lo) : "v"(hi), "v"(b));
#else
  const f16x2v h = __builtin_bit_cast(f16x2v, hi);
  lo = pack_f16x2(a - (float)h[0], b - (float)h[1]);
#endif
}
__device__ __forceinline__ void split2(float w, uint32_t& hi, uint32_t& lo) {
  uint32_t h2, l2;
  split2x2(w, 0.f, h2, l2);
  hi = h2 & 0xFFFFu;
  lo = l2 & 0xFFFFu;
}

// exponent k with amax * 2^k in [2^14, 2^15) (0 for an all-zero tensor), clamped
__device__ __forceinline__ int amax_exp(uint32_t amax_bits) {
  if (amax_bits == 0u) return 0;
  const int e = (int)((amax_bits >> 23) & 255u) - 127;   // floor(log2(amax)), normal amax
  return max(-100, min(100, 14 - e));
}
__device__ __forceinline__ float exp2i(int k) { return __int_as_float((k + 127) << 23); }

// split-family policy: NS planes per operand and the cross products that are kept
template <int NS>
struct SplitP;
template <>
struct SplitP<3> {   // bf16 hi/mid/lo: a1b1, a1b2, a2b1, a1b3, a2b2, a3b1
  static constexpr int NPROD = 6;
  __device__ static constexpr int pa(int p) { return p == 2 || p == 4 ? 1 : (p == 5 ? 2 : 0); }
  __device__ static constexpr int pb(int p) { return p == 1 || p == 4 ? 1 : (p == 3 ? 2 : 0); }
  __device__ static __forceinline__ f32x4 mfma(const u32x4& a, const u32x4& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                   __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
  }
  // two values -> NS packed planes (no scaling: bf16 has fp32's exponent range)
  __device__ static __forceinline__ void split(float a, float b, float, uint32_t (&o)[3]) {
    split3x2(a, b, o[0], o[1], o[2]);
  }
};
template <>
struct SplitP<2> {   // scaled fp16 hi/lo: a1b1, a1b2, a2b1
  static constexpr int NPROD = 3;
  __device__ static constexpr int pa(int p) { return p == 2 ? 1 : 0; }
  __device__ static constexpr int pb(int p) { return p == 1 ? 1 : 0; }
  __device__ static __forceinline__ f32x4 mfma(const u32x4& a, const u32x4& b, const f32x4& c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                  __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
  }
  __device__ static __forceinline__ void split(float a, float b, float scale, uint32_t (&o)[2]) {
    split2x2(a * scale, b * scale, o[0], o[1]);
  }
};

struct Conv0S {
  static constexpr int HS = 84, WS = 84, C = 4, COUT = 32, KT = 5, NTAP = 25;
  static constexpr int HO = 80, WO = 80, RB = 16, NBANDS = HO / RB, SROWS = RB + KT - 1;
  static constexpr int KSTEPS = 4;                 // 4 x 32 K = 32 tap slots (25 used)
  static constexpr int MAXSPLIT = 3;
  static constexpr int PROWS_W = RB / 2 / 4;       // pooled rows per wave (2)
  static constexpr int MBROW = (WO / 2) / 4;       // m-blocks per pooled row (10)
  static constexpr int MBW = PROWS_W * MBROW;      // m-blocks per wave (20)
#ifndef BA3C_C0F_PIPE
#define BA3C_C0F_PIPE 1   // chunk c's MFMAs interleaved with chunk c - 1's pool epilogue (two accumulator sets)
#endif
#ifndef BA3C_C0F_POSPK
#define BA3C_C0F_POSPK 1  // ReLU positives by saturating pack + byte gather + popcount (A/B: 0)
#endif
#ifndef BA3C_C0F_MCH
#define BA3C_C0F_MCH (BA3C_C0F_PIPE ? 2 : 5)
#endif
  static constexpr int MCH = BA3C_C0F_MCH;          // m-blocks per accumulator chunk
  // prepared weights: [split][nt][kstep][lane] x 16 bytes (room for the 3-plane family)
  static constexpr int WB_U4 = MAXSPLIT * 2 * KSTEPS * 64;
  static_assert(RB % 8 == 0 && HO % RB == 0 && MBW % MCH == 0, "conv0 split geometry");
};

// K order of conv0's forward: the two taps of a LANE's A fragment are (t, t + 10) = (kh, kw)
// and (kh + 2, kw), two LDS rows apart for every lane and k-step, so the fragment is ONE
// 16-byte LDS entry (see C0E_ROWS).  Pair P = 4s + q: P < 10 holds taps (P, P + 10);
// P = 10..14 holds (P, P + 10) with the first half padding (weight 0, reads the in-band row
// kh = 2) and the second the kh = 4 tap; P = 15 is padding in both halves.  A 16-lane group
// reads 2 rows x 8 pixels; with the 88-entry pitch those 16 addresses are distinct mod 128 B.
// The tap whose pixels slot (s, q, h) reads (always a real tap: in-bounds, finite values):
__host__ __device__ constexpr int conv0_atap(int s, int q, int h) { return (4 * s + q < 15 ? 4 * s + q : 0) + 10 * h; }
// the tap whose weight slot (s, q, h) carries, -1 for padding
__host__ __device__ constexpr int conv0_wtap(int s, int q, int h) {
  return 4 * s + q < 10 ? 4 * s + q + 10 * h : (4 * s + q < 15 && h ? 4 * s + q + 10 : -1);
}

// real-channel weight of conv0/W [5,5,16,32] (TARGET_CHANNELS = 16, train.py:99) at
// K position (kstep s, lane group q, element e) = tap conv0_wtap(s, q, e >> 2), channel e & 3
__device__ __forceinline__ float conv0_w(const float* __restrict__ w, int s, int q, int e, int n) {
  const int tap = conv0_wtap(s, q, e >> 2), c = e & 3;
  return tap >= 0 ? w[((size_t)tap * 16 + c) * 32 + n] : 0.f;
}

// max |w| over conv0's real-channel weights, reduced over the calling workgroup (256 threads)
__device__ __forceinline__ float conv0_wmax_block(const float* __restrict__ w, float* red4) {
  float m = 0.f;
  for (int i = threadIdx.x; i < Conv0S::NTAP * 4 * 32; i += 256) {
    const int tap = i / 128, c = (i >> 5) & 3, n = i & 31;
    m = fmaxf(m, fabsf(w[((size_t)tap * 16 + c) * 32 + n]));
  }
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
  __syncthreads();
  return fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
}

// conv0 weights -> 2 fp16 split planes of w * 2^kexp in MFMA B-fragment order.  One thread
// per (nt, kstep, lane).
__device__ __forceinline__ void conv0s_wprep_one(const float* __restrict__ w, uint4* __restrict__ wb, int t,
                                                 int kexp) {
  using G = Conv0S;
  if (t >= 2 * G::KSTEPS * 64) return;
  const int lane = t & 63, s = (t >> 6) % G::KSTEPS, nt = t / (64 * G::KSTEPS);
  const int n = nt * 16 + (lane & 15), q = lane >> 4;
  const float sc = exp2i(kexp);
  uint32_t part[2][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) split2(conv0_w(w, s, q, e, n) * sc, part[0][e], part[1][e]);
#pragma unroll
  for (int sp = 0; sp < 2; ++sp)
    wb[((sp * 2 + nt) * G::KSTEPS + s) * 64 + lane] =
        make_uint4(part[sp][0] | (part[sp][1] << 16), part[sp][2] | (part[sp][3] << 16),
                   part[sp][4] | (part[sp][5] << 16), part[sp][6] | (part[sp][7] << 16));
}

// Persistent workgroups walk bands (one image x RB output rows = RB/2 pooled rows); wave w
// owns pooled rows 2w, 2w+1 of a band = 20 m-blocks of 4 windows, both 16-channel n-tiles.
// The weight splits are loaded into registers once per workgroup, and the next band's frame
// rows are loaded into registers before the current band's MFMAs, so HBM latency hides
// behind the arithmetic.  M rows are ordered (window, sub) so a lane's 4 accumulator rows
// are one 2x2 window.  Frame bytes are exact in bf16 and in fp16 alike (no scaling); the
// weights carry 2^kw (NS = 2), removed with the 1/255 in the epilogue.
struct Conv0SArgs {
  const uint8_t* x;        // frames [B,84,84,4]
  const uint4* wb;         // prepared weight splits
  float* out;              // pooled [B,40,40,32]
  uint8_t* out_code;       // argmax codes (may be null)
  unsigned long long* relu_count;
  int batch;
  const int* wexp;         // NS = 2: exponent of the weight scale
  uint32_t* amax_out;      // NS = 2: per-image max of the pooled output (may be null)
  // chained launch (launch_prep_conv0_multi): the workgroup splits its own weight fragments
  // from w0 (conv0/W) instead of reading wb / wexp, and waits for the zeroing workgroups'
  // signal count (*zsig >= zneed) only before its first publication into the ReLU counters /
  // max slots they zero
  const float* w0;
  const unsigned* zsig;
  unsigned zneed;
  unsigned* zerr;
};

// 1 if the fp32 bits x are a positive value (x > 0 as a signed integer), else 0: one
// v_med3_i32 (x, 0, 1); in C the clamp is turned back into a compare + select through VCC.
// x is an MFMA result: inline asm is not seen by the MFMA -> VALU read hazard check, so the
// asm also takes `after`, a compiler-visible VALU result of the same accumulator (the window
// max), which orders it behind the wait states the compiler inserted for that read.
__device__ __forceinline__ int c0w_pos1(int x, int after) {
  int r;
  asm("v_med3_i32 %0, %1, 0, 1" : "=v"(r) : "v"(x), "v"(after));
  return r;
}

// max(t, x, 0) in one v_max3_i32; x an MFMA result read after t, a compiler-visible VALU
// result of the same accumulator (as c0w_pos1)
__device__ __forceinline__ int c0w_max3z(int t, int x) {
  int r;
  asm("v_max3_i32 %0, %1, %2, 0" : "=v"(r) : "v"(t), "v"(x));
  return r;
}

// a frame byte pair -> packed 16-bit pair of the split family
template <int NS>
__device__ __forceinline__ uint32_t u8pair(uint32_t a, uint32_t b) {
  if constexpr (NS == 3) return u8_bf16(a) | (u8_bf16(b) << 16);
  else return pack_f16x2((float)a, (float)b);
}

// Layout 3 stores every 16-bit pixel twice: LDS entry (r, x) is 16 bytes [pixel (r, x) |
// pixel (r + 2, x)] (rows of the band, 4 channels each), so a lane's A fragment of taps
// (t, t + 10) is ONE aligned ds_read_b128 (two 8-byte reads let the compiler pair halves of
// different m-blocks and re-copy them: ~3 v_mov per fragment).  Entry rows 0 .. SROWS-3 are
// read (row r + kh, kh <= 2); the entry pitch 88 (= 8 mod 16 entries) puts a 16-lane group's
// two output rows in disjoint bank halves.
constexpr int C0E_ROWS = Conv0S::SROWS - 2, C0E_PITCH = 88;
// four frame bytes (one pixel's 4 channels) -> two packed 16-bit pairs of the split family.
// fp16: 0x6400 | b is 1024 + b exactly, so one v_perm_b32 per pair builds the magic values and
// one v_pk_add_f16 of -1024 leaves b exactly (bits identical to a float conversion)
template <int NS>
__device__ __forceinline__ void u8quad(uint32_t px, uint32_t& o01, uint32_t& o23) {
  if constexpr (NS == 3) {
    o01 = u8pair<NS>(px & 255u, (px >> 8) & 255u);
    o23 = u8pair<NS>((px >> 16) & 255u, px >> 24);
  } else {
    const f16x2v m1024 = {(_Float16)-1024.0f, (_Float16)-1024.0f};
    const uint32_t k = 0x64646464u;
    const f16x2v a = __builtin_bit_cast(f16x2v, __builtin_amdgcn_perm(k, px, 0x04010400u)) + m1024;
    const f16x2v b = __builtin_bit_cast(f16x2v, __builtin_amdgcn_perm(k, px, 0x04030402u)) + m1024;
    o01 = __builtin_bit_cast(uint32_t, a);
    o23 = __builtin_bit_cast(uint32_t, b);
  }
}

constexpr int conv0s_band_bytes() { return C0E_ROWS * C0E_PITCH * 16; }
// per wave: one pooled row of the band's output (40 windows x 32 channels) as fp32 + codes,
// staged so the global stores are whole 16-byte pieces (see the epilogue)
constexpr int C0_WST_BYTES = (Conv0S::WO / 2) * Conv0S::COUT * 5;
constexpr int conv0s_fwd_lds_bytes() { return conv0s_band_bytes() + 4 * C0_WST_BYTES; }

// raw buffer resource over `base` (gfx9 descriptor word 3; offsets stay < 2^31 bytes)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFFF, 0x00020000);
}

// bx / gx: first band and persistent stride (blockIdx.x / gridDim.x of a plain launch);
// lds: conv0s_fwd_lds_bytes() bytes
template <bool TRAIN>
__device__ __forceinline__ void conv0s_fwd_body_t(const Conv0SArgs& a, int bx, int gx, char* lds);

__device__ __forceinline__ void conv0s_fwd_body(const Conv0SArgs& a, int bx, int gx, char* lds) {
  // training (codes + ReLU count) and predictor variants: no per-store branch in the loop
  if (a.out_code) conv0s_fwd_body_t<true>(a, bx, gx, lds);
  else conv0s_fwd_body_t<false>(a, bx, gx, lds);
}

template <bool TRAIN>
__device__ __forceinline__ void conv0s_fwd_body_t(const Conv0SArgs& a, int bx, int gx, char* lds) {
  using G = Conv0S;
  using SP = SplitP<2>;
  // wave index in an SGPR: the wave's LDS areas and output rows are scalar arithmetic
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nbands = a.batch * G::NBANDS;

  // ---- rows [y0, y0 + SROWS) of a band: one thread per 16-byte ENTRY (r, x) = [pixel (r, x)
  // | pixel (r + 2, x)]: two dword loads (coalesced over consecutive x), one ds_write_b128 —
  // consecutive lanes write consecutive entries, conflict-free (r03e PMC: the 4-pixel runs
  // written as 8-byte halves at a 64-byte lane stride made 52 % of the LDS cycles conflicts)
  constexpr int NV = C0E_ROWS * G::WS;             // entries
  constexpr int NPT = (NV + 255) / 256;
  uint32_t ev[NPT][2];
  auto load_band = [&](int band) {
    const int img = band / G::NBANDS, y0 = (band - img * G::NBANDS) * G::RB;
    const uint32_t* src = reinterpret_cast<const uint32_t*>(a.x + ((size_t)img * G::HS + y0) * G::WS * G::C);
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = tid + 256 * i;                 // entry e = row r * 84 + x: pixel index e
      // branch-free (past the band: entry 0 again, stored nowhere): the conditional loads made
      // the compiler wait for this prefetch before the band's first MFMA (r04 ISA)
      const int ec = e < NV ? e : 0;
      ev[i][0] = src[ec];
      ev[i][1] = src[ec + 2 * G::WS];
    }
  };
  auto store_band = [&]() {
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int e = tid + 256 * i;
      if (e < NV) {
        const int r = e / G::WS, x = e - r * G::WS;
        uint32_t o[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) u8quad<2>(ev[i][h], o[2 * h], o[2 * h + 1]);
        reinterpret_cast<uint4*>(lds)[r * C0E_PITCH + x] = make_uint4(o[0], o[1], o[2], o[3]);
      }
    }
  };

  int band = bx;
  if (band < nbands) load_band(band);

  const int li = lane & 15, lq = lane >> 4;
  bool zdone = a.zsig == nullptr;                   // the zeroing signal seen (chained launch)
  u32x4 wf[2][2][G::KSTEPS];
  int wx;
  if (a.w0) {
    // the fragments conv0s_wprep_one writes for thread lane + 64 (s + KSTEPS nt), bit for bit
    // (LDS word 0..3 as the max reduction's scratch: the band loop's barrier precedes its use)
    wx = amax_exp(__float_as_uint(conv0_wmax_block(a.w0, reinterpret_cast<float*>(lds))));
    const float sc = exp2i(wx);
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        uint32_t part[2][8];
#pragma unroll
        for (int e = 0; e < 8; ++e) split2(conv0_w(a.w0, s, lq, e, nt * 16 + li) * sc, part[0][e], part[1][e]);
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
          wf[sp][nt][s] = u32x4{part[sp][0] | (part[sp][1] << 16), part[sp][2] | (part[sp][3] << 16),
                                part[sp][4] | (part[sp][5] << 16), part[sp][6] | (part[sp][7] << 16)};
      }
  } else {
    wx = a.wexp[0];
#pragma unroll
    for (int sp = 0; sp < 2; ++sp)
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int s = 0; s < G::KSTEPS; ++s) {
          const uint4 u = a.wb[((sp * 2 + nt) * G::KSTEPS + s) * 64 + lane];
          wf[sp][nt][s] = u32x4{u.x, u.y, u.z, u.w};
        }
  }
  // the weights are complete before the band loop: otherwise the loop's merged wait state
  // made every band's first MFMA wait for all loads, the next band's prefetch included
#pragma unroll
  for (int sp = 0; sp < 2; ++sp)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) asm volatile("" : "+v"(wf[sp][nt][s]));
  // this lane's row (window li>>2, sub li&3) of m-block 0 of the wave, per (kstep, tap half)
  const int wi = li >> 2, sub = li & 3;
  constexpr int RP = C0E_PITCH;                     // entry index pitch
  const int pix0 = (4 * wave + (sub >> 1)) * RP + 2 * wi + (sub & 1);
  int lb[G::KSTEPS][2];
#pragma unroll
  for (int s = 0; s < G::KSTEPS; ++s)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int tap = conv0_atap(s, lq, h);
      lb[s][h] = pix0 + (tap / G::KT) * RP + tap % G::KT;
    }

  int pos = 0;                                      // this lane's ReLU positives (TRAIN; 8x with BA3C_C0F_POSPK)
  // (sum_k u8 * w 2^kw) * (2^-kw / 255): scaling by a power of two commutes with the rounding
  const float oscale = (1.0f / 255.0f) * exp2i(-wx);
  // Epilogue stores go through a wave-private LDS area holding one pooled row of outputs
  // (40 windows x 32 channels: 5 KB fp32 + 1.25 KB codes, contiguous in global memory too):
  // each lane writes its window / channel values there, then the wave copies the row out in
  // 16-byte pieces, consecutive lanes consecutive pieces — 7 buffer_store_dwordx4 per pooled
  // row instead of 40 dword + 40 byte stores (r03i: a byte store per value cost ~7 cycles of
  // the CU's store path each)
  float* wst = reinterpret_cast<float*>(lds + conv0s_band_bytes() + wave * C0_WST_BYTES);
  uint8_t* wsc = reinterpret_cast<uint8_t*>(wst + (G::WO / 2) * G::COUT);
  const int lane_el = lq * G::COUT + li;           // (window lq, channel li) in the row area
  for (; band < nbands; band += gx) {
    const int img = band / G::NBANDS, y0 = (band - img * G::NBANDS) * G::RB;
    __syncthreads();                                 // previous band's LDS reads are done
    store_band();
    __syncthreads();
    if (band + gx < nbands) load_band(band + gx);
    const size_t band_el = (size_t)(img * (G::HO / 2) + y0 / 2) * (G::WO / 2) * G::COUT;
    int bmaxi = 0;                                  // max window-max bits of the band
    constexpr int NCH = G::MBW / G::MCH, CPR = G::MBROW / G::MCH;   // chunks per band / pooled row
    static_assert(G::MBROW % G::MCH == 0, "whole chunks per pooled row");
    // the chunk's MFMAs into `acc`
    auto chunk_mma = [&](int ch, f32x4 (&acc)[G::MCH][2]) {
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < G::KSTEPS; ++s) {
        u32x4 af[G::MCH];
#pragma unroll
        for (int j = 0; j < G::MCH; ++j) {
          const int jj = ch * G::MCH + j;
          const int off = (jj / G::MBROW) * 2 * RP + (jj % G::MBROW) * 8;   // immediate
          // both taps of the fragment in one 16-byte entry: one ds_read_b128
          const uint4 u = reinterpret_cast<const uint4*>(lds)[lb[s][0] + off];
          af[j] = u32x4{u.x, u.y, u.z, u.w};
        }
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int j = 0; j < G::MCH; ++j)
              acc[j][nt] = SP::mfma(af[j], wf[sp][nt][s], acc[j][nt]);
      }
    };
    // its pool epilogue, and the copy-out of a completed pooled row
    auto chunk_epi = [&](int ch, const f32x4 (&acc)[G::MCH][2]) {
      // pool epilogue: lane holds the 4 subs of window 4*mb + lq, channel nt*16 + li.
      // Max of the ReLU'd window = max(v0..v3, +0), taken on the fp32 BITS as signed
      // integers (negative values are negative integers, positive ones order like floats;
      // integer max needs no NaN canonicalisation): two v_max3_i32.  Its argmax = the FIRST
      // k with v_k == max (TF's strict-'<' update, models/pool.py:14-33); 255 when max <= 0.
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) {
        const int jj = ch * G::MCH + j;
#pragma unroll
        for (int nt = 0; nt < 2; ++nt) {
          // element of (window 4 (jj % 10), n-tile) in the row area, from lane_el
          const int cofs = 4 * (jj % G::MBROW) * G::COUT + nt * 16;
          const int b0 = __float_as_int(acc[j][nt][0]), b1 = __float_as_int(acc[j][nt][1]);
          const int b2 = __float_as_int(acc[j][nt][2]), b3 = __float_as_int(acc[j][nt][3]);
          // max3 (b0, b1, b2) then max3 (., b3, 0): two v_max3_i32 (the compiler splits the
          // second into a max and a max with 0)
          const int m = c0w_max3z(max(max(b0, b1), b2), b3);
          bmaxi = max(bmaxi, m);
          wst[lane_el + cofs] = __int_as_float(m) * oscale;
          if constexpr (TRAIN) {
            uint32_t arg = b2 == m ? 2u : 3u;
            arg = b1 == m ? 1u : arg;
            arg = b0 == m ? 0u : arg;
            wsc[lane_el + cofs] = (uint8_t)(m != 0 ? arg : 255u);
            // positives by v_cmp -> SGPR mask -> s_bcnt1 (one VALU instruction per value; the
            // bits compare as signed integers: x > 0 exactly for positive x)
            // ReLU positives: the bits compare as signed integers (x > 0 exactly for x > 0).
            // Per-lane compare + add; a v_cmp -> SGPR ballot + s_bcnt1 form has fewer VALU
            // instructions but measured slower (0.189 -> 0.209 ms, VALU-to-SALU dependencies)
            // (x > 0) as med3(x, 0, 1) on the bits (v_med3_i32) and three-input adds: no VCC
            // round trips (a compare + add-with-carry per value chained the four through VCC)
#if BA3C_C0F_POSPK
            // 8 x (positives): v_cvt_pk_i16_i32 saturates the bits of a positive value to
            // 0x7FFF, of zero to 0, of a negative one to 0x8000, so the low byte of each half is
            // 0xFF exactly for a positive value; one v_perm_b32 gathers the four low bytes and
            // v_bcnt_u32_b32 adds 8 per positive (4 VALU per window instead of 6)
            pos += __builtin_popcount(__builtin_amdgcn_perm(
                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(b2, b3)),
                __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_pk_i16(b0, b1)), 0x06040200u));
#else
            pos += (c0w_pos1(b0, m) + c0w_pos1(b1, m)) + (c0w_pos1(b2, m) + c0w_pos1(b3, m));
#endif
            // materialise the count here: otherwise it is sunk to its only use after the band
            // loop, keeping every accumulator of the chunk live (r03g: > 256 registers)
            asm volatile("" : "+v"(pos));
          }
        }
      }
      if (ch % CPR == CPR - 1) {
        // the wave's pooled row 2 wave + ch / CPR is complete in its LDS area: copy it out
        const size_t row_el = band_el + (size_t)(2 * wave + ch / CPR) * (G::WO / 2) * G::COUT;
        const __amdgpu_buffer_rsrc_t rout = buf_rsrc(a.out + row_el);
        constexpr int NF = (G::WO / 2) * G::COUT * 4 / 16;     // 320 pieces of 16 B
#pragma unroll
        for (int i = 0; i < NF / 64; ++i) {
          const uint4 v = reinterpret_cast<const uint4*>(wst)[lane + 64 * i];
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rout, 16 * (lane + 64 * i), 0, 0);
        }
        if constexpr (TRAIN) {
          const __amdgpu_buffer_rsrc_t rcode = buf_rsrc(a.out_code + row_el);
          constexpr int NC = (G::WO / 2) * G::COUT / 16;       // 80 pieces of 16 B
#pragma unroll
          for (int i = 0; i < (NC + 63) / 64; ++i) {
            const int piece = lane + 64 * i;
            if (piece < NC) {
              const uint4 v = reinterpret_cast<const uint4*>(wsc)[piece];
              __builtin_amdgcn_raw_buffer_store_b128(u32x4{v.x, v.y, v.z, v.w}, rcode, 16 * piece, 0, 0);
            }
          }
        }
      }
    };
    if constexpr (BA3C_C0F_PIPE) {
      // software pipeline over the band's chunks: the epilogue of chunk c - 1 (VALU) issues
      // between the MFMAs of chunk c, which do not depend on it, so one wave keeps the matrix
      // core and the VALU busy together (two MCH = 2 accumulator sets: 32 registers, fewer than
      // one MCH = 5 set)
      f32x4 acc[2][G::MCH][2];
      chunk_mma(0, acc[0]);
#pragma unroll
      for (int ch = 1; ch < NCH; ++ch) {
        chunk_mma(ch, acc[ch & 1]);
        chunk_epi(ch - 1, acc[(ch - 1) & 1]);
      }
      chunk_epi(NCH - 1, acc[(NCH - 1) & 1]);
    } else {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        // chunks do not overlap inside a wave (the two waves per SIMD overlap each other's
        // epilogue and MFMAs): without this fence the scheduler interleaves chunk c + 1's A reads
        // and MFMAs with chunk c's epilogue, two MCH = 5 accumulator sets live -> > 256
        // registers and one wave per SIMD (r03g: 0.35 ms)
        __builtin_amdgcn_sched_barrier(0);
        f32x4 acc[G::MCH][2];
        chunk_mma(ch, acc);
        chunk_epi(ch, acc);
      }
    }
    // max over the window maxima, then the scale: a positive scale is monotone in fp32
    if (!zdone) {
      chain_wait_wave(a.zsig, a.zneed, a.zerr);
      zdone = true;
    }
    amax_publish(a.amax_out, img, __int_as_float(bmaxi) * oscale, lane);
  }
  if (!zdone) chain_wait_wave(a.zsig, a.zneed, a.zerr);
  if (TRAIN && a.relu_count)
    relu_count_add(a.relu_count, (unsigned long long)(BA3C_C0F_POSPK ? pos >> 3 : pos), lane);
}

#if !BA3C_SHARED_KERNELS  // emitted by ba3c_conv0.hip only
__global__ void __launch_bounds__(256) conv0s_fwd_kernel(const Conv0SArgs a) {
  __shared__ uint4 xs4[conv0s_fwd_lds_bytes() / 16];
  conv0s_fwd_body(a, blockIdx.x, gridDim.x, reinterpret_cast<char*>(xs4));
}
#endif

// ---------------------------------------------------------------------------------------
// conv0 weight gradient (Conv2DBackpropFilter of conv0, train.py:177 under TF autodiff):
//   dW[tap, c, o] = (1/255) * sum_{n, pixel p} u8[n, p + tap, c] * dY[n, p, o]
// with dY the un-pooled output gradient (dP routed to each window's argmax, ReLU folded in).
// M = (tap, c) = 100 rows (7 m-tiles), N = o (2 n-tiles), K = pixels; dY is split into NS
// planes (NS = 3: bf16 hi/mid/lo; NS = 2: fp16 hi/lo of dY * 2^ky, ky from the dP0 tensor's
// max), the frames are exact in either type, so NS MFMAs per (m-tile, n-tile, 32 px).
//
// Persistent workgroups walk bands of RB output rows.  LDS per band:
//   X: two copies of the RB + 4 input rows, channel-planar 16-bit, copy h shifted left by h
//      pixels, so the 8 pixels a lane feeds for tap (kh, kw) start at an even column of copy
//      kw & 1 (dword aligned);
//   Y: the POOLED gradient dP of the band, split: [split][pooled row][o][pooled col] 16-bit,
//      plus its argmax codes [pooled row][o][pooled col] u8 — a quarter of the un-pooled
//      dY's bytes.  The MFMA B fragment (8 un-pooled pixels = 4 windows x 2 sub-columns of
//      one row) is un-pooled in registers: window j's dword is (v, v) & mask, mask =
//      0x0000FFFF / 0xFFFF0000 for the argmax sub-column, 0 when the argmax is in the other
//      row or there is no gradient.  o pitch 40 = 20 dwords: the 16 o of a lane group land on
//      16 distinct bank pairs.
// K-step s of a band = pixels 32s .. 32s + 31 (row-major over the band), lane group q
// supplies pixels 32s + 8q .. + 7 (one row, since 80 % 8 == 0); waves take K-steps
// s = wave, wave + 4, ...  The next band's global loads are issued into registers before
// the MFMA phase of the current one.  Each workgroup writes one partial slab (x 1/255).
// ---------------------------------------------------------------------------------------
// A-row slot -> tap of conv0's weight gradient (7 m-tiles x 4 slots; see Conv0W's pitches):
// C0W_TAP_ADDR is the tap whose pixels a slot reads, C0W_TAP_OUT the tap it computes (-1:
// padding, discarded).  A slot's MFMA row is independent of the others, so the order changes
// nothing in any output's arithmetic.
__device__ constexpr int C0W_TAP_ADDR[28] = {0, 2, 1, 3, 8, 5, 4, 6, 11, 13, 7, 9, 14, 16,
                                             10, 12, 17, 19, 18, 15, 20, 22, 21, 23, 0, 2, 24, 3};
__device__ constexpr int C0W_TAP_OUT[28] = {0, 2, 1, 3, 8, 5, 4, 6, 11, 13, 7, 9, 14, 16,
                                            10, 12, 17, 19, 18, 15, 20, 22, 21, 23, -1, -1, 24, -1};

template <int NS>
struct Conv0W {
  static constexpr int HS = 84, WS = 84, C = 4, COUT = 32, KT = 5, NTAP = 25;
  static constexpr int HO = 80, WO = 80, PH = 40, PW = 40;
  static constexpr int RB = 8, NBANDS = HO / RB, XROWS = RB + KT - 1;   // 12 rows (<= 84)
  static constexpr int PRB = RB / 2;               // pooled rows per band (4)
  static constexpr int KPB = RB * WO;              // 640 pixels per band
  static constexpr int KSTEPS = KPB / 32;          // 20
  static constexpr int KSW = KSTEPS / 4;           // 5 per wave
  static constexpr int Y_16 = NS * PRB * COUT * PW;                   // 16-bit words
  static constexpr int YC_BYTES = PRB * COUT * PW;                    // 5120
  // Row / channel-plane / copy pitches (16-bit units) and the tap order of the A rows, from the
  // bank model of the A-fragment dword reads (2 x 32-lane groups, bank = dword mod 32).  A
  // 32-lane group reads 4 taps x 4 channels x 2 pixel runs; channel planes add multiples of 8
  // dwords (XPL / 2 = 552 = 8 mod 32), pixel runs 4, so the reads are conflict-free when the 4
  // taps of an m-tile have distinct tap offsets mod 4 dwords.  With XP / 2 = 45 (1 mod 4) and
  // XCP / 2 = 2210 (2 mod 4) the 25 taps fall 6 / 6 / 7 / 6 into the residues and C0W_TAP puts
  // one of each into every m-tile (padding slots read a tap of the missing residue): 1.00 LDS
  // cycles per read (r02: 1.43 with 88 / 1072 / 4292 and taps in order; r01: 3.71 dense)
  static constexpr int XP = 90;
  static constexpr int XPL = 1104;                 // >= XROWS * XP = 1080
  static constexpr int XCP = 4420;                 // >= C * XPL = 4416
  static constexpr int X_16 = 2 * XCP;
  static constexpr int LDS_U4 = ((Y_16 + X_16) * 2 + YC_BYTES) / 16;
  static constexpr int MT = 7, M = NTAP * C;
  static constexpr int SLAB_U4 = 4 * M * COUT * 4 / 16;            // epilogue: 4 wave slabs
  static constexpr int ALLOC_U4 = LDS_U4 > SLAB_U4 ? LDS_U4 : SLAB_U4;
  static constexpr int NITEM = COUT * PRB * (PW / 4) / 256;            // dP items per thread
  static constexpr int NXV = XROWS * WS * C / 16;                      // uint4 of frame rows
  static_assert(KSTEPS % 4 == 0 && COUT * PRB * (PW / 4) % 256 == 0 && NXV <= 256, "geom");
  static_assert(HO % RB == 0 && RB + KT - 1 + HO - RB <= HS, "band rows stay inside the frame");
  static_assert(WO % 8 == 0 && ((Y_16 + X_16) * 2) % 16 == 0, "layout");
  static_assert(XPL >= XROWS * XP && XCP >= C * XPL && XP % 2 == 0 && XPL % 2 == 0 && XCP % 2 == 0,
                "X planes: disjoint, dword-aligned pixel pairs");
};

struct Conv0WArgs {
  const uint8_t* x;        // frames [B,84,84,4]
  const float* dp;         // dP0 [B,40,40,32]
  const uint8_t* code;     // argmax codes of dP0
  float* part;             // [gridDim.x][100][32] partial slabs
  int batch;
  const uint32_t* amax_dp; // NS = 2: per-image max |dP0| slots
};

// packed 16-bit halves: 0xFFFF where the half is zero, else 0 — two packed VALU ops (the plain
// C form of mask16_eq0 is rewritten by the compiler into a compare + select per half)
__device__ __forceinline__ uint32_t c0w_mask16_eq0(uint32_t d) {
  uint32_t m;
  // (the constants go in SGPRs: an inline constant of a packed op is not replicated to the high
  // half the way the C vector (1, 1) is)
  asm("v_pk_min_u16 %0, %1, %2\n\tv_pk_add_u16 %0, %0, %3" : "=&v"(m) : "v"(d), "s"(0x00010001u), "s"(0xFFFFFFFFu));
  return m;
}

// bx / gx: first band and persistent stride (blockIdx.x / gridDim.x of the plain kernel; a
// paired launch passes its own); lds: Conv0W<NS>::ALLOC_U4 uint4 of LDS, red4: 4 words
#ifndef BA3C_C0W_SPARSE
#define BA3C_C0W_SPARSE 1
#endif
template <int NS>
__device__ __forceinline__ void conv0s_wgrad_body(const Conv0WArgs& a, int bx, int gx, uint4* lds, uint32_t* red4) {
  using G = Conv0W<NS>;
  using SP = SplitP<NS>;
  constexpr bool C0W_SPARSE = BA3C_C0W_SPARSE && NS == 2;
#ifndef BA3C_C0W_XFIRST
#define BA3C_C0W_XFIRST 1
#endif
  // X first: its A-fragment addresses are then lane offset + k-step offset with no LDS base to
  // add (the base of a region past 1 KB does not fit the ds_read2 offset fields, and the
  // compiler added it to each of the 14 dword-pair reads of a k-step)
  uint16_t* xs = reinterpret_cast<uint16_t*>(lds) + (BA3C_C0W_XFIRST ? 0 : G::Y_16);
  uint16_t* ys = reinterpret_cast<uint16_t*>(lds) + (BA3C_C0W_XFIRST ? G::X_16 : 0);
  uint8_t* yc8 = reinterpret_cast<uint8_t*>(reinterpret_cast<uint16_t*>(lds) + G::X_16 + G::Y_16);
  const int tid = threadIdx.x, lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, lq = lane >> 4;
  const int nbands = a.batch * G::NBANDS;
  const int ky = NS == 2 ? amax_exp(amax_all(a.amax_dp, a.batch, red4)) : 0;
  const float ysc = exp2i(ky);

  // ---- per-thread prefetch registers for one band ----
  float yv[G::NITEM][4];
  uint32_t yc[G::NITEM];
  uint4 xv;
  auto load_band = [&](int band) {
    const int img = band / G::NBANDS, y0 = (band - img * G::NBANDS) * G::RB;
#pragma unroll
    for (int i = 0; i < G::NITEM; ++i) {
      const int f = tid + 256 * i, o = f & 31, rest = f >> 5;
      const int pr = rest / (G::PW / 4), q4 = rest - pr * (G::PW / 4);
      const size_t base = ((size_t)(img * G::PH + y0 / 2 + pr) * G::PW + 4 * q4) * G::COUT + o;
      uint32_t c = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        yv[i][j] = a.dp[base + j * G::COUT];
        c |= (uint32_t)a.code[base + j * G::COUT] << (8 * j);
      }
      yc[i] = c;
    }
    // branch-free (threads past the rows re-read entry 0 and store nothing)
    xv = reinterpret_cast<const uint4*>(a.x + ((size_t)img * G::HS + y0) * G::WS * G::C)[tid < G::NXV ? tid : 0];
  };
  auto store_band = [&]() {
#pragma unroll
    for (int i = 0; i < G::NITEM; ++i) {
      const int f = tid + 256 * i, o = f & 31, rest = f >> 5;
      const int pr = rest / (G::PW / 4), q4 = rest - pr * (G::PW / 4);
      uint32_t s0[NS], s1[NS];
      SP::split(yv[i][0], yv[i][1], ysc, s0);
      SP::split(yv[i][2], yv[i][3], ysc, s1);
      const int e = (pr * G::COUT + o) * G::PW + 4 * q4;
      constexpr int SPL = G::PRB * G::COUT * G::PW;
#pragma unroll
      for (int sp = 0; sp < NS; ++sp)
        *reinterpret_cast<uint2*>(ys + sp * SPL + e) = make_uint2(s0[sp], s1[sp]);
      *reinterpret_cast<uint32_t*>(yc8 + e) = yc[i];
    }
    if (tid < G::NXV) {
      const int p = 4 * tid, r = p / G::WS, x = p - r * G::WS;    // 4 pixels of one row
      const uint32_t px[4] = {xv.x, xv.y, xv.z, xv.w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        uint32_t b[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) b[j] = u8pair<NS>((px[j] >> (8 * c)) & 255u, 0u) & 0xFFFFu;
        uint16_t* p0 = xs + c * G::XPL + r * G::XP + x;              // copy 0 (4-byte aligned:
        reinterpret_cast<uint32_t*>(p0)[0] = b[0] | (b[1] << 16);       // odd rows sit at 4 mod 8)
        reinterpret_cast<uint32_t*>(p0)[1] = b[2] | (b[3] << 16);
        uint16_t* p1 = xs + G::XCP + c * G::XPL + r * G::XP + x;     // copy 1: column x - 1
        if (x > 0) p1[-1] = (uint16_t)b[0];
        *reinterpret_cast<uint32_t*>(p1) = b[1] | (b[2] << 16);
        p1[2] = (uint16_t)b[3];
      }
    }
  };

  // per-lane A offsets (16-bit units) for m-tile mt: row m = 16 mt + li = (tap, c)
  int aoff[G::MT];
#pragma unroll
  for (int mt = 0; mt < G::MT; ++mt) {
    const int tap = C0W_TAP_ADDR[4 * mt + (li >> 2)];   // padding slots: discarded rows
    const int c = li & 3, kh = tap / G::KT, kw = tap % G::KT, h = kw & 1;
    aoff[mt] = h * G::XCP + c * G::XPL + kh * G::XP + (kw - h);
  }

  f32x4 acc[G::MT][2];
#pragma unroll
  for (int mt = 0; mt < G::MT; ++mt) acc[mt][0] = acc[mt][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  int band = bx;
  if (band < nbands) load_band(band);
  for (; band < nbands; band += gx) {
    __syncthreads();                                   // previous band's LDS reads are done
    store_band();
    __syncthreads();
    if (band + gx < nbands) load_band(band + gx);
#pragma unroll
    for (int i = 0; i < G::KSW; ++i) {
      const int s = wave + 4 * i;
      const int pb = 32 * s + 8 * lq, r = pb / G::WO, x0 = pb - r * G::WO;
      const int xo = r * G::XP + x0;
      u32x4 av[G::MT];
#pragma unroll
      for (int mt = 0; mt < G::MT; ++mt) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(xs + aoff[mt] + xo);
        av[mt] = u32x4{p[0], p[1], p[2], p[3]};
      }
      // B: un-pool 4 windows (pooled cols x0/2 .. +3 of pooled row r/2) for channel o
      const uint32_t sy = (uint32_t)(r & 1);
      const int e0 = ((r >> 1) * G::COUT + li) * G::PW + (x0 >> 1);
      if constexpr (C0W_SPARSE) {
        // 2:4-sparse form (BA3C_C0W_SPARSE): dY^T on the sparse A side of
        // v_smfmac_f32_16x16x32_f16 (rows o, the lane's 8 pixels = 2 quads of 2 windows each),
        // the frames' fragments above as its dense B (columns (tap, c)).  Per quad the two kept
        // values are the windows' gradients where their argmax lies in this pixel row (else 0)
        // at positions (argmax column) and (2 + argmax column): no un-pooling at all.
        const uint32_t sx = sy * 0x00020002u;
#pragma unroll
        for (int m = 0; m < 2; ++m) {
          const int e = e0 + 16 * m * G::PW;
          const uint32_t cw = *reinterpret_cast<const uint32_t*>(yc8 + e);
          // (code ^ 2 sy) & ~1 == 0 <=> the argmax is in this pixel row (255 never is)
          const uint32_t m01 = c0w_mask16_eq0((__builtin_amdgcn_perm(cw, cw, 0x0C010C00u) ^ sx) & 0x00FE00FEu);
          const uint32_t m23 = c0w_mask16_eq0((__builtin_amdgcn_perm(cw, cw, 0x0C030C02u) ^ sx) & 0x00FE00FEu);
          // index nibbles: quad 0 = (c0 & 1) | (2 + (c1 & 1)) << 2, quad 1 from c2, c3
          const uint32_t t = cw & 0x01010101u;
          const uint32_t t1 = t | (t >> 6);
          const int ix = (int)(((t1 | (t1 >> 12)) & 0x55u) | 0x88u);
#pragma unroll
          for (int sp = 0; sp < NS; ++sp) {
            const uint2 u = *reinterpret_cast<const uint2*>(ys + sp * (G::PRB * G::COUT * G::PW) + e);
            typedef _Float16 f16x4c __attribute__((ext_vector_type(4)));
            const f16x4c av4 = __builtin_bit_cast(f16x4c, make_uint2(u.x & m01, u.y & m23));
#pragma unroll
            for (int mt = 0; mt < G::MT; ++mt)
              acc[mt][m] = __builtin_amdgcn_smfmac_f32_16x16x32_f16(av4, __builtin_bit_cast(f16x8, av[mt]), acc[mt][m], ix, 0, 0);
          }
        }
        continue;
      }
      u32x4 bv[NS][2];
#ifndef BA3C_C0W_PKMASK
#define BA3C_C0W_PKMASK 1
#endif
#pragma unroll
      for (int nt = 0; nt < 2; ++nt) {
        const int e = e0 + 16 * nt * G::PW;
        const uint32_t cw = *reinterpret_cast<const uint32_t*>(yc8 + e);
        if constexpr (BA3C_C0W_PKMASK) {
          // the four windows' codes as 16-bit halves, xor 2 sy: a window's argmax is in this
          // pixel row at sub-column h exactly when its half equals h (255 ^ 2 sy never does);
          // m0 / m1 = 0xFFFF halves where it is sub-column 0 / 1 (packed 16-bit compares:
          // 14 VALU per n-tile for what took a bfe + compare + select per window and mask)
          const uint32_t sx = sy * 0x00020002u;
          const uint32_t k01 = __builtin_amdgcn_perm(cw, cw, 0x0C010C00u) ^ sx;
          const uint32_t k23 = __builtin_amdgcn_perm(cw, cw, 0x0C030C02u) ^ sx;
          const uint32_t m0a = c0w_mask16_eq0(k01), m1a = c0w_mask16_eq0(k01 ^ 0x00010001u);
          const uint32_t m0b = c0w_mask16_eq0(k23), m1b = c0w_mask16_eq0(k23 ^ 0x00010001u);
#pragma unroll
          for (int sp = 0; sp < NS; ++sp) {
            const uint2 u = *reinterpret_cast<const uint2*>(ys + sp * (G::PRB * G::COUT * G::PW) + e);
            // window j's dword = (v_j at sub-column 0, v_j at sub-column 1): low halves of
            // (u & m0, u & m1) for even j, high halves for odd j
            const uint32_t a0 = u.x & m0a, b0 = u.x & m1a, a1 = u.y & m0b, b1 = u.y & m1b;
            bv[sp][nt] = u32x4{__builtin_amdgcn_perm(b0, a0, 0x05040100u), __builtin_amdgcn_perm(b0, a0, 0x07060302u),
                               __builtin_amdgcn_perm(b1, a1, 0x05040100u), __builtin_amdgcn_perm(b1, a1, 0x07060302u)};
          }
          continue;
        }
        uint32_t mk[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t k = (cw >> (8 * j)) & 255u;   // 0..3, or 255 (no gradient)
          mk[j] = (k >> 1) == sy ? ((k & 1u) ? 0xFFFF0000u : 0x0000FFFFu) : 0u;
        }
#pragma unroll
        for (int sp = 0; sp < NS; ++sp) {
          const uint2 u = *reinterpret_cast<const uint2*>(ys + sp * (G::PRB * G::COUT * G::PW) + e);
          // (lo, lo) and (hi, hi) half-word pairs of each dword
          bv[sp][nt] = u32x4{__builtin_amdgcn_perm(u.x, u.x, 0x01000100u) & mk[0],
                             __builtin_amdgcn_perm(u.x, u.x, 0x03020302u) & mk[1],
                             __builtin_amdgcn_perm(u.y, u.y, 0x01000100u) & mk[2],
                             __builtin_amdgcn_perm(u.y, u.y, 0x03020302u) & mk[3]};
        }
      }
#pragma unroll
      for (int sp = 0; sp < NS; ++sp)
#pragma unroll
        for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
          for (int nt = 0; nt < 2; ++nt)
            acc[mt][nt] = SP::mfma(av[mt], bv[sp][nt], acc[mt][nt]);
    }
  }

  // ---- epilogue: the four waves' accumulators go through LDS and are summed in wave order
  // into ONE slab per workgroup (dense: lane holds rows (tap, c) 16 mt + 4 lq + r, column
  // o = 16 nt + li; sparse: rows o = 16 m + 4 lq + r, column (tap, c) = 16 mt + li) ----
  static_assert(4 * G::M * G::COUT * 4 <= G::ALLOC_U4 * 16, "slab staging fits the band LDS");
  float* red = reinterpret_cast<float*>(lds);
  __syncthreads();                                     // last band's LDS reads are done
#pragma unroll
  for (int mt = 0; mt < G::MT; ++mt)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if constexpr (C0W_SPARSE) {
          const int tap = C0W_TAP_OUT[4 * mt + (li >> 2)], c = li & 3, o = 16 * nt + 4 * lq + r;
          if (tap >= 0) red[(wave * G::M + tap * G::C + c) * G::COUT + o] = acc[mt][nt][r];
        } else {
          const int tap = C0W_TAP_OUT[4 * mt + lq];      // row 4 lq + r = (slot lq, channel r)
          if (tap >= 0) red[(wave * G::M + tap * G::C + r) * G::COUT + 16 * nt + li] = acc[mt][nt][r];
        }
      }
  __syncthreads();
  float* pz = a.part + (size_t)bx * G::M * G::COUT;
  const float oscale = (1.0f / 255.0f) * exp2i(-ky);
  for (int e = tid; e < G::M * G::COUT; e += 256) {
    constexpr int W = G::M * G::COUT;
    pz[e] = (((red[e] + red[W + e]) + red[2 * W + e]) + red[3 * W + e]) * oscale;
  }
}

template <int NS>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) conv0s_wgrad_kernel(const Conv0WArgs a) {
  __shared__ uint4 lds[Conv0W<NS>::ALLOC_U4];
  __shared__ uint32_t red4[4];
  conv0s_wgrad_body<NS>(a, blockIdx.x, gridDim.x, lds, red4);
}

}  // namespace ba3c
