// ba3c_problems.h — operand gathers and fused epilogues for each product of the BA3C net.
//
// Geometry is compile-time (84x84 frames, train.py:92; conv stack train.py:177-212), so all
// index decodes are multiply-shift.  Activations are NHWC fp32; a max-pooled layer stores
// its pooled output plus a 1-byte argmax code per element (0..3 = row-major position of
// the FIRST maximum of the 2x2 window, TF's tie rule; 255 = window max <= 0, i.e. the ReLU
// gradient is zero).  Backward loaders "unpool" on the fly from (dP, code), so no
// full-resolution gradient map is ever written.
#pragma once
#include <type_traits>

#include "ba3c_gemm.h"

namespace ba3c {


// count_nonzero of ReLU outputs (train.py:271): one integer add per wave, spread over
// RELU_SLOTS counters so 10^5 waves do not serialise on one address (summed by the scalars
// kernel; integer adds are exact in any order).
constexpr int RELU_SLOTS = 1024;
// the ReLU-count region holds one more word: the heads kernel's completion counter (its last
// workgroup reduces the per-sample loss terms), zeroed with the counters every training step
constexpr int RELU_WORDS = RELU_SLOTS + 1;
__device__ __forceinline__ void relu_count_add(unsigned long long* slots, unsigned long long pos, int lane) {
  pos = wave_sum_u64(pos);
  if (lane == 0 && pos) {
    const unsigned slot = (blockIdx.x * 4u + (threadIdx.x >> 6) + blockIdx.y * 977u) & (RELU_SLOTS - 1);
    atomicAdd(slots + slot, pos);
  }
}

// Wave-uniform variant: count positives with v_cmp -> SGPR mask + s_bcnt1 (scalar ALU), one
// VALU instruction per value instead of a compare, a select and a 64-bit add.
__device__ __forceinline__ unsigned long long count_pos4(float v0, float v1, float v2, float v3) {
  return (unsigned long long)(__popcll(__ballot(v0 > 0.f)) + __popcll(__ballot(v1 > 0.f)) +
                              __popcll(__ballot(v2 > 0.f)) + __popcll(__ballot(v3 > 0.f)));
}
__device__ __forceinline__ void relu_count_add_uniform(unsigned long long* slots, unsigned long long pos,
                                                       int lane) {
  if (lane == 0 && pos) {
    const unsigned slot = (blockIdx.x * 4u + (threadIdx.x >> 6) + blockIdx.y * 977u) & (RELU_SLOTS - 1);
    atomicAdd(slots + slot, pos);
  }
}

// Max |x| of a tensor, published for the scaled-fp16 split kernels that consume it
// (ba3c_split.h): lane 0 of a wave adds the wave's max of image img to slot [1 + img]
// (atomicMax on the bits of a non-negative float orders like the float; a few tens of waves
// per image, so the adds do not contend — one chip-wide slot measured +0.2 ms per producer).
// Every lane of the wave must call it (wave-wide reduction).
// Device-coherent (agent-scope: global_store / global_load sc1) accesses for data handed
// between the jobs of one chained launch (ba3c_multi.h launch_chain): they leave / bypass the
// XCD's non-coherent L2, so neither side needs a fence.
__device__ __forceinline__ void st_agent_u32(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent_u64(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// One wave waits until a chained launch's signal count reaches `need` (bounded: gives up with
// bit 0 of *err set rather than hang the device).
__device__ __forceinline__ void chain_wait_wave(const unsigned* sig, unsigned need, unsigned* err) {
  unsigned spins = 0;
  while (__hip_atomic_load(const_cast<unsigned*>(sig), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < need) {
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1u << 22)) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 1u);
      break;
    }
  }
}

// chained launches' spread signal counters: one per 64-byte line
constexpr int CHAIN_STRIDE = 16;
// wave-wide: wait until the `n` (<= 64) spread counters sum to `need` (bounded)
__device__ __forceinline__ void chain_wait_spread(const unsigned* ctr, int n, unsigned need, unsigned* err) {
  const int lane = threadIdx.x & 63;
  unsigned spins = 0;
  while (true) {
    unsigned v = lane < n ? __hip_atomic_load(const_cast<unsigned*>(ctr) + CHAIN_STRIDE * lane, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT)
                          : 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    if (v >= need) break;
    __builtin_amdgcn_s_sleep(2);
    if (++spins > (1u << 22)) {
      if (lane == 0) atomicOr(err, 1u);
      break;
    }
  }
}

__device__ __forceinline__ void amax_publish(uint32_t* slots, int img, float m, int lane) {
  if (!slots) return;
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
  if (lane == 0 && m > 0.f) atomicMax(slots + 1 + img, __float_as_uint(m));
}

// The whole tensor's max (bits) from its per-image slots [1, 1 + B), for every thread of a
// 256-thread workgroup (red4: 4 words of LDS).
__device__ __forceinline__ uint32_t amax_all(const uint32_t* slots, int B, uint32_t* red4) {
  uint32_t m = 0;
  for (int i = threadIdx.x; i < B; i += 256) m = max(m, slots[1 + i]);
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
  if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
  __syncthreads();
  const uint32_t r = max(max(red4[0], red4[1]), max(red4[2], red4[3]));
  __syncthreads();
  return r;
}

// dY at conv-output position (y, x) from pooled grad dP and argmax codes (0 where !ok).
template <int PW, int COUT>
__device__ __forceinline__ UnpoolRaw unpool4(const float* __restrict__ dP, const uint8_t* __restrict__ code,
                                             int n_ph_base, int y, int x, int c, bool ok = true) {
  const size_t e = (size_t)(n_ph_base + (y >> 1) * PW + (x >> 1)) * COUT + c;
  UnpoolRaw r;
  r.g = ld4(dP + e, ok);
  r.cd = ld_u8x4(code + e, ok);
  r.sub = ok ? ((y & 1) << 1) | (x & 1) : 256u;   // 256: matches no code
  return r;
}

// ------------------------------------------------------------------------------------
// Forward conv (Conv2D VALID stride 1, no bias; models/conv2d.py:63-73, train.py:177-212)
// MODE 0: ReLU + 2x2 max-pool + argmax code (codes when `code` is set)   MODE 1: same without codes
// MODE 2: ReLU only, plain NHWC store (conv3)
// M rows: MODE 0/1 = (n, ph, pw, sub) so a lane's 4 consecutive accumulator rows are one
// pooling window; MODE 2 = (n, oh, ow).  K = (kh, kw, c) over the REAL input channels
// (conv0's 16-channel zero padding, train.py:173-174, contributes exactly 0).
// ------------------------------------------------------------------------------------
template <bool SRC_U8, int HIN, int WIN, int CIN, int CINPAD, int KH, int KW, int COUT, int MODE>
struct ConvFwd {
  static constexpr bool A_KCONTIG = true, B_KCONTIG = false;
  static constexpr int HO = HIN - KH + 1, WO = WIN - KW + 1, PH = HO / 2, PW = WO / 2;
  static constexpr int KDIM = KH * KW * CIN;
  using ARow = int;
  using BRow = int;
  using ARaw = typename std::conditional<SRC_U8, uint32_t, float4>::type;
  using BRaw = float4;
  const void* src;
  const float* w;
  float* out;
  uint8_t* code;
  unsigned long long* relu_count;
  float scale;
  int M, N, K, kchunk;
  uint32_t* amax;        // MODE 0/1: max of the pooled output per image (may be null)

  __device__ int a_row(int m) const {
    if (m >= M) return -1;
    int n, oh, ow;
    if constexpr (MODE != 2) {
      const int win = m >> 2, sub = m & 3;
      n = win / (PH * PW);
      const int r = win - n * (PH * PW);
      const int ph = r / PW, pw = r - ph * PW;
      oh = 2 * ph + (sub >> 1);
      ow = 2 * pw + (sub & 1);
    } else {
      n = m / (HO * WO);
      const int r = m - n * (HO * WO);
      oh = r / WO;
      ow = r - oh * WO;
    }
    return ((n * HIN + oh) * WIN + ow) * CIN;
  }
  __device__ ARaw a_load(int row, int k, int kend) const {
    const bool ok = row >= 0 && k < kend;
    const int kh = k / (KW * CIN);
    const int r = k - kh * (KW * CIN);
    const int kw = r / CIN, c = r - kw * CIN;
    const int off = row + (kh * WIN + kw) * CIN + c;
    if constexpr (SRC_U8)
      return ld_u8x4(static_cast<const uint8_t*>(src) + off, ok);
    else
      return ld4(static_cast<const float*>(src) + off, ok);
  }
  __device__ int b_col(int n) const { return n < N ? n : -1; }
  __device__ BRaw b_load_t(int ncol, int k, int kend) const {
    const bool ok = ncol >= 0 && k < kend;
    const int kh = k / (KW * CIN);
    const int r = k - kh * (KW * CIN);
    const int kw = r / CIN, c = r - kw * CIN;
    return ld4(w + ((kh * KW + kw) * CINPAD + c) * COUT + ncol, ok);
  }
  template <int TM, int TN>
  __device__ void epilogue(const f32x16 (&acc)[TM][TN], int mrow, int ncol, int lane, int) const {
    const int j = lane & 31, h = lane >> 5;
    unsigned long long pos = 0;
    constexpr int WPI = MODE != 2 ? PH * PW : 1;       // pooling windows per image
    static_assert(MODE == 2 || TM * 8 <= WPI, "a wave's windows span at most two images");
    const int n0 = (mrow >> 2) / WPI;
    float m0 = 0.f, m1 = 0.f;   // max pooled output of images n0, n0 + 1 in this lane's rows
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = ncol + b * 32 + j;
        if constexpr (MODE != 2) {
          const int wbase = (mrow + a * 32) >> 2;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v0 = acc[a][b][4 * q + 0] * scale, v1 = acc[a][b][4 * q + 1] * scale;
            const float v2 = acc[a][b][4 * q + 2] * scale, v3 = acc[a][b][4 * q + 3] * scale;
            pos += (v0 > 0.f) + (v1 > 0.f) + (v2 > 0.f) + (v3 > 0.f);
            float mx = v0;
            uint32_t arg = 0;
            if (v1 > mx) { mx = v1; arg = 1; }
            if (v2 > mx) { mx = v2; arg = 2; }
            if (v3 > mx) { mx = v3; arg = 3; }
            const int win = wbase + 2 * q + h;
            if (win * 4 < M && col < N) {
              const float o = fmaxf(mx, 0.f);
              out[(size_t)win * COUT + col] = o;
              if (win / WPI == n0) m0 = fmaxf(m0, o);
              else m1 = fmaxf(m1, o);
              if (MODE == 0 && code) code[(size_t)win * COUT + col] = mx > 0.f ? (uint8_t)arg : (uint8_t)255;
            }
          }
        } else {
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow + a * 32 + acc_row(r, lane);
            const float v = acc[a][b][r] * scale;
            pos += (v > 0.f);
            if (m < M && col < N) out[(size_t)m * COUT + col] = fmaxf(v, 0.f);
          }
        }
      }
    if (relu_count) relu_count_add(relu_count, pos, lane);
    if (MODE != 2 && amax) {
      amax_publish(amax, n0, m0, lane);
      if (((mrow + TM * 32 - 1) >> 2) / WPI > n0) amax_publish(amax, n0 + 1, m1, lane);
    }
  }
};

// ------------------------------------------------------------------------------------
// Conv2DBackpropInput: dX[n,y,x,ci] = sum_{kh,kw,o} dY[n,y-kh,x-kw,o] W[kh,kw,ci,o]
// M = (n, y, x) over the input map, N = ci, K = (kh, kw, o).  POOLED: dY is unpooled from
// (dP, code) of the max-pool that follows this conv (MaxPoolGrad + ReluGrad fused).
// ------------------------------------------------------------------------------------
template <int HIN, int WIN, int CIN, int KH, int KW, int COUT, bool POOLED>
struct ConvDgrad {
  static constexpr bool A_KCONTIG = true, B_KCONTIG = true;
  static constexpr int HO = HIN - KH + 1, WO = WIN - KW + 1, PH = HO / 2, PW = WO / 2;
  struct ARow { int n, y, x; };
  using BRow = int;
  using ARaw = typename std::conditional<POOLED, UnpoolRaw, float4>::type;
  using BRaw = float4;
  const float* dy;       // POOLED: dP [B,PH,PW,COUT]  else dY [B,HO,WO,COUT]
  const uint8_t* code;   // POOLED only
  const float* w;        // [KH,KW,CIN,COUT]
  float* dx;             // [B,HIN,WIN,CIN]
  int M, N, K, kchunk;
  uint32_t* amax;        // max |dx| per image (amax_publish slots; may be null)

  __device__ ARow a_row(int m) const {
    ARow r;
    if (m >= M) { r.n = -1; r.y = 0; r.x = 0; return r; }
    r.n = m / (HIN * WIN);
    const int q = m - r.n * (HIN * WIN);
    r.y = q / WIN;
    r.x = q - r.y * WIN;
    return r;
  }
  __device__ ARaw a_load(const ARow& r, int k, int kend) const {
    const int kh = k / (KW * COUT);
    const int q = k - kh * (KW * COUT);
    const int kw = q / COUT, o = q - kw * COUT;
    const int yy = r.y - kh, xx = r.x - kw;
    const bool ok = r.n >= 0 && k < kend && yy >= 0 && yy < HO && xx >= 0 && xx < WO;
    if constexpr (POOLED)
      return unpool4<PW, COUT>(dy, code, r.n * (PH * PW), yy, xx, o, ok);
    else
      return ld4(dy + ((size_t)(r.n * HO + yy) * WO + xx) * COUT + o, ok);
  }
  __device__ int b_row(int n) const { return n < N ? n : -1; }
  __device__ BRaw b_load(int ci, int k, int kend) const {
    const bool ok = ci >= 0 && k < kend;
    const int kh = k / (KW * COUT);
    const int q = k - kh * (KW * COUT);
    const int kw = q / COUT, o = q - kw * COUT;
    return ld4(w + ((kh * KW + kw) * CIN + ci) * COUT + o, ok);
  }
  template <int TM, int TN>
  __device__ void epilogue(const f32x16 (&acc)[TM][TN], int mrow, int ncol, int lane, int) const {
    static_assert(TM * 32 <= HIN * WIN, "a wave's rows span at most two images");
    const int j = lane & 31;
    const int n0 = mrow / (HIN * WIN);
    float m0 = 0.f, m1 = 0.f;   // max |dx| of images n0 and n0 + 1 in this lane's rows
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = ncol + b * 32 + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow + a * 32 + acc_row(r, lane);
          if (m < M && col < N) {
            const float v = acc[a][b][r];
            dx[(size_t)m * CIN + col] = v;
            if (m / (HIN * WIN) == n0) m0 = fmaxf(m0, fabsf(v));
            else m1 = fmaxf(m1, fabsf(v));
          }
        }
      }
    if (amax) {
      amax_publish(amax, n0, m0, lane);
      if ((mrow + TM * 32 - 1) / (HIN * WIN) > n0) amax_publish(amax, n0 + 1, m1, lane);
    }
  }
};

// ------------------------------------------------------------------------------------
// Conv2DBackpropFilter: dW[kh,kw,c,o] = sum_{n,y,x} X[n,y+kh,x+kw,c] dY[n,y,x,o]
// M = (kh, kw, c) (real channels), N = o, K = (n, y, x) split over blockIdx.z.
// Writes fp32 partial slabs part[z][m][n]; scale = 1/255 for the uint8 frame input.
// ------------------------------------------------------------------------------------
template <bool SRC_U8, int HIN, int WIN, int CIN, int KH, int KW, int COUT, bool POOLED>
struct ConvWgrad {
  static constexpr bool A_KCONTIG = false, B_KCONTIG = false;
  static constexpr int HO = HIN - KH + 1, WO = WIN - KW + 1, PH = HO / 2, PW = WO / 2;
  using ARow = int;
  using BRow = int;
  using ARaw = typename std::conditional<SRC_U8, uint32_t, float4>::type;
  using BRaw = typename std::conditional<POOLED, UnpoolRaw, float4>::type;
  const void* src;       // X [B,HIN,WIN,CIN] (u8 or f32)
  const float* dy;       // POOLED: dP [B,PH,PW,COUT] else dY [B,HO,WO,COUT]
  const uint8_t* code;
  float* part;
  float scale;
  int M, N, K, kchunk;

  __device__ int a_col(int m) const {
    if (m >= M) return -1;
    const int kh = m / (KW * CIN);
    const int q = m - kh * (KW * CIN);
    const int kw = q / CIN, c = q - kw * CIN;
    return (kh * WIN + kw) * CIN + c;
  }
  __device__ ARaw a_load_t(int mo, int k, int kend) const {
    const bool ok = mo >= 0 && k < kend;
    const int n = k / (HO * WO);
    const int q = k - n * (HO * WO);
    const int y = q / WO, x = q - y * WO;
    const size_t off = ((size_t)(n * HIN + y) * WIN + x) * CIN + mo;
    if constexpr (SRC_U8)
      return ld_u8x4(static_cast<const uint8_t*>(src) + off, ok);
    else
      return ld4(static_cast<const float*>(src) + off, ok);
  }
  __device__ int b_col(int n) const { return n < N ? n : -1; }
  __device__ BRaw b_load_t(int c, int k, int kend) const {
    const bool ok = c >= 0 && k < kend;
    const int n = k / (HO * WO);
    const int q = k - n * (HO * WO);
    const int y = q / WO, x = q - y * WO;
    if constexpr (POOLED)
      return unpool4<PW, COUT>(dy, code, n * (PH * PW), y, x, c, ok);
    else
      return ld4(dy + (size_t)k * COUT + c, ok);
  }
  template <int TM, int TN>
  __device__ void epilogue(const f32x16 (&acc)[TM][TN], int mrow, int ncol, int lane, int z) const {
    const int j = lane & 31;
    float* pz = part + (size_t)z * M * N;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = ncol + b * 32 + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow + a * 32 + acc_row(r, lane);
          if (m < M && col < N) pz[(size_t)m * N + col] = acc[a][b][r] * scale;
        }
      }
  }
};

// ------------------------------------------------------------------------------------
// FC1 forward (train.py:216-243): h[b][f] = sum_j a3[b][j] W1[j][f], W1 = concat of the
// S split tensors along f (each [1600, per], row-major; the 5x5x64 conv form flattens
// (h,w,c) exactly like batch_flatten).  Legacy (--use_normal_fc): + bias, ReLU.
// ------------------------------------------------------------------------------------
struct FcFwd {
  static constexpr bool A_KCONTIG = true, B_KCONTIG = false;
  using ARow = int;
  using BRow = int;
  using ARaw = float4;
  using BRaw = float4;
  const float* a3;      // [B,1600]
  const float* w1;      // split 0 base
  float* h;             // [B,F]
  unsigned long long* relu_count;
  int per, wstride, legacy;
  int M, N, K, kchunk;
  float* part;          // split-K (kchunk > 0): raw partial slabs [z][M][N]; the heads kernel
                        // (ba3c_small.h) sums them in z order and applies the legacy epilogue

  __device__ int a_row(int m) const { return m < M ? m * 1600 : -1; }
  __device__ ARaw a_load(int row, int k, int kend) const {
    return ld4(a3 + (size_t)row + k, row >= 0 && k < kend);
  }
  __device__ int b_col(int n) const {
    if (n >= N) return -1;
    const int s = n / per;
    return s * wstride + (n - s * per);
  }
  __device__ BRaw b_load_t(int c, int k, int kend) const {
    return ld4(w1 + c + (size_t)k * per, c >= 0 && k < kend);
  }
  template <int TM, int TN>
  __device__ void epilogue(const f32x16 (&acc)[TM][TN], int mrow, int ncol, int lane, int z) const {
    const int j = lane & 31;
    if (part) {
      float* pz = part + (size_t)z * M * N;
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b) {
          const int col = ncol + b * 32 + j;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int m = mrow + a * 32 + acc_row(r, lane);
            if (m < M && col < N) pz[(size_t)m * N + col] = acc[a][b][r];
          }
        }
      return;
    }
    unsigned long long pos = 0;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = ncol + b * 32 + j;
        float bias = 0.f;
        if (legacy && col < N) {
          const int s = col / per;
          bias = w1[s * wstride + 1600 * per + (col - s * per)];
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow + a * 32 + acc_row(r, lane);
          float v = acc[a][b][r];
          if (legacy) {
            v = fmaxf(v + bias, 0.f);
            pos += (v > 0.f) && (m < M);
          }
          if (m < M && col < N) h[(size_t)m * N + col] = v;
        }
      }
    if (legacy && relu_count) relu_count_add(relu_count, pos, lane);
  }
};

// FC1 input gradient: dY3[b][j] = (sum_f dh[b][f] W1[j][f]) * (a3[b][j] > 0)
struct FcDgrad {
  static constexpr bool A_KCONTIG = true, B_KCONTIG = true;
  using ARow = int;
  using BRow = int;
  using ARaw = float4;
  using BRaw = float4;
  const float* dh;   // [B,F]
  const float* w1;
  const float* a3;   // [B,1600] relu mask source
  float* dy3;        // [B,1600]
  int per, wstride;
  int M, N, K, kchunk;  // M=B, N=1600, K=F

  __device__ int a_row(int m) const { return m < M ? m * K : -1; }
  __device__ ARaw a_load(int row, int k, int kend) const {
    return ld4(dh + (size_t)row + k, row >= 0 && k < kend);
  }
  __device__ int b_row(int n) const { return n < N ? n * per : -1; }
  __device__ BRaw b_load(int row, int k, int kend) const {
    const int s = k / per;
    return ld4(w1 + (size_t)s * wstride + row + (k - s * per), row >= 0 && k < kend);
  }
  template <int TM, int TN>
  __device__ void epilogue(const f32x16 (&acc)[TM][TN], int mrow, int ncol, int lane, int) const {
    const int j = lane & 31;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = ncol + b * 32 + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow + a * 32 + acc_row(r, lane);
          if (m < M && col < N) {
            const size_t o = (size_t)m * 1600 + col;
            dy3[o] = a3[o] > 0.f ? acc[a][b][r] : 0.f;
          }
        }
      }
  }
};

// Weight gradient of a [B,Kin] x [Kin,Nout] product with the batch as reduction:
// part[z][m][n] = sum_b X[b][m] G[b][n] over the chunk; row m == Kin is the bias row
// (X == 1) when has_bias.  Used for fc1 (X=a3, G=dh) and the heads (X=h, G=[dz|dv]).
struct BatchWgrad {
  static constexpr bool A_KCONTIG = false, B_KCONTIG = false;
  using ARow = int;
  using BRow = int;
  using ARaw = float4;
  using BRaw = float4;
  const float* x;    // [B, kin]
  const float* g;    // [B, gld]
  float* part;
  int kin, gld, has_bias;
  int M, N, K, kchunk;   // M = kin (+1), N = columns of g used, K = B

  __device__ int a_col(int m) const {
    if (m < kin) return m;
    if (has_bias && m == kin) return -2;
    return -1;
  }
  __device__ ARaw a_load_t(int c, int k, int kend) const {
    // the bias row (c == -2) reads {1, 0, 0, 0}
    const float* q = (c == -2 && k < kend) ? kOne4 : x + (size_t)k * kin + c;
    return ld4(q, (c >= 0 || c == -2) && k < kend);
  }
  __device__ int b_col(int n) const { return n < N ? n : -1; }
  __device__ BRaw b_load_t(int c, int k, int kend) const {
    return ld4(g + (size_t)k * gld + c, c >= 0 && k < kend);
  }
  template <int TM, int TN>
  __device__ void epilogue(const f32x16 (&acc)[TM][TN], int mrow, int ncol, int lane, int z) const {
    const int j = lane & 31;
    float* pz = part + (size_t)z * M * N;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b) {
        const int col = ncol + b * 32 + j;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = mrow + a * 32 + acc_row(r, lane);
          if (m < M && col < N) pz[(size_t)m * N + col] = acc[a][b][r];
        }
      }
  }
};

}  // namespace ba3c
