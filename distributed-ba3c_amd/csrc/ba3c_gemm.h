// ba3c_gemm.h — fp32-MFMA implicit-GEMM engine for gfx950 (CDNA4).
//
// Every conv / FC product of the BA3C net (OpenAIGym/train.py:177-264 forward, and the TF
// autodiff Conv2DBackpropInput / Conv2DBackpropFilter / MatMul grads of
// train/multigpu.py:85-86) is C[M][N] = sum_k A[m][k] B[k][n] where A and B are gathered
// on the fly from NHWC activations / HWIO weights by a problem struct P (ba3c_problems.h).
//
// Tile: BM x BN x 32 per 256-thread workgroup (4 waves as WGM x WGN), each wave owning a
// (BM/WGM) x (BN/WGN) block of 32x32 accumulators fed by v_mfma_f32_32x32x2_f32 (exact f32,
// 64 FLOP/clk/SIMD — gfx950 has no xf32).  Operands are staged through LDS in k-major
// layout ([k][m], [k][n]) so every MFMA fragment read is one conflict-free ds_read_b32 per
// 32-lane half; gathered rows that are contiguous along k are transposed on the LDS write
// (row pitch BM+1 keeps those ds_write_b32 conflict-free).  The next k-tile's global loads
// are issued before the current tile's MFMAs (register prefetch, one LDS buffer).
// Split-K over blockIdx.z (P::kchunk > 0) writes fp32 partial slabs reduced by a separate,
// deterministic kernel.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// Non-template kernels defined in the shared headers are emitted by one translation unit only
// (ba3c_capi.hip); the other units (ba3c_conv0.hip) set this to 0.
#ifndef BA3C_SHARED_KERNELS
#define BA3C_SHARED_KERNELS 1
#endif

namespace ba3c {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int GEMM_BK = 32;

__device__ __forceinline__ float4 u8x4_to_f4(uint32_t v) {
  return make_float4((float)(v & 255u), (float)((v >> 8) & 255u), (float)((v >> 16) & 255u),
                     (float)(v >> 24));
}

// Operand fetches are branch-free and return the RAW loaded words; `fin` turns them into the
// float4 operand when the k-tile is staged.  An out-of-range element is fetched from a
// 16-byte zero block instead of its tensor (no select on the data), so nothing consumes a
// load before it is staged: a load under a branch, or an op on its result right after it,
// makes the compiler drain every outstanding load (vmcnt(0)) there, which would serialise
// the k-tile register ring of gemm6_kernel.
__device__ __attribute__((aligned(16))) float kZero4[4] = {0.f, 0.f, 0.f, 0.f};
__device__ __attribute__((aligned(16))) float kOne4[4] = {1.f, 0.f, 0.f, 0.f};

__device__ __forceinline__ float4 ld4(const float* p, bool ok) {
  return *reinterpret_cast<const float4*>(ok ? p : kZero4);
}
__device__ __forceinline__ uint32_t ld_u8x4(const uint8_t* p, bool ok) {
  return *reinterpret_cast<const uint32_t*>(ok ? p : reinterpret_cast<const uint8_t*>(kZero4));
}
struct UnpoolRaw {
  float4 g;
  uint32_t cd, sub;
};
// pin(): an empty volatile asm that "redefines" the raw words where a k-tile is staged, so
// no pass can hoist the staging arithmetic of a later tile (and the wait for its loads)
// ahead of the current one
__device__ __forceinline__ void pin(float4& v) { asm volatile("" : "+v"(v.x), "+v"(v.y), "+v"(v.z), "+v"(v.w)); }
__device__ __forceinline__ void pin(uint32_t& u) { asm volatile("" : "+v"(u)); }
__device__ __forceinline__ float4 fin(const float4& v) { return v; }
__device__ __forceinline__ float4 fin(uint32_t u) { return u8x4_to_f4(u); }
__device__ __forceinline__ void pin(UnpoolRaw& r) {
  pin(r.g);
  asm volatile("" : "+v"(r.cd), "+v"(r.sub));
}
__device__ __forceinline__ float4 fin(const UnpoolRaw& r) {
  float4 g = r.g;
  g.x = ((r.cd & 255u) == r.sub) ? g.x : 0.f;
  g.y = (((r.cd >> 8) & 255u) == r.sub) ? g.y : 0.f;
  g.z = (((r.cd >> 16) & 255u) == r.sub) ? g.z : 0.f;
  g.w = ((r.cd >> 24) == r.sub) ? g.w : 0.f;
  return g;
}

constexpr int GEMM_THREADS = 256;

__device__ __forceinline__ float4 f4zero() { return make_float4(0.f, 0.f, 0.f, 0.f); }

__device__ __forceinline__ float f4get(const float4& v, int j) {
  return j == 0 ? v.x : (j == 1 ? v.y : (j == 2 ? v.z : v.w));
}

template <int BM, int BN, int WGM, int WGN, class P>
__global__ void __launch_bounds__(GEMM_THREADS) gemm_kernel(const P p) {
  static_assert(WGM * WGN == 4, "4 waves per workgroup");
  constexpr int BK = GEMM_BK;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  constexpr int PADA = P::A_KCONTIG ? 1 : 4;
  constexpr int PADB = P::B_KCONTIG ? 1 : 4;
  constexpr int LDA = BM + PADA, LDB = BN + PADB;
  constexpr int NA = BM * BK / 4 / GEMM_THREADS;  // float4 per thread per k-tile
  constexpr int NB = BN * BK / 4 / GEMM_THREADS;
  static_assert(NA >= 1 && NB >= 1, "tile too small for 256 threads");
  // !KCONTIG operands: a float4 spans 4 consecutive m (n); QA quads per k-row.
  constexpr int QA = BM / 4, QB = BN / 4;
  constexpr int RA = GEMM_THREADS / QA, RB = GEMM_THREADS / QB;  // k-rows per pass

  __shared__ __attribute__((aligned(16))) float lds[BK * LDA + BK * LDB];
  float* As = lds;
  float* Bs = lds + BK * LDA;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;
  int kbeg = 0, kend = p.K;
  if (p.kchunk > 0) {
    kbeg = blockIdx.z * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }

  // per-thread operand coordinates that do not change along k
  typename P::ARow arow[P::A_KCONTIG ? NA : 1];
  typename P::BRow brow[P::B_KCONTIG ? NB : 1];
  if constexpr (P::A_KCONTIG) {
#pragma unroll
    for (int i = 0; i < NA; ++i) arow[i] = p.a_row(m0 + (tid >> 3) + 32 * i);
  } else {
    arow[0] = p.a_col(m0 + (tid % QA) * 4);
  }
  if constexpr (P::B_KCONTIG) {
#pragma unroll
    for (int i = 0; i < NB; ++i) brow[i] = p.b_row(n0 + (tid >> 3) + 32 * i);
  } else {
    brow[0] = p.b_col(n0 + (tid % QB) * 4);
  }

  float4 ra[NA], rb[NB];
  auto load = [&](int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (P::A_KCONTIG)
        ra[i] = fin(p.a_load(arow[i], k0 + (tid & 7) * 4, kend));
      else
        ra[i] = fin(p.a_load_t(arow[0], k0 + tid / QA + RA * i, kend));
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (P::B_KCONTIG)
        rb[i] = fin(p.b_load(brow[i], k0 + (tid & 7) * 4, kend));
      else
        rb[i] = fin(p.b_load_t(brow[0], k0 + tid / QB + RB * i, kend));
    }
  };
  auto store = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (P::A_KCONTIG) {
        const int ml = (tid >> 3) + 32 * i, kq = (tid & 7) * 4;
        As[(kq + 0) * LDA + ml] = ra[i].x;
        As[(kq + 1) * LDA + ml] = ra[i].y;
        As[(kq + 2) * LDA + ml] = ra[i].z;
        As[(kq + 3) * LDA + ml] = ra[i].w;
      } else {
        const int kl = tid / QA + RA * i, mq = (tid % QA) * 4;
        *reinterpret_cast<float4*>(&As[kl * LDA + mq]) = ra[i];
      }
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (P::B_KCONTIG) {
        const int nl = (tid >> 3) + 32 * i, kq = (tid & 7) * 4;
        Bs[(kq + 0) * LDB + nl] = rb[i].x;
        Bs[(kq + 1) * LDB + nl] = rb[i].y;
        Bs[(kq + 2) * LDB + nl] = rb[i].z;
        Bs[(kq + 3) * LDB + nl] = rb[i].w;
      } else {
        const int kl = tid / QB + RB * i, nq = (tid % QB) * 4;
        *reinterpret_cast<float4*>(&Bs[kl * LDB + nq]) = rb[i];
      }
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int a = 0; a < TM; ++a)
#pragma unroll
    for (int b = 0; b < TN; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  const int li = lane & 31, lh = lane >> 5;
  const float* Aw = As + wm * WTM + li;
  const float* Bw = Bs + wn * WTN + li;

  if (kbeg < kend) load(kbeg);
  for (int k0 = kbeg; k0 < kend; k0 += BK) {
    store();
    __syncthreads();
    if (k0 + BK < kend) load(k0 + BK);
#pragma unroll
    for (int s = 0; s < BK / 2; ++s) {
      const int kr = 2 * s + lh;
      float av[TM], bv[TN];
#pragma unroll
      for (int a = 0; a < TM; ++a) av[a] = Aw[kr * LDA + a * 32];
#pragma unroll
      for (int b = 0; b < TN; ++b) bv[b] = Bw[kr * LDB + b * 32];
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
          acc[a][b] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[b], acc[a][b], 0, 0, 0);
    }
    __syncthreads();
  }

  p.template epilogue<TM, TN>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, blockIdx.z);
}

// C/D layout of a 32x32 block (v_mfma_f32_32x32x2_f32): lane l holds column (l & 31),
// register r holds row (r & 3) + 8 * (r >> 2) + 4 * (l >> 5).
__device__ __forceinline__ int acc_row(int r, int lane) {
  return (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
}

__device__ __forceinline__ unsigned long long wave_sum_u64(unsigned long long v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- wave-wide reductions on DPP + gfx950 permlane swaps (VALU-only; ds_bpermute-based
// __shfl_xor went through the LDS unit, ~6 round trips per reduction).  Steps: quad xor 1,
// quad xor 2, half-row mirror, row mirror (DPP), then row pairs (v_permlane16_swap) and halves
// (v_permlane32_swap).  Every step combines a lane with a partner that combines the same two
// operands, so all 64 lanes end with the bit-identical result.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp32(uint32_t x) {
  return __builtin_amdgcn_update_dpp(0u, x, CTRL, 0xF, 0xF, false);
}
template <int CTRL>
__device__ __forceinline__ float dppf(float v) { return __uint_as_float(dpp32<CTRL>(__float_as_uint(v))); }
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
  const unsigned long long u = __double_as_longlong(v);
  const uint32_t lo = dpp32<CTRL>((uint32_t)u), hi = dpp32<CTRL>((uint32_t)(u >> 32));
  return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// (even-row value, odd-row value) of this lane's row pair / (low-half, high-half) values
__device__ __forceinline__ void swap16f(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap32f(float v, float& a, float& b) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  a = __uint_as_float(r[0]);
  b = __uint_as_float(r[1]);
}
__device__ __forceinline__ void swap16d(double v, double& a, double& b) {
  const unsigned long long u = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane16_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}
__device__ __forceinline__ void swap32d(double v, double& a, double& b) {
  const unsigned long long u = __double_as_longlong(v);
  const auto lo = __builtin_amdgcn_permlane32_swap((uint32_t)u, (uint32_t)u, false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap((uint32_t)(u >> 32), (uint32_t)(u >> 32), false, false);
  a = __longlong_as_double((long long)(((unsigned long long)hi[0] << 32) | lo[0]));
  b = __longlong_as_double((long long)(((unsigned long long)hi[1] << 32) | lo[1]));
}

struct OpAdd {
  template <class T>
  __device__ T operator()(T a, T b) const { return a + b; }
};
struct OpMax {
  __device__ float operator()(float a, float b) const { return fmaxf(a, b); }
  __device__ double operator()(double a, double b) const { return fmax(a, b); }
};

// reduction over the first `w` lanes (w <= 4, 8, 16 or 64 — the others must hold the
// identity) in every lane: the narrow forms stop after the DPP steps that cover w lanes and
// broadcast lane 0 (v_readlane)
template <class Op>
__device__ __forceinline__ float wave_reduce_f(float v, Op op, int w = 64) {
  v = op(v, dppf<0xB1>(v));
  v = op(v, dppf<0x4E>(v));
  if (w <= 4) return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 0));
  v = op(v, dppf<0x141>(v));
  if (w <= 8) return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 0));
  v = op(v, dppf<0x140>(v));
  if (w <= 16) return __uint_as_float(__builtin_amdgcn_readlane(__float_as_uint(v), 0));
  float a, b;
  swap16f(v, a, b);
  v = op(a, b);
  swap32f(v, a, b);
  return op(a, b);
}
template <class Op>
__device__ __forceinline__ double wave_reduce_d(double v, Op op, int w = 64) {
  auto bcast0 = [](double x) {
    const unsigned long long u = __double_as_longlong(x);
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, 0), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), 0);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
  };
  v = op(v, dppd<0xB1>(v));
  v = op(v, dppd<0x4E>(v));
  if (w <= 4) return bcast0(v);
  v = op(v, dppd<0x141>(v));
  if (w <= 8) return bcast0(v);
  v = op(v, dppd<0x140>(v));
  if (w <= 16) return bcast0(v);
  double a, b;
  swap16d(v, a, b);
  v = op(a, b);
  swap32d(v, a, b);
  return op(a, b);
}

__device__ __forceinline__ float wave_sum_f(float v) { return wave_reduce_f(v, OpAdd{}); }
__device__ __forceinline__ double wave_sum_d(double v, int w = 64) { return wave_reduce_d(v, OpAdd{}, w); }
__device__ __forceinline__ float wave_max_f(float v) { return wave_reduce_f(v, OpMax{}); }

}  // namespace ba3c
