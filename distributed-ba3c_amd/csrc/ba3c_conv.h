// ba3c_conv.h — direct convolution over an LDS-staged input band (gfx950, fp32 MFMA 16x16x4).
//
// Used for the big forward convs (conv1/conv2 of train.py:187-204, with ReLU + 2x2 max-pool +
// argmax code fused) and for their input gradients (Conv2DBackpropInput), which are the same
// VALID convolution applied to the zero-padded, un-pooled output gradient with the kernel
// rotated by 180 degrees and its channel axes swapped.
//
// One workgroup (4 waves) = one image x one band of RB output rows.  The input rows the band
// needs are copied ONCE into LDS ([row][col][CPITCH] fp32, CPITCH = CIN + 4); every MFMA
// operand is then read from LDS with ds_read_b128 at compile-time offsets, so the MFMA loop
// carries no address arithmetic and no bounds checks (the band holds the zero padding).
// K is consumed in 16-channel chunks; lane group q of MFMA step t supplies channel 4q + t so
// that each lane's 4 consecutive K values are one 16-byte read.  The B operand (weights) is
// read from a per-step [N][K] transposed copy (L2-resident, 16 bytes per lane per 4 MFMAs).
//
// Wave w owns n-block (w % NB) and m-blocks w / NB, w / NB + 4 / NB, ... (16 output rows each),
// with one 4-register accumulator per m-block; rows of a pooled layer are ordered
// (window, sub) so a lane's 4 accumulator rows are exactly one 2x2 window.
#pragma once
#include "ba3c_problems.h"

namespace ba3c {

typedef float f32x4 __attribute__((ext_vector_type(4)));

// ---------------------------------------------------------------------------------------
// Geometry of one band conv.  SRC: 0 = fp32 NHWC input map, 1 = un-pool (dP, code) of the
// map that follows the conv being differentiated, zero-padded by PADY/PADX.
// ---------------------------------------------------------------------------------------
template <int HS_, int WS_, int CIN_, int COUT_, int KH_, int KW_, int RB_, bool POOL_, int SRC_,
          int CPAD_, int PADY_ = 0, int PADX_ = 0, int UPH_ = 0, int UPW_ = 0, int UHO_ = 0,
          int UWO_ = 0>
struct BandGeom {
  static constexpr int HS = HS_, WS = WS_;        // full (padded) input map height / width
  static constexpr int CIN = CIN_, COUT = COUT_, KH = KH_, KW = KW_, RB = RB_;
  static constexpr bool POOL = POOL_;
  static constexpr int SRC = SRC_, PADY = PADY_, PADX = PADX_;
  static constexpr int UPH = UPH_, UPW = UPW_, UHO = UHO_, UWO = UWO_;  // un-pool source dims
  static constexpr int HO = HS - KH + 1, WO = WS - KW + 1;
  static constexpr int NBANDS = (HO + RB - 1) / RB;
  static constexpr int SROWS = RB + KH - 1;       // staged input rows per band
  // pixel pitch: CIN + CPAD floats, CPAD chosen per geometry to minimise ds_read_b128
  // bank conflicts over the 16-lane groups (brute-forced over the lane->pixel map)
  static constexpr int CPITCH = CIN + CPAD_;
  static_assert(CPAD_ % 4 == 0, "16-byte pixel pitch");
  static constexpr int LDS_FLOATS = SROWS * WS * CPITCH;
  static constexpr int NB = COUT / 16;
  static constexpr int MROWS = POOL ? (RB / 2) * (WO / 2) * 4 : RB * WO;   // rows per band
  static constexpr int MB = (MROWS + 15) / 16;
  static constexpr int WPN = 4 / NB;                // waves per n-block
  static constexpr int MBW = (MB + WPN - 1) / WPN;  // m-blocks per wave (max)
  static constexpr int KCH = CIN / 16;              // 16-channel chunks per tap
  static constexpr int KDIM = KH * KW * CIN;
  static_assert(CIN % 16 == 0 && COUT % 16 == 0 && 4 % NB == 0, "band geometry");
  static_assert(!POOL || (RB % 2 == 0 && HO % 2 == 0 && WO % 2 == 0), "pool geometry");
};

struct BandArgs {
  const float* src;        // SRC 0: input map [B,HS,WS,CIN];  SRC 1: dP [B,UPH,UPW,CIN]
  const uint8_t* code;     // SRC 1: argmax codes of dP
  const float* wt;         // [COUT][KH*KW*CIN] (prepared per step)
  float* out;              // POOL: pooled [B,HO/2,WO/2,COUT]; else [B,HO,WO,COUT]
  uint8_t* out_code;       // POOL: argmax codes (may be null: predictor)
  unsigned long long* relu_count;
  int batch;
};

template <class G>
__global__ void __launch_bounds__(256) conv_band_kernel(const BandArgs a) {
  // float4 elements: every LDS access is a 16-byte-aligned ds_read/write_b128 whose
  // compile-time part folds into the instruction's offset field
  __shared__ float4 band4[G::LDS_FLOATS / 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.x / G::NBANDS;
  const int bnd = blockIdx.x - img * G::NBANDS;
  const int y0 = bnd * G::RB;                       // first output row of the band
  const int rows_out = min(G::RB, G::HO - y0);

  // ---- stage input rows [y0, y0 + rows_out + KH - 1) of the (padded) input map ----
  // All of a thread's global loads are issued before any LDS store (one HBM round trip per
  // band instead of one per element).
  {
    constexpr int Q = G::CIN / 4;                   // float4 per pixel
    constexpr int NTOT = (G::SROWS * G::WS * Q + 255) / 256;
    constexpr int NPT = NTOT < 8 ? NTOT : 8;        // loads in flight per thread per chunk
    const int srows = rows_out + G::KH - 1;
    const int nvec = srows * G::WS * Q;
    for (int base = 0; base < NTOT; base += NPT) {
    float4 v[NPT];
    uint32_t cd[G::SRC == 1 ? NPT : 1];
    int sub[G::SRC == 1 ? NPT : 1];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int f = tid + 256 * (base + i);
      const int pix = f / Q, cq = f - pix * Q;
      const int ry = pix / G::WS, x = pix - ry * G::WS;
      const int y = y0 + ry;
      if constexpr (G::SRC == 0) {
        v[i] = f < nvec ? *reinterpret_cast<const float4*>(
                              a.src + ((size_t)(img * G::HS + y) * G::WS + x) * G::CIN + cq * 4)
                        : f4zero();
      } else {
        const int uy = y - G::PADY, ux = x - G::PADX;   // position in the un-pooled map
        sub[i] = -1;
        v[i] = f4zero();
        cd[i] = 0;
        if (f < nvec && uy >= 0 && uy < G::UHO && ux >= 0 && ux < G::UWO) {
          const int pidx = img * (G::UPH * G::UPW) + (uy >> 1) * G::UPW + (ux >> 1);
          v[i] = *reinterpret_cast<const float4*>(a.src + (size_t)pidx * G::CIN + cq * 4);
          cd[i] = *reinterpret_cast<const uint32_t*>(a.code + (size_t)pidx * G::CIN + cq * 4);
          sub[i] = ((uy & 1) << 1) | (ux & 1);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int f = tid + 256 * (base + i);
      if (f < nvec) {
        const int pix = f / Q, cq = f - pix * Q;
        float4 x = v[i];
        if constexpr (G::SRC == 1) {
          const uint32_t s = (uint32_t)sub[i], c = cd[i];
          x.x = ((c & 255u) == s) ? x.x : 0.f;
          x.y = (((c >> 8) & 255u) == s) ? x.y : 0.f;
          x.z = (((c >> 16) & 255u) == s) ? x.z : 0.f;
          x.w = ((c >> 24) == s) ? x.w : 0.f;
        }
        band4[pix * (G::CPITCH / 4) + cq] = x;
      }
    }
    }
  }
  __syncthreads();

  const int nb = wave % G::NB;
  const int mb0 = wave / G::NB;
  const int li = lane & 15, lq = lane >> 4;
  // per-m-block LDS base (in floats) of this lane's A row, and row validity
  int abase[G::MBW];
#pragma unroll
  for (int j = 0; j < G::MBW; ++j) {
    const int mb = mb0 + j * G::WPN;
    const int row = mb * 16 + li;
    int oy, ox;
    if constexpr (G::POOL) {
      const int w = row >> 2, sub = row & 3;
      const int ph = w / (G::WO / 2), pw = w - ph * (G::WO / 2);
      oy = 2 * ph + (sub >> 1);
      ox = 2 * pw + (sub & 1);
    } else {
      oy = row / G::WO;
      ox = row - oy * G::WO;
    }
    const bool ok = mb < G::MB && row < G::MROWS && oy < rows_out;
    abase[j] = (ok ? (oy * G::WS + ox) * G::CPITCH + lq * 4 : lq * 4) / 4;   // float4 units
  }

  f32x4 acc[G::MBW];
#pragma unroll
  for (int j = 0; j < G::MBW; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const float* wrow = a.wt + (size_t)(nb * 16 + li) * G::KDIM + lq * 4;
  // Every tap (kh, kw, 16-channel chunk) fully unrolled: the A reads are ds_read_b128 with
  // immediate offsets from one per-m-block base register; the B fragment of tap t + LA is
  // loaded (global, L2-resident) while tap t computes, through a ring of LA + 1 registers.
  constexpr int NT = G::KH * G::KW * G::KCH;
  constexpr int LA = 3;
  float4 bring[LA + 1];
#pragma unroll
  for (int t = 0; t < LA && t < NT; ++t) bring[t] = *reinterpret_cast<const float4*>(wrow + t * 16);
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    if (t + LA < NT) bring[(t + LA) % (LA + 1)] = *reinterpret_cast<const float4*>(wrow + (t + LA) * 16);
    const float4 b = bring[t % (LA + 1)];
    const int kh = t / (G::KW * G::KCH), kw = (t / G::KCH) % G::KW, ch = t % G::KCH;
    const int toff = (kh * G::WS + kw) * G::CPITCH + ch * 16;
    // all A fragments of the tap first, then the 4 k-steps interleaved across m-blocks so
    // consecutive MFMAs never depend on each other (16x16x4 f32: 32-cycle issue, 40 latency)
    float4 av[G::MBW];
#pragma unroll
    for (int j = 0; j < G::MBW; ++j) av[j] = band4[abase[j] + toff / 4];
#pragma unroll
    for (int j = 0; j < G::MBW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].x, b.x, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < G::MBW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].y, b.y, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < G::MBW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].z, b.z, acc[j], 0, 0, 0);
#pragma unroll
    for (int j = 0; j < G::MBW; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].w, b.w, acc[j], 0, 0, 0);
  }

  // ---- epilogue: C layout of 16x16x4: lane holds column (lane & 15), rows 4*(lane>>4)+r ----
  const int col = nb * 16 + li;
  unsigned long long pos = 0;
#pragma unroll
  for (int j = 0; j < G::MBW; ++j) {
    const int mb = mb0 + j * G::WPN;
    if (mb >= G::MB) continue;
    if constexpr (G::POOL) {
      const int w = mb * 4 + lq;                    // window of this lane's 4 rows
      const int ph = w / (G::WO / 2), pw = w - ph * (G::WO / 2);
      const float v0 = acc[j][0], v1 = acc[j][1], v2 = acc[j][2], v3 = acc[j][3];
      if (w * 4 < G::MROWS && 2 * ph < rows_out) {
        pos += (v0 > 0.f) + (v1 > 0.f) + (v2 > 0.f) + (v3 > 0.f);
        float mx = v0;
        uint32_t arg = 0;
        if (v1 > mx) { mx = v1; arg = 1; }
        if (v2 > mx) { mx = v2; arg = 2; }
        if (v3 > mx) { mx = v3; arg = 3; }
        const size_t o = ((size_t)(img * (G::HO / 2) + y0 / 2 + ph) * (G::WO / 2) + pw) * G::COUT + col;
        a.out[o] = fmaxf(mx, 0.f);
        if (a.out_code) a.out_code[o] = mx > 0.f ? (uint8_t)arg : (uint8_t)255;
      }
    } else {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = mb * 16 + lq * 4 + r;
        const int oy = row / G::WO, ox = row - oy * G::WO;
        if (row < G::MROWS && oy < rows_out)
          a.out[((size_t)(img * G::HO + y0 + oy) * G::WO + ox) * G::COUT + col] = acc[j][r];
      }
    }
  }
  if (G::POOL && a.relu_count) relu_count_add(a.relu_count, pos, lane);
}

// ---------------------------------------------------------------------------------------
// conv0 forward (train.py:167-185): uint8 frames [B,84,84,4] -> ReLU -> 2x2 max-pool.
// The band (RB0 + 4 input rows) is staged as x = u8 / 255.0f (exactly train.py:167), one
// float4 (the 4 frame channels) per pixel.  K = 25 taps x 4 channels is consumed in 7 groups
// of 4 taps (taps 25..27 have zero weights); in group g, MFMA step t and lane group q cover
// tap 4g + q, channel t, so one ds_read_b128 of a pixel feeds a lane's 4 steps.  All 112 K
// values of the wave's 16 output channels stay in 28 registers for the whole band.
// ---------------------------------------------------------------------------------------
struct Conv0Geom {
  static constexpr int HS = 84, WS = 84, C = 4, COUT = 32, KT = 5, NTAP = 25;
  static constexpr int HO = 80, WO = 80, RB = 8, NBANDS = HO / RB, SROWS = RB + KT - 1;
  static constexpr int NTG = 7;                             // tap groups of 4
  static constexpr int KDIM = NTG * 16;                     // 112 (zero-padded K)
  static constexpr int MROWS = (RB / 2) * (WO / 2) * 4;     // 640 rows = 160 windows
  static constexpr int MB = MROWS / 16;                     // 40 m-blocks
  static constexpr int MBW = MB / 2;                        // 20 per wave (2 waves per n-block)
  static constexpr int MCH = 10;                            // m-blocks per register chunk
};

#if BA3C_SHARED_KERNELS  // non-template kernel: emitted by ba3c_capi.hip only
__global__ void __launch_bounds__(256) conv0_band_kernel(const BandArgs a) {
  using G = Conv0Geom;
  __shared__ float4 xs4[G::SROWS * G::WS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int img = blockIdx.x / G::NBANDS;
  const int y0 = (blockIdx.x - img * G::NBANDS) * G::RB;
  const uint8_t* src = reinterpret_cast<const uint8_t*>(a.src);
  {
    constexpr int NV = G::SROWS * G::WS;                    // 1008 pixels
    constexpr int NPT = (NV + 255) / 256;
    uint32_t v[NPT];
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int f = tid + 256 * i;
      v[i] = f < NV ? *reinterpret_cast<const uint32_t*>(src + ((size_t)img * G::HS * G::WS + (size_t)y0 * G::WS + f) * G::C) : 0u;
    }
#pragma unroll
    for (int i = 0; i < NPT; ++i) {
      const int f = tid + 256 * i;
      if (f < NV)
        xs4[f] = make_float4((float)(v[i] & 255u) / 255.0f, (float)((v[i] >> 8) & 255u) / 255.0f,
                             (float)((v[i] >> 16) & 255u) / 255.0f, (float)(v[i] >> 24) / 255.0f);
    }
  }
  const int nb = wave & 1, mb0 = wave >> 1;
  const int li = lane & 15, lq = lane >> 4;
  // weights of output channel nb*16+li for this lane's taps 4g+lq, channels 0..3
  float4 b[G::NTG];
  const float* wrow = a.wt + (size_t)(nb * 16 + li) * G::KDIM + lq * 4;
#pragma unroll
  for (int g = 0; g < G::NTG; ++g) b[g] = *reinterpret_cast<const float4*>(wrow + g * 16);
  int toff[G::NTG];                                         // this lane's tap offset per group
#pragma unroll
  for (int g = 0; g < G::NTG; ++g) {
    const int tap = 4 * g + lq;
    toff[g] = tap < G::NTAP ? (tap / G::KT) * G::WS + tap % G::KT : 0;
  }
  __syncthreads();

  unsigned long long pos = 0;
#pragma unroll
  for (int ch = 0; ch < G::MBW / G::MCH; ++ch) {
    int pbase[G::MCH];
#pragma unroll
    for (int j = 0; j < G::MCH; ++j) {
      const int mb = mb0 + 2 * (ch * G::MCH + j);
      const int row = mb * 16 + li;
      const int w = row >> 2, sub = row & 3;
      const int ph = w / (G::WO / 2), pw = w - ph * (G::WO / 2);
      pbase[j] = (2 * ph + (sub >> 1)) * G::WS + 2 * pw + (sub & 1);
    }
    f32x4 acc[G::MCH];
#pragma unroll
    for (int j = 0; j < G::MCH; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int g = 0; g < G::NTG; ++g) {
      float4 av[G::MCH];
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) av[j] = xs4[pbase[j] + toff[g]];
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].x, b[g].x, acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].y, b[g].y, acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].z, b[g].z, acc[j], 0, 0, 0);
#pragma unroll
      for (int j = 0; j < G::MCH; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j].w, b[g].w, acc[j], 0, 0, 0);
    }
    // pool epilogue: lane holds the 4 subs of window 4*mb + lq, channel nb*16 + li
    const int col = nb * 16 + li;
#pragma unroll
    for (int j = 0; j < G::MCH; ++j) {
      const int mb = mb0 + 2 * (ch * G::MCH + j);
      const int w = mb * 4 + lq;
      const int ph = w / (G::WO / 2), pw = w - ph * (G::WO / 2);
      const float v0 = acc[j][0], v1 = acc[j][1], v2 = acc[j][2], v3 = acc[j][3];
      pos += (v0 > 0.f) + (v1 > 0.f) + (v2 > 0.f) + (v3 > 0.f);
      float mx = v0;
      uint32_t arg = 0;
      if (v1 > mx) { mx = v1; arg = 1; }
      if (v2 > mx) { mx = v2; arg = 2; }
      if (v3 > mx) { mx = v3; arg = 3; }
      const size_t o = ((size_t)(img * (G::HO / 2) + y0 / 2 + ph) * (G::WO / 2) + pw) * G::COUT + col;
      a.out[o] = fmaxf(mx, 0.f);
      if (a.out_code) a.out_code[o] = mx > 0.f ? (uint8_t)arg : (uint8_t)255;
    }
  }
  if (a.relu_count) relu_count_add(a.relu_count, pos, lane);
}
#endif

// conv0 weights as [32][112]: k = (tap, c) for taps < 25 of the real channels, zero beyond
#if BA3C_SHARED_KERNELS  // non-template kernel: emitted by ba3c_capi.hip only
__global__ void __launch_bounds__(256) conv0_wprep_kernel(const float* __restrict__ w,
                                                          float* __restrict__ wt) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= 32 * Conv0Geom::KDIM) return;
  const int o = e / Conv0Geom::KDIM, k = e - o * Conv0Geom::KDIM;
  const int tap = k >> 2, c = k & 3;
  // conv0/W is [5,5,16,32] (TARGET_CHANNELS = 16, train.py:99); real channels c < 4
  wt[e] = tap < Conv0Geom::NTAP ? w[((size_t)tap * 16 + c) * 32 + o] : 0.f;
}
#endif

// ---------------------------------------------------------------------------------------
// Per-step weight preparation: B operand of a band conv as [N][K] with K = (kh, kw, c).
//   forward:  wt[o][(kh,kw,c)]  = W[kh, kw, c, o]                         (W: [KH,KW,CI,CO])
//   dgrad:    wt[ci][(a,b,o)]   = W[KH-1-a, KW-1-b, ci, o]
// ---------------------------------------------------------------------------------------
struct WPrepJob {
  const float* w;
  float* wt;
  int KH, KW, CI, CO, dgrad, n;   // n = total elements
};
struct WPrepArgs {
  WPrepJob job[4];
  int njobs;
};

// element e of job j's [N][K] copy (forward: [CO][KH*KW*CI]; dgrad: rotated [CI][KH*KW*CO])
__device__ __forceinline__ float wprep_value(const WPrepJob& j, int e) {
  if (!j.dgrad) {
    const int K = j.KH * j.KW * j.CI;
    const int o = e / K, k = e - o * K;            // k = (kh*KW+kw)*CI + c
    return j.w[(size_t)k * j.CO + o];
  }
  const int K = j.KH * j.KW * j.CO;
  const int ci = e / K, k = e - ci * K;            // k = (a*KW+b)*CO + o
  const int ab = k / j.CO, o = k - ab * j.CO;
  const int aa = ab / j.KW, bb = ab - aa * j.KW;
  const int kh = j.KH - 1 - aa, kw = j.KW - 1 - bb;
  return j.w[((size_t)(kh * j.KW + kw) * j.CI + ci) * j.CO + o];
}

#if BA3C_SHARED_KERNELS  // non-template kernel: emitted by ba3c_capi.hip only
__global__ void __launch_bounds__(256) wprep_kernel(const WPrepArgs a) {
  const WPrepJob& j = a.job[blockIdx.y];
  for (int e = blockIdx.x * 256 + threadIdx.x; e < j.n; e += gridDim.x * 256) j.wt[e] = wprep_value(j, e);
}
#endif

}  // namespace ba3c
