// ba3c_wgrad.h — weight gradients of the pooled convs (Conv2DBackpropFilter of conv0/1/2,
// train.py:177-204 differentiated by TF autodiff, train/multigpu.py:85-86) as a persistent
// band kernel on fp32 MFMA 16x16x4.
//
//   dW[kh,kw,c,o] = sum_{n,y,x} X[n, y+kh, x+kw, c] * dY[n, y, x, o]
//
// A persistent workgroup walks bands (image n, RB output rows).  Per band it stages into LDS
// the input rows the band touches (X; conv0's uint8 frames become x = u8/255 exactly as
// train.py:167) and the un-pooled output gradient (dY from dP + argmax codes, ReLU gradient
// folded in) at the same row pitch WS, so a pixel p = y*WS + x addresses both with the same
// affine offset and every LDS read in the MFMA loop has a compile-time immediate offset.
// The columns x >= WO of dY are zero (their MFMAs are wasted, WS/WO - 1 = 5-29 %).
// The reduction index k runs over 16-pixel groups; MFMA step s, lane group q covers pixel
// 16*(s/4) + s%4 + 4q, which puts the two 16-lane halves of a 32-lane LDS access 4 pixels
// apart: with a pixel pitch of CIN + 4 floats that is 16 banks apart (conflict-free).
// Accumulators stay in registers across all bands; each workgroup writes one fp32 partial
// slab at the end, reduced deterministically by wgrad_reduce_kernel.
#pragma once
#include "ba3c_conv.h"

namespace ba3c {

template <int HS_, int WS_, int CIN_, int KH_, int KW_, int COUT_, int RB_, bool U8_, int NSPLIT_>
struct WgGeom {
  static constexpr int HS = HS_, WS = WS_, CIN = CIN_, KH = KH_, KW = KW_, COUT = COUT_;
  static constexpr int RB = RB_, NSPLIT = NSPLIT_;
  static constexpr bool U8 = U8_;
  static constexpr int HO = HS - KH + 1, WO = WS - KW + 1, PH = HO / 2, PW = WO / 2;
  static constexpr int NBANDS = (HO + RB - 1) / RB;
  static constexpr int KB = ((RB * WS + 15) / 16) * 16;   // pixels (reduction length) per band
  static constexpr int XROWS = RB + KH;                   // +1 zero row covers the K padding
  static constexpr int CPX = U8 ? CIN : CIN + 4;          // X pixel pitch (floats)
  static constexpr int CPY = 36;                          // dY pixel pitch: 32 channels + 4
  static constexpr int X_F4 = XROWS * WS * CPX / 4;
  static constexpr int Y_F4 = KB * CPY / 4;
  static constexpr int NT = KH * KW;
  static constexpr int M = NT * CIN;                      // rows of dW (tap, c)
  // units per wave: conv1/conv2 -> one M-block per tap at channel half (wave >> 1);
  // conv0 (CIN = 4) -> M-blocks of 4 taps x 4 channels, (wave >> 1) + 2j
  static constexpr int MB_U8 = (M + 15) / 16;
  static constexpr int UPW = U8 ? (MB_U8 + 1) / 2 : NT;
  static_assert(U8 ? CIN == 4 : CIN == 32, "wgrad band geometry");
  static_assert((COUT / NSPLIT) == 32, "32 output channels per workgroup");
  static_assert(CPX % 4 == 0 && (4 * CPX) % 32 == 16, "conflict-free pixel pitch");
};

struct WgArgs {
  const void* x;          // X [B,HS,WS,CIN] (u8 frames for conv0, fp32 pooled map otherwise)
  const float* dp;        // dP [B,PH,PW,COUT] (grad of the max-pool output)
  const uint8_t* code;    // argmax codes of dP (255 = no gradient)
  float* part;            // [gridDim.x][M][COUT] partial slabs
  int batch;
};

template <class G>
__global__ void __launch_bounds__(256) wgrad_band_kernel(const WgArgs a) {
  __shared__ float4 xs4[G::X_F4];
  __shared__ float4 ys4[G::Y_F4];
  const float* xs = reinterpret_cast<const float*>(xs4);
  const float* ys = reinterpret_cast<const float*>(ys4);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int li = lane & 15, lq = lane >> 4;
  const int nb = wave & 1, half = wave >> 1;
  const int o0 = blockIdx.y * 32;                         // this workgroup's output channels

  // per-lane LDS bases (floats); MFMA step offsets are compile-time immediates
  int xbase[G::U8 ? G::UPW : 1];
  if constexpr (G::U8) {
#pragma unroll
    for (int j = 0; j < G::UPW; ++j) {
      const int mb = half + 2 * j;
      int tap = 4 * mb + (li >> 2);
      if (tap >= G::NT) tap = 0;                          // padded rows: discarded
      const int toff = (tap / G::KW) * G::WS + tap % G::KW;
      xbase[j] = (4 * lq + toff) * G::CPX + (li & 3);
    }
  } else {
    xbase[0] = 4 * lq * G::CPX + half * 16 + li;
  }
  const int ybase = 4 * lq * G::CPY + nb * 16 + li;

  f32x4 acc[G::UPW];
#pragma unroll
  for (int u = 0; u < G::UPW; ++u) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nbands = a.batch * G::NBANDS;
  for (int band = blockIdx.x; band < nbands; band += gridDim.x) {
    const int img = band / G::NBANDS;
    const int y0 = (band - img * G::NBANDS) * G::RB;
    const int rows_out = min(G::RB, G::HO - y0);
    __syncthreads();                                      // previous band's reads are done
    // ---- stage X rows [y0, y0 + XROWS) (zero beyond the map) ----
    {
      constexpr int Q = G::CPX / 4;                       // float4 per staged pixel
      constexpr int NV = G::XROWS * G::WS * Q;
      constexpr int NTOT = (NV + 255) / 256;
      constexpr int NPT = NTOT < 8 ? NTOT : 8;            // loads in flight per chunk
      for (int c0 = 0; c0 < NTOT; c0 += NPT) {
      float4 v[NPT];
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int f = tid + 256 * (c0 + i);
        const int pix = f / Q, cq = f - pix * Q;
        const int ry = pix / G::WS, x = pix - ry * G::WS;
        const int y = y0 + ry;
        v[i] = f4zero();
        if (f < NV && y < G::HS) {
          if constexpr (G::U8) {
            const uint32_t w = *reinterpret_cast<const uint32_t*>(
                static_cast<const uint8_t*>(a.x) + ((size_t)(img * G::HS + y) * G::WS + x) * G::CIN);
            v[i] = make_float4((float)(w & 255u) / 255.0f, (float)((w >> 8) & 255u) / 255.0f,
                               (float)((w >> 16) & 255u) / 255.0f, (float)(w >> 24) / 255.0f);
          } else {
            v[i] = *reinterpret_cast<const float4*>(
                static_cast<const float*>(a.x) + ((size_t)(img * G::HS + y) * G::WS + x) * G::CIN + cq * 4);
          }
        }
      }
#pragma unroll
      for (int i = 0; i < NPT; ++i) {
        const int f = tid + 256 * (c0 + i);
        if (f < NV) {
          const int pix = f / Q, cq = f - pix * Q;
          xs4[pix * (G::CPX / 4) + cq] = v[i];
        }
      }
      }
    }
    // ---- stage dY (un-pooled) for pixels p in [0, KB) of the band, channels o0..o0+31 ----
    {
      constexpr int NV = G::KB * 8;                       // 8 float4 per pixel
      constexpr int NPT = (NV + 255) / 256;
      constexpr int CH = NPT < 8 ? NPT : 8;
      for (int c0 = 0; c0 < NPT; c0 += CH) {
        float4 v[CH];
        uint32_t cd[CH];
        int sub[CH];
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int f = tid + 256 * (c0 + i);
          const int pix = f >> 3, cq = f & 7;
          const int ry = pix / G::WS, x = pix - ry * G::WS;
          v[i] = f4zero();
          cd[i] = 0;
          sub[i] = -1;
          if (f < NV && ry < rows_out && x < G::WO) {
            const int y = y0 + ry;
            const int pidx = (img * G::PH + (y >> 1)) * G::PW + (x >> 1);
            v[i] = *reinterpret_cast<const float4*>(a.dp + (size_t)pidx * G::COUT + o0 + cq * 4);
            cd[i] = *reinterpret_cast<const uint32_t*>(a.code + (size_t)pidx * G::COUT + o0 + cq * 4);
            sub[i] = ((y & 1) << 1) | (x & 1);
          }
        }
#pragma unroll
        for (int i = 0; i < CH; ++i) {
          const int f = tid + 256 * (c0 + i);
          if (f < NV) {
            const int pix = f >> 3, cq = f & 7;
            const uint32_t s = (uint32_t)sub[i], c = cd[i];
            float4 g = v[i];
            g.x = ((c & 255u) == s) ? g.x : 0.f;
            g.y = (((c >> 8) & 255u) == s) ? g.y : 0.f;
            g.z = (((c >> 16) & 255u) == s) ? g.z : 0.f;
            g.w = ((c >> 24) == s) ? g.w : 0.f;
            ys4[pix * (G::CPY / 4) + cq] = g;
          }
        }
      }
    }
    __syncthreads();
    // ---- MFMA over the band's pixels: runtime loop over 16-pixel groups, 4 steps unrolled ----
#pragma unroll 1
    for (int g = 0; g < G::KB / 16; ++g) {
      const int gp = 16 * g;
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        const int pix = gp + t;                           // + 4q via the lane base
        const float b = ys[ybase + pix * G::CPY];
        if constexpr (G::U8) {
#pragma unroll
          for (int u = 0; u < G::UPW; ++u) {
            const float av = xs[xbase[u] + pix * G::CPX];
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b, acc[u], 0, 0, 0);
          }
        } else {
          float av[G::UPW];
#pragma unroll
          for (int u = 0; u < G::UPW; ++u) {
            const int toff = (u / G::KW) * G::WS + (u % G::KW);
            av[u] = xs[xbase[0] + (pix + toff) * G::CPX];
          }
#pragma unroll
          for (int u = 0; u < G::UPW; ++u)
            acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], b, acc[u], 0, 0, 0);
        }
      }
    }
  }

  // ---- epilogue: partial slab z = blockIdx.x; lane (col li, rows 4*lq + r) ----
  float* pz = a.part + (size_t)blockIdx.x * G::M * G::COUT;
  const int n = o0 + nb * 16 + li;
#pragma unroll
  for (int u = 0; u < G::UPW; ++u) {
    int mrow0;
    if constexpr (G::U8) {
      const int mb = half + 2 * u;
      mrow0 = 16 * mb + 4 * lq;
    } else {
      mrow0 = u * G::CIN + half * 16 + 4 * lq;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = mrow0 + r;
      if (m < G::M) pz[(size_t)m * G::COUT + n] = acc[u][r];
    }
  }
}

}  // namespace ba3c
