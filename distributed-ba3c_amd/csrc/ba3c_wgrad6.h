// ba3c_wgrad6.h — weight gradients of conv1/conv2 (Conv2DBackpropFilter, train.py:187-204
// under TF autodiff, train/multigpu.py:85-86) on bf16 MFMA with fp32-accurate splitting.
//
//   dW[kh,kw,c,o] = sum_{n,y,x} X[n, y+kh, x+kw, c] * dY[n, y, x, o]
//
// GEMM view: M = (tap, c), N = o, K = output pixels.  X and dY are fp32; each is split into
// three bf16 planes (hi + mid + lo == value exactly, split3x2) and the six significant
// cross products (a1b1, a1b2, a2b1, a1b3, a2b2, a3b1) run on v_mfma_f32_16x16x32_bf16 with
// fp32 accumulation (dropped terms < 2^-23 relative: fp32 accuracy, see ba3c_band6.h).
//
// Persistent workgroups walk bands (image, RB output rows); blockIdx.y selects a group of
// CW input channels x OW output channels, so one workgroup's LDS holds
//   X  [XROWS][WS][split][CW]  bf16, pixel pitch PX bytes  (the band's input rows + 4)
//   dY [KPAD][split][OW]       bf16, pixel pitch PY bytes  (un-pooled: dP routed to each
//                                                         window's argmax, ReLU folded in)
// with dY's pixels compacted (p = y*WO + x: no MFMA spent on the WS - WO dead columns) and
// zero-padded to a multiple of 32.  Both operands have K = pixels on the LDS row axis, so
// they are read with ds_read_b64_tr_b16 (hardware transpose: 4 pixel rows x 16 channel
// columns per 16-lane group).  Within a k-step the 32 pixels are permuted so the 8 rows a
// 32-lane half reads are consecutive pixels: with PX = 3*32 and PY = 7*32 bytes those land
// in 8 distinct 32-byte bank slots (conflict-free except where a run wraps a row of X).
// Each lane's address is per k-step (compacted pixel -> (y, x)); the tap offset is an
// immediate.  Accumulators stay in registers across all bands; one fp32 partial slab per
// workgroup, reduced deterministically by wgrad_reduce_kernel.
#pragma once
#include "ba3c_split.h"

namespace ba3c {

typedef short i16x4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 lds_tr16(const char* p) {
  const i16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) i16x4*)(p));
  return __builtin_bit_cast(uint2, v);
}

// packed 16-bit halves: 0xFFFF where the half is zero, else 0
__device__ __forceinline__ uint32_t w6_mask16_eq0(uint32_t d) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  u16x2 x = __builtin_bit_cast(u16x2, d);
  x = __builtin_elementwise_min(x, (u16x2){1, 1});
  x = x + (u16x2){0xFFFF, 0xFFFF};
  return __builtin_bit_cast(uint32_t, x);
}

template <int HS_, int WS_, int CIN_, int COUT_, int RB_, int CW_, int OW_, int PX_, int PY_, int NS_ = 3>
struct Wg6Geom {
  static constexpr int NS = NS_;                          // split planes (3 bf16 / 2 fp16)
  static constexpr int HS = HS_, WS = WS_, CIN = CIN_, COUT = COUT_, RB = RB_, CW = CW_, OW = OW_;
  static constexpr int KH = 5, KW = 5, NTAP = 25;
  static constexpr int HO = HS - KH + 1, WO = WS - KW + 1, PH = HO / 2, PW = WO / 2;
  static constexpr int NBANDS = (HO + RB - 1) / RB;
  static constexpr int KP = RB * WO;                      // output pixels of a full band
  static constexpr int KS = (KP + 31) / 32, KPAD = 32 * KS;
  static constexpr int XROWS = RB + KH - 1;
  // RING: a workgroup that walks the bands of whole images keeps the 4 halo rows of band i as
  // the first rows of band i + 1 and loads only RB new rows per band (halves X's HBM reads).
  // Row groups of RB rows live in three LDS slots: group g in slot g & 1 and, for even g, also
  // in slot 2, so the two groups (i, i + 1) a band reads are always contiguous from slot i & 1.
  static constexpr bool RING = NBANDS > 1 && XROWS == 2 * RB;
  static constexpr int XSLOTROWS = RING ? 3 * RB : XROWS;
  static constexpr int PX = PX_, PY = PY_;                // pixel pitches (bytes)
  static constexpr int XSB = 2 * CW, YSB = 2 * OW;        // bytes per split
  static constexpr int X_BYTES = XSLOTROWS * WS * PX, Y_BYTES = KPAD * PY;
  static constexpr int NCG = CIN / CW, NOG = COUT / OW;
  static constexpr int TBASE = NTAP / 4, TREM = NTAP % 4;  // taps per wave: 7, 6, 6, 6
  static constexpr int TW = TBASE + (TREM > 0);
  static constexpr int M = NTAP * CIN;
  static_assert(CW == 16 && OW == 32, "16 input x 32 output channels per workgroup");
  static_assert(PX >= NS * XSB && PY >= NS * YSB && PX % 8 == 0 && PY % 8 == 0, "pitches");
  static_assert(X_BYTES % 16 == 0 && RB % 2 == 0, "wgrad6 geometry");
};

struct Wg6Args {
  const float* x;          // X [B,HS,WS,CIN] pooled fp32 map
  const float* dp;         // dP [B,PH,PW,COUT]
  const uint8_t* code;     // argmax codes of dP (255 = no gradient)
  float* part;             // [gridDim.x][M][COUT] partial slabs
  int batch;
  const uint32_t* amax_x;  // NS = 2: per-image max |X| slots
  const uint32_t* amax_dp; // NS = 2: per-image max |dP| slots
};

// bx / by / gx: the workgroup's band start, channel group and the persistent stride (blockIdx.x,
// blockIdx.y, gridDim.x of a plain launch; ba3c_multi.h passes its own); xs: X_BYTES + Y_BYTES
// of LDS, red4: 4 words of LDS scratch.
template <class G>
__device__ __forceinline__ void wgrad6_body(const Wg6Args& a, int bx, int by, int gx, char* xs, uint32_t* red4) {
  using SP = SplitP<G::NS>;
  // NS = 2: both operands scaled by their whole tensor's max (the sum runs over images)
  const int kx = G::NS == 2 ? amax_exp(amax_all(a.amax_x, a.batch, red4)) : 0;
  const int ky = G::NS == 2 ? amax_exp(amax_all(a.amax_dp, a.batch, red4)) : 0;
  const float xsc = exp2i(kx), ysc = exp2i(ky);
  char* ys = xs + G::X_BYTES;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int cg = by / G::NOG, og = by - cg * G::NOG;
  const int c0 = cg * G::CW, o0 = og * G::OW;
  // wave w owns a contiguous run of taps and both 16-column n-blocks, so every X fragment it
  // reads from LDS feeds two MFMA chains (LDS reads per MFMA 1.08 -> 0.64)
  const int tap0 = wave * G::TBASE + min(wave, G::TREM);
  const int ntap = G::TBASE + (wave < G::TREM);

  // tr-read lane roles: group g = lane >> 4, row q, column quad p
  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  const int kperm = 16 * (g >> 1) + 4 * (g & 1) + q;      // + 8 r for read r

  f32x4 acc[G::TW][2];
#pragma unroll
  for (int t = 0; t < G::TW; ++t) acc[t][0] = acc[t][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  // ---- staging work per thread ----
  constexpr int XQ = G::CW / 4;                           // float4 per X pixel (4)
  constexpr int XN = G::XROWS * G::WS * XQ;
  constexpr int XPT = (XN + 255) / 256;
  constexpr int YQ = G::OW / 4;                           // float4 per dY pixel (8)
  // UNP (BA3C_W6_UNPOOL, default): dY staged per POOLED element — each (pooled pixel, 4
  // channels) of dP is loaded and split once and written to the four pixels of its window
  // under per-channel code masks (as wgrad6s / band6r_up): a quarter of the loads and splits,
  // and 5 float4 + 5 code registers per thread fewer held through the k-loop (conv2's pair
  // launch spilled 20 B/lane at 256 VGPRs).  The staged LDS image is the per-pixel one bit for
  // bit (a masked split of v is the split of the masked v; the padded pixels KP .. KPAD - 1 are
  // zeroed once and never written again)
#ifndef BA3C_W6_UNPOOL
#define BA3C_W6_UNPOOL 1
#endif
  constexpr bool UNP = BA3C_W6_UNPOOL && G::HO % G::RB == 0 && G::RB % 2 == 0;
  constexpr int YN = UNP ? (G::RB / 2) * G::PW * YQ : G::KPAD * YQ;
  constexpr int YPT = (YN + 255) / 256;
  float4 xv[XPT], yv[YPT];
  uint32_t yc[YPT];                                       // (un-loaded: dY is zero)
  if constexpr (UNP) {
    for (int i = tid; i < (G::KPAD - G::KP) * G::PY / 16; i += 256)
      reinterpret_cast<uint4*>(ys + G::KP * G::PY)[i] = make_uint4(0, 0, 0, 0);
  }

  const int nbands = a.batch * G::NBANDS;
  // band walk: whole images per workgroup (ring reuse of the halo rows) when the images split
  // evenly over the workgroups (or nearly: >= 8 each), else bands bx, bx + gx, ... (balanced
  // at any batch)
  const bool ring = G::RING && a.batch >= gx && (a.batch % gx == 0 || a.batch >= 8 * gx);
  int band_end = nbands;
  int band = bx;
  if (ring) {
    const int ipw = (a.batch + gx - 1) / gx;
    band = min(a.batch, bx * ipw) * G::NBANDS;
    band_end = min(a.batch, (bx + 1) * ipw) * G::NBANDS;
  }
  const int bstep = ring ? 1 : gx;
  // rows [r0, XROWS) of the band's input window: all of them, or (ring, not the image's first
  // band) only the RB rows that are new
  int xr0 = 0;
  auto load_band = [&](int band) {
    const int img = band / G::NBANDS;
    const int bi = band - img * G::NBANDS;
    const int y0 = bi * G::RB;
    const int rows_out = min(G::RB, G::HO - y0);
    xr0 = (ring && bi > 0) ? G::RB : 0;
    const int xn = (G::XROWS - xr0) * G::WS * XQ;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int f = tid + 256 * i;
      const int pix = f / XQ, cq = f - pix * XQ;
      const int ry = xr0 + pix / G::WS, x = pix - (pix / G::WS) * G::WS;
      const int y = y0 + ry;
      // branch-free (ld4 reads zeros for a rejected element): a load in a branch made the
      // compiler wait for every outstanding load at the join, serialising the prefetch
      const bool ok = f < xn && y < G::HS;
      xv[i] = ld4(a.x + (ok ? ((size_t)(img * G::HS + y) * G::WS + x) * G::CIN + c0 + cq * 4 : 0), ok);
    }
    if constexpr (UNP) {
#pragma unroll
      for (int i = 0; i < YPT; ++i) {
        const int f = tid + 256 * i;
        const int oq = f % YQ, rest = f / YQ;
        const int pc = rest % G::PW, py = (y0 >> 1) + rest / G::PW;
        const bool ok = f < YN;
        const size_t e = ok ? ((size_t)(img * G::PH + py) * G::PW + pc) * G::COUT + o0 + oq * 4 : 0;
        yv[i] = ld4(a.dp + e, ok);
        yc[i] = ld_u8x4(a.code + e, ok);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + 256 * i;
      const int p = f / YQ, oq = f - p * YQ;
      const int ry = p / G::WO, x = p - ry * G::WO;
      const bool ok = f < YN && ry < rows_out;
      const size_t e = ok ? ((size_t)(img * G::PH + ((y0 + ry) >> 1)) * G::PW + (x >> 1)) * G::COUT + o0 + oq * 4 : 0;
      yv[i] = ld4(a.dp + e, ok);
      yc[i] = ld_u8x4(a.code + e, ok);
    }
  };
  auto store_band = [&](int band) {
    const int bi = band - (band / G::NBANDS) * G::NBANDS;
    const int y0 = bi * G::RB;
    const int xn = (G::XROWS - xr0) * G::WS * XQ;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int f = tid + 256 * i;
      if (f < xn) {
        const int pix = f / XQ, cq = f - pix * XQ;
        const int ry = xr0 + pix / G::WS, x = pix - (pix / G::WS) * G::WS;
        uint32_t s0[G::NS], s1[G::NS];
        SP::split(xv[i].x, xv[i].y, xsc, s0);
        SP::split(xv[i].z, xv[i].w, xsc, s1);
        // window row ry of band bi is row ry % RB of group bi + ry / RB
        const int g = bi + ry / G::RB, rr = ry - (ry / G::RB) * G::RB;
        const int prow = ring ? (g & 1) * G::RB + rr : ry;
        char* p = xs + (prow * G::WS + x) * G::PX + cq * 8;
#pragma unroll
        for (int sp = 0; sp < G::NS; ++sp)
          *reinterpret_cast<uint2*>(p + sp * G::XSB) = make_uint2(s0[sp], s1[sp]);
        if (ring && (g & 1) == 0) {                       // even groups also in slot 2
          char* q = p + 2 * G::RB * G::WS * G::PX;
#pragma unroll
          for (int sp = 0; sp < G::NS; ++sp)
            *reinterpret_cast<uint2*>(q + sp * G::XSB) = make_uint2(s0[sp], s1[sp]);
        }
      }
    }
    if constexpr (UNP) {
#pragma unroll
      for (int i = 0; i < YPT; ++i) {
        const int f = tid + 256 * i;
        if (f < YN) {
          const int oq = f % YQ, rest = f / YQ;
          const int pc = rest % G::PW, pr = rest / G::PW;
          uint32_t s0[G::NS], s1[G::NS];
          SP::split(yv[i].x, yv[i].y, ysc, s0);
          SP::split(yv[i].z, yv[i].w, ysc, s1);
          const uint32_t c01 = __builtin_amdgcn_perm(yc[i], yc[i], 0x0C010C00u);   // codes as halves
          const uint32_t c23 = __builtin_amdgcn_perm(yc[i], yc[i], 0x0C030C02u);
          char* base = ys + ((2 * pr) * G::WO + 2 * pc) * G::PY + oq * 8;
#pragma unroll
          for (int sub = 0; sub < 4; ++sub) {
            const uint32_t S = (uint32_t)sub * 0x00010001u;
            const uint32_t m01 = w6_mask16_eq0(c01 ^ S), m23 = w6_mask16_eq0(c23 ^ S);
            char* d = base + ((sub >> 1) * G::WO + (sub & 1)) * G::PY;
#pragma unroll
            for (int sp = 0; sp < G::NS; ++sp)
              *reinterpret_cast<uint2*>(d + sp * G::YSB) = make_uint2(s0[sp] & m01, s1[sp] & m23);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + 256 * i;
      if (f < YN) {
        const int p = f / YQ, oq = f - p * YQ;
        const int ry = p / G::WO, x = p - ry * G::WO;
        const uint32_t s = (((y0 + ry) & 1) << 1) | (x & 1), c = yc[i];
        float e[4] = {yv[i].x, yv[i].y, yv[i].z, yv[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = ((c >> (8 * k)) & 255u) == s ? e[k] : 0.f;
        uint32_t s0[G::NS], s1[G::NS];
        SP::split(e[0], e[1], ysc, s0);
        SP::split(e[2], e[3], ysc, s1);
        char* d = ys + p * G::PY + oq * 8;
#pragma unroll
        for (int sp = 0; sp < G::NS; ++sp)
          *reinterpret_cast<uint2*>(d + sp * G::YSB) = make_uint2(s0[sp], s1[sp]);
      }
    }
  };

  if (band < band_end) load_band(band);
  for (; band < band_end; band += bstep) {
    const int img = band / G::NBANDS;
    const int bi = band - img * G::NBANDS;
    const int rows_out = min(G::RB, G::HO - bi * G::RB);
    const int kvalid = rows_out * G::WO;
    // first window row of this band in the X slots (ring: slot bi & 1)
    const int xbase = ring ? (bi & 1) * G::RB * G::WS * G::PX : 0;
#ifndef BA3C_DIAG_W6
#define BA3C_DIAG_W6 0        // diagnostics only (A/B timing): 1 = no staging, 2 = no MFMA loop
#endif
    __syncthreads();                                      // previous band's LDS reads done
    if (BA3C_DIAG_W6 != 1) store_band(band);
    __syncthreads();
    if (BA3C_DIAG_W6 != 1 && band + bstep < band_end) load_band(band + bstep);

#ifndef BA3C_W6_UNROLL
#define BA3C_W6_UNROLL 2      // k-steps unrolled per loop iteration: 2 since the pooled staging
#endif                        // freed the registers (r06l: conv2 pair 0.2157 -> 0.2105 ms; r03: 1 -> 2 spilled)
#pragma unroll BA3C_W6_UNROLL
    for (int s = 0; s < (BA3C_DIAG_W6 == 2 ? 0 : G::KS); ++s) {
      // this lane's pixel rows for tr reads r = 0, 1
      int xb[2], yb[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        int p = 32 * s + kperm + 8 * r;
        yb[r] = p * G::PY + 8 * pq;
        if (p >= kvalid) p = 0;                           // padded pixels: dY is zero
        const int y = p / G::WO, x = p - y * G::WO;
        xb[r] = xbase + (y * G::WS + x) * G::PX + 8 * pq;
      }
      u32x4 b[2][G::NS];
#pragma unroll
      for (int nb = 0; nb < 2; ++nb)
#pragma unroll
        for (int sp = 0; sp < G::NS; ++sp) {
          const uint2 u0 = lds_tr16(ys + yb[0] + nb * 32 + sp * G::YSB);
          const uint2 u1 = lds_tr16(ys + yb[1] + nb * 32 + sp * G::YSB);
          b[nb][sp] = u32x4{u0.x, u0.y, u1.x, u1.y};
        }
      // A fragments of tap t + 1 are read into the second register set before tap t's MFMAs
      // (one set made every tap wait a full LDS round trip before its MFMAs)
      auto read_a = [&](int t, u32x4 (&av)[G::NS]) {
        const int tap = tap0 + t;
        const int kh = tap / G::KW, kw = tap - kh * G::KW;
        const int toff = (kh * G::WS + kw) * G::PX;
#pragma unroll
        for (int sp = 0; sp < G::NS; ++sp) {
          const uint2 u0 = lds_tr16(xs + xb[0] + toff + sp * G::XSB);
          const uint2 u1 = lds_tr16(xs + xb[1] + toff + sp * G::XSB);
          av[sp] = u32x4{u0.x, u0.y, u1.x, u1.y};
        }
      };
#ifndef BA3C_W6_DBUF
#define BA3C_W6_DBUF 1
#endif
      u32x4 avb[2][G::NS];
      if (BA3C_W6_DBUF) read_a(0, avb[0]);
#pragma unroll
      for (int t = 0; t < G::TW; ++t) {
        if (t >= ntap) break;
        if (BA3C_W6_DBUF) {
          if (t + 1 < ntap) read_a(t + 1, avb[(t + 1) & 1]);
          __builtin_amdgcn_sched_barrier(0);              // keep those reads ahead of the MFMAs
        } else {
          read_a(t, avb[t & 1]);
        }
        const u32x4 (&av)[G::NS] = avb[t & 1];
        // the family's cross products, interleaved over the two n-blocks
#pragma unroll
        for (int pr = 0; pr < SP::NPROD; ++pr)
#pragma unroll
          for (int nb = 0; nb < 2; ++nb)
            acc[t][nb] = SP::mfma(av[SP::pa(pr)], b[nb][SP::pb(pr)], acc[t][nb]);
      }
    }
  }

  // ---- epilogue: C layout 16x16: lane holds column (lane & 15) = o, rows 4*(lane>>4)+r = c ----
  float* pz = a.part + (size_t)bx * G::M * G::COUT;
  const float us1 = exp2i(-kx), us2 = exp2i(-ky);
#pragma unroll
  for (int t = 0; t < G::TW; ++t) {
    if (t >= ntap) break;
    const int tap = tap0 + t;
#pragma unroll
    for (int nb = 0; nb < 2; ++nb) {
      const int o = o0 + nb * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = c0 + 4 * (lane >> 4) + r;
        pz[((size_t)tap * G::CIN + c) * G::COUT + o] = acc[t][nb][r] * us1 * us2;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// Whole-channel variant (conv1 at large batches, scaled fp16 family).  wgrad6_body gives each
// workgroup 16 of the 32 input channels, so the un-pooled, split dY of every band was loaded and
// split twice (once per channel group: r02 PMC 978 MB per launch against 550 MB algorithmic).
// Here one workgroup takes all (tap, c) rows of its images: dY is staged once, X (all 32
// channels) lives in an XROWS-row window — band i + 1's first HALO rows are band i's last ones
// and move down with one LDS-to-LDS copy, so only RB new rows are loaded and split — and the
// workgroup writes one full [M][COUT] partial slab.  Wave w owns a run of 7 / 6 / 6 / 6 taps x
// both 16-channel c-blocks x both 16-column n-blocks.  Per output the accumulation runs over
// the same k-steps in the same order as wgrad6_body's (bands in order, 32 permuted pixels per
// k-step); only the grouping of images into slabs differs.

template <int HS_, int WS_, int CIN_, int COUT_, int RB_, int PX_, int PY_>
struct Wg6WGeom {
  static constexpr int NS = 2;
  static constexpr int HS = HS_, WS = WS_, CIN = CIN_, COUT = COUT_, RB = RB_;
  static constexpr int KH = 5, KW = 5, NTAP = 25;
  static constexpr int HO = HS - KH + 1, WO = WS - KW + 1, PH = HO / 2, PW = WO / 2;
  static constexpr int NBANDS = HO / RB;
  static constexpr int KP = RB * WO, KS = (KP + 31) / 32, KPAD = 32 * KS;
  static constexpr int HALO = KH - 1, XROWS = RB + HALO;
  static constexpr int PX = PX_, PY = PY_;
  static constexpr int XSB = 2 * CIN, YSB = 2 * COUT;
  static constexpr int X_BYTES = XROWS * WS * PX, Y_BYTES = KPAD * PY;
  static constexpr int CB = CIN / 16, NB = COUT / 16;
  static constexpr int TBASE = NTAP / 4, TREM = NTAP % 4, TW = TBASE + (TREM > 0);
  static constexpr int M = NTAP * CIN;
  static_assert(HO % RB == 0 && RB == HALO, "whole bands; the halo copy's ranges are disjoint");
  static_assert(PX >= NS * XSB && PY >= NS * YSB && PX % 32 == 0 && PY % 32 == 0, "pitches");
  static_assert(RB * WS * (CIN / 4) % 256 == 0, "new X rows: whole float4 per thread");
  static_assert(X_BYTES % 16 == 0 && (HALO * WS * PX) % 16 == 0, "wgrad6w geometry");
  // 2:4-sparse layout (wgrad6s_units): K = quads of 4 consecutive output pixels of one row (two
  // pooling windows), QPR per row, 16 quads per k-step of v_smfmac_f32_16x16x64_f16; the pooled
  // dY as one masked (window 2p, window 2p + 1) dword per (plane, o, quad) and one index nibble
  // per (o, quad)
  static constexpr int QPR = WO / 4, NQ = RB * QPR, SKS = (NQ + 15) / 16, NQPAD = 16 * SKS;
  static constexpr int QS = NQPAD + 4;                     // dwords per (plane, o) row
  static constexpr int SYQ_BYTES = 2 * COUT * QS * 4, SYI_BYTES = (COUT * QS + 15) / 16 * 16;
  static constexpr int S_BYTES = X_BYTES + SYQ_BYTES + SYI_BYTES;
  static_assert(WO % 4 == 0 && COUT == 32 && CIN == 32, "sparse layout: whole quads per row");
};

// conv1's whole-channel weight-gradient geometry (ba3c_capi.hip Lay<2>::W1W, ba3c_conv0.hip)
using Conv1W6W = Wg6WGeom<40, 40, 32, 32, 4, 160, 160>;

// Work units of a workgroup: (tap, c-block) pairs u = 2 tap + cb, 50 of them for 25 taps x 2
// c-blocks; a unit's A fragments feed both n-blocks (6 MFMAs per k-step).  Wave w owns units
// [U0, U0 + NU).  BA3C_W6W_BAL=1 (default): 13 / 13 / 12 / 12 units — the r03/r04 split was
// whole taps, 7 / 6 / 6 / 6 = 14 / 12 / 12 / 12 units, and every band waited for the 14-unit
// wave (25 / 28 of the MFMA pipes busy).  Per output the k-order is unchanged, so the slabs
// are bit-identical either way.
#ifndef BA3C_W6W_BAL
#define BA3C_W6W_BAL 1
#endif
#ifndef BA3C_W6W_PF
#define BA3C_W6W_PF 1
#endif
template <class G>
struct Wg6WUnits {
  static constexpr int UNITS = G::NTAP * G::CB;
  static constexpr int BASE = UNITS / 4, REM = UNITS % 4;
  __host__ __device__ static constexpr int u0(int w) {
    return BA3C_W6W_BAL ? w * BASE + (w < REM ? w : REM)
                        : G::CB * (w * G::TBASE + (w < G::TREM ? w : G::TREM));
  }
  __host__ __device__ static constexpr int nu(int w) { return u0(w + 1) - u0(w); }
  static constexpr int MAXU = BA3C_W6W_BAL ? BASE + (REM > 0) : G::CB * G::TW;
};

template <class G, int U0, int NU>
__device__ __forceinline__ void wgrad6w_units(const Wg6Args& a, int bx, int gx, char* xs, uint32_t* red4) {
  using SP = SplitP<G::NS>;
  const int kx = amax_exp(amax_all(a.amax_x, a.batch, red4));
  const int ky = amax_exp(amax_all(a.amax_dp, a.batch, red4));
  const float xsc = exp2i(kx), ysc = exp2i(ky);
  char* ys = xs + G::X_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  const int kperm = 16 * (g >> 1) + 4 * (g & 1) + q;      // + 8 r for read r (wgrad6_body)

  f32x4 acc[NU][G::NB];
#pragma unroll
  for (int u = 0; u < NU; ++u)
#pragma unroll
    for (int nb = 0; nb < G::NB; ++nb) acc[u][nb] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int XQ = G::CIN / 4;                          // float4 per X pixel
  constexpr int XPT = G::RB * G::WS * XQ / 256;           // float4 of RB rows per thread
  constexpr int YQ = G::COUT / 4;
#ifndef BA3C_W6W_UNPOOL
#define BA3C_W6W_UNPOOL 1     // dY staged per pooled element (0: per un-pooled pixel, A/B)
#endif
  // UNP: each (pooled pixel, 4 channels) of dP is loaded and split once and written to the four
  // pixels of its window with per-channel masks (as band6r_up_body); the padded pixels KP ..
  // KPAD - 1 are zeroed once and never written again
  constexpr bool UNP = BA3C_W6W_UNPOOL;
  constexpr int YN = UNP ? (G::RB / 2) * G::PW * YQ : G::KPAD * YQ;
  constexpr int YPT = (YN + 255) / 256;
  float4 xv[XPT], yv[YPT];
  uint32_t yc[YPT];

  const int ipw = (a.batch + gx - 1) / gx;                // whole images per workgroup
  const int img0 = min(a.batch, bx * ipw), img1 = min(a.batch, img0 + ipw);
  const int band_end = img1 * G::NBANDS;

  // RB image rows from row y of image img -> registers
  auto load_x = [&](int img, int y, float4 (&v)[XPT]) {
    const float* src = a.x + ((size_t)(img * G::HS + y) * G::WS) * G::CIN;
#pragma unroll
    for (int i = 0; i < XPT; ++i) v[i] = reinterpret_cast<const float4*>(src)[tid + 256 * i];
  };
  auto load_y = [&](int img, int bi) {
    const int y0 = bi * G::RB;
    if constexpr (UNP) {
#pragma unroll
      for (int i = 0; i < YPT; ++i) {
        const int f = tid + 256 * i;
        const int oq = f % YQ, rest = f / YQ;
        const int pc = rest % G::PW, py = (y0 >> 1) + rest / G::PW;
        const bool ok = f < YN;                         // branch-free (see wgrad6_body)
        const size_t off = ok ? ((size_t)(img * G::PH + py) * G::PW + pc) * G::COUT + oq * 4 : 0;
        yv[i] = ld4(a.dp + off, ok);
        yc[i] = ld_u8x4(a.code + off, ok);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + 256 * i;
      const int p = f / YQ, oq = f - p * YQ;
      const int ry = p / G::WO, x = p - ry * G::WO;
      yv[i] = f4zero();
      yc[i] = 0;
      if (f < YN && ry < G::RB) {
        const int y = y0 + ry;
        const size_t pidx = (size_t)(img * G::PH + (y >> 1)) * G::PW + (x >> 1);
        yv[i] = *reinterpret_cast<const float4*>(a.dp + pidx * G::COUT + oq * 4);
        yc[i] = *reinterpret_cast<const uint32_t*>(a.code + pidx * G::COUT + oq * 4);
      }
    }
  };
  // RB rows -> window rows wr .. wr + RB - 1, split
  auto store_x = [&](int wr, const float4 (&v)[XPT]) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int f = tid + 256 * i;
      const int pix = f / XQ, cq = f - pix * XQ;
      uint32_t s0[G::NS], s1[G::NS];
      SP::split(v[i].x, v[i].y, xsc, s0);
      SP::split(v[i].z, v[i].w, xsc, s1);
      char* p = xs + (wr * G::WS + pix) * G::PX + cq * 8;
#pragma unroll
      for (int sp = 0; sp < G::NS; ++sp) *reinterpret_cast<uint2*>(p + sp * G::XSB) = make_uint2(s0[sp], s1[sp]);
    }
  };
  auto store_y = [&](int bi) {
    const int y0 = bi * G::RB;
    if constexpr (UNP) {
#pragma unroll
      for (int i = 0; i < YPT; ++i) {
        const int f = tid + 256 * i;
        if (f < YN) {
          const int oq = f % YQ, rest = f / YQ;
          const int pc = rest % G::PW, pr = rest / G::PW;
          uint32_t s0[G::NS], s1[G::NS];
          SP::split(yv[i].x, yv[i].y, ysc, s0);
          SP::split(yv[i].z, yv[i].w, ysc, s1);
          const uint32_t c01 = __builtin_amdgcn_perm(yc[i], yc[i], 0x0C010C00u);   // codes as halves
          const uint32_t c23 = __builtin_amdgcn_perm(yc[i], yc[i], 0x0C030C02u);
          char* base = ys + ((2 * pr) * G::WO + 2 * pc) * G::PY + oq * 8;
#pragma unroll
          for (int sub = 0; sub < 4; ++sub) {
            const uint32_t S = (uint32_t)sub * 0x00010001u;
            const uint32_t m01 = w6_mask16_eq0(c01 ^ S), m23 = w6_mask16_eq0(c23 ^ S);
            char* d = base + ((sub >> 1) * G::WO + (sub & 1)) * G::PY;
#pragma unroll
            for (int sp = 0; sp < G::NS; ++sp)
              *reinterpret_cast<uint2*>(d + sp * G::YSB) = make_uint2(s0[sp] & m01, s1[sp] & m23);
          }
        }
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + 256 * i;
      if (f < YN) {
        const int p = f / YQ, oq = f - p * YQ;
        const int ry = p / G::WO, x = p - ry * G::WO;
        const uint32_t sb = (((y0 + ry) & 1) << 1) | (x & 1), c = yc[i];
        float e[4] = {yv[i].x, yv[i].y, yv[i].z, yv[i].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) e[k] = ((c >> (8 * k)) & 255u) == sb ? e[k] : 0.f;
        uint32_t s0[G::NS], s1[G::NS];
        SP::split(e[0], e[1], ysc, s0);
        SP::split(e[2], e[3], ysc, s1);
        char* d = ys + p * G::PY + oq * 8;
#pragma unroll
        for (int sp = 0; sp < G::NS; ++sp) *reinterpret_cast<uint2*>(d + sp * G::YSB) = make_uint2(s0[sp], s1[sp]);
      }
    }
  };

  if constexpr (UNP) {
    // padded pixels KP .. KPAD - 1 of dY stay zero (the pooled items never write them)
    for (int i = tid; i < (G::KPAD - G::KP) * G::PY / 16; i += 256)
      reinterpret_cast<uint4*>(ys + G::KP * G::PY)[i] = make_uint4(0, 0, 0, 0);
  }
  int band = img0 * G::NBANDS;
  if (band < band_end) {
    load_x(img0, G::HALO, xv);
    load_y(img0, 0);
  }
  for (; band < band_end; ++band) {
    const int img = band / G::NBANDS;
    const int bi = band - img * G::NBANDS;
    __syncthreads();                                      // previous band's LDS reads are done
    if (bi > 0) {
      // window rows RB .. RB + HALO - 1 -> 0 .. HALO - 1 (disjoint); every wave's copy is
      // complete before any wave stores the new rows over the source rows (barrier)
      constexpr int N16 = G::HALO * G::WS * G::PX / 16;
      const uint4* src = reinterpret_cast<const uint4*>(xs + G::RB * G::WS * G::PX);
      uint4* dst = reinterpret_cast<uint4*>(xs);
      for (int i = tid; i < N16; i += 256) dst[i] = src[i];
      __syncthreads();
    }
    store_x(G::HALO, xv);
    store_y(bi);
    if (bi == 0) {                                        // an image's first HALO rows
      load_x(img, 0, xv);
      store_x(0, xv);
    }
    __syncthreads();
    if (band + 1 < band_end) {
      const int ni = (band + 1) / G::NBANDS, nbi = band + 1 - ni * G::NBANDS;
      load_x(ni, nbi * G::RB + G::HALO, xv);
      load_y(ni, nbi);
    }
    // software-pipelined k-steps: unit u + 1's A fragments are read before unit u's MFMAs, and
    // during the last unit of a k-step the next k-step's B fragments and its first unit's A
    // fragments (r04 ISA: each tap's reads were issued ~2 MFMAs ahead of their use and every
    // k-step opened with a full LDS round trip, at one wave per SIMD nothing hid them)
    int xb[2];
    auto addr = [&](int s, int (&xbo)[2], int (&ybo)[2]) {
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        int p = 32 * s + kperm + 8 * r;
        ybo[r] = p * G::PY + 8 * pq;
        if (p >= G::KP) p = 0;                            // padded pixels: dY is zero
        const int y = p / G::WO, x = p - y * G::WO;
        xbo[r] = (y * G::WS + x) * G::PX + 8 * pq;
      }
    };
    auto read_b = [&](const int (&ybo)[2], u32x4 (&bo)[G::NB][G::NS]) {
#pragma unroll
      for (int nb = 0; nb < G::NB; ++nb)
#pragma unroll
        for (int sp = 0; sp < G::NS; ++sp) {
          const uint2 u0 = lds_tr16(ys + ybo[0] + nb * 32 + sp * G::YSB);
          const uint2 u1 = lds_tr16(ys + ybo[1] + nb * 32 + sp * G::YSB);
          bo[nb][sp] = u32x4{u0.x, u0.y, u1.x, u1.y};
        }
    };
    auto read_a = [&](int u, const int (&xbo)[2], u32x4 (&av)[G::NS]) {
      const int unit = U0 + u, tap = unit / G::CB, cb = unit - tap * G::CB;
      const int kh = tap / G::KW, kw = tap - kh * G::KW;
      const int off = (kh * G::WS + kw) * G::PX + cb * 32;   // compile-time
#pragma unroll
      for (int sp = 0; sp < G::NS; ++sp) {
        const uint2 u0 = lds_tr16(xs + xbo[0] + off + sp * G::XSB);
        const uint2 u1 = lds_tr16(xs + xbo[1] + off + sp * G::XSB);
        av[sp] = u32x4{u0.x, u0.y, u1.x, u1.y};
      }
    };
    // D: units of lookahead for the A fragments (BA3C_W6W_PF, A/B)
    constexpr int D = BA3C_W6W_PF, NBUF = D + 1;
    static_assert(D >= 1 && D < NU, "prefetch distance");
    u32x4 b[G::NB][G::NS], bn[G::NB][G::NS], avb[NBUF][G::NS];
    {
      int yb[2];
      addr(0, xb, yb);
      read_b(yb, b);
#pragma unroll
      for (int j = 0; j < D; ++j) read_a(j, xb, avb[j]);
    }
    // one k-step; PF: prefetch the next k-step's B and first D units' A fragments (all but
    // the last k-step of a band)
    auto kstep = [&](int s, auto pf) {
      constexpr bool PF = decltype(pf)::value;
      int xbn[2], ybn[2];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        const int v = u + D;                              // the unit whose A is read now
        if (v < NU) {
          read_a(v, xb, avb[v % NBUF]);
        } else if (PF) {
          if (v == NU) {
            addr(s + 1, xbn, ybn);
            read_b(ybn, bn);
          }
          read_a(v - NU, xbn, avb[v % NBUF]);
        }
        __builtin_amdgcn_sched_barrier(0);                // keep those reads ahead of the MFMAs
        const u32x4 (&av)[G::NS] = avb[u % NBUF];
#pragma unroll
        for (int pr = 0; pr < SP::NPROD; ++pr)
#pragma unroll
          for (int nb = 0; nb < G::NB; ++nb)
            acc[u][nb] = SP::mfma(av[SP::pa(pr)], b[nb][SP::pb(pr)], acc[u][nb]);
      }
      if (PF) {
#pragma unroll
        for (int nb = 0; nb < G::NB; ++nb)
#pragma unroll
          for (int sp = 0; sp < G::NS; ++sp) b[nb][sp] = bn[nb][sp];
        xb[0] = xbn[0];
        xb[1] = xbn[1];
        // the next step's units 0 .. D - 1 were read into buffers NU % NBUF ..: rotate
        u32x4 t[D][G::NS];
#pragma unroll
        for (int j = 0; j < D; ++j)
#pragma unroll
          for (int sp = 0; sp < G::NS; ++sp) t[j][sp] = avb[(NU + j) % NBUF][sp];
#pragma unroll
        for (int j = 0; j < D; ++j)
#pragma unroll
          for (int sp = 0; sp < G::NS; ++sp) avb[j][sp] = t[j][sp];
      }
    };
#ifndef BA3C_W6W_PRIO
#define BA3C_W6W_PRIO 0       // A/B: the k-steps at wave priority 1 (the staging at 0)
#endif
    if (BA3C_W6W_PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll 1
    for (int s = 0; s + 1 < G::KS; ++s) kstep(s, std::true_type{});
    kstep(G::KS - 1, std::false_type{});
    if (BA3C_W6W_PRIO) __builtin_amdgcn_s_setprio(0);
  }

  // ---- epilogue: one full slab per workgroup (lane: column o = 16 nb + (lane & 15), rows
  // c = 16 cb + 4 (lane >> 4) + r) ----
  float* pz = a.part + (size_t)bx * G::M * G::COUT;
  const float us1 = exp2i(-kx), us2 = exp2i(-ky);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int unit = U0 + u, tap = unit / G::CB, cb = unit - tap * G::CB;
#pragma unroll
    for (int nb = 0; nb < G::NB; ++nb) {
      const int o = nb * 16 + (lane & 15);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = cb * 16 + 4 * (lane >> 4) + r;
        pz[((size_t)tap * G::CIN + c) * G::COUT + o] = acc[u][nb][r] * us1 * us2;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------
// 2:4-sparse conv1 weight gradient (BA3C_W6W_SPARSE=1, default).  The un-pooled output
// gradient dY = MaxPoolGrad(dP) * ReluGrad has at most ONE non-zero per 2x2 window and channel,
// so along a row of output pixels every group of 4 consecutive pixels (two windows) holds at
// most 2 non-zeros per channel: exactly the 2:4 structured sparsity of gfx950's
// v_smfmac_f32_16x16x64_f16, whose sparse A operand covers 64 K values in the issue time of the
// dense 16x16x32 MFMA (scripts/probes/smfmac_probe.hip: layout, index encoding and rate).  The
// GEMM is transposed to put dY on that side: dW^T[o][(tap, c)] = sum_p dY[p][o] X[p + tap][c]
// with M = o (2 m-tiles), N = (tap, 16-channel block) units, K = pixels in quads.
//  * A (dY^T): lane l = row o = l & 15 (+ 16 m), quads 4 (l >> 4) .. + 3 of the k-step, two
//    values per quad — window 2p's and 2p+1's gradient where the window's argmax lies in this
//    pixel row (else 0) — and a nibble per quad: the two positions (argmax column in window 0:
//    0 / 1, in window 1: 2 / 3).  Staged once per band from the POOLED dP (no un-pooling).
//  * B (X): lane l = channel l & 15 of the unit, K = quads 2g, 2g + 1, 8 + 2g, 9 + 2g (g = l >>
//    4) of the k-step: four ds_read_b64_tr_b16 of 4 pixels each per plane.
// Same products (dY_hi X_hi, dY_hi X_lo, dY_lo X_hi), same scales, same slabs; the k-order
// differs from the dense body, so the sums agree to rounding, not bit for bit.
// ---------------------------------------------------------------------------------------
#ifndef BA3C_W6W_SPARSE
#define BA3C_W6W_SPARSE 1
#endif
#ifndef BA3C_W6S_HALF
#define BA3C_W6S_HALF 1       // the band's last 4 quads on a half-size sparse k-step (0: a padded full one)
#endif
#ifndef BA3C_DIAG_W6S
#define BA3C_DIAG_W6S 0       // diagnostics only (A/B timing): 1 = no band staging, 2 = no MFMA loop
#endif
typedef _Float16 f16x16v __attribute__((ext_vector_type(16)));

// Logical quad J (the MFMA's K / 4) -> physical quad of the k-step: bits 0 and 1 swapped
// within each group of 4 (an involution).  A 32-lane half of a B read (ds_read_b64_tr_b16)
// holds lane groups g and g + 1, whose quads are J and J + 2: in physical order they are
// neighbours, 4 pixels = 4 x 40 dwords apart = the other 32 banks (row order put them 8 pixels
// = 320 dwords apart: the same banks, a 2-way conflict on every B read, PMC r05i).
__device__ __forceinline__ constexpr int s_pi(int j) { return (j & ~3) | ((j & 1) << 1) | ((j >> 1) & 1); }

template <class G, int U0, int NU>
__device__ __forceinline__ void wgrad6s_units(const Wg6Args& a, int bx, int gx, char* xs, uint32_t* red4) {
  using SP = SplitP<2>;
  const int kx = amax_exp(amax_all(a.amax_x, a.batch, red4));
  const int ky = amax_exp(amax_all(a.amax_dp, a.batch, red4));
  const float xsc = exp2i(kx), ysc = exp2i(ky);
  char* yq = xs + G::X_BYTES;                              // [plane][o][QS] dwords
  uint8_t* yi = reinterpret_cast<uint8_t*>(yq + G::SYQ_BYTES);   // [o][QS] index nibbles
  const int tid = threadIdx.x, lane = tid & 63;
  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3, li = lane & 15;

  f32x4 acc[NU][2];
#pragma unroll
  for (int u = 0; u < NU; ++u) acc[u][0] = acc[u][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  constexpr int XQ = G::CIN / 4;
  constexpr int XPT = G::RB * G::WS * XQ / 256;
  // dY items of a band: (pooled row, window pair p, o), o fastest (coalesced dP loads)
  constexpr int YN = (G::RB / 2) * G::QPR * G::COUT;
  constexpr int YPT = (YN + 255) / 256;
  float4 xv[XPT];
  float yv[YPT][2];
  uint32_t yc[YPT];

  const int ipw = (a.batch + gx - 1) / gx;
  const int img0 = min(a.batch, bx * ipw), img1 = min(a.batch, img0 + ipw);
  const int band_end = img1 * G::NBANDS;

  auto load_x = [&](int img, int y, float4 (&v)[XPT]) {
    const float* src = a.x + ((size_t)(img * G::HS + y) * G::WS) * G::CIN;
#pragma unroll
    for (int i = 0; i < XPT; ++i) v[i] = reinterpret_cast<const float4*>(src)[tid + 256 * i];
  };
  auto load_y = [&](int img, int bi) {
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + 256 * i;
      const int o = f % G::COUT, rest = f / G::COUT;
      const int p = rest % G::QPR, pr = bi * (G::RB / 2) + rest / G::QPR;
      // unconditional loads (past YN: element 0 again, never stored): a load in a branch made
      // the compiler wait for every outstanding load at the join
      const size_t e = f < YN ? ((size_t)(img * G::PH + pr) * G::PW + 2 * p) * G::COUT + o : 0;
      yv[i][0] = a.dp[e];
      yv[i][1] = a.dp[e + G::COUT];
      yc[i] = (uint32_t)a.code[e] | ((uint32_t)a.code[e + G::COUT] << 8);
    }
  };
  auto store_x = [&](int wr, const float4 (&v)[XPT]) {
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int f = tid + 256 * i;
      const int pix = f / XQ, cq = f - pix * XQ;
      uint32_t s0[2], s1[2];
      SP::split(v[i].x, v[i].y, xsc, s0);
      SP::split(v[i].z, v[i].w, xsc, s1);
      char* p = xs + (wr * G::WS + pix) * G::PX + cq * 8;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) *reinterpret_cast<uint2*>(p + sp * G::XSB) = make_uint2(s0[sp], s1[sp]);
    }
  };
  // the band's quads: (pixel row y = 2 pr' + dy, pair p) -> masked dwords + nibbles
  auto store_y = [&]() {
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + 256 * i;
      if (f < YN) {
        const int o = f % G::COUT, rest = f / G::COUT;
        const int p = rest % G::QPR, prl = rest / G::QPR;     // pooled row within the band
        uint32_t h[2];                                       // (hi, lo) of window 2p / 2p+1
        {
          uint32_t s0[2];
          SP::split(yv[i][0], yv[i][1], ysc, s0);
          h[0] = s0[0];
          h[1] = s0[1];
        }
        const uint32_t c0 = yc[i] & 255u, c1 = yc[i] >> 8;
#pragma unroll
        for (int dy = 0; dy < 2; ++dy) {
          const bool m0 = c0 != 255u && (c0 >> 1) == (uint32_t)dy;
          const bool m1 = c1 != 255u && (c1 >> 1) == (uint32_t)dy;
          const uint32_t mk = (m0 ? 0x0000FFFFu : 0u) | (m1 ? 0xFFFF0000u : 0u);
          const int Qp = (2 * prl + dy) * G::QPR + p;     // physical quad -> logical slot
          const int Q = (Qp & ~15) | s_pi(Qp & 15);
#pragma unroll
          for (int sp = 0; sp < 2; ++sp)
            reinterpret_cast<uint32_t*>(yq)[(sp * G::COUT + o) * G::QS + Q] = h[sp] & mk;
          yi[o * G::QS + Q] = (uint8_t)((m0 ? (c0 & 1u) : 0u) | ((2u + (m1 ? (c1 & 1u) : 0u)) << 2));
        }
      }
    }
  };

  // padding quads NQ .. NQPAD - 1: zero values, positions (0, 2); written once
  for (int i = tid; i < 2 * G::COUT * (G::NQPAD - G::NQ); i += 256) {
    const int row = i / (G::NQPAD - G::NQ), Q = G::NQ + i % (G::NQPAD - G::NQ);
    reinterpret_cast<uint32_t*>(yq)[row * G::QS + Q] = 0u;
    if (row < G::COUT) yi[row * G::QS + Q] = (uint8_t)(2u << 2);
  }
  // BA3C_W6S_XPF: 1 = the next band's new X rows are loaded into registers before this band's
  // k-steps and held through them; 0 (default) = loaded at the start of the band's staging.
  // Holding them put the pair kernel at 256 VGPRs with 44 B/lane of scratch (loop constants
  // spilled and reloaded in every band's staging); the exposed load is hidden by the conv0
  // workgroup beside it: same-box r06j, pair 0.4218 -> 0.3928 ms, step 1.739 -> 1.712 ms
#ifndef BA3C_W6S_XPF
#define BA3C_W6S_XPF 0
#endif
  // BA3C_W6S_APF (A/B): 1 (default) = the next k-step's A words and index nibbles are read
  // during the last unit of a k-step; 0 = at the k-step's end (16 + 2 fewer live VGPRs)
#ifndef BA3C_W6S_APF
#define BA3C_W6S_APF 1
#endif
  int band = img0 * G::NBANDS;
  if (band < band_end) {
    if (BA3C_W6S_XPF) load_x(img0, G::HALO, xv);
    load_y(img0, 0);
  }
  for (; band < band_end; ++band) {
    const int img = band / G::NBANDS;
    const int bi = band - img * G::NBANDS;
    if (!BA3C_W6S_XPF && BA3C_DIAG_W6S != 1) load_x(img, bi * G::RB + G::HALO, xv);
    __syncthreads();                                      // previous band's LDS reads are done
    if (BA3C_DIAG_W6S != 1 && bi > 0) {
      constexpr int N16 = G::HALO * G::WS * G::PX / 16;
      const uint4* src = reinterpret_cast<const uint4*>(xs + G::RB * G::WS * G::PX);
      uint4* dst = reinterpret_cast<uint4*>(xs);
      for (int i = tid; i < N16; i += 256) dst[i] = src[i];
      __syncthreads();
    }
    if (BA3C_DIAG_W6S != 1) {
      store_x(G::HALO, xv);
      store_y();
      if (bi == 0) {
        load_x(img, 0, xv);
        store_x(0, xv);
      }
    }
    __syncthreads();
    if (BA3C_DIAG_W6S != 1 && band + 1 < band_end) {
      const int ni = (band + 1) / G::NBANDS, nbi = band + 1 - ni * G::NBANDS;
      if (BA3C_W6S_XPF) load_x(ni, nbi * G::RB + G::HALO, xv);
      load_y(ni, nbi);
    }
    if (BA3C_DIAG_W6S == 2) continue;

    // per k-step: the lane's four quad pixel bases (B reads) and its A / index words
    int xq[4];
    auto addr = [&](int s, int (&xo)[4]) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        // logical quad J of the read; its pixels sit in physical quad s_pi(J) (see below)
        const int Q = 16 * s + s_pi((r >> 1) * 8 + 2 * g + (r & 1));
        const int y = Q < G::NQ ? Q / G::QPR : 0, p = Q < G::NQ ? Q - (Q / G::QPR) * G::QPR : 0;
        xo[r] = (y * G::WS + 4 * p + q) * G::PX + 8 * pq;
      }
    };
    auto read_a = [&](int s, u32x4 (&av)[2][2], uint32_t (&ix)[2]) {
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int o = 16 * m + li;
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const uint4 u = *reinterpret_cast<const uint4*>(yq + ((sp * G::COUT + o) * G::QS + 16 * s + 4 * g) * 4);
          av[m][sp] = u32x4{u.x, u.y, u.z, u.w};
        }
        const uint32_t b = *reinterpret_cast<const uint32_t*>(yi + o * G::QS + 16 * s + 4 * g);
        const uint32_t t = (b | (b >> 4)) & 0x00FF00FFu;     // nibbles of quads 0..3 -> 16 bits
        ix[m] = (t | (t >> 8)) & 0xFFFFu;
      }
    };
    auto read_b = [&](int u, const int (&xo)[4], u32x4 (&bv)[2][2]) {
      const int unit = U0 + u, tap = unit / G::CB, cb = unit - tap * G::CB;
      const int kh = tap / G::KW, kw = tap - kh * G::KW;
      const int off = (kh * G::WS + kw) * G::PX + cb * 32;    // compile-time
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const uint2 r0 = lds_tr16(xs + xo[0] + off + sp * G::XSB);
        const uint2 r1 = lds_tr16(xs + xo[1] + off + sp * G::XSB);
        const uint2 r2 = lds_tr16(xs + xo[2] + off + sp * G::XSB);
        const uint2 r3 = lds_tr16(xs + xo[3] + off + sp * G::XSB);
        bv[sp][0] = u32x4{r0.x, r0.y, r1.x, r1.y};
        bv[sp][1] = u32x4{r2.x, r2.y, r3.x, r3.y};
      }
    };
    u32x4 av[2][2], avn[2][2];
    uint32_t ix[2], ixn[2];
    u32x4 bb[2][2][2];                                    // [buffer][plane][half]
    addr(0, xq);
    read_a(0, av, ix);
    read_b(0, xq, bb[0]);
    auto kstep = [&](int s, auto pf) {
      constexpr bool PF = decltype(pf)::value;
      int xn[4];
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (u + 1 < NU) {
          read_b(u + 1, xq, bb[(u + 1) & 1]);
        } else if (PF) {
          addr(s + 1, xn);
          if (BA3C_W6S_APF) read_a(s + 1, avn, ixn);
          read_b(0, xn, bb[NU & 1]);
        }
        __builtin_amdgcn_sched_barrier(0);                // keep those reads ahead of the MFMAs
        const u32x4 (&bu)[2][2] = bb[u & 1];
        f16x16v b16[2];
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const u32x4 lo = bu[sp][0], hi = bu[sp][1];
          typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));
          const u32x8 w = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          b16[sp] = __builtin_bit_cast(f16x16v, w);
        }
        // dY_hi X_hi, dY_hi X_lo, dY_lo X_hi (SplitP<2>'s products, dY on the sparse side)
#pragma unroll
        for (int pr = 0; pr < 3; ++pr)
#pragma unroll
          for (int m = 0; m < 2; ++m)
            acc[u][m] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(
                __builtin_bit_cast(f16x8, av[m][pr == 2 ? 1 : 0]), b16[pr == 1 ? 1 : 0], acc[u][m], (int)ix[m], 0, 0);
      }
      if (PF) {
        if (BA3C_W6S_APF) {
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            av[m][0] = avn[m][0];
            av[m][1] = avn[m][1];
            ix[m] = ixn[m];
          }
        } else {
          read_a(s + 1, av, ix);                          // (not prefetched: read here)
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) xq[r] = xn[r];
        if (NU & 1) {                                     // the next step's unit 0 is in bb[1]
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) {
            bb[0][sp][0] = bb[1][sp][0];
            bb[0][sp][1] = bb[1][sp][1];
          }
        }
      }
    };
    // a band of NQ = 16 SKF + r quads with 0 < r <= 8 ends in a half k-step: the last 8 slots on
    // v_smfmac_f32_16x16x32_f16 (conv1: 36 quads issue 40 instead of 48)
    constexpr bool HALF = BA3C_W6S_HALF && G::NQ % 16 != 0 && G::NQ % 16 <= 8;
    constexpr int SKF = HALF ? G::SKS - 1 : G::SKS;
#pragma unroll 1
    for (int s = 0; s + 1 < SKF; ++s) kstep(s, std::true_type{});
    kstep(SKF - 1, std::false_type{});
    if constexpr (HALF) {
      // 16x16x32 lane layouts (scripts/probes/smfmac_probe.hip): group g holds logical K 8g .. 8g + 7
      // of A and B = the half step's logical quads 2g, 2g + 1 = slots 16 SKF + 2g, + 1 (addr()'s
      // r = 0, 1 give their pixels)
      typedef _Float16 f16x4h __attribute__((ext_vector_type(4)));
      int xh[4];
      addr(SKF, xh);
      uint2 ah[2][2];
      int ixh[2];
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const int o = 16 * m + li;
#pragma unroll
        for (int sp = 0; sp < 2; ++sp)
          ah[m][sp] = *reinterpret_cast<const uint2*>(yq + ((sp * G::COUT + o) * G::QS + 16 * SKF + 2 * g) * 4);
        const uint32_t b = *reinterpret_cast<const uint16_t*>(yi + o * G::QS + 16 * SKF + 2 * g);
        ixh[m] = (int)((b | (b >> 4)) & 0xFFu);
      }
      auto read_bh = [&](int u, u32x4 (&bv)[2]) {
        const int unit = U0 + u, tap = unit / G::CB, cb = unit - tap * G::CB;
        const int kh = tap / G::KW, kw = tap - kh * G::KW;
        const int off = (kh * G::WS + kw) * G::PX + cb * 32;
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const uint2 r0 = lds_tr16(xs + xh[0] + off + sp * G::XSB);
          const uint2 r1 = lds_tr16(xs + xh[1] + off + sp * G::XSB);
          bv[sp] = u32x4{r0.x, r0.y, r1.x, r1.y};
        }
      };
      u32x4 bh[2][2];                                     // [buffer][plane]
      read_bh(0, bh[0]);
#pragma unroll
      for (int u = 0; u < NU; ++u) {
        if (u + 1 < NU) read_bh(u + 1, bh[(u + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int pr = 0; pr < 3; ++pr)
#pragma unroll
          for (int m = 0; m < 2; ++m)
            acc[u][m] = __builtin_amdgcn_smfmac_f32_16x16x32_f16(
                __builtin_bit_cast(f16x4h, ah[m][pr == 2 ? 1 : 0]), __builtin_bit_cast(f16x8, bh[u & 1][pr == 1 ? 1 : 0]),
                acc[u][m], ixh[m], 0, 0);
      }
    }
  }

  // ---- epilogue: C 16x16: lane holds column li = channel 16 cb + li, rows o = 16 m + 4 g + r
  float* pz = a.part + (size_t)bx * G::M * G::COUT;
  const float us1 = exp2i(-kx), us2 = exp2i(-ky);
#pragma unroll
  for (int u = 0; u < NU; ++u) {
    const int unit = U0 + u, tap = unit / G::CB, cb = unit - tap * G::CB;
    const int c = 16 * cb + li;
#pragma unroll
    for (int m = 0; m < 2; ++m)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int o = 16 * m + 4 * g + r;
        pz[((size_t)tap * G::CIN + c) * G::COUT + o] = acc[u][m][r] * us1 * us2;
      }
  }
}

template <class G>
__device__ __forceinline__ void wgrad6w_body(const Wg6Args& a, int bx, int gx, char* xs, uint32_t* red4) {
  using U = Wg6WUnits<G>;
  static_assert(U::u0(4) == U::UNITS && U::nu(0) <= U::MAXU, "unit partition");
  switch (__builtin_amdgcn_readfirstlane(threadIdx.x >> 6)) {
#define BA3C_W6W_CASE(w)                                                                  \
    if constexpr (BA3C_W6W_SPARSE) wgrad6s_units<G, U::u0(w), U::nu(w)>(a, bx, gx, xs, red4); \
    else wgrad6w_units<G, U::u0(w), U::nu(w)>(a, bx, gx, xs, red4);
    case 0: BA3C_W6W_CASE(0) break;
    case 1: BA3C_W6W_CASE(1) break;
    case 2: BA3C_W6W_CASE(2) break;
    default: BA3C_W6W_CASE(3) break;
#undef BA3C_W6W_CASE
  }
}

// LDS bytes of wgrad6w_body (dense: X window + un-pooled dY; sparse: X window + quads)
template <class G>
__host__ __device__ constexpr int wgrad6w_lds_bytes() {
  return BA3C_W6W_SPARSE ? G::S_BYTES : G::X_BYTES + G::Y_BYTES;
}

template <class G>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) wgrad6w_kernel(const Wg6Args a) {
  __shared__ uint4 lds4[wgrad6w_lds_bytes<G>() / 16];
  __shared__ uint32_t red4[4];
  wgrad6w_body<G>(a, blockIdx.x, gridDim.x, reinterpret_cast<char*>(lds4), red4);
}

template <class G>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) wgrad6_kernel(const Wg6Args a) {
  __shared__ uint4 lds4[(G::X_BYTES + G::Y_BYTES) / 16];
  __shared__ uint32_t red4[4];
  wgrad6_body<G>(a, blockIdx.x, blockIdx.y, gridDim.x, reinterpret_cast<char*>(lds4), red4);
}

}  // namespace ba3c
