// ba3c_dgrad1s.h — conv1's input gradient (dP0 = the un-pooled dY1 correlated with the
// flipped conv1/W, OpenAIGym/train.py:187-195 differentiated) on gfx950's 2:4-structured-sparse
// MFMA (v_smfmac_f32_16x16x64_f16), scaled fp16 hi/lo (3 products).
//
// Structure.  A max-pool gradient has at most one non-zero per 2x2 window and channel, so along
// a row of the un-pooled dY any two window-aligned neighbours hold at most one non-zero and any
// window-aligned run of 4 pixels at most two: exactly the 2:4 pattern of the MFMA's sparse A
// operand.  The dense input gradient of output pixel (y, x) sums, per tap row kh and channel o,
// the 5 pixels x-4 .. x of dY row y+kh-4.  Split the output columns by parity:
//   x = 2j   : taps kw 0..3 read windows (j-2, j-1) — one aligned quad; kw 4 reads window j col 0;
//   x = 2j+1 : taps kw 1..4 read windows (j-1, j) — one aligned quad; kw 0 reads window j-2 col 1.
// Per (kh, o) the aligned quad is one sparse quad (the two windows' pooled gradients, masked by
// their argmax row, at positions col(w) and 2 + col(w+1)); the single taps of channels o, o+1
// share one quad whose dummy positions carry zero weights (logical K (o, col 0), (o, col 1),
// (o+1, col 0), (o+1, col 1)).  Per kh: 32 aligned quads + 16 single quads = 3 k-steps of 64
// logical K, 15 k-steps in all against the dense kernel's 25 of 32 — 40 % fewer matrix
// instructions, the same sums (every dropped product is an exact zero).  The layout was proved
// on the CPU first (scripts/probes/sparse_dgrad_model.py) with the lane layouts measured by
// scripts/probes/smfmac_probe.hip.
//
// Staging (per band of RB = 4 output rows): no un-pooled map is built.  For each staged dY row
// (8: the band's rows shifted by the 4-row halo), window pair (w', w' + 1) of the 22 windows (2
// of padding each side) and channel, the dword (masked pooled value of w', that of w' + 1) is
// written (PV; one ds_read_b128 gives a lane its 4 aligned quads, two and four v_perm its 4
// single-tap quads), split into fp16 hi / lo planes with the image's power-of-two scale, and the
// 4-bit quad indices (IXF / IXS) are precomputed from the argmax columns.  Pitches come from a
// bank search over the lane -> address map of the A reads.
//
// Work split: two 256-thread workgroups per CU (58 KB of LDS each: one's staging runs under the
// other's MFMAs), persistent over bands; wave w takes column parity w >> 1 and channel block
// w & 1: 5 m-tiles of 4 rows x 4 same-parity columns.  The B operand (weights in the sparse
// logical K order, both parities) is prepared per step by the wprep job WJ_C1S (ba3c_band6.h)
// and read from L2 through a register ring.  (A first version with 8-row bands in one
// 512-thread workgroup per CU exposed its staging: 0.41 ms against the dense ring's 0.34.)
#pragma once
#include "ba3c_band6.h"

namespace ba3c {

typedef _Float16 f16x16s __attribute__((ext_vector_type(16)));

// a: src = dP1 [B,18,18,32], code = its argmax codes, wt6 = the WJ_C1S fragments (hi plane;
// lo at + WPLANE), out = dP0 [B,40,40,32], amax_in = max |dP1| per image, wexp = the
// weights' scale exponent, amax_out = max |dP0| per image.  bx / gx: first band and stride.
__device__ __forceinline__ void dgrad1s_body(const Band6Args& a, int bx, int gx, char* lds) {
  using G = D1S;
  using SP = SplitP<2>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int eps = wave >> 1, nt = wave & 1;
  const int li = lane & 15, g = lane >> 4, ry = li >> 2, ii = li & 3;
  const float us2 = exp2i(-a.wexp[0]);
  uint32_t* pv = reinterpret_cast<uint32_t*>(lds);
  uint32_t* mv = reinterpret_cast<uint32_t*>(lds + G::MV_OFF);
  uint16_t* ixf = reinterpret_cast<uint16_t*>(lds + G::IXF_OFF);
  uint8_t* ixs = reinterpret_cast<uint8_t*>(lds + G::IXS_OFF);

  // ---- staging items f = (pooled row pr of the band's 4, window w', 4 channels), f = (pr NW +
  // w') 8 + o4; windows w' and w' + 1 loaded (the PV dword pairs them); rows / windows outside
  // the map load as zero.  An image's first band stages all 704 items (three synchronous
  // passes); the others only pooled rows 2, 3 (items 352 ..: two per thread, prefetched into
  // registers mid-band), rows 0 .. 3 being the previous band's rows 4 .. 7 moved down in LDS
  constexpr int FNEW = 2 * G::NW * 8, IPN = (G::NITEM - FNEW + 255) / 256;
  auto item_load = [&](int img, int y0, int f, float4& v0, float4& v1, uint32_t& c0, uint32_t& c1) {
    const int o4 = f & 7, rest = f >> 3, wp = rest % G::NW, pr = rest / G::NW;
    const int py = y0 / 2 - 2 + pr, w = wp - 2;
    const bool rok = f < G::NITEM && (unsigned)py < (unsigned)G::UP;
    const bool ok0 = rok && (unsigned)w < (unsigned)G::UP, ok1 = rok && (unsigned)(w + 1) < (unsigned)G::UP;
    const size_t e = ((size_t)(img * G::UP + (rok ? py : 0)) * G::UP) * G::O + 4 * o4;
    const size_t e0 = ok0 ? e + (size_t)w * G::O : 0, e1 = ok1 ? e + (size_t)(w + 1) * G::O : 0;
    v0 = ld4(a.src + e0, ok0);
    c0 = ld_u8x4(a.code + e0, ok0);
    v1 = ld4(a.src + e1, ok1);
    c1 = ld_u8x4(a.code + e1, ok1);
  };
  auto item_store = [&](float asc, int f, const float4& v0, const float4& v1, uint32_t c0, uint32_t c1) {
    const int o4 = f & 7, rest = f >> 3, wp = rest % G::NW, pr = rest / G::NW;
    uint32_t a01[2], a23[2], b01[2], b23[2];           // [plane]: split halves of channels (0,1), (2,3)
    SP::split(v0.x, v0.y, asc, a01);
    SP::split(v0.z, v0.w, asc, a23);
    SP::split(v1.x, v1.y, asc, b01);
    SP::split(v1.z, v1.w, asc, b23);
    const uint32_t ca01 = __builtin_amdgcn_perm(c0, c0, 0x0C010C00u), ca23 = __builtin_amdgcn_perm(c0, c0, 0x0C030C02u);
    const uint32_t cb01 = __builtin_amdgcn_perm(c1, c1, 0x0C010C00u), cb23 = __builtin_amdgcn_perm(c1, c1, 0x0C030C02u);
#pragma unroll
    for (int t = 0; t < 2; ++t) {                      // staged row 2 pr + t: argmax row t
      const uint32_t T = (uint32_t)(2 * t) * 0x00010001u;
      const uint32_t ma01 = c0w_mask16_eq0((ca01 ^ T) & 0x00FE00FEu), ma23 = c0w_mask16_eq0((ca23 ^ T) & 0x00FE00FEu);
      const uint32_t mb01 = c0w_mask16_eq0((cb01 ^ T) & 0x00FE00FEu), mb23 = c0w_mask16_eq0((cb23 ^ T) & 0x00FE00FEu);
      const int r = 2 * pr + t;
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const uint32_t x01 = a01[sp] & ma01, x23 = a23[sp] & ma23, y01 = b01[sp] & mb01, y23 = b23[sp] & mb23;
        *reinterpret_cast<uint2*>(mv + sp * G::MV_PLANE + r * G::MV_RS + wp * G::MV_WS + 2 * o4) = make_uint2(x01, x23);
        if (wp < G::NW - 1)
          *reinterpret_cast<uint4*>(pv + sp * G::PV_PLANE + r * G::PV_RS + wp * G::PV_WS + 4 * o4) =
              make_uint4(__builtin_amdgcn_perm(y01, x01, 0x05040100u), __builtin_amdgcn_perm(y01, x01, 0x07060302u),
                         __builtin_amdgcn_perm(y23, x23, 0x05040100u), __builtin_amdgcn_perm(y23, x23, 0x07060302u));
      }
    }
    // quad indices (argmax columns; per pooled row)
    const uint32_t ka = c0 & 0x01010101u, kb = c1 & 0x01010101u;
    const uint32_t nf = ka | (kb << 2) | 0x08080808u;                       // nibble per channel
    const uint32_t tf = (nf | (nf >> 4)) & 0x00FF00FFu;
    const uint16_t xf = (uint16_t)((tf | (tf >> 8)) & 0xFFFFu);
    const uint32_t ns = ka | ((ka >> 8) << 2) | 0x00080008u;                // channel pairs (0,1), (2,3)
    const uint8_t xs = (uint8_t)((ns & 15u) | (((ns >> 16) & 15u) << 4));
    if (wp < G::NW - 1) ixf[pr * G::IXF_RS + wp * 8 + o4] = xf;
    ixs[(pr * G::IXS_RS + wp * 4) * 2 + o4] = xs;
  };
  float4 v0[IPN], v1[IPN];
  uint32_t c0[IPN], c1[IPN];
  auto load_new = [&](int img, int y0) {
#pragma unroll
    for (int i = 0; i < IPN; ++i) item_load(img, y0, FNEW + tid + 256 * i, v0[i], v1[i], c0[i], c1[i]);
  };

  // per-lane A offsets of m-tile jt at tap row 0 (kh adds a row; all compile-time beyond this)
  // single taps read window j + 2 - 2 eps (padded), 8 channels from 8 g; the index rows are
  // per pooled row: (ry + kh) >> 1 is added per item
  int pvo[5], mvo[5], ixo[5], iso[5];
#pragma unroll
  for (int jt = 0; jt < 5; ++jt) {
    const int j = 4 * jt + ii;
    pvo[jt] = ry * G::PV_RS + (j + eps) * G::PV_WS + 4 * g;
    mvo[jt] = ry * G::MV_RS + (j + 2 - 2 * eps) * G::MV_WS + 4 * g;
    ixo[jt] = (j + eps) * 8 + g;
    iso[jt] = (j + 2 - 2 * eps) * 4 + g;
  }
  // B fragments of this wave (parity eps, channel block nt): k-step s at + s * 2 * 64 * 16
  const uint16_t* wb = a.wt6 + ((size_t)(eps * G::KSTEPS * 2 + nt) * 64 + lane) * G::WFRAG;
  constexpr size_t BSTEP = 2 * 64 * G::WFRAG;

#ifndef BA3C_DIAG_D1S
#define BA3C_DIAG_D1S 0       // diagnostics only (A/B timing): 1 = no staging, 2 = no MFMA loop,
                              // 3 = weight fragments of the first k-steps reused (no L2 weight stream)
#endif
  // whole images per workgroup, bands in order (the halo rows move down in LDS)
  const int ipw = (a.batch + gx - 1) / gx;
  const int img0 = bx * ipw, img1 = min(a.batch, img0 + ipw);
  for (int img = img0; img < img1; ++img) {
    const int ka = amax_exp(a.amax_in[1 + img]);
    const float asc = exp2i(ka), us1 = exp2i(-ka);
    for (int bi = 0; bi < G::NBANDS; ++bi) {
    const int y0 = bi * G::RB;
    __syncthreads();                                   // previous band's LDS reads are done
    if (BA3C_DIAG_D1S != 1 && bi > 0) {
      // staged rows 4 .. 7 -> 0 .. 3 (PV and MV planes) and pooled index rows 2, 3 -> 0, 1;
      // every copy completes before any new row is stored over its source
      constexpr int NPV = G::PV_RS, NMV = G::MV_RS;    // uint4 per plane (4 rows)
      constexpr int NF = 2 * G::IXF_RS * 2 / 16, NS = 2 * G::IXS_RS * 2 / 16;
      static_assert(G::PV_RS % 4 == 0 && G::MV_RS % 4 == 0 && (2 * G::IXF_RS * 2) % 16 == 0 &&
                    (2 * G::IXS_RS * 2) % 16 == 0 && G::IXF_OFF % 16 == 0 && G::IXS_OFF % 16 == 0, "copy units");
      uint4* pv4 = reinterpret_cast<uint4*>(pv);
      uint4* mv4 = reinterpret_cast<uint4*>(mv);
      uint4* f4 = reinterpret_cast<uint4*>(lds + G::IXF_OFF);
      uint4* s4 = reinterpret_cast<uint4*>(lds + G::IXS_OFF);
      for (int k = tid; k < 2 * NPV + 2 * NMV + NF + NS; k += 256) {
        if (k < 2 * NPV) {
          const int sp = k / NPV, e = k - sp * NPV;
          pv4[(sp * G::PV_PLANE) / 4 + e] = pv4[(sp * G::PV_PLANE + 4 * G::PV_RS) / 4 + e];
        } else if (k < 2 * NPV + 2 * NMV) {
          const int kk = k - 2 * NPV, sp = kk / NMV, e = kk - sp * NMV;
          mv4[(sp * G::MV_PLANE) / 4 + e] = mv4[(sp * G::MV_PLANE + 4 * G::MV_RS) / 4 + e];
        } else if (k < 2 * NPV + 2 * NMV + NF) {
          const int e = k - 2 * NPV - 2 * NMV;
          f4[e] = f4[e + NF];
        } else {
          const int e = k - 2 * NPV - 2 * NMV - NF;
          s4[e] = s4[e + NS];
        }
      }
      __syncthreads();
    }
    if (BA3C_DIAG_D1S != 1) {
      if (bi == 0) {
#pragma unroll 1
        for (int f = tid; f < G::NITEM; f += 256) {
          float4 x0, x1;
          uint32_t k0, k1;
          item_load(img, y0, f, x0, x1, k0, k1);
          item_store(asc, f, x0, x1, k0, k1);
        }
      } else {
#pragma unroll
        for (int i = 0; i < IPN; ++i)
          if (FNEW + tid + 256 * i < G::NITEM) item_store(asc, FNEW + tid + 256 * i, v0[i], v1[i], c0[i], c1[i]);
      }
    }
    __syncthreads();
    f32x4 acc[5];
#pragma unroll
    for (int jt = 0; jt < 5; ++jt) acc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B ring: k-step s = 3 kh + t in slot t (two k-steps of lookahead).  A ring: item i = 5 t + jt
    // of tap row kh in slot i % 3, read two items ahead (across tap rows: 15 items per row, so
    // the slot of an item does not depend on its row).  The tap-row loop stays rolled (fully
    // unrolled, the scheduler hoisted A reads across k-steps: 124 B/lane of scratch)
    constexpr int LA = 2;
    uint4 br[3][2][2];                                 // [slot][plane][half of the 16 halves]
#pragma unroll
    for (int s = 0; s < LA; ++s)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const uint4* p = reinterpret_cast<const uint4*>(wb + s * BSTEP + (size_t)sp * G::WPLANE);
        br[s][sp][0] = p[0];
        br[s][sp][1] = p[1];
      }
    auto read_item = [&](int kh, int t, int jt, u32x4 (&av)[2], int& ix) {
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        if (t < 2) {
          const uint4 u = *reinterpret_cast<const uint4*>(pv + sp * G::PV_PLANE + pvo[jt] + kh * G::PV_RS + 16 * t);
          av[sp] = u32x4{u.x, u.y, u.z, u.w};
        } else {
          const uint4 u = *reinterpret_cast<const uint4*>(mv + sp * G::MV_PLANE + mvo[jt] + kh * G::MV_RS);
          av[sp] = u32x4{u.x, u.y, u.z, u.w};
        }
      }
      const int prl = (ry + kh) >> 1;
      ix = t < 2 ? (int)ixf[prl * G::IXF_RS + ixo[jt] + 4 * t]
                 : (int)reinterpret_cast<const uint16_t*>(ixs)[prl * G::IXS_RS + iso[jt]];
    };
    u32x4 ar[3][2];
    int xr[3];
    if (BA3C_DIAG_D1S != 2) {
      read_item(0, 0, 0, ar[0], xr[0]);
      read_item(0, 0, 1, ar[1], xr[1]);
    }
#pragma unroll 1
    for (int kh = 0; kh < (BA3C_DIAG_D1S == 2 ? 0 : 5); ++kh) {
      // the next band's new rows mid-band (vmcnt waits are in issue order: loads issued before
      // the first weight-ring loads would hold up this band's first k-steps)
      if (BA3C_DIAG_D1S != 1 && kh == 1 && bi + 1 < G::NBANDS) load_new(img, y0 + G::RB);
#pragma unroll
      for (int i = 0; i < 15; ++i) {
        const int t = i / 5, jt = i - 5 * t, s = 3 * kh + t;
        if (jt == 0 && s + LA < G::KSTEPS && BA3C_DIAG_D1S != 3) {
#pragma unroll
          for (int sp = 0; sp < 2; ++sp) {
            const uint4* p = reinterpret_cast<const uint4*>(wb + (s + LA) * BSTEP + (size_t)sp * G::WPLANE);
            br[(t + LA) % 3][sp][0] = p[0];
            br[(t + LA) % 3][sp][1] = p[1];
          }
        }
        {
          const int i2 = i + 2, kh2 = kh + (i2 >= 15 ? 1 : 0), j2 = i2 >= 15 ? i2 - 15 : i2;
          if (kh2 < 5) read_item(kh2, j2 / 5, j2 % 5, ar[i2 % 3], xr[i2 % 3]);
        }
        __builtin_amdgcn_sched_barrier(0);             // those reads ahead of this item's MFMAs
        f16x16s b16[2];
#pragma unroll
        for (int sp = 0; sp < 2; ++sp) {
          const uint4 lo = br[t][sp][0], hi = br[t][sp][1];
          typedef unsigned int u32x8 __attribute__((ext_vector_type(8)));
          const u32x8 w8 = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
          b16[sp] = __builtin_bit_cast(f16x16s, w8);
        }
        // dY_hi W_hi, dY_hi W_lo, dY_lo W_hi (dY on the sparse side)
#pragma unroll
        for (int pr = 0; pr < 3; ++pr)
          acc[jt] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(__builtin_bit_cast(f16x8, ar[i % 3][pr == 2 ? 1 : 0]),
                                                             b16[pr == 1 ? 1 : 0], acc[jt], xr[i % 3], 0, 0);
      }
    }
    // ---- epilogue: lane holds channel 16 nt + li, rows 4 g + r = (row g, column 2 (4 jt + r) + eps)
    float omax = 0.f;
    const int y = y0 + g;
#pragma unroll
    for (int jt = 0; jt < 5; ++jt)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int x = 2 * (4 * jt + r) + eps;
        const float out = acc[jt][r] * us1 * us2;
        omax = fmaxf(omax, fabsf(out));
        a.out[((size_t)(img * G::HO + y) * G::WO + x) * G::C + 16 * nt + li] = out;
      }
    amax_publish(a.amax_out, img, omax, lane);
    }
  }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) dgrad1s_kernel(const Band6Args a) {
  __shared__ uint4 lds4[D1S::LDS_BYTES / 16];
  dgrad1s_body(a, blockIdx.x, gridDim.x, reinterpret_cast<char*>(lds4));
}

}  // namespace ba3c
