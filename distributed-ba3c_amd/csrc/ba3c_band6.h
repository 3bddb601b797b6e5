// ba3c_band6.h — band convolutions on bf16 MFMA with fp32-accurate operand splitting.
//
// gfx950 has no xf32 and its fp32 MFMA runs at 1/16 of the bf16 rate.  Every fp32 value v is
// exactly hi + mid + lo with hi, mid, lo bf16 (8 significant bits each, split3 in
// ba3c_split.h), so for fp32 operands a = a1 + a2 + a3, b = b1 + b2 + b3:
//
//   a*b = a1b1 + (a1b2 + a2b1) + (a1b3 + a2b2 + a3b1) + O(2^-24 |a||b|)
//
// Each bf16 x bf16 product is exact in fp32 and v_mfma_f32_16x16x32_bf16 accumulates in fp32,
// so the six products give the convolution at fp32 accuracy (the three dropped terms are
// below 2^-23 relative — the size of one fp32 rounding) at 16/6 = 2.7x the fp32 MFMA rate.
//
// Same band structure as conv_band_kernel (ba3c_conv.h): one workgroup = one image x RB
// output rows; the input rows the band needs are staged ONCE into LDS — here already split,
// [row][col][split][CIN] bf16 with a pixel pitch PP and row pitch RP (bytes) chosen by a
// bank-conflict search (affine, so every MFMA operand read is a ds_read_b128 at a
// compile-time immediate offset from one per-m-block base).  K-step t = (tap, 32-channel
// chunk); lane group q supplies channels 8q..8q+7, so a lane's A fragment of one split is
// 16 contiguous bytes.  B (weights) comes from a per-step [split][N][K] bf16 copy (L2
// resident) through a register ring.  Pooled epilogues are unchanged: rows are ordered
// (window, sub) so a lane's 4 accumulator rows are one 2x2 window (16x16 C layout).
#pragma once
#include "ba3c_split.h"

#ifndef BA3C_STAGE_NPT
#define BA3C_STAGE_NPT 16   // staging loads in flight per thread (one-band kernels)
#endif

namespace ba3c {

// G: BandGeom (ba3c_conv.h).  PP_: pixel pitch in bytes (>= 6 KPH), RPX_: extra row bytes,
// MCH_: m-blocks per accumulator chunk, KPH_: input channels staged per phase (0 = all CIN).
// With KPH < CIN the band is staged in CIN/KPH channel phases through the same LDS (smaller
// footprint => more workgroups per CU to hide the staging); accumulators persist across
// phases, so a phased layout needs all of a wave's m-blocks in one chunk.
template <class G_, int PP_, int RPX_, int MCH_, int KPH_ = 0, int NS_ = 3, bool DBUF_ = false,
          bool TILE4_ = false, bool PADSKIP_ = false>
struct Band6 {
  // DBUF: A fragments of k-step t + 1 read into a second register set before k-step t's
  // MFMAs (only where the registers allow it without spilling)
  static constexpr bool DBUF = DBUF_;
  // TILE4 (input-gradient layouts with 4-row bands): an m-block is a 4 x 4 pixel tile (rows
  // 0..3 of the band x 4 columns) instead of 16 consecutive pixels, and the two waves of an
  // n-block take tiles 0..4 / 5..9 of the band.  The input gradient is a VALID conv over the
  // zero-padded un-pooled dY, so whole taps of a tile read only padding: kw = 0 for the left
  // edge tile, kw = KW-1 for the right one, kh = 0 / KH-1 for every tile of the first / last
  // band.  Those MFMAs multiply exact zeros and are not issued (8 % of conv1's input-gradient
  // MFMAs); an MFMA adds its products to the accumulator exactly, so nothing else changes.
  static constexpr bool TILE4 = TILE4_;
  // PADSKIP (input-gradient layouts whose one band is the whole map): an m-block of 16
  // consecutive pixels spans one or two output rows; tap rows kh that read only the zero
  // padding for all of them are not issued.  The band is fixed, so the skipped (m-block, tap)
  // pairs are compile-time (conv2: 22 % of the MFMAs, the same count for both waves of an
  // n-block).
  static constexpr bool PADSKIP = PADSKIP_;
  using G = G_;
  __host__ __device__ static constexpr bool pad_kh(int mb, int kh) {
    return 16 * mb >= G_::MROWS ||
           kh < G_::PADY - (16 * mb + 15 < G_::MROWS ? 16 * mb + 15 : G_::MROWS - 1) / G_::WO ||
           kh > G_::PADY - (16 * mb) / G_::WO + G_::UHO - 1;
  }
  static constexpr int NS = NS_;                         // split planes (3 bf16 / 2 fp16)
  static constexpr int KPH = KPH_ ? KPH_ : G_::CIN;
  static constexpr int NPH = G_::CIN / KPH;
  static constexpr int PP = PP_, RP = G::WS * PP_ + RPX_, MCH = MCH_;
  static constexpr int SPB = 2 * KPH;                    // bytes per split of a pixel
  static constexpr int LDS_BYTES = G::SROWS * RP;
  static constexpr int K32 = KPH / 32;                   // 32-channel chunks per tap and phase
  static constexpr int NT = G::KH * G::KW * K32;         // k-steps per phase
  static constexpr int NCH = (G::MBW + MCH - 1) / MCH;   // m-block chunks per wave
  static_assert(KPH % 32 == 0 && G::CIN % KPH == 0 && PP % 16 == 0 && RP % 16 == 0 &&
                PP >= NS * SPB, "band6 layout");
  static_assert(NPH == 1 || NCH == 1, "phased staging keeps every accumulator live");
  static_assert(LDS_BYTES <= 160 * 1024, "band6 LDS");
  static_assert(!TILE4 || (!G::POOL && G::SRC == 1 && G::RB == 4 && G::WO % 4 == 0 &&
                           G::MB == 2 * G::MBW && G::WPN == 2 && NCH == 1 &&
                           G::WO / 4 == G::MB && G::HO % 4 == 0 && G::PADX == G::KW - 1 &&
                           G::PADY == G::KH - 1 && G::UWO + 2 * G::PADX == G::WS &&
                           G::UHO + 2 * G::PADY == G::HS),
                "4x4 tiles: input-gradient bands of 4 rows, one m-block chunk per wave");
  static_assert(!PADSKIP || (!TILE4 && !G::POOL && G::SRC == 1 && G::NBANDS == 1 && G::WPN == 2 &&
                             NCH == 1 && G::UHO + 2 * G::PADY == G::HS),
                "padding skip: one whole-map band, one m-block chunk per wave");
};

struct Band6Args {
  const float* src;        // SRC 0: input map [B,HS,WS,CIN];  SRC 1: dP [B,UPH,UPW,CIN]
  const uint8_t* code;     // SRC 1: argmax codes of dP
  const uint16_t* wt6;     // [NS][COUT][KH*KW*CIN] 16-bit splits (prepared per step)
  float* out;              // POOL: pooled [B,HO/2,WO/2,COUT]; else [B,HO,WO,COUT]
  uint8_t* out_code;       // POOL: argmax codes (may be null: predictor)
  unsigned long long* relu_count;
  int batch;
  // NS = 2 (scaled fp16): max |src| slots of the staged map (per image at [1 + img]), the
  // weight scale exponent, and the slots that receive max |out| (may be null)
  const uint32_t* amax_in;
  const int* wexp;
  uint32_t* amax_out;
  // ring walks only (conv_band6r_kernel): non-null = a dynamic image queue (one ticket word,
  // zeroed by the step's weight-prep launch); null = static contiguous image ranges
  unsigned* ticket;
};

// Dynamic image queue of the ring walks (BA3C_DYNQ, default on where a workgroup walks several
// images): workgroup b starts with image b; thread 0 draws each further image (gx + ticket) with
// one agent-scope atomic when the workgroup STARTS an image and parks it in an LDS slot one
// band later, so the round trip hides behind the band's work; the workgroup reads it at the
// image's end.  Every image's outputs depend only on
// the image, so the results equal the static partition's bit for bit; what changes is that a
// workgroup held off the chip (a collective's workgroups on its CU) no longer leaves its images
// for the end of the launch.
// (an increment, not an add: the compiler's atomic optimizer rewrites a uniform-address add into
// a wave-aggregated one whose result is read back at once, a full vmcnt wait right at the draw)
__device__ __forceinline__ unsigned draw_ticket(unsigned* t) {
  return __builtin_amdgcn_atomic_inc32(t, 0xFFFFFFFFu, __ATOMIC_RELAXED, "agent");
}

// packed 16-bit halves: 0xFFFF where the half is zero, else 0 (code-mask of the pooled staging)
__device__ __forceinline__ uint32_t mask16_eq0(uint32_t d) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  u16x2 x = __builtin_bit_cast(u16x2, d);
  x = __builtin_elementwise_min(x, (u16x2){1, 1});   // 0 where the half matched, else 1
  x = x + (u16x2){0xFFFF, 0xFFFF};                    // 0xFFFF where matched, else 0
  return __builtin_bit_cast(uint32_t, x);
}

// Staging and compute of one band, shared by the one-band-per-workgroup kernel and the
// pipelined persistent kernel below.
template <class L>
struct Band6Ops {
  using G = typename L::G;
  using SP = SplitP<L::NS>;
  static constexpr unsigned Q = L::KPH / 4;                 // float4 per pixel and phase
  static constexpr int NTOT = (G::SROWS * G::WS * Q + 255) / 256;

  __device__ static void band_geom(int b, int& img, int& y0, int& rows_out) {
    img = b / G::NBANDS;
    y0 = (b - img * G::NBANDS) * G::RB;
    rows_out = min(G::RB, G::HO - y0);
  }

  // ---- staging of input rows [y0, y0 + rows_out + KH - 1) (channels of phase ph), split
  // into NS planes, by 256 threads (t = 0..255).  Index math is 32-bit from per-band base
  // pointers (the band of an SRC 0 map is one contiguous run of rows); unsigned division by
  // the compile-time Q / WS is a mul-hi.  SRC 1 un-pools (dP, code) on the fly (sub =
  // position in the 2x2 window).
  __device__ static void load1(const Band6Args& a, int img, int y0, int rows_out, int cb, unsigned f,
                               float4& v, uint32_t& cd) {
    const unsigned nvec = (unsigned)(rows_out + G::KH - 1) * G::WS * Q;
    const unsigned pix = f / Q, cq = f - pix * Q;
    if constexpr (G::SRC == 0) {
      // (the forward layouts keep the branch: branch-free measured 0.289 -> 0.297 ms for conv1's
      // ring walk, 0.093 -> 0.094 ms for conv2)
      v = f4zero();
      cd = 0;
      const float* srcb = a.src + ((size_t)(img * G::HS + y0) * G::WS) * G::CIN + cb;
      if (f < nvec) v = *reinterpret_cast<const float4*>(srcb + pix * G::CIN + cq * 4);
    } else {
      // branch-free loads (ld4 / ld_u8x4 read zeros for a rejected element): a load in a
      // branch made the compiler wait for every outstanding load at the join
      const unsigned ry = pix / G::WS, x = pix - ry * G::WS;
      const int uy = (int)(y0 + ry) - G::PADY, ux = (int)x - G::PADX;
      const bool ok = f < nvec && (unsigned)uy < (unsigned)G::UHO && (unsigned)ux < (unsigned)G::UWO;
      const size_t e = ok ? (size_t)img * (G::UPH * G::UPW) * G::CIN + cb +
                                ((uy >> 1) * G::UPW + (ux >> 1)) * G::CIN + cq * 4
                          : 0;
      v = ld4(a.src + e, ok);
      cd = ld_u8x4(a.code + e, ok);
    }
  }
  __device__ static void store1(char* lds, int y0, int rows_out, unsigned f, const float4& v, uint32_t cd,
                                float asc) {
    const unsigned nvec = (unsigned)(rows_out + G::KH - 1) * G::WS * Q;
    if (f >= nvec) return;
    const unsigned pix = f / Q, cq = f - pix * Q;
    const unsigned ry = pix / G::WS;
    float e[4] = {v.x, v.y, v.z, v.w};
    if constexpr (G::SRC == 1) {
      const unsigned x = pix - ry * G::WS;
      const int uy = (int)(y0 + ry) - G::PADY, ux = (int)x - G::PADX;
      const uint32_t sb = ((uy & 1) << 1) | (ux & 1);      // cd == 0 outside: no code matches
      const bool in = (unsigned)uy < (unsigned)G::UHO && (unsigned)ux < (unsigned)G::UWO;
#pragma unroll
      for (int k = 0; k < 4; ++k) e[k] = (in && ((cd >> (8 * k)) & 255u) == sb) ? e[k] : 0.f;
    }
    uint32_t s0[L::NS], s1[L::NS];
    SP::split(e[0], e[1], asc, s0);
    SP::split(e[2], e[3], asc, s1);
    // ry * RP + x * PP == pix * PP + ry * (RP - WS * PP)
    char* p = lds + pix * L::PP + ry * (L::RP - G::WS * L::PP) + cq * 8;
#pragma unroll
    for (int sp = 0; sp < L::NS; ++sp) *reinterpret_cast<uint2*>(p + sp * L::SPB) = make_uint2(s0[sp], s1[sp]);
  }
#ifndef BA3C_UNPOOL_STAGE
#define BA3C_UNPOOL_STAGE 1   // 0: A/B build with the per-pixel staging (store1) everywhere
#endif
  // Whole-map input-gradient bands (conv2's): the zero-padded un-pooled dY staged from the
  // POOLED map, each (pooled pixel, 4 channels) loaded and split once and written to its 2x2
  // window with per-channel masks (mask16_eq0 on the codes as 16-bit halves); store1 instead
  // loads and splits every staged float4 (4 loads + 4 splits per pooled element, 3 of zeros).
  // The padding cells are zeroed in phase 0 and never written again.  Same LDS image bit for bit.
  static constexpr bool UPSTAGE = BA3C_UNPOOL_STAGE && G::SRC == 1 && L::NS == 2 && G::NBANDS == 1 &&
                                  G::UHO == 2 * G::UPH && G::UWO == 2 * G::UPW &&
                                  G::UHO + 2 * G::PADY == G::HS && G::UWO + 2 * G::PADX == G::WS &&
                                  G::PADY % 2 == 0 && G::PADX % 2 == 0;
  __device__ static void stage_up(const Band6Args& a, char* lds, int t, int img, int ph, float asc) {
    using SP = SplitP<L::NS>;
    constexpr int PARTS = L::NS * L::SPB / 16;             // uint4 per staged pixel
    if (ph == 0) {
      constexpr int NZ = G::SROWS * G::WS * PARTS;
      for (int f = t; f < NZ; f += 256) {
        const int cell = f / PARTS, part = f - cell * PARTS;
        const int r = cell / G::WS, x = cell - r * G::WS;
        if ((unsigned)(r - G::PADY) >= (unsigned)G::UHO || (unsigned)(x - G::PADX) >= (unsigned)G::UWO)
          *reinterpret_cast<uint4*>(lds + r * L::RP + x * L::PP + part * 16) = make_uint4(0, 0, 0, 0);
      }
    }
    constexpr int NPI = G::UPH * G::UPW * (int)Q;
    constexpr int IT = (NPI + 255) / 256;
    float4 v[IT];
    uint32_t c[IT];
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int f = t + 256 * i;
      const bool ok = f < NPI;                           // branch-free (see load1)
      const int cq = f % Q, rest = f / Q;
      const size_t off = ok ? ((size_t)img * (G::UPH * G::UPW) + rest) * G::CIN + ph * L::KPH + cq * 4 : 0;
      v[i] = ld4(a.src + off, ok);
      c[i] = ld_u8x4(a.code + off, ok);
    }
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int f = t + 256 * i;
      if (f < NPI) {
        const int cq = f % Q, rest = f / Q;
        const int pc = rest % G::UPW, py = rest / G::UPW;
        uint32_t s0[2], s1[2];
        SP::split(v[i].x, v[i].y, asc, s0);
        SP::split(v[i].z, v[i].w, asc, s1);
        const uint32_t c01 = __builtin_amdgcn_perm(c[i], c[i], 0x0C010C00u);   // codes as halves
        const uint32_t c23 = __builtin_amdgcn_perm(c[i], c[i], 0x0C030C02u);
        char* base = lds + (G::PADY + 2 * py) * L::RP + (G::PADX + 2 * pc) * L::PP + cq * 8;
#pragma unroll
        for (int sub = 0; sub < 4; ++sub) {
          const uint32_t S = (uint32_t)sub * 0x00010001u;
          const uint32_t m01 = mask16_eq0(c01 ^ S), m23 = mask16_eq0(c23 ^ S);
          char* p = base + (sub >> 1) * L::RP + (sub & 1) * L::PP;
#pragma unroll
          for (int sp = 0; sp < 2; ++sp)
            *reinterpret_cast<uint2*>(p + sp * L::SPB) = make_uint2(s0[sp] & m01, s1[sp] & m23);
        }
      }
    }
  }

  // loads in chunks of NPT (<= NPTMAX), then their stores
  template <int NPTMAX = 8>
  __device__ static void stage(const Band6Args& a, char* lds, int t, int img, int y0, int rows_out, int ph,
                               float asc) {
    constexpr int NPT = NTOT < NPTMAX ? NTOT : NPTMAX;
    for (int base = 0; base < NTOT; base += NPT) {
      float4 v[NPT];
      uint32_t cd[NPT];
#pragma unroll
      for (int i = 0; i < NPT; ++i) load1(a, img, y0, rows_out, ph * L::KPH, t + 256u * (base + i), v[i], cd[i]);
#pragma unroll
      for (int i = 0; i < NPT; ++i) store1(lds, y0, rows_out, t + 256u * (base + i), v[i], cd[i], asc);
    }
  }

  // ---- MFMA main loop + epilogue of one band by the 4 compute waves (wave = 0..3).  For a
  // phased layout (NPH > 1) `stage_phase(ph)` stages phase ph between the barriers; with
  // NPH == 1 the band must already be in LDS.  ReLU positives add to `pos`, the band's max
  // |out| to `omax`.
  template <class StageFn>
  __device__ static void compute(const Band6Args& a, const char* lds, int wave, int lane, int img, int y0,
                                 int rows_out, float us1, float us2, unsigned long long& pos, float& omax,
                                 StageFn&& stage_phase) {
    if constexpr (L::TILE4 || L::PADSKIP) {
      // TILE4: the wave's edge tile (left for waves of tiles 0..4, right for 5..9) and PADSKIP:
      // the wave's m-blocks are compile-time
      if (wave / G::NB == 0) compute_t<0>(a, lds, wave, lane, img, y0, rows_out, us1, us2, pos, omax, stage_phase);
      else compute_t<1>(a, lds, wave, lane, img, y0, rows_out, us1, us2, pos, omax, stage_phase);
    } else {
      compute_t<0>(a, lds, wave, lane, img, y0, rows_out, us1, us2, pos, omax, stage_phase);
    }
  }
  template <int MB0, class StageFn>
  __device__ static void compute_t(const Band6Args& a, const char* lds, int wave, int lane, int img, int y0,
                                   int rows_out, float us1, float us2, unsigned long long& pos, float& omax,
                                   StageFn&& stage_phase) {
    // lane-derived addressing goes through an empty asm: recomputed per band (a few VALU)
    // instead of being hoisted out of a persistent caller's band loop into live registers
    asm volatile("" : "+v"(lane));
    const int nb = wave % G::NB;
    const int mb0 = (L::TILE4 || L::PADSKIP) ? MB0 : wave / G::NB;
    // TILE4: tap row kh_skip reads only padding for every tile of this band (-1: none)
    const int kh_skip = !L::TILE4 ? -1 : (y0 == 0 ? 0 : (y0 + G::RB == G::HO ? G::KH - 1 : -1));
    const int li = lane & 15, lq = lane >> 4;
    const int col = nb * 16 + li;
    // B: lane reads n = col, k = 32 t + 8 lq of split s, stored in MFMA fragment order
    // [s][K / 32][COUT / 16][lane] x 16 B (wprep6_body), so one wave's fragment is 1 KB
    // contiguous.  The offset goes through an empty asm so a persistent caller's band loop
    // cannot hoist the (band-invariant) weight loads of all k-steps out of the loop into
    // registers.
#ifndef BA3C_WFRAG
#define BA3C_WFRAG 1          // 0: A/B build with the plain [s][COUT][KDIM] weight order
#endif
    int woff = BA3C_WFRAG ? nb * 512 + lane * 8 : col * G::KDIM + 8 * lq;
    asm volatile("" : "+v"(woff));
    const uint16_t* wrow = a.wt6 + woff;
    constexpr size_t WSPLIT = (size_t)G::COUT * G::KDIM;
    // fragment offset (16-bit units) of K index k0 (a multiple of 32)
    auto kfrag = [](int k0) { return BA3C_WFRAG ? (k0 / 32) * G::NB * 512 : k0; };
    // K index (tap, channel) of k-step t of a phase, relative to the phase's first channel
    auto koff = [&](int t) { return kfrag((t / L::K32) * G::CIN + (t % L::K32) * 32); };

#pragma unroll
    for (int chn = 0; chn < L::NCH; ++chn) {
      constexpr int MCH = L::MCH;
      int abase[MCH];                                       // bytes
      bool live[MCH];
#pragma unroll
      for (int j = 0; j < MCH; ++j) {
        const int mb = L::TILE4 ? mb0 * G::MBW + j : mb0 + (chn * MCH + j) * G::WPN;
        const int row = mb * 16 + li;
        int oy, ox;
        if constexpr (L::TILE4) {
          oy = li >> 2;
          ox = 4 * mb + (li & 3);
        } else if constexpr (G::POOL) {
          const int w = row >> 2, sb = row & 3;
          const int ph = w / (G::WO / 2), pw = w - ph * (G::WO / 2);
          oy = 2 * ph + (sb >> 1);
          ox = 2 * pw + (sb & 1);
        } else {
          oy = row / G::WO;
          ox = row - oy * G::WO;
        }
        live[j] = chn * MCH + j < G::MBW && mb < G::MB;
        const bool ok = live[j] && row < G::MROWS && oy < rows_out;
        abase[j] = (ok ? oy * L::RP + ox * L::PP : 0) + 16 * lq;
      }
      f32x4 acc[MCH];
#pragma unroll
      for (int j = 0; j < MCH; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};

#ifndef BA3C_B6_PRIO
#define BA3C_B6_PRIO 1        // the MFMA main loop at wave priority 1, the staging at 0 (r05 A/B: conv1 fwd -1 %, dgrad -2 %)
#endif
#pragma unroll 1
      for (int ph = 0; ph < L::NPH; ++ph) {
        if constexpr (L::NPH > 1) stage_phase(ph);
        if (BA3C_B6_PRIO) __builtin_amdgcn_s_setprio(1);
        const uint16_t* wph = wrow + kfrag(ph * L::KPH);
        constexpr int LA = 3;
        uint4 bring[LA + 1][L::NS];
#pragma unroll
        for (int t = 0; t < LA && t < L::NT; ++t)
#pragma unroll
          for (int s = 0; s < L::NS; ++s) bring[t][s] = *reinterpret_cast<const uint4*>(wph + s * WSPLIT + koff(t));
        // A fragments double-buffered in registers: k-step t + 1's LDS reads are issued before
        // k-step t's MFMAs, so their latency hides behind the MFMA chain
        auto read_a = [&](int t, u32x4 (&av)[L::NS][MCH]) {
          const int tap = t / L::K32, ch = t - tap * L::K32;
          const int kh = tap / G::KW, kw = tap - kh * G::KW;
          const int toff = kh * L::RP + kw * L::PP + ch * 64;
#pragma unroll
          for (int j = 0; j < MCH; ++j)
#pragma unroll
            for (int s = 0; s < L::NS; ++s) {
              const uint4 u = *reinterpret_cast<const uint4*>(lds + abase[j] + toff + s * L::SPB);
              av[s][j] = u32x4{u.x, u.y, u.z, u.w};
            }
        };
        constexpr int NB2 = L::DBUF ? 2 : 1;
        u32x4 avb[NB2][L::NS][MCH];
        if constexpr (L::DBUF) read_a(0, avb[0]);
#pragma unroll
        for (int t = 0; t < L::NT; ++t) {
#ifndef BA3C_DIAG_NOB
#define BA3C_DIAG_NOB 0       // diagnostics only: B fragments of the first k-steps reused
#endif
          if (!BA3C_DIAG_NOB && t + LA < L::NT) {
#pragma unroll
            for (int s = 0; s < L::NS; ++s)
              bring[(t + LA) % (LA + 1)][s] = *reinterpret_cast<const uint4*>(wph + s * WSPLIT + koff(t + LA));
          }
          if constexpr (L::DBUF) {
            if (t + 1 < L::NT) read_a(t + 1, avb[(t + 1) & 1]);
            __builtin_amdgcn_sched_barrier(0);                // keep those reads ahead of the MFMAs
          } else {
#ifndef BA3C_B6_RINGFENCE
#define BA3C_B6_RINGFENCE 1   // 0: A/B build without the fence below
#endif
            // the weight-ring loads of k-step t + LA stay here: the scheduler otherwise sank them
            // next to their use, leaving one k-step of lookahead (a vmcnt(0) per k-step, r04 ISA).
            // Input-gradient layouts only: conv2's whole-map input gradient + weight gradient
            // 0.265 -> 0.221 ms with the branch-free staging; conv2's forward 0.093 -> 0.095 ms
            if (BA3C_B6_RINGFENCE && !G::POOL) __builtin_amdgcn_sched_barrier(0);
            read_a(t, avb[0]);
          }
          u32x4 b[L::NS];
#pragma unroll
          for (int s = 0; s < L::NS; ++s) {
            const uint4 u = bring[BA3C_DIAG_NOB ? t % LA : t % (LA + 1)][s];
            b[s] = u32x4{u.x, u.y, u.z, u.w};
          }
          // NS = 3: a1b1, a1b2, a2b1, a1b3, a2b2, a3b1;  NS = 2: a1b1, a1b2, a2b1 —
          // interleaved over m-blocks
          auto mfmas = [&]() {
#pragma unroll
            for (int pr = 0; pr < SP::NPROD; ++pr)
#pragma unroll
              for (int j = 0; j < MCH; ++j) {
                if constexpr (L::TILE4) {
                  // edge tile: tap column kw = 0 (left) / KW-1 (right) reads only padding
                  const int kw = (t / L::K32) % G::KW;
                  if ((MB0 == 0 && j == 0 && kw == 0) || (MB0 == 1 && j == MCH - 1 && kw == G::KW - 1)) continue;
                }
                if constexpr (L::PADSKIP) {
                  if (L::pad_kh(MB0 + j * G::WPN, (t / L::K32) / G::KW)) continue;
                }
                acc[j] = SP::mfma(avb[L::DBUF ? (t & 1) : 0][SP::pa(pr)][j], b[SP::pb(pr)], acc[j]);
              }
          };
          if constexpr (L::TILE4) {
            if ((t / L::K32) / G::KW != kh_skip) mfmas();     // wave-uniform branch
          } else {
            mfmas();
          }
        }
        if (BA3C_B6_PRIO) __builtin_amdgcn_s_setprio(0);
      }

      // ---- epilogue (16x16 C layout: lane holds column li, rows 4 lq + r) ----
      // un-scale by 2^-(ka + kw) (two exact power-of-two products)
#pragma unroll
      for (int j = 0; j < MCH; ++j) {
        const int mb = L::TILE4 ? mb0 * G::MBW + j : mb0 + (chn * MCH + j) * G::WPN;
        if (!live[j]) continue;
        if constexpr (G::POOL) {
          const int w = mb * 4 + lq;
          const int ph = w / (G::WO / 2), pw = w - ph * (G::WO / 2);
          const float v0 = acc[j][0], v1 = acc[j][1], v2 = acc[j][2], v3 = acc[j][3];
          if (w * 4 < G::MROWS && 2 * ph < rows_out) {
            pos += count_pos4(v0, v1, v2, v3);   // uniform over the active lanes (lane 0 among them)
            float mx = v0;
            uint32_t arg = 0;
            if (v1 > mx) { mx = v1; arg = 1; }
            if (v2 > mx) { mx = v2; arg = 2; }
            if (v3 > mx) { mx = v3; arg = 3; }
            const size_t o = ((size_t)(img * (G::HO / 2) + y0 / 2 + ph) * (G::WO / 2) + pw) * G::COUT + col;
            const float out = fmaxf(mx, 0.f) * us1 * us2;
            omax = fmaxf(omax, out);
            a.out[o] = out;
            if (a.out_code) a.out_code[o] = mx > 0.f ? (uint8_t)arg : (uint8_t)255;
          }
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = mb * 16 + lq * 4 + r;
            // TILE4: accumulator row 4 lq + r of tile mb is pixel (lq, 4 mb + r)
            const int oy = L::TILE4 ? lq : row / G::WO, ox = L::TILE4 ? 4 * mb + r : row - oy * G::WO;
            if (row < G::MROWS && oy < rows_out) {
              const float out = acc[j][r] * us1 * us2;
              omax = fmaxf(omax, fabsf(out));
              a.out[((size_t)(img * G::HO + y0 + oy) * G::WO + ox) * G::COUT + col] = out;
            }
          }
        }
      }
    }
  }
};

// One workgroup = one band (image x RB output rows); two workgroups per CU overlap one's
// staging with the other's MFMAs.  The body takes its band index and LDS from the caller, so
// a multi-job launch (ba3c_multi.h) can run it beside another kernel's workgroups.
template <class L>
__device__ __forceinline__ void band6_body(const Band6Args& a, int bx, char* lds) {
  using O = Band6Ops<L>;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  int img, y0, rows_out;
  O::band_geom(bx, img, y0, rows_out);
  const int ka = L::NS == 2 ? amax_exp(a.amax_in[1 + img]) : 0;   // per-image operand scale
  const float asc = exp2i(ka), us1 = exp2i(-ka);
  const float us2 = L::NS == 2 ? exp2i(-a.wexp[0]) : 1.0f;
  unsigned long long pos = 0;
  float omax = 0.f;
  // every staging load of the band in flight at once (one global round trip, not two)
  if constexpr (L::NPH == 1) {
    if constexpr (O::UPSTAGE) O::stage_up(a, lds, tid, img, 0, asc);
    else O::template stage<BA3C_STAGE_NPT>(a, lds, tid, img, y0, rows_out, 0, asc);
    __syncthreads();
  }
  O::compute(a, lds, wave, lane, img, y0, rows_out, us1, us2, pos, omax, [&](int ph) {
    if (ph) __syncthreads();                                // previous phase's reads are done
    if constexpr (O::UPSTAGE) O::stage_up(a, lds, tid, img, ph, asc);
    else O::template stage<BA3C_STAGE_NPT>(a, lds, tid, img, y0, rows_out, ph, asc);
    __syncthreads();
  });
  if (L::NS == 2) amax_publish(a.amax_out, img, omax, lane);
  if (L::G::POOL && a.relu_count) relu_count_add_uniform(a.relu_count, pos, lane);
}

template <class L>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) conv_band6_kernel(const Band6Args a) {
  __shared__ uint4 lds4[L::LDS_BYTES / 16];
  band6_body<L>(a, blockIdx.x, reinterpret_cast<char*>(lds4));
}

// Ring-walk persistent variant (NPH == 1 layouts, large batches): each workgroup walks the
// bands of whole images in order.  Band i + 1's first KH - 1 input rows are band i's last ones,
// already split in LDS: they move down with one LDS-to-LDS copy (rows RB .. SROWS-1 -> 0 ..
// KH-2, disjoint ranges) and only the RB new rows are loaded, un-pooled and split — the
// band's staging VALU and global reads drop by (KH - 1) / SROWS (40 % for conv1 fwd's 6-row
// bands, 50 % for conv1 dgrad's 4-row ones).  Per band the LDS image and the MFMA stream are
// the one-band kernel's, so the outputs are bit-identical.  (Round 2 ran the copy and the new-row
// stores with no barrier in between: a cross-wave write-after-read race in LDS; fixed in r03.)
template <class L, bool PRE_ = L::G::SRC == 1>
__device__ __forceinline__ void band6r_body(const Band6Args& a, int bx, int gx, char* lds, int* tslot) {
  static_assert(L::NPH == 1 && L::G::SROWS > L::G::RB, "ring walk: unphased layouts with a halo");
  static_assert(L::G::NBANDS >= 3, "dynamic queue: the ticket is parked at band 1 and read after the last");
  using O = Band6Ops<L>;
  using G = typename L::G;
  constexpr int HALO = G::SROWS - G::RB;                    // KH - 1 rows carried over
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float us2 = L::NS == 2 ? exp2i(-a.wexp[0]) : 1.0f;
  const bool dyn = a.ticket != nullptr;
  const int ipw = (a.batch + gx - 1) / gx;
  int img0 = bx * ipw, img1 = min(a.batch, img0 + ipw);
  if (dyn) {                  // first image bx (no draw: gx simultaneous same-address draws at
    img0 = bx;                // the start serialise), then images gx + ticket
    img1 = a.batch;
  }
  // PRE (input-gradient layouts, whose registers allow it): the next band's RB new rows are
  // loaded into registers before this band's MFMAs, so their global latency hides behind them
#ifndef BA3C_RING_PRE
#define BA3C_RING_PRE 1
#endif
  constexpr bool PRE = BA3C_RING_PRE && PRE_;
  constexpr unsigned FNEW = (unsigned)HALO * G::WS * O::Q;  // first float4 index of the new rows
  constexpr int NNEW = (G::RB * G::WS * O::Q + 255) / 256;
  float4 pv[PRE ? NNEW : 1];
  uint32_t pc[PRE ? NNEW : 1];
  unsigned long long pos = 0;
  for (int img = img0; img < img1;) {
    const int ka = L::NS == 2 ? amax_exp(a.amax_in[1 + img]) : 0;   // per-image operand scale
    const float asc = exp2i(ka), us1 = exp2i(-ka);
    float omax = 0.f;
    unsigned nt = 0;
    // the image after this one, drawn once the scale's load is consumed (the asm pins the
    // order: a wait for that load at the branch join would otherwise also wait for the draw)
    if (dyn) {
      asm volatile("" ::"v"(asc) : "memory");
      if (tid == 0) nt = draw_ticket(a.ticket);
    }
    for (int bi = 0; bi < G::NBANDS; ++bi) {
      const int y0 = bi * G::RB;
      const int rows_out = min(G::RB, G::HO - y0);
      __syncthreads();                                      // previous band's LDS reads are done
      if (dyn && tid == 0 && bi == 1) *tslot = (int)nt;     // (read after the image's last band)
      unsigned fbase = 0;
#ifndef BA3C_DIAG_NOSTAGE
#define BA3C_DIAG_NOSTAGE 0   // diagnostics only (A/B timing builds): skip the band staging
#endif
#ifndef BA3C_DIAG_NOCOMPUTE
#define BA3C_DIAG_NOCOMPUTE 0 // diagnostics only: skip the MFMA main loop and epilogue
#endif
      if (BA3C_DIAG_NOSTAGE) {
        __syncthreads();
      } else if (bi > 0) {
        // carry the halo rows down: source rows RB .. SROWS-1 -> rows 0 .. HALO-1.  The new
        // rows then go to rows HALO .. SROWS-1, which overlap the source rows (RB >= HALO), and
        // a thread's copy elements are not the rows its stores write: every wave's copy must
        // be complete before any wave stores (the barrier below; without it a fast wave could
        // overwrite halo bytes a slower wave has not copied yet)
        constexpr int N16 = HALO * L::RP / 16;
        const uint4* src = reinterpret_cast<const uint4*>(lds + G::RB * L::RP);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (int i = tid; i < N16; i += 256) dst[i] = src[i];
        fbase = FNEW;                                       // stage rows HALO .. SROWS-1 only
        __syncthreads();
      }
      if (BA3C_DIAG_NOSTAGE) {
      } else if (PRE && bi > 0) {
        // the new rows were prefetched during the previous band's MFMAs
#pragma unroll
        for (int i = 0; i < NNEW; ++i) O::store1(lds, y0, rows_out, FNEW + tid + 256u * i, pv[i], pc[i], asc);
      } else {
        // staging of rows [fbase / (WS Q), rows_out + KH - 1), loads in chunks, then the stores
        const unsigned nvec = (unsigned)(rows_out + G::KH - 1) * G::WS * O::Q;
        constexpr int NPT = O::NTOT < BA3C_STAGE_NPT ? O::NTOT : BA3C_STAGE_NPT;
        for (unsigned base = fbase; base < nvec; base += 256u * NPT) {
          float4 v[NPT];
          uint32_t cd[NPT];
#pragma unroll
          for (int i = 0; i < NPT; ++i) O::load1(a, img, y0, rows_out, 0, base + tid + 256u * i, v[i], cd[i]);
#pragma unroll
          for (int i = 0; i < NPT; ++i) O::store1(lds, y0, rows_out, base + tid + 256u * i, v[i], cd[i], asc);
        }
      }
      __syncthreads();
      if (PRE && !BA3C_DIAG_NOSTAGE && bi + 1 < G::NBANDS) {
        const int y1 = y0 + G::RB, ro1 = min(G::RB, G::HO - y1);
#pragma unroll
        for (int i = 0; i < NNEW; ++i) O::load1(a, img, y1, ro1, 0, FNEW + tid + 256u * i, pv[i], pc[i]);
      }
      if (!BA3C_DIAG_NOCOMPUTE) O::compute(a, lds, wave, lane, img, y0, rows_out, us1, us2, pos, omax, [](int) {});
    }
    if (L::NS == 2) amax_publish(a.amax_out, img, omax, lane);
    img = dyn ? gx + *tslot : img + 1;   // (written at band 1; bands >= 2 put barriers in between)
  }
  if (G::POOL && a.relu_count) relu_count_add_uniform(a.relu_count, pos, lane);
}

// zero-padded un-pooled dY staged from the POOLED map (ring walk of an input-gradient layout,
// scaled fp16 family).  Band6Ops::store1 builds every staged float4 from the pooled float4 of
// its 2x2 window: four global loads and four splits per pooled element, three of them splits
// of zeros.  Here each (pooled pixel, 4 channels) is loaded and split ONCE and written to the
// four pixels of its window with per-channel masks (code == position, compared as packed
// 16-bit halves); the padding columns are zeroed once per workgroup and never written again,
// padding rows are written as zeros.  Split values of zero are +0 either way, so the staged LDS
// image is bit for bit the one store1 builds.

template <class L>
__device__ __forceinline__ void band6r_up_body(const Band6Args& a, int bx, int gx, char* lds, int* tslot) {
  using O = Band6Ops<L>;
  using G = typename L::G;
  using SP = SplitP<L::NS>;
  constexpr int HALO = G::SROWS - G::RB;
  static_assert(L::NS == 2 && G::SRC == 1 && L::NPH == 1 && !G::POOL && G::PADY == HALO &&
                G::RB % 2 == 0 && G::UHO == 2 * G::UPH && G::UWO == 2 * G::UPW &&
                G::UWO + 2 * G::PADX == G::WS && G::HO % G::RB == 0 && G::NBANDS >= 2,
                "pooled staging: padded input-gradient rings with whole windows per band");
  constexpr int Q = O::Q;                                   // float4 per pixel
  constexpr int NPI = (G::RB / 2) * G::UPW * Q;             // pooled items of the new rows
  constexpr int IT = (NPI + 255) / 256;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const float us2 = exp2i(-a.wexp[0]);
  const bool dyn = a.ticket != nullptr;
  const int ipw = (a.batch + gx - 1) / gx;
  int img0 = bx * ipw, img1 = min(a.batch, img0 + ipw);
  if (dyn) {                                                // first image bx, then gx + ticket
    img0 = bx;
    img1 = a.batch;
  }

  // pooled rows bi * RB / 2 .. of image img (new rows of band bi: un-pooled rows y0 .. y0 +
  // RB - 1 = staged rows HALO ..); rows past the map load as zero (value and code 0: the
  // masked writes then store zeros)
  auto load_items = [&](int img, int bi, float4 (&v)[IT], uint32_t (&c)[IT]) {
    const int py0 = bi * (G::RB / 2);
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int f = tid + 256 * i;
      v[i] = f4zero();
      c[i] = 0;
      const int cq = f % Q, rest = f / Q;
      const int pc = rest % G::UPW, py = py0 + rest / G::UPW;
      if (f < NPI && py < G::UPH) {
        const size_t off = ((size_t)(img * G::UPH + py) * G::UPW + pc) * G::CIN + cq * 4;
        v[i] = *reinterpret_cast<const float4*>(a.src + off);
        c[i] = *reinterpret_cast<const uint32_t*>(a.code + off);
      }
    }
  };
  auto store_items = [&](const float4 (&v)[IT], const uint32_t (&c)[IT], float asc) {
#pragma unroll
    for (int i = 0; i < IT; ++i) {
      const int f = tid + 256 * i;
      if (f < NPI) {
        const int cq = f % Q, rest = f / Q;
        const int pc = rest % G::UPW, pr = rest / G::UPW;
        uint32_t s0[2], s1[2];
        SP::split(v[i].x, v[i].y, asc, s0);
        SP::split(v[i].z, v[i].w, asc, s1);
        const uint32_t c01 = __builtin_amdgcn_perm(c[i], c[i], 0x0C010C00u);   // codes as halves
        const uint32_t c23 = __builtin_amdgcn_perm(c[i], c[i], 0x0C030C02u);
        char* base = lds + (HALO + 2 * pr) * L::RP + (G::PADX + 2 * pc) * L::PP + cq * 8;
#pragma unroll
        for (int sub = 0; sub < 4; ++sub) {
          const uint32_t S = (uint32_t)sub * 0x00010001u;
          const uint32_t m01 = mask16_eq0(c01 ^ S), m23 = mask16_eq0(c23 ^ S);
          char* p = base + (sub >> 1) * L::RP + (sub & 1) * L::PP;
#pragma unroll
          for (int sp = 0; sp < 2; ++sp)
            *reinterpret_cast<uint2*>(p + sp * L::SPB) = make_uint2(s0[sp] & m01, s1[sp] & m23);
        }
      }
    }
  };

  // the whole band image starts zero: the padding columns are never written again
  for (int i = tid; i < L::LDS_BYTES / 16; i += 256) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0, 0, 0, 0);
  float4 pv[IT];
  uint32_t pc[IT];
  if (img0 < img1) load_items(img0, 0, pv, pc);
  unsigned long long pos = 0;
  for (int img = img0; img < img1;) {
    const int ka = amax_exp(a.amax_in[1 + img]);            // per-image operand scale
    const float asc = exp2i(ka), us1 = exp2i(-ka);
    float omax = 0.f;
    unsigned nt = 0;
    if (dyn) {                                              // the image after this one (as above)
      asm volatile("" ::"v"(asc) : "memory");
      if (tid == 0) nt = draw_ticket(a.ticket);
    }
    int nimg = img + 1;
    for (int bi = 0; bi < G::NBANDS; ++bi) {
      const int y0 = bi * G::RB;
      __syncthreads();                                      // previous band's LDS reads are done
      if (dyn && tid == 0 && bi == 1) *tslot = (int)nt;     // read after the store barrier below
      if (bi > 0) {
        // halo rows RB .. SROWS-1 -> 0 .. HALO-1; every wave's copy completes before any wave
        // stores new rows over the source rows
        constexpr int N16 = HALO * L::RP / 16;
        const uint4* src = reinterpret_cast<const uint4*>(lds + G::RB * L::RP);
        uint4* dst = reinterpret_cast<uint4*>(lds);
        for (int i = tid; i < N16; i += 256) dst[i] = src[i];
        __syncthreads();
      } else {
        // the first band's rows 0 .. HALO-1 are top padding
        for (int i = tid; i < HALO * L::RP / 16; i += 256) reinterpret_cast<uint4*>(lds)[i] = make_uint4(0, 0, 0, 0);
      }
      store_items(pv, pc, asc);
      __syncthreads();
      if (dyn && bi == 1) nimg = gx + *tslot;
      {
        // prefetch the workgroup's next band (the next image's first band after the last)
        const int nb = bi + 1 < G::NBANDS ? bi + 1 : 0;
        const int ni = bi + 1 < G::NBANDS ? img : nimg;
        if (ni < img1) load_items(ni, nb, pv, pc);
      }
      O::compute(a, lds, wave, lane, img, y0, G::RB, us1, us2, pos, omax, [](int) {});
    }
    amax_publish(a.amax_out, img, omax, lane);
    img = nimg;
  }
}

template <class L, bool PRE_ = L::G::SRC == 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) conv_band6r_kernel(const Band6Args a) {
  __shared__ uint4 lds4[L::LDS_BYTES / 16];
  __shared__ int tslot[1];
  if constexpr (BA3C_UNPOOL_STAGE && L::G::SRC == 1 && L::NS == 2)
    band6r_up_body<L>(a, blockIdx.x, gridDim.x, reinterpret_cast<char*>(lds4), tslot);
  else
    band6r_body<L, PRE_>(a, blockIdx.x, gridDim.x, reinterpret_cast<char*>(lds4), tslot);
}

// conv1's 2:4-sparse input gradient (ba3c_dgrad1s.h): geometry and the B operand of its
// sparse logical K order, prepared by wprep job WJ_C1S
struct D1S {
  static constexpr int HO = 40, WO = 40, C = 32, O = 32, UP = 18;  // dX map / channels; pooled dY
  static constexpr int RB = 4, NBANDS = HO / RB;                     // output rows per band
  static constexpr int SR = RB + 4;                                  // staged dY rows
  static constexpr int NW = 22;                                      // windows (w' = w + 2)
  // PV: dword (window w', window w' + 1) per staged row, w' 0..20, channel; MV: the masked value
  // of window w', w' 0..21, channel (single taps); the quad indices per POOLED row.  Pitches from
  // a bank search over the A-read lane maps (conflict-free ds_read_b128)
  static constexpr int PV_WS = 40, PV_RS = 864;
  static constexpr int MV_WS = 16, MV_RS = 360;
  static constexpr int PV_PLANE = SR * PV_RS, MV_PLANE = SR * MV_RS;  // dwords
  static constexpr int IXF_RS = 21 * 8, IXS_RS = NW * 4;             // u16 per pooled row
  static constexpr int MV_OFF = 2 * PV_PLANE * 4;                    // bytes
  static constexpr int IXF_OFF = MV_OFF + 2 * MV_PLANE * 4;
  static constexpr int IXS_OFF = IXF_OFF + (SR / 2) * IXF_RS * 2;
  static constexpr int LDS_BYTES = IXS_OFF + (SR / 2) * IXS_RS * 2;
  static constexpr int KSTEPS = 15;                                  // 5 tap rows x 3
  static constexpr int WFRAG = 16;                                   // halves per lane and plane
  static constexpr int WPLANE = 2 * KSTEPS * 2 * 64 * WFRAG;         // halves per plane (2 parities)
  static constexpr int NITEM = (SR / 2) * NW * (O / 4);              // (pooled row, window, 4 ch)
  static constexpr int IPT = (NITEM + 255) / 256;
  static_assert(2 * LDS_BYTES <= 160 * 1024 && 21 * PV_WS <= PV_RS && NW * MV_WS <= MV_RS,
                "d1s layout: two workgroups per CU");
};

// The weight of B element (parity eps, k-step s, column c, logical K) — the wprep job's value
// (scripts/probes/sparse_dgrad_model.py bweight): W is conv1/W [5][5][C][O] (HWIO).
__device__ __forceinline__ float d1s_weight(const float* __restrict__ w, int eps, int s, int c, int K) {
  const int kh = s / 3, t = s - 3 * kh, q = K >> 2, p = K & 3;
  if (t < 2) {                                     // aligned quad: channel 16 t + q, tap kw = p + eps
    const int o = 16 * t + q, kw = p + eps;
    return w[((size_t)((4 - kh) * 5 + (4 - kw)) * D1S::C + c) * D1S::O + o];
  }
  const int o = 2 * q + (p >> 1), cl = p & 1;      // single taps: channel pair, pixel column cl
  if (eps == 0) return cl == 0 ? w[((size_t)((4 - kh) * 5 + 0) * D1S::C + c) * D1S::O + o] : 0.f;
  return cl == 1 ? w[((size_t)((4 - kh) * 5 + 4) * D1S::C + c) * D1S::O + o] : 0.f;
}
// fragment element d of one plane: [eps][s][n-tile][lane][16]; B lane layout of the 16x16x64
// sparse MFMA: column lane & 15, logical K 8 g + e (e < 8) / 32 + 8 g + e - 8 (g = lane >> 4)
__device__ __forceinline__ float d1s_wprep_value(const float* __restrict__ w, int d) {
  const int e = d & 15, lane = (d >> 4) & 63, nt = (d >> 10) & 1, rest = d >> 11;
  const int s = rest % D1S::KSTEPS, eps = rest / D1S::KSTEPS, g = lane >> 4;
  const int K = e < 8 ? 8 * g + e : 32 + 8 * g + (e - 8);
  return d1s_weight(w, eps, s, 16 * nt + (lane & 15), K);
}

// One launch per step for all weight preparation on the split path: job y < njobs writes the
// NS split planes of band-conv copy y straight from the parameters (no fp32 [N][K] copy and no
// second pass), job y == njobs (when w0 is set) prepares conv0's MFMA B fragments.  With the
// scaled fp16 family every workgroup of a job first reduces max |W| over the whole tensor
// (L2-resident, <= 200 KB) and splits W * 2^kw; workgroup 0 publishes kw.  The same launch
// zeroes the step's ReLU counters and max-|x| slots (nothing reads them before it ends).
struct WPrep6Args {
  WPrepArgs jobs;
  uint16_t* wt6;
  int off[7];              // fp32 offset of job i; its splits start at NS * off[i]
  const float* w0;         // conv0/W (null: no conv0 job)
  uint4* wb0;
  unsigned long long* relu;  // training: ReLU-count slots zeroed here (no separate memset)
  uint32_t* amax;          // max-|x| slots zeroed here (n_amax words; may be null)
  int n_amax;
  int* wexp;               // [8]: weight scale exponents of jobs 0..5 and conv0 (slot 7)
  int coherent;            // 1: zero with agent-scope stores (read inside the same chained launch)
};

// (bx, by, gx): blockIdx.x, blockIdx.y, gridDim.x of a plain launch; red4: 4 floats of LDS
__device__ __forceinline__ void wprep6_body(const WPrep6Args& a, int bx, int by, int gx, float* red4) {
  const int y = by;
  if (y == 0) {
    if (a.relu)
      for (int i = bx * 256 + threadIdx.x; i < RELU_WORDS; i += gx * 256) {
        if (a.coherent) st_agent_u64(a.relu + i, 0ull);
        else a.relu[i] = 0ull;
      }
    if (a.amax)
      for (int i = bx * 256 + threadIdx.x; i < a.n_amax; i += gx * 256) {
        if (a.coherent) st_agent_u32(a.amax + i, 0u);
        else a.amax[i] = 0u;
      }
  }
  if (y == a.jobs.njobs) {
    if (!a.w0) return;                 // zeroing only (conv0 splits its own fragments)
    const int k = amax_exp(__float_as_uint(conv0_wmax_block(a.w0, red4)));
    if (bx == 0 && threadIdx.x == 0) a.wexp[7] = k;
    conv0s_wprep_one(a.w0, a.wb0, bx * 256 + threadIdx.x, k);
    return;
  }
  const WPrepJob& j = a.jobs.job[y];
  float sc = 1.f;
  {
    // max |W| over the tensor (L2-resident): four independent float4 loads in flight per
    // thread (a single dependent chain was ~15 us of the B=32 step)
    const float4* w4 = reinterpret_cast<const float4*>(j.w);
    auto amax4 = [](float m, const float4& v) {
      return fmaxf(fmaxf(m, fmaxf(fabsf(v.x), fabsf(v.y))), fmaxf(fabsf(v.z), fabsf(v.w)));
    };
    const int n4 = (j.dgrad == 2 ? j.KH * j.KW * j.CI * j.CO : j.n) / 4;   // the source tensor
    float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
    int i = threadIdx.x;
    for (; i + 768 < n4; i += 1024) {
      const float4 v0 = w4[i], v1 = w4[i + 256], v2 = w4[i + 512], v3 = w4[i + 768];
      m0 = amax4(m0, v0);
      m1 = amax4(m1, v1);
      m2 = amax4(m2, v2);
      m3 = amax4(m3, v3);
    }
    for (; i < n4; i += 256) m0 = amax4(m0, w4[i]);
    float m = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if ((threadIdx.x & 63) == 0) red4[threadIdx.x >> 6] = m;
    __syncthreads();
    const int k = amax_exp(__float_as_uint(fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]))));
    if (bx == 0 && threadIdx.x == 0) a.wexp[y] = k;
    sc = exp2i(k);
  }
  uint16_t* dst = a.wt6 + 2 * (size_t)a.off[y];
  if (j.dgrad == 2) {                  // conv1's sparse input-gradient fragments (ba3c_dgrad1s.h)
    for (int d = bx * 256 + threadIdx.x; d < j.n; d += gx * 256) {
      uint32_t hi, lo;
      split2(d1s_wprep_value(j.w, d) * sc, hi, lo);
      dst[d] = (uint16_t)hi;
      dst[j.n + d] = (uint16_t)lo;
    }
    return;
  }
  // destination d in the band kernels' MFMA B-fragment order [K / 32][N / 16][lane][8]: lane
  // (lq, li) holds column n = 16 nb + li, K = 32 k32 + 8 lq .. + 7 (Band6Ops::compute)
  const int K = j.KH * j.KW * (j.dgrad ? j.CO : j.CI);
  const int NB = j.n / K / 16;
  for (int d = bx * 256 + threadIdx.x; d < j.n; d += gx * 256) {
    const int kk = d & 7, li = (d >> 3) & 15, lq = (d >> 7) & 3, rest = d >> 9;
    const int k32 = rest / NB, nb = rest - k32 * NB;
    const int e = BA3C_WFRAG ? (nb * 16 + li) * K + k32 * 32 + lq * 8 + kk : d;
    const float v = wprep_value(j, e);
    uint32_t hi, lo;
    split2(v * sc, hi, lo);
    dst[d] = (uint16_t)hi;
    dst[j.n + d] = (uint16_t)lo;
  }
}

#if BA3C_SHARED_KERNELS  // non-template kernel: emitted by ba3c_capi.hip only
__global__ void __launch_bounds__(256) wprep6_kernel(const WPrep6Args a) {
  __shared__ float red4[4];
  wprep6_body(a, blockIdx.x, blockIdx.y, gridDim.x, red4);
}
#endif

}  // namespace ba3c
