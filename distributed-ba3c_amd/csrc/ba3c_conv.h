// ba3c_conv.h — geometry of the band convolutions (ba3c_band6.h) and the per-step weight
// preparation jobs.
//
// A band convolution stages one image's RB output rows worth of input rows into LDS once and
// runs every MFMA operand read from there at compile-time offsets (no address arithmetic or
// bounds checks in the MFMA loop: the band holds the zero padding).  It is used for the big
// forward convs (conv1/conv2 of train.py:187-204, with ReLU + 2x2 max-pool + argmax code fused)
// and for their input gradients (Conv2DBackpropInput), which are the same VALID convolution
// applied to the zero-padded, un-pooled output gradient with the kernel rotated by 180
// degrees and its channel axes swapped.  Rows of a pooled layer are ordered (window, sub) so a
// lane's 4 accumulator rows are exactly one 2x2 window.
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

// conv0's zero-padded K (25 taps x 4 channels in 7 groups of 16): sizes its workspace region
struct Conv0Geom {
  static constexpr int KDIM = 7 * 16;
};

// ---------------------------------------------------------------------------------------
// Per-step weight preparation: B operand of a band conv as [N][K] with K = (kh, kw, c).
//   forward:  wt[o][(kh,kw,c)]  = W[kh, kw, c, o]                         (W: [KH,KW,CI,CO])
//   dgrad:    wt[ci][(a,b,o)]   = W[KH-1-a, KW-1-b, ci, o]
// ---------------------------------------------------------------------------------------
struct WPrepJob {
  const float* w;
  float* wt;
  int KH, KW, CI, CO, dgrad, n;   // n = total elements; dgrad 2: conv1's sparse input gradient
};
struct WPrepArgs {
  WPrepJob job[7];
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

}  // namespace ba3c
