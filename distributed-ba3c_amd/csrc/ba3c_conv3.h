// ba3c_conv3.h — conv3 (train.py:206-209: Conv2D 3x3, 64 -> 64 channels, VALID, ReLU, on the
// 7x7 pooled conv2 map) and its input gradient (Conv2DBackpropInput under TF autodiff,
// train/multigpu.py:85-86) as persistent whole-image convolutions on the scaled fp16 hi/lo
// MFMA family (ba3c_split.h: three v_mfma_f32_16x16x32_f16 per fp32 product).
//
//   forward:  a3[n,y,x,o]  = ReLU(sum_{kh,kw,c} p2[n,y+kh,x+kw,c] W3[kh,kw,c,o])       5x5 out
//   DG:       dP2[n,y,x,c] = sum_{a,b,o} dY3pad[n,y+a,x+b,o] W3[2-a,2-b,c,o]            7x7 out
//
// (the input gradient is the VALID convolution of the 2-padded dY3 with the kernel rotated by
// 180 degrees and its channel axes swapped: wprep6's dgrad copy).  The bf16x6 GEMM engine ran
// these as im2col GEMMs: every workgroup re-gathered and re-split its 64 x 64 tile of both
// operands for each k-tile (VALU:MFMA 13-14, r03 PMC), i.e. each p2 / dY3 element 9 times and
// the whole of W3 once per workgroup.  Here one workgroup owns an image at a time:
//   * the image (p2: 12.5 KB, dY3: 6.4 KB) is loaded once, its max |x| reduced in the
//     workgroup (the per-image scale: results do not depend on the batch), split once into
//     hi / lo fp16 planes and stored into LDS with the zero padding around it;
//   * wave w computes output channels 16w .. 16w + 15 for all of the image's output pixels
//     (m-blocks of 16 pixels: 2 forward, 4 DG); its B fragments (the prepared weights in MFMA
//     fragment order, 18 k-steps x 2 planes x 16 B per lane = 144 VGPRs) are loaded once per
//     workgroup and stay in registers for every image it walks;
//   * every A read is a ds_read_b128 at a compile-time offset from one per-m-block base
//     (pixel / row pitches from scripts/lds_bank_search.py);
//   * the next image's input is loaded into registers while the MFMAs of this one run.
// Forward epilogue: ReLU, the count of positive outputs (TfDictOp's active_relus), a3 in the
// [B,1600] layout fc1 reads.  DG epilogue: dP2 and its per-image max |x| (amax_publish) for
// conv2's split kernels.
#pragma once
#include "ba3c_split.h"
#include "ba3c_wgrad6.h"   // lds_tr16

namespace ba3c {

template <bool DG>
struct Conv3G {
  static constexpr int CIN = 64, COUT = 64, KH = 3, KW = 3;  // of the band conv (DG: swapped)
  static constexpr int HI = DG ? 5 : 7;                 // input map: p2 7x7 / dY3 5x5
  static constexpr int PAD = DG ? 2 : 0;                // DG: zero padding of dY3
  static constexpr int HS = HI + 2 * PAD;               // staged map: 7 / 9
  static constexpr int HO = HS - KH + 1;                // output map: 5 / 7
  static constexpr int MROWS = HO * HO;                 // output pixels: 25 / 49
  static constexpr int MB = (MROWS + 15) / 16;          // m-blocks: 2 / 4
  static constexpr int NB = COUT / 16;                  // n-blocks = waves
  static constexpr int K32 = CIN / 32;
  static constexpr int NT = KH * KW * K32;              // 32-wide k-steps: 18
  static constexpr int SPB = 2 * CIN;                   // bytes of one plane of a pixel
  // pixel / row pitches: 6.0 (forward) / 5.0 (DG) LDS cycles per ds_read_b128, ideal 4
  static constexpr int PP = DG ? 288 : 272, RP = HS * PP + (DG ? 192 : 240);
  static constexpr int LDS_BYTES = HS * RP;
  static constexpr int NV4 = HI * HI * CIN / 4;         // float4 of one input image
  static constexpr int V4PT = (NV4 + 255) / 256;        // per thread
  static constexpr int WSPLIT = KH * KW * CIN * COUT;   // 16-bit elements between weight planes
  static_assert(PP >= 2 * SPB && PP % 16 == 0 && RP % 16 == 0 && NB == 4, "conv3 layout");
  // DG: does tap (kh, kw) of m-block j read any non-padding input for a real output pixel?
  // (m-block 3 holds pixel 48 alone, whose only such tap is (0, 0): its other 16 k-steps
  // multiply zeros and are not issued — 22 % of the input gradient's MFMAs.  The first MBL
  // m-blocks use every tap and run in the main k-loop; the rest (DG: m-block 3) run their live
  // k-steps in a loop of their own — skipping inside the main loop made the compiler spill.)
  __host__ __device__ static constexpr bool live(int j, int kh, int kw) {
    for (int r = 16 * j; r < 16 * j + 16 && r < MROWS; ++r) {
      const int y = r / HO + kh - PAD, x = r % HO + kw - PAD;
      if (y >= 0 && y < HI && x >= 0 && x < HI) return true;
    }
    return false;
  }
  static constexpr int MBL = DG ? 3 : MB;
  static_assert(LDS_BYTES <= 64 * 1024, "two workgroups per CU");
};

struct Conv3Args {
  const float* src;                 // forward: p2 [B,7,7,64];  DG: dY3 [B,5,5,64]
  const uint16_t* wt6;              // hi / lo planes of the prepared weights (wprep6 job)
  const int* wexp;                  // their scale exponent
  float* out;                       // forward: a3 [B,5,5,64];  DG: dP2 [B,7,7,64]
  unsigned long long* relu_count;   // forward, training: ReLU-count slots (may be null)
  uint32_t* amax_out;               // DG: max |dP2| per image (may be null)
  int batch;
  uint32_t* amax_in;                // DG: receives max |dY3| per image (conv3_wgrad_body's scale)
};

// (bx, gx): first image and image stride of this workgroup; lds: LDS_BYTES, red4: 4 words
template <bool DG>
__device__ __forceinline__ void conv3_body(const Conv3Args& a, int bx, int gx, char* lds, float* red4) {
  using G = Conv3G<DG>;
  using SP = SplitP<2>;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // = the wave's n-block
  const int li = lane & 15, lq = lane >> 4;

  // B fragments of this wave's n-block for every k-step: lane (li, lq) holds column
  // 16 wave + li, K 32 t + 8 lq .. + 7 ([K/32][N/16][lane] order, wprep6_body)
  u32x4 bw[G::NT][2];
  {
    const uint16_t* wp = a.wt6 + wave * 512 + lane * 8;
#pragma unroll
    for (int t = 0; t < G::NT; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const uint4 u = *reinterpret_cast<const uint4*>(wp + s * G::WSPLIT + t * G::NB * 512);
        bw[t][s] = u32x4{u.x, u.y, u.z, u.w};
      }
  }
  const float us2 = exp2i(-a.wexp[0]);
  if constexpr (DG) {   // the padding ring is never written again
    for (int f = tid; f < G::LDS_BYTES / 16; f += 256) reinterpret_cast<uint4*>(lds)[f] = make_uint4(0, 0, 0, 0);
  }
  // A-fragment base of each m-block: lane row li = output pixel 16 j + li (rows past the map
  // read pixel 0; their results are dropped), K 8 lq .. + 7 of the k-step's 32 channels
  int abase[G::MB];
#pragma unroll
  for (int j = 0; j < G::MB; ++j) {
    const int row = 16 * j + li, oy = row / G::HO, ox = row - oy * G::HO;
    abase[j] = (row < G::MROWS ? oy * G::RP + ox * G::PP : 0) + 16 * lq;
  }

  const float4* src4 = reinterpret_cast<const float4*>(a.src);
  float4 v[G::V4PT];
  auto load = [&](int img) {
#pragma unroll
    for (int i = 0; i < G::V4PT; ++i) {
      const int f = tid + 256 * i;
      v[i] = (img < a.batch && f < G::NV4) ? src4[(size_t)img * G::NV4 + f] : f4zero();
    }
  };
  unsigned long long pos = 0;
  load(bx);
  for (int img = bx; img < a.batch; img += gx) {
    // the image's max |x| -> its scale exponent
    float m = 0.f;
#pragma unroll
    for (int i = 0; i < G::V4PT; ++i)
      m = fmaxf(m, fmaxf(fmaxf(fabsf(v[i].x), fabsf(v[i].y)), fmaxf(fabsf(v[i].z), fabsf(v[i].w))));
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = fmaxf(m, __shfl_xor(m, o, 64));
    if (lane == 0) red4[wave] = m;
    __syncthreads();   // also: every wave's MFMA reads of the previous image are done
    const float imax = fmaxf(fmaxf(red4[0], red4[1]), fmaxf(red4[2], red4[3]));
    if (DG && a.amax_in && tid == 0 && imax > 0.f) a.amax_in[1 + img] = __float_as_uint(imax);
    const int ka = amax_exp(__float_as_uint(imax));
    const float asc = exp2i(ka), us1 = exp2i(-ka);
    // split and store: float4 f = pixel f / 16, channels 4 (f % 16) .. + 3
#pragma unroll
    for (int i = 0; i < G::V4PT; ++i) {
      const int f = tid + 256 * i;
      if (f < G::NV4) {
        const int pix = f >> 4, cq = f & 15;
        const int y = pix / G::HI, x = pix - y * G::HI;
        uint32_t s0[2], s1[2];
        SP::split(v[i].x, v[i].y, asc, s0);
        SP::split(v[i].z, v[i].w, asc, s1);
        char* p = lds + (y + G::PAD) * G::RP + (x + G::PAD) * G::PP + cq * 8;
        *reinterpret_cast<uint2*>(p) = make_uint2(s0[0], s1[0]);
        *reinterpret_cast<uint2*>(p + G::SPB) = make_uint2(s0[1], s1[1]);
      }
    }
    __syncthreads();
    load(img + gx);   // in flight during the MFMAs

    f32x4 acc[G::MB];
#pragma unroll
    for (int j = 0; j < G::MB; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the m-blocks past MBL: only their live k-steps
#pragma unroll
    for (int j = G::MBL; j < G::MB; ++j)
#pragma unroll
      for (int t = 0; t < G::NT; ++t) {
        const int tap = t / G::K32, ch = t - tap * G::K32;
        const int kh = tap / G::KW, kw = tap - kh * G::KW;
        if (!G::live(j, kh, kw)) continue;
        const int toff = kh * G::RP + kw * G::PP + ch * 64;
        u32x4 av[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint4 u = *reinterpret_cast<const uint4*>(lds + abase[j] + toff + s * G::SPB);
          av[s] = u32x4{u.x, u.y, u.z, u.w};
        }
#pragma unroll
        for (int pr = 0; pr < SP::NPROD; ++pr) acc[j] = SP::mfma(av[SP::pa(pr)], bw[t][SP::pb(pr)], acc[j]);
      }
    // A fragments double-buffered: k-step t + 1's LDS reads are issued before k-step t's
    // MFMAs (one set left every k-step waiting a full LDS round trip)
    auto read_a = [&](int t, u32x4 (&av)[2][G::MB]) {
      const int tap = t / G::K32, ch = t - tap * G::K32;
      const int kh = tap / G::KW, kw = tap - kh * G::KW;
      const int toff = kh * G::RP + kw * G::PP + ch * 64;
#pragma unroll
      for (int j = 0; j < G::MBL; ++j)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const uint4 u = *reinterpret_cast<const uint4*>(lds + abase[j] + toff + s * G::SPB);
          av[s][j] = u32x4{u.x, u.y, u.z, u.w};
        }
    };
    // (the input gradient's four m-blocks leave no registers for a second set: single-buffered)
    constexpr bool DBUF = !DG;
    u32x4 avb[DBUF ? 2 : 1][2][G::MB];
    if constexpr (DBUF) read_a(0, avb[0]);
#pragma unroll
    for (int t = 0; t < G::NT; ++t) {
      if constexpr (DBUF) {
        if (t + 1 < G::NT) read_a(t + 1, avb[(t + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);   // keep those reads ahead of the MFMAs
      } else {
        const int tap = t / G::K32, ch = t - tap * G::K32;
        const int toff = (tap / G::KW) * G::RP + (tap % G::KW) * G::PP + ch * 64;
#pragma unroll
        for (int j = 0; j < G::MBL; ++j)
#pragma unroll
          for (int s = 0; s < 2; ++s) {
            const uint4 u = *reinterpret_cast<const uint4*>(lds + abase[j] + toff + s * G::SPB);
            avb[0][s][j] = u32x4{u.x, u.y, u.z, u.w};
          }
      }
      // a1b1, a1b2, a2b1, interleaved over the m-blocks
#pragma unroll
      for (int pr = 0; pr < SP::NPROD; ++pr)
#pragma unroll
        for (int j = 0; j < G::MBL; ++j)
          acc[j] = SP::mfma(avb[DBUF ? (t & 1) : 0][SP::pa(pr)][j], bw[t][SP::pb(pr)], acc[j]);
    }

    // epilogue (16x16 C layout: lane holds column li, rows 4 lq + r of each m-block); the
    // scale comes off as two exact power-of-two products
    const int col = 16 * wave + li;
    float omax = 0.f;
#pragma unroll
    for (int j = 0; j < G::MB; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * j + 4 * lq + r;
        if (row < G::MROWS) {
          const float o = acc[j][r] * us1 * us2;
          float* dst = a.out + ((size_t)img * G::MROWS + row) * G::COUT + col;
          if constexpr (DG) {
            omax = fmaxf(omax, fabsf(o));
            *dst = o;
          } else {
            pos += o > 0.f;
            *dst = fmaxf(o, 0.f);
          }
        }
      }
    if constexpr (DG) amax_publish(a.amax_out, img, omax, lane);
  }
  if constexpr (!DG) {
    if (a.relu_count) relu_count_add(a.relu_count, pos, lane);
  }
}

template <bool DG>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) conv3_band_kernel(const Conv3Args a) {
  __shared__ uint4 lds4[Conv3G<DG>::LDS_BYTES / 16];
  __shared__ float red4[4];
  conv3_body<DG>(a, blockIdx.x, gridDim.x, reinterpret_cast<char*>(lds4), red4);
}

// the input-gradient kernel as a multi-job launch job (ba3c_multi.h: x = first image, gx = the
// job's own grid)
struct Conv3DJob {
  using Args = Conv3Args;
  static constexpr int LDS = Conv3G<true>::LDS_BYTES;
  __device__ static void run(const Args& a, int x, int, int, int gx, char* lds, uint32_t* red4) {
    conv3_body<true>(a, x, gx, lds, reinterpret_cast<float*>(red4));
  }
};

// ---------------------------------------------------------------------------------------
// conv3's weight gradient (Conv2DBackpropFilter, train.py:206-209 under TF autodiff):
//   dW3[kh,kw,c,o] = sum_{n, y<5, x<5} p2[n, y+kh, x+kw, c] * dY3[n, y, x, o]
// GEMM view M = (tap, c) = 576, N = o = 64, K = the 25 output pixels of every image (one
// 32-wide k-step per image, rows 25..31 of dY3 zero).  One 512-thread workgroup per CU walks
// images; its 576 x 64 accumulators stay in registers (wave w: m-blocks 9 (w & 3) .. + 8 of
// n-blocks 2 (w >> 2), + 1: 72 VGPRs) and are written once as the workgroup's fp32 partial
// slab (reduced in the deferred reduction launch).  The image's p2 and dY3 are split into
// fp16 hi / lo planes in LDS ([pixel][plane][channel], the natural NHWC order) and read with
// ds_read_b64_tr_b16 (4 pixel rows x 16 channels per 16-lane group, transposed in hardware), the
// A reads of tap (kh, kw) at the affine offset (7 kh + kw) x pixel pitch.  The sum runs over
// images, so both operands take the whole tensor's scale: the maxima of p2 (published by
// conv2's forward) and of dY3 (by conv3's input-gradient kernel, which runs first).
// The GEMM engine gathered 64 x 32 transposed tiles per k-tile from HBM: 176 MB of traffic per
// launch for 39 MB of operands (r03 PMC).
// ---------------------------------------------------------------------------------------
struct Conv3WG {
  static constexpr int NPX = 49, NPY = 25, KP = 32, M = 576, N = 64;
  // pixel pitches 288 = 32 x 9 (mod 256): the 8 pixel rows of a 32-lane tr read land in
  // distinct 32-byte bank windows when the rows are consecutive
  static constexpr int PX = 288, PY = 288, SPB = 128;
  static constexpr int X_BYTES = NPX * PX, Y_BYTES = KP * PY;
  static constexpr int NV4X = NPX * 64 / 4, NV4Y = NPY * 64 / 4;   // float4 per image: 784 / 400
};

struct Conv3WArgs {
  const float* x;              // p2 [B,7,7,64]
  const float* dy;             // dY3 [B,5,5,64]
  float* part;                 // [gridDim.x][576][64] partial slabs
  int batch;
  const uint32_t* amax_x;      // per-image max |p2| slots
  const uint32_t* amax_dy;     // per-image max |dY3| slots
  int self_dy;                 // 1: max |dY3| reduced from dY3 itself (amax_dy unused)
};

// NT = 512: one workgroup per slab (waves 4..7 take n-blocks 2, 3); NT = 256: two workgroups
// per slab, n-half `nhw` each (a multi-job launch beside conv3's input gradient: every output
// element's k order is the same, so the slabs are bit-identical).  bx / gx: first image and
// image stride; lds: X_BYTES + Y_BYTES; red: NT / 64 words
template <int NT>
__device__ __forceinline__ void conv3_wgrad_body(const Conv3WArgs& a, int bx, int gx, int nhw, char* lds, uint32_t* red) {
  using G = Conv3WG;
  using SP = SplitP<2>;
  constexpr int NW = NT / 64;
  constexpr int XPT = (G::NV4X + NT - 1) / NT, YPT = (G::NV4Y + NT - 1) / NT;
  static_assert(NT == 512 || NT == 256, "conv3 weight gradient: 8 or 4 waves");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mg = wave & 3, nh = NT == 512 ? wave >> 2 : nhw;
  char* xs = lds;
  char* ys = lds + G::X_BYTES;
  // whole-tensor scales (the sum runs over images)
  auto amax_wg = [&](uint32_t m) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o, 64));
    if (lane == 0) red[wave] = m;
    __syncthreads();
    uint32_t r = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) r = max(r, red[w]);
    __syncthreads();
    return r;
  };
  auto amax_slots = [&](const uint32_t* slots) {
    uint32_t m = 0;
    for (int i = tid; i < a.batch; i += NT) m = max(m, slots[1 + i]);
    return amax_wg(m);
  };
  // self_dy: max |dY3| over the tensor (the bits of |x| order like the values: the maximum the
  // input-gradient kernel would publish), four float4 in flight per thread
  auto amax_dy_self = [&]() {
    const uint4* y = reinterpret_cast<const uint4*>(a.dy);
    const int n4 = a.batch * G::NV4Y;
    uint32_t m = 0;
    auto m4 = [](uint32_t m, const uint4& v) {
      return max(max(m, max(v.x & 0x7FFFFFFFu, v.y & 0x7FFFFFFFu)), max(v.z & 0x7FFFFFFFu, v.w & 0x7FFFFFFFu));
    };
    int i = tid;
    for (; i + 3 * NT < n4; i += 4 * NT) {
      const uint4 v0 = y[i], v1 = y[i + NT], v2 = y[i + 2 * NT], v3 = y[i + 3 * NT];
      m = m4(m4(m4(m4(m, v0), v1), v2), v3);
    }
    for (; i < n4; i += NT) m = m4(m, y[i]);
    return amax_wg(m);
  };
  const int kx = amax_exp(amax_slots(a.amax_x));
  const int ky = amax_exp(a.self_dy ? amax_dy_self() : amax_slots(a.amax_dy));
  const float xsc = exp2i(kx), ysc = exp2i(ky);
  // dY3 rows 25..31 (the k-step's padding) are zero and never written
  for (int f = tid; f < (G::KP - G::NPY) * G::PY / 16; f += NT)
    reinterpret_cast<uint4*>(ys + G::NPY * G::PY)[f] = make_uint4(0, 0, 0, 0);

  // tr-read lane roles (as wgrad6_body): group g = lane >> 4, K row q, channel quad pq; this
  // lane's pixel rows are kperm and kperm + 8 of the 32
  const int g = lane >> 4, q = (lane >> 2) & 3, pq = lane & 3;
  const int kperm = 16 * (g >> 1) + 4 * (g & 1) + q;
  int xb[2], yb[2];
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int p = kperm + 8 * r;
    yb[r] = p * G::PY + 8 * pq;
    const int pc = p < G::NPY ? p : 0;                   // dY3 is zero there
    xb[r] = ((pc / 5) * 7 + pc % 5) * G::PX + 8 * pq;
  }

  f32x4 acc[9][2];
#pragma unroll
  for (int j = 0; j < 9; ++j) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};

  float4 xv[XPT], yv[YPT];
  // NT = 256: branch-free (ld4 reads zeros for a rejected element), so the loads stay in flight
  // together; the 512-thread kernel keeps the selects (branch-free measured 0.0242 -> 0.0256 ms)
  auto load = [&](int img) {
    const float4* x4 = reinterpret_cast<const float4*>(a.x);
    const float4* y4 = reinterpret_cast<const float4*>(a.dy);
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int f = tid + NT * i;
      const bool ok = img < a.batch && f < G::NV4X;
      if constexpr (NT == 256) xv[i] = ld4(a.x + ((size_t)img * G::NV4X + f) * 4, ok);
      else xv[i] = ok ? x4[(size_t)img * G::NV4X + f] : f4zero();
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + NT * i;
      const bool ok = img < a.batch && f < G::NV4Y;
      if constexpr (NT == 256) yv[i] = ld4(a.dy + ((size_t)img * G::NV4Y + f) * 4, ok);
      else yv[i] = ok ? y4[(size_t)img * G::NV4Y + f] : f4zero();
    }
  };
  load(bx);
  for (int img = bx; img < a.batch; img += gx) {
    __syncthreads();                                     // the previous image's reads are done
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int f = tid + NT * i;
      if (f < G::NV4X) {
        uint32_t s0[2], s1[2];
        SP::split(xv[i].x, xv[i].y, xsc, s0);
        SP::split(xv[i].z, xv[i].w, xsc, s1);
        char* p = xs + (f >> 4) * G::PX + (f & 15) * 8;
        *reinterpret_cast<uint2*>(p) = make_uint2(s0[0], s1[0]);
        *reinterpret_cast<uint2*>(p + G::SPB) = make_uint2(s0[1], s1[1]);
      }
    }
#pragma unroll
    for (int i = 0; i < YPT; ++i) {
      const int f = tid + NT * i;
      if (f < G::NV4Y) {
        uint32_t s0[2], s1[2];
        SP::split(yv[i].x, yv[i].y, ysc, s0);
        SP::split(yv[i].z, yv[i].w, ysc, s1);
        char* p = ys + (f >> 4) * G::PY + (f & 15) * 8;
        *reinterpret_cast<uint2*>(p) = make_uint2(s0[0], s1[0]);
        *reinterpret_cast<uint2*>(p + G::SPB) = make_uint2(s0[1], s1[1]);
      }
    }
    __syncthreads();
    load(img + gx);                                      // in flight during the MFMAs

    u32x4 b[2][2];
#pragma unroll
    for (int nl = 0; nl < 2; ++nl)
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const int off = (2 * nh + nl) * 32 + sp * G::SPB;
        const uint2 u0 = lds_tr16(ys + yb[0] + off), u1 = lds_tr16(ys + yb[1] + off);
        b[nl][sp] = u32x4{u0.x, u0.y, u1.x, u1.y};
      }
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int mb = 9 * mg + j, tap = mb >> 2, cb = mb & 3;
      const int toff = ((tap / 3) * 7 + tap % 3) * G::PX + cb * 32;
      u32x4 av[2];
#pragma unroll
      for (int sp = 0; sp < 2; ++sp) {
        const uint2 u0 = lds_tr16(xs + xb[0] + toff + sp * G::SPB), u1 = lds_tr16(xs + xb[1] + toff + sp * G::SPB);
        av[sp] = u32x4{u0.x, u0.y, u1.x, u1.y};
      }
#pragma unroll
      for (int pr = 0; pr < SP::NPROD; ++pr)
#pragma unroll
        for (int nl = 0; nl < 2; ++nl) acc[j][nl] = SP::mfma(av[SP::pa(pr)], b[nl][SP::pb(pr)], acc[j][nl]);
    }
  }
  // the partial slab (16x16 C layout: lane holds column li, rows 4 lq + r), unscaled by two
  // exact power-of-two products
  const float u1 = exp2i(-kx), u2 = exp2i(-ky);
  const int li = lane & 15, lq = lane >> 4;
  float* slab = a.part + (size_t)bx * G::M * G::N;
#pragma unroll
  for (int j = 0; j < 9; ++j)
#pragma unroll
    for (int nl = 0; nl < 2; ++nl)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = (9 * mg + j) * 16 + 4 * lq + r, n = (2 * nh + nl) * 16 + li;
        slab[m * G::N + n] = acc[j][nl][r] * u1 * u2;
      }
}

#if BA3C_SHARED_KERNELS  // non-template kernel: emitted by ba3c_capi.hip only
__global__ void __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2))) conv3_wgrad_kernel(const Conv3WArgs a) {
  __shared__ uint4 lds4[(Conv3WG::X_BYTES + Conv3WG::Y_BYTES) / 16];
  __shared__ uint32_t red8[8];
  conv3_wgrad_body<512>(a, blockIdx.x, gridDim.x, 0, reinterpret_cast<char*>(lds4), red8);
}
#endif

// the 256-thread weight gradient as a multi-job launch job: x = slab (first image), y = n-half
struct Conv3WJob {
  using Args = Conv3WArgs;
  static constexpr int LDS = Conv3WG::X_BYTES + Conv3WG::Y_BYTES;
  __device__ static void run(const Args& a, int x, int y, int, int gx, char* lds, uint32_t* red4) {
    conv3_wgrad_body<256>(a, x, gx, y, lds, red4);
  }
};

}  // namespace ba3c
