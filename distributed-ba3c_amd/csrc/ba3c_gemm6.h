// ba3c_gemm6.h — the implicit-GEMM engine of ba3c_gemm.h on bf16 MFMA with fp32-accurate
// operand splitting (conv3 fwd/dgrad/wgrad, fc1 fwd/dgrad/wgrad, head wgrad).
//
// Same problem structs (ba3c_problems.h: gathers, unpooling, fused epilogues), same tiles
// and split-K, same 32x32 accumulator layout — only the product changes: every fp32 operand
// value is split exactly into bf16 hi + mid + lo (split3x2, ba3c_split.h) as it is staged,
// and each 32x32x16 block product is the six bf16 MFMAs a1b1, a1b2, a2b1, a1b3, a2b2, a3b1
// (v_mfma_f32_32x32x16_bf16, fp32 accumulation; the dropped terms are below 2^-23 relative).
// Per unit of K that is 6 x 32 cycles per 16 K against 64 cycles per 2 K for
// v_mfma_f32_32x32x2_f32: 2.7x the fp32-MFMA rate, and 2.7x shorter dependent MFMA chains for
// the small-batch (latency-bound) launches.  bf16 keeps fp32's exponent range, so these
// kernels need no operand scaling.
//
// LDS, per operand and split plane (bf16):
//  * k-contiguous gathers (a float4 = 4 K of one row): [row][BK], 80-byte row pitch; a lane of
//    the 32x32x16 MFMA supplies row (l & 31) and K 8 (l >> 5) + 0..7 — one ds_read_b128 (the
//    eight 16-byte reads of a lane octet hit disjoint banks);
//  * row-contiguous gathers (a float4 = 4 rows at one K): [BK][rows] with a pitch = 64 or 192
//    (mod 256) bytes, stored with one ds_write_b64 per float4 and plane, and read with two
//    ds_read_b64_tr_b16 (hardware transpose: lane 4q + p of a 16-lane group addresses K row q,
//    rows 4p..4p+3 of the operand; lane i receives operand row i of the 4 K rows) — the
//    4 K rows of each 32-lane half land in 4 distinct 64-byte bank windows.
#pragma once
#include "ba3c_gemm.h"
#include "ba3c_split.h"
#include "ba3c_wgrad6.h"   // lds_tr16

namespace ba3c {

typedef __bf16 bf16x8v __attribute__((ext_vector_type(8)));

constexpr int G6_RP = GEMM_BK * 2 + 16;
  // row pitch (bytes) of a k-contiguous plane
// K-row pitch of a transposed plane of `rows` operand rows: 64 or 192 mod 256 bytes
constexpr int tr_pitch(int rows) { return rows * 2 + (64 - (rows * 2) % 128 + 128) % 128; }

// G6_DEPTH: k-tiles in flight per thread (register ring); 2 = classic one-ahead prefetch.
// Small-batch launches (a few workgroups walking a long K each) take 4, large ones 2 (the
// deeper ring's registers cost occupancy that the big launches need more).
template <int BM, int BN, class P>
struct Gemm6Lds {
  static constexpr int TPA = tr_pitch(BM), TPB = tr_pitch(BN);
  static constexpr int PA = P::A_KCONTIG ? BM * G6_RP : GEMM_BK * TPA;
  static constexpr int PB = P::B_KCONTIG ? BN * G6_RP : GEMM_BK * TPB;
  static constexpr int BYTES = 3 * (PA + PB);
};

// (bx, by, bz): the output tile and K chunk (blockIdx of a plain launch; ba3c_multi.h passes
// its own); lds: KS * Gemm6Lds<BM, BN, P>::BYTES, 16-byte aligned.
// KS = 2: 512 threads, two groups of 4 waves split the tile's k-tiles in halves (group 0 the
// first ceil(n/2), group 1 the rest, each with its own staging LDS and the same trip count),
// and group 0 adds group 1's accumulators (acc0 + acc1) before the epilogue.  Small launches
// (a few workgroups walking a long K) run their serial k-tile chain at half the length.
// PAR: the k-tiles split by parity instead of in halves — KS = 2: group g takes tiles g, g + 2,
// ...; KS = 1: even tiles into one accumulator set and odd ones into a second (compile-time:
// G6_DEPTH is even), added at the end.  Both forms compute (sum of even tiles) + (sum of odd
// tiles) with the same order inside each sum, so a problem can run two groups at small batches
// and one at large ones with every output rounded the same.
template <int BM, int BN, int WGM, int WGN, class P, int G6_DEPTH = 2, int KS = 1, bool PAR = false>
__device__ __forceinline__ void gemm6_body(const P& p, int bx, int by, int bz, char* lds) {
  static_assert(WGM * WGN == 4, "4 waves per group");
  static_assert(KS == 1 || KS == 2, "k groups");
  static_assert(!PAR || G6_DEPTH % 2 == 0, "parity sets need an even ring depth");
  constexpr int NSET = PAR && KS == 1 ? 2 : 1;
  constexpr int BK = GEMM_BK;
  constexpr int WTM = BM / WGM, WTN = BN / WGN;
  constexpr int TM = WTM / 32, TN = WTN / 32;
  static_assert(TM >= 1 && TN >= 1 && WTM % 32 == 0 && WTN % 32 == 0, "wave tile");
  constexpr int NA = BM * BK / 4 / GEMM_THREADS;
  constexpr int NB = BN * BK / 4 / GEMM_THREADS;
  static_assert(NA >= 1 && NB >= 1, "tile too small for 256 threads");
  constexpr int QA = BM / 4, QB = BN / 4;
  constexpr int RA = GEMM_THREADS / QA, RB = GEMM_THREADS / QB;
  // plane bytes and pitches of the two operands (see the layout note above)
  constexpr int TPA = Gemm6Lds<BM, BN, P>::TPA, TPB = Gemm6Lds<BM, BN, P>::TPB;
  constexpr int PA = Gemm6Lds<BM, BN, P>::PA, PB = Gemm6Lds<BM, BN, P>::PB;
  const int grp = KS == 2 ? (int)(threadIdx.x >> 8) : 0;
  char* As = lds + grp * 3 * (PA + PB);
  char* Bs = As + 3 * PA;

  const int tid = threadIdx.x & 255;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave / WGN, wn = wave % WGN;
  const int m0 = bx * BM;
  const int n0 = by * BN;
  int kbeg = 0, kend = p.K;
  if (p.kchunk > 0) {
    kbeg = bz * p.kchunk;
    kend = min(p.K, kbeg + p.kchunk);
  }
  // k-tiles of this group; both groups run the same trip count (a tile past the group's
  // kend reads the zero block)
  int ntiles = (kend - kbeg + BK - 1) / BK;
  // k offset of this group's i-th tile (PAR, KS = 2: tile 2 i + grp; past kend: the zero block)
  int kstep = BK;
  if constexpr (KS == 2 && PAR) {
    ntiles = (ntiles + 1) / 2;
    kbeg += grp * BK;
    kstep = 2 * BK;
  } else if constexpr (KS == 2) {
    ntiles = (ntiles + 1) / 2;
    kbeg += grp * ntiles * BK;
    kend = min(kend, kbeg + ntiles * BK);
  }

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

  // register ring of G6_DEPTH k-tiles: the loads of tile t + G6_DEPTH - 1 are issued before
  // tile t is staged, so G6_DEPTH - 1 tiles of global-load latency overlap the MFMA loop (the
  // small-batch launches have a few workgroups each walking a long K: one exposed load round
  // trip per k-tile was their whole time).  Stage indices are compile-time after unrolling.
  typename P::ARaw ra[G6_DEPTH][NA];
  typename P::BRaw rb[G6_DEPTH][NB];
  auto load = [&](int st, int k0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (P::A_KCONTIG)
        ra[st][i] = p.a_load(arow[i], k0 + (tid & 7) * 4, kend);
      else
        ra[st][i] = p.a_load_t(arow[0], k0 + tid / QA + RA * i, kend);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (P::B_KCONTIG)
        rb[st][i] = p.b_load(brow[i], k0 + (tid & 7) * 4, kend);
      else
        rb[st][i] = p.b_load_t(brow[0], k0 + tid / QB + RB * i, kend);
    }
  };
  // split a float4 into 3 planes and store it (8 bytes per plane): KC -> 4 K of row r at
  // [r][k]; !KC -> rows r..r+3 at K row k of the transposed image [k][r] (pitch tp)
  auto put = [&](char* base, int plane_bytes, bool kc, int tp, int r, int k, const float4& v) {
    uint32_t h0, m0_, l0, h1, m1, l1;
    split3x2(v.x, v.y, h0, m0_, l0);
    split3x2(v.z, v.w, h1, m1, l1);
    const uint32_t hs[3][2] = {{h0, h1}, {m0_, m1}, {l0, l1}};
    const int off = kc ? r * G6_RP + k * 2 : k * tp + r * 2;
#pragma unroll
    for (int s = 0; s < 3; ++s)
      *reinterpret_cast<uint2*>(base + s * plane_bytes + off) = make_uint2(hs[s][0], hs[s][1]);
  };
  auto store = [&](int st) {
    if constexpr (G6_DEPTH > 2) {
#pragma unroll
      for (int i = 0; i < NA; ++i) pin(ra[st][i]);
#pragma unroll
      for (int i = 0; i < NB; ++i) pin(rb[st][i]);
    }
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      if constexpr (P::A_KCONTIG)
        put(As, PA, true, TPA, (tid >> 3) + 32 * i, (tid & 7) * 4, fin(ra[st][i]));
      else
        put(As, PA, false, TPA, (tid % QA) * 4, tid / QA + RA * i, fin(ra[st][i]));
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      if constexpr (P::B_KCONTIG)
        put(Bs, PB, true, TPB, (tid >> 3) + 32 * i, (tid & 7) * 4, fin(rb[st][i]));
      else
        put(Bs, PB, false, TPB, (tid % QB) * 4, tid / QB + RB * i, fin(rb[st][i]));
    }
  };

  f32x16 accs[NSET][TM][TN];
#pragma unroll
  for (int q = 0; q < NSET; ++q)
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) accs[q][a][b][r] = 0.f;
  f32x16 (&acc)[TM][TN] = accs[0];

  const int li = lane & 31, lh = lane >> 5;
  // fragment base of this lane: row reads at [row li][K 8 lh]; transposed reads: lane 4q + p
  // of group g = lane >> 4 addresses K row 8 (g >> 1) + q (+ 4 for the second read), operand
  // rows 16 (g & 1) + 4p .. + 3
  const int tg = lane >> 4, tq = (lane >> 2) & 3, tpp = lane & 3;
  const int tr_row = 8 * (tg >> 1) + tq, tr_col = 16 * (tg & 1) + 4 * tpp;
  const char* Aw = P::A_KCONTIG ? As + (wm * WTM + li) * G6_RP + lh * 16
                                : As + tr_row * TPA + (wm * WTM + tr_col) * 2;
  const char* Bw = P::B_KCONTIG ? Bs + (wn * WTN + li) * G6_RP + lh * 16
                                : Bs + tr_row * TPB + (wn * WTN + tr_col) * 2;
  // one 32x32x16 operand fragment (8 K of one row) of block a at k-step ks
  auto frag = [](const char* w, bool kc, int tp, int blk, int ks) -> bf16x8v {
    if (kc) return __builtin_bit_cast(bf16x8v, *reinterpret_cast<const uint4*>(w + blk * 32 * G6_RP + ks * 32));
    const char* q = w + ks * 16 * tp + blk * 64;
    const uint2 u0 = lds_tr16(q), u1 = lds_tr16(q + 4 * tp);
    return __builtin_bit_cast(bf16x8v, u32x4{u0.x, u0.y, u1.x, u1.y});
  };

  auto tile = [&](int k0, f32x16 (&ac)[TM][TN]) {
#pragma unroll
    for (int ks = 0; ks < BK / 16; ++ks) {
      bf16x8v av[3][TM], bv[3][TN];
#pragma unroll
      for (int s = 0; s < 3; ++s) {
#pragma unroll
        for (int a = 0; a < TM; ++a) av[s][a] = frag(Aw + s * PA, P::A_KCONTIG, TPA, a, ks);
#pragma unroll
        for (int b = 0; b < TN; ++b) bv[s][b] = frag(Bw + s * PB, P::B_KCONTIG, TPB, b, ks);
      }
      // a1b1, a1b2, a2b1, a1b3, a2b2, a3b1 (SplitP<3> order), interleaved over the blocks
      constexpr int PA_[6] = {0, 0, 1, 0, 1, 2}, PB_[6] = {0, 1, 0, 2, 1, 0};
#pragma unroll
      for (int pr = 0; pr < 6; ++pr)
#pragma unroll
        for (int a = 0; a < TM; ++a)
#pragma unroll
          for (int b = 0; b < TN; ++b)
            ac[a][b] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[PA_[pr]][a], bv[PB_[pr]][b], ac[a][b], 0, 0, 0);
    }
  };

  // Prologue loads and the steady-state prefetches are unconditional (a tile past kend reads
  // the zero block): a conditionally issued load leaves the compiler unsure how many loads are
  // outstanding where the paths join, and it then waits for all of them.  Full groups of
  // G6_DEPTH tiles (the last may be partial: its loads mask k >= kend) run branch-free; the
  // < G6_DEPTH tail tiles are already in the ring.
#pragma unroll
  for (int st = 0; st < G6_DEPTH - 1; ++st) load(st, kbeg + st * kstep);
  int it = 0;
  for (; it + G6_DEPTH - 1 < ntiles; it += G6_DEPTH) {   // >= G6_DEPTH tiles left
    const int kk = kbeg + it * kstep;
#pragma unroll
    for (int st = 0; st < G6_DEPTH; ++st) {
      // sched barriers: the split arithmetic of a later stage would otherwise be hoisted to
      // the top of the group, waiting for loads that are meant to stay in flight
      __builtin_amdgcn_sched_barrier(0);
      load((st + G6_DEPTH - 1) % G6_DEPTH, kk + (st + G6_DEPTH - 1) * kstep);
      store(st);
      __syncthreads();
      tile(kk + st * kstep, accs[st % NSET]);   // (it is a multiple of the even depth)
      __syncthreads();
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int st = 0; st < G6_DEPTH - 1; ++st) {
    if (it + st < ntiles) {                    // uniform
      store(st);
      __syncthreads();
      tile(kbeg + (it + st) * kstep, accs[st % NSET]);
      __syncthreads();
    }
  }
  if constexpr (NSET == 2) {                   // (even tiles) + (odd tiles)
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = accs[0][a][b][r] + accs[1][a][b][r];
  }

  if constexpr (KS == 2) {
    // group 1 hands its accumulators to group 0 through LDS (lane-major: conflict-free)
    float* xch = reinterpret_cast<float*>(lds);
    constexpr int NV = TM * TN * 16;
    static_assert(NV * 256 * 4 <= 3 * (PA + PB), "exchange fits a group's staging LDS");
    if (grp == 1) {
#pragma unroll
      for (int a = 0; a < TM; ++a)
#pragma unroll
        for (int b = 0; b < TN; ++b)
#pragma unroll
          for (int r = 0; r < 16; ++r) xch[((a * TN + b) * 16 + r) * 256 + tid] = acc[a][b][r];
    }
    __syncthreads();
    if (grp == 1) return;
#pragma unroll
    for (int a = 0; a < TM; ++a)
#pragma unroll
      for (int b = 0; b < TN; ++b)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[a][b][r] = acc[a][b][r] + xch[((a * TN + b) * 16 + r) * 256 + tid];
  }
  p.template epilogue<TM, TN>(acc, m0 + wm * WTM, n0 + wn * WTN, lane, bz);
}

template <int BM, int BN, int WGM, int WGN, class P, int G6_DEPTH = 2, int KS = 1, bool PAR = false>
__global__ void __launch_bounds__(GEMM_THREADS * KS) gemm6_kernel(const P p) {
  __shared__ __attribute__((aligned(16))) char lds[KS * Gemm6Lds<BM, BN, P>::BYTES];
  gemm6_body<BM, BN, WGM, WGN, P, G6_DEPTH, KS, PAR>(p, blockIdx.x, blockIdx.y, blockIdx.z, lds);
}

}  // namespace ba3c
