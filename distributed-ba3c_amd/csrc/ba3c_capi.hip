// ba3c_capi.hip — C ABI (include/ba3c.h) and step orchestration of libba3c.so.
//
// One call of ba3c_train_grads runs, on the caller's stream, the whole tower of
// train.py:164-327 plus its TF autodiff (train/multigpu.py:85-86):
//   conv0..conv3 forward (ReLU, max-pool + argmax codes fused), fc1, heads+softmax+loss,
//   then backward: head/fc1/conv weight gradients (split-K MFMA + deterministic reduce)
//   and input gradients (MFMA dgrad with MaxPoolGrad/ReluGrad fused into the loaders).
// No device allocation and no synchronisation happen inside any entry point.
#include <hip/hip_runtime.h>
#include <dlfcn.h>
#include <rccl/rccl.h>   // types only: the functions are resolved from the loaded RCCL (dlsym)

#include <cmath>
#include <cstdio>
#include <cstring>
#include <optional>
#include <string>
#include <vector>

#include "../../include/ba3c.h"
#include "ba3c_band6.h"
#include "ba3c_conv.h"
#include "ba3c_conv3.h"
#include "ba3c_dgrad1s.h"
#include "ba3c_gemm6.h"
#include "ba3c_launch.h"
#include "ba3c_multi.h"
#include "ba3c_problems.h"
#include "ba3c_rollout.h"
#include "ba3c_small.h"
#include "ba3c_split.h"
#include "ba3c_wgrad6.h"

using namespace ba3c;

// The TfDictOp scalar reduction (scalars_block) as one workgroup of a multi-job launch: at
// large batches it rides on conv3's input-gradient launch instead of its own dependent
// launch after the heads (nothing in the step reads the scalars).
struct ScalarsJob {
  struct Args {
    const float* terms;
    int B;
    float beta;
    const unsigned long long* relu;
    double* out;
  };
  static constexpr int LDS = 0;
  __device__ static void run(const Args& a, int, int, int, int, char*, uint32_t*) {
    scalars_block(a.terms, a.B, a.beta, a.relu, a.out);
  }
};

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_TRY(expr)                                                                      \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess)                                                                  \
      return fail(BA3C_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(_e));        \
  } while (0)

#ifndef BA3C_WGRAD_TARGET
#define BA3C_WGRAD_TARGET 1024   // split-K workgroups a GEMM-engine weight gradient aims for (A/B)
#endif
constexpr int kWgradTargetBlocks = BA3C_WGRAD_TARGET;
constexpr int kMaxBatch = 16384;

inline int64_t align64(int64_t x) { return (x + 63) & ~int64_t(63); }
inline size_t align256(size_t x) { return (x + 255) & ~size_t(255); }

}  // namespace

struct TensorDesc {
  std::string name;
  int64_t offset;
  int64_t numel;
  int32_t shape[4];
  int32_t ndim;
};

constexpr int CHAIN_SITES = 2;   // chained launch sites (launch_chain)
constexpr int CHAIN_SPREAD = 32; // spread signal counters of a site with many signalling workgroups

struct ba3c_handle {
  ba3c_config cfg;
  std::vector<TensorDesc> tensors;
  int64_t flat;
  int idx_conv[4];
  int idx_fc1;        // first fc1 tensor
  int idx_piW, idx_pib, idx_vW, idx_vb;
  int per, wstride;
  TensorTable table;
  // split-MFMA kernels (band convolutions, conv0, weight gradients, the bf16x6 GEMM engine);
  // BA3C_GENERIC=1: every convolution and GEMM on the fp32-MFMA GEMM engine instead (a
  // parity configuration with exact fp32 products)
  bool band = true;
  // large batches: conv1's weight gradient shares a launch with (2, default) conv0's weight
  // gradient, (1) conv1's input gradient, or (0) runs alone (BA3C_C1PAIR)
  int c1pair = 2;
  uint32_t merged[BA3C_NUM_KERNELS] = {};   // ba3c_kernel_merged, per training pass
  // large-batch (B > OVERLAP_B) scalar reduction deferred from run_heads onto conv3's
  // input-gradient launch as one extra workgroup (default; also across the phase-1/phase-2
  // split of the N>1 step); when no launch takes it, finish() launches it at the end of phase
  // 0 or phase 2.  BA3C_SCALARS_RIDE=0: its own launch after the heads.
  // r04 same-box A/B: step 1.954 -> 1.935 ms
  bool scalars_ride = true;
  bool pend_scalars = false;
  ScalarsJob::Args scalars_args{};
  // conv1 fwd / dgrad (multi-band layouts) as ring-walk persistent kernels at batches that
  // give every workgroup whole images (conv_band6r_kernel; BA3C_RING=0: one band per workgroup)
  bool ring = true;
  int cus = 256;      // compute units of the device (persistent grids)
  bool g6 = true;     // implicit-GEMM launches (conv3, fc1, heads; C=12 conv0) on bf16x6 split
                      // MFMA (ba3c_gemm6.h; off with BA3C_GENERIC=1: fp32 MFMA)
  // backward weight gradients on a side stream (created on the first training call that is
  // not being captured): 0 never (BA3C_OVERLAP=0), 1 always (BA3C_OVERLAP=1), 2 (default) for
  // batches <= OVERLAP_B only.  Large batches: r01t/u measured +0.5% step throughput (561k vs
  // 557k samples/s) because conv1's dgrad and wgrad kernels each fill the chip, and concurrent
  // kernels make the per-kernel durations (roofline, rocprof) meaningless.  Small batches: each
  // backward kernel is a few latency-bound workgroups, so the weight-gradient chain runs in
  // the input-gradient chain's shadow.
  int overlap = 2;
  // batches <= OVERLAP_B on the split path: each layer's input- and weight-gradient kernels
  // run as ONE multi-job launch (ba3c_multi.h) on the main stream instead of on two streams
  // joined by events (r02k trace at B=32: 6-11 us of idle queue per fork / join).
  // BA3C_MULTI=0: side stream as before.
  bool multi = true;
  // Backward pairs run as multi-job launches at batches > OVERLAP_B too (BA3C_MULTI_BIG bits:
  // 1 fc1 + heads — r02x at B=2048, 84 -> 64 us for the three products; 2 conv2 — r02aa, 300 ->
  // 292 us).  conv3's pair measured slower there (116 -> 134 us), and conv1's products stay
  // on their own (the dominant kernel's roofline probe needs conv1 dgrad alone).
  int multi_big = 3;
  // fused-clip optimizer applies as one clip_update_kernel launch (ba3c_small.h) when the chunk
  // count fits one workgroup per CU; its grid-barrier words live in `bar` (device, zeroed at
  // create).  BA3C_FUSED_UPDATE=0: sumsq_kernel + update_kernel.
  bool fused_update = true;
  // clip_update_kernel's tagged partials (nchunks words) + error flag: device, zeroed at create;
  // clip_range_kernel's (a generation space of their own) follow them
  unsigned long long* utag = nullptr;
  unsigned long long* ctag = nullptr;
  // chained multi-job launches (ba3c_multi.h: an in-launch dependency instead of a kernel
  // boundary): CHAIN_SITES x 4 words + an error word after the tags (null: no device memory,
  // unchained launches).  BA3C_CHAIN=0: unchained.
  bool chain_on = true;
  unsigned* chain = nullptr;
  unsigned* spread = nullptr;   // CHAIN_SPREAD counters, CHAIN_STRIDE words apart (64-byte aligned)
  // conv1's input gradient on 2:4-sparse MFMA (ba3c_dgrad1s.h) at the ring-walk batches
  // (B >= 2 x CUs) with BA3C_C1D_SPARSE=1; default 0, the dense ring walk: the sparse kernel
  // issues 40 % fewer matrix instructions but measured 0.40 against 0.33 ms (r05x-y: its L2
  // weight-fragment stream and its staging, which two workgroups per CU do not hide, cost
  // 0.07 and 0.13 ms)
  bool c1s = false;
  // BA3C_DYNQ=1: ring walks with several images per workgroup draw their images after the
  // first from a dynamic queue (Band6Args::ticket) instead of static contiguous ranges;
  // bit-identical either way.  Default 0: same-box r06g, the queue costs ~9 us per step with
  // the chip to itself (conv1 fwd + dgrad), and with 16 CUs held for 50 us by a stand-in for
  // RCCL (bench --occupy) conv1 dgrad's slowdown is the same 1.08 either way; it only pays when
  // CUs are held for the whole launch (1.55 -> 1.14)
  bool dynq = false;
  // BA3C_C3W_RIDE (large batches, conv2's gradients in one multi-job launch): conv3's weight
  // gradient as a third job of that launch instead of a launch of its own (two 256-thread
  // workgroups per slab, bit-identical slabs); 1: after conv2's jobs, 2: before them, 0: own
  // launch (default: r06n, conv2's launch grows by conv3's whole 22 us either way, since both
  // fill every workgroup slot; the step gains 0-3 us, within box noise)
  int c3ride = 0;
  // ba3c_train_grads_phase(phase 3): the pass's weight-gradient reduction is left pending and
  // the next fused-clip apply on the handle runs it as the signalling job of a chained launch
  // (reduce -> clip + update, one launch fewer); any other entry point launches it first
  bool pend_reduce = false;
  hipStream_t pend_stream = nullptr;
  const float* pend_grads = nullptr;
  hipEvent_t ev_pend = nullptr;   // orders a flush on the pass's stream before another stream
  bool defer_final = false;   // set by train_grads_impl for phase 3
  // phase 4 (phase 1 with its reduction held): the fc1 + heads weight-gradient reduction is
  // kept here, unlaunched, until ba3c_launch_held puts it on the caller's stream (the exchange
  // stream of the N>1 step); phase 2 does not launch it, every other entry point does
  bool held = false;
  hipStream_t held_stream = nullptr;
  ReduceJobs held_jobs{};
  // recorded on the pass's stream after conv3's gradient launches of every phase-2 pass
  // (ba3c_set_phase2_event; null: none)
  hipEvent_t ev_mid = nullptr;
  hipStream_t side = nullptr;
  hipEvent_t ev_fork[4] = {}, ev_join = nullptr;
  // weight-gradient reductions of the running backward pass, launched together at its end
  bool defer_reduce = false;
  ReduceJobs rjobs{};
  // RCCL communicator of the C-ABI gradient exchange (ba3c_comm_init; null: none)
  ncclComm_t comm = nullptr;
  int comm_ranks = 0;
  // timing probe
  int probe_kernel = -1;
  std::vector<hipEvent_t> ev_begin, ev_end;
  int probe_used = 0;
  int probe_every = 1;        // ba3c_probe_every: bracket one launch in `probe_every`
  unsigned probe_seen = 0;    // launches of probe_kernel since ba3c_probe_enable
  int probe_launches = 0;
  double probe_ms = 0.0;
};

namespace {

// ---- workspace layout -----------------------------------------------------------------
// band-conv geometries (ba3c_conv.h): forward conv1/conv2 with pooling, and the input
// gradients of conv1/conv2 as VALID convs over the 4-padded un-pooled output gradient
using GConv1F = BandGeom<40, 40, 32, 32, 5, 5, 6, true, 0, 4>;
using GConv2F = BandGeom<18, 18, 32, 64, 5, 5, 14, true, 0, 4>;
using GConv1D = BandGeom<44, 44, 32, 32, 5, 5, 4, false, 1, 8, 4, 4, 18, 18, 36, 36>;
using GConv2D = BandGeom<22, 22, 64, 32, 5, 5, 6, false, 1, 8, 4, 4, 7, 7, 14, 14>;
// split-family variants (ba3c_band6.h): pixel pitch / extra row bytes from a bank-conflict
// search (scripts/lds_bank_search.py), per family (3 bf16 planes or 2 fp16 planes per pixel)
//  C2D: conv2 input gradient, the whole 18x18 map per workgroup in two 32-channel phases
//       (r01r: 0.44 ms at 6-row bands -> 0.31 ms: no halo re-staging, 11 m-blocks per wave
//       hide the weight-fragment latency; 6 and 9-row bands and 8-row conv1 / 12-row
//       conv1-fwd bands measured slower)
//  C2FS / C2DS: small batches (B <= SMALL_B, e.g. configs[1]'s B=32): conv2 forward / input
//       gradient in 2- / 3-row bands, so the launch has 7x / 6x the workgroups of the
//       whole-map kernels — at B=32 those are 32 workgroups on 256 CUs, one latency-bound
//       wave of work.  Every output's K order (phase, tap, channel chunk, product) is the same
//       in both geometries, so results are bit-identical across the switch.
constexpr int SMALL_B = 128;
constexpr int OVERLAP_B = 128;   // default side-stream weight gradients up to this batch
using GConv2DW = BandGeom<22, 22, 64, 32, 5, 5, 18, false, 1, 8, 4, 4, 7, 7, 14, 14>;
using GConv2FS = BandGeom<18, 18, 32, 64, 5, 5, 2, true, 0, 4>;
using GConv2DS = BandGeom<22, 22, 64, 32, 5, 5, 3, false, 1, 8, 4, 4, 7, 7, 14, 14>;
// split-kernel layouts (scaled fp16 hi/lo planes)
struct Lay {
  using C1F = Band6<GConv1F, 160, 128, 7, 0, 2, true>;
  using C2F = Band6<GConv2F, 160, 64, 7, 0, 2>;   // (double-buffered: 256 VGPRs, neutral, r04)
#ifndef BA3C_C1D_TILE4
#define BA3C_C1D_TILE4 1
#endif
#if BA3C_C1D_TILE4
  using C1D = Band6<GConv1D, 160, 0, 5, 0, 2, true, true>;   // 4x4 tiles: RP = 128 mod 256 B
#else
  using C1D = Band6<GConv1D, 160, 128, 5, 0, 2, true>;
#endif
#ifndef BA3C_C2D_PADSKIP
#define BA3C_C2D_PADSKIP 1
#endif
#ifndef BA3C_C2D_DBUF
#define BA3C_C2D_DBUF 0
#endif
  using C2D = Band6<GConv2DW, 160, 128, 11, 32, 2, BA3C_C2D_DBUF, false, BA3C_C2D_PADSKIP>;
  using C2FS = Band6<GConv2FS, 160, 64, 2, 0, 2, true>;
  using C2DS = Band6<GConv2DS, 160, 128, 2, 32, 2, true>;
  using W1 = Wg6Geom<40, 40, 32, 32, 4, 16, 32, 96, 160, 2>;
  using W2 = Wg6Geom<18, 18, 32, 64, 14, 16, 32, 96, 160, 2>;
  using W1W = Wg6WGeom<40, 40, 32, 32, 4, 160, 160>;   // conv1, B >= W6W_MIN_B (76.8 KB LDS)
};
// persistent grid bound of conv1's partial slabs
constexpr int WG_P1 = 512;
constexpr int W6_P1 = 256, W6_P2 = 128;   // x (c-groups x o-groups) = 512 workgroups
// conv1 weight-gradient workgroups: ~4 bands each, at least 64 (at B=32 one band per
// workgroup made 256 partial slabs of 100 KB — 26 MB written and read back by the reduction
// for 3.3 MB of input).  A function of B alone, so every launch path sums the same slabs.
#ifndef BA3C_C1W_BPW
#define BA3C_C1W_BPW 3        // conv1 weight-gradient bands per workgroup below the ring sizes (r03: 4 -> 3, B=32 0.1966 -> 0.1925 ms)
#endif
inline int conv1_wgrad_p(int B) { return std::max(64, std::min(W6_P1, B * 9 / BA3C_C1W_BPW)); }
// conv1 weight gradient with all 32 input channels per workgroup (wgrad6w_kernel) from this
// batch on: whole images per workgroup, two workgroups per CU, one slab each
constexpr int W6W_MIN_B = 512, W6W_P = 512;
static_assert(W6W_P <= WG_P1, "conv1 partial slabs: the allocation covers WG_P1 slabs");
// its slab count: one per CU (whole images, B / CUs each) where the input gradient can run beside
// it in one launch (conv1_pair), else up to W6W_P; a function of B and the CU count alone, so
// the paired and the separate launches sum the same slabs bit for bit
inline bool conv1_pair_geometry(int B, int cus) { return B >= 2 * W6W_MIN_B && B % cus == 0 && cus <= WG_P1; }
inline int conv1_w6w_p(int B, int cus) { return conv1_pair_geometry(B, cus) ? cus : std::min(W6W_P, B); }
constexpr int FW_P0S = 512;   // conv0s_fwd_kernel: persistent, two workgroups per CU
constexpr int C3W_P = 256;    // conv3_wgrad_kernel: one 512-thread workgroup (and slab) per CU, at most
inline int conv3_wgrad_p(int B, int cus) { return std::min(B, std::min(C3W_P, cus)); }
constexpr int WG_P0S = 512;   // conv0s_wgrad_kernel: 52 KB LDS, two workgroups per CU
constexpr int WT_C1F = 0, WT_C2F = WT_C1F + 800 * 32, WT_C3F = WT_C2F + 800 * 64,
              WT_C1D = WT_C3F + 576 * 64, WT_C2D = WT_C1D + 800 * 32, WT_C3D = WT_C2D + 1600 * 32,
              WT_C1S = WT_C3D + 576 * 64, WT_C0F = WT_C1S + D1S::WPLANE,
              WT_C0S = WT_C0F + 32 * Conv0Geom::KDIM,            // uint4 [Conv0S::WB_U4]
              WT_TOTAL = WT_C0S + 4 * Conv0S::WB_U4;

// max-|x| slot arrays (ba3c_split.h, fp16 family)
enum { AM_P0 = 0, AM_P1 = 1, AM_DP0 = 2, AM_DP1 = 3, AM_DP2 = 4, AM_P2 = 5, AM_DY3 = 6, AMAX_N = 7 };
// dynamic image-queue tickets of the ring walks (Band6Args::ticket), right after the max slots
// so the step's weight-prep launch zeroes them with those
enum { TK_C1F = 0, TK_C1D = 1, TK_N = 4 };
struct Workspace {
  float *p0, *p1, *p2, *a3, *h, *fcpart, *dh, *dy3, *dp2, *dp1, *dp0, *dzv, *terms, *part0, *sumsq, *wt;
  // split-K / per-workgroup partial slabs of each weight gradient (reduced in one launch at the
  // end of the backward pass, so each layer needs a region of its own)
  float *part_h, *part_f, *part_3, *part_2, *part_1;
  uint16_t* wt6;   // [3][N][K] bf16 splits of the four band-conv weight copies
  uint8_t *c0, *c1, *c2;
  unsigned long long* relu;
  uint32_t* amax;  // [AMAX_N][1 + max_batch]: max |x| of split operands (global, per image)
  int* wexp;       // [8]: weight scale exponents (wprep jobs WJ_*, conv0 = WX_CONV0)
  size_t bytes;
  uint32_t* am(int t, const ba3c_handle* h) const { return amax + (size_t)t * (1 + h->cfg.max_batch); }
  unsigned* ticket(int k, const ba3c_handle* h) const { return amax + (size_t)AMAX_N * (1 + h->cfg.max_batch) + k; }
};
// weight-preparation jobs (forward copies first: inference prepares only those) and the
// index of each one's scale exponent in Workspace::wexp
enum { WJ_C1F = 0, WJ_C2F = 1, WJ_C3F = 2, WJ_C1D = 3, WJ_C2D = 4, WJ_C3D = 5, WJ_C1S = 6, WJ_N = 7, WJ_FWD = 3,
       WX_CONV0 = 7 };

struct WgradPlan {
  int M, N, K, S, kchunk, mt, nt;
};

WgradPlan plan_wgrad(int M, int N, int K, int BM, int BN, int target = kWgradTargetBlocks) {
  WgradPlan w;
  w.M = M;
  w.N = N;
  w.K = K;
  w.mt = (M + BM - 1) / BM;
  w.nt = (N + BN - 1) / BN;
  const int ktiles = (K + GEMM_BK - 1) / GEMM_BK;
  int S = (target + w.mt * w.nt - 1) / (w.mt * w.nt);
  S = std::max(1, std::min(S, (ktiles + 3) / 4));   // >= 4 k-tiles per split
  const int tiles_per = (ktiles + S - 1) / S;
  w.kchunk = tiles_per * GEMM_BK;
  w.S = (K + w.kchunk - 1) / w.kchunk;
  return w;
}

// fc1's backward at large batches (the multi-job launch): 128 x 128 tiles for the input and
// weight gradients instead of 64 x 64 / 128 x 64.  The engine splits every staged fp32 value
// into three bf16 planes (ba3c_gemm6.h), and at the small tiles that staging issued 10.8 VALU
// instructions per MFMA (PMC): four times the MFMAs per staged value.  The weight gradient
// takes fewer, longer K slabs (BA3C_FC1W_TARGET workgroups: 5 slabs at B = 2048, F = 512).
// Measured (r06v, r06w): the launch 0.0600 -> 0.0586 ms and the all-layer reduction 29.2 ->
// 28.0 us (half the fc1 slabs); not the 3x the VALU count suggested — the two workgroups per CU
// that 60 KB of LDS allows leave each k-tile's staging exposed, and 3- / 4-deep load rings
// (BA3C_FCD_DEPTH) made it 0.079 / 0.080 ms.
#ifndef BA3C_FC1_BIGTILE
#define BA3C_FC1_BIGTILE 1
#endif
#ifndef BA3C_FC1W_TARGET
#define BA3C_FC1W_TARGET 256
#endif
WgradPlan fc1w_plan(int F, int B, bool legacy, bool bigtile) {
  return bigtile ? plan_wgrad(1600 + (legacy ? 1 : 0), F, B, 128, 128, BA3C_FC1W_TARGET)
                 : plan_wgrad(1600 + (legacy ? 1 : 0), F, B, 128, 64);
}

// geometry constants (train.py:92, :177-212)
constexpr int P0 = 40 * 40 * 32, P1 = 18 * 18 * 32, P2 = 7 * 7 * 64, A3 = 1600;
// FC1 fwd split-K: 5 fixed chunks of 10 k-tiles (batch-independent rounding), each the sum
// of its even and its odd k-tiles (BA3C_FC_HALVES, gemm6_body PAR: two groups at B <= 64, one
// group with two accumulator sets above; the same association, so every row rounds the same
// at any batch).
// r02: 416 (4 chunks of 13 k-tiles) left B=32 with 8 workgroups walking 13 dependent k-tiles
// (17.6 us).  r06aa / r06ab: 5 chunks instead of 10 (half the partial sums written by fc1 and
// read by the heads kernel) took the B=2048 step 1.713 -> 1.685 and 1.685 -> 1.665 ms, but
// B=32 0.1565 -> 0.1612 ms with 10 k-tiles per workgroup in series: hence the two groups.
#ifndef BA3C_FC_HALVES
#define BA3C_FC_HALVES 1
#endif
#ifndef BA3C_FC_KCHUNK
#define BA3C_FC_KCHUNK (BA3C_FC_HALVES ? 320 : 160)
#endif
constexpr int FC_KCHUNK = BA3C_FC_KCHUNK, FC_SPLIT = (A3 + FC_KCHUNK - 1) / FC_KCHUNK;
static_assert(FC_SPLIT <= FC_SPLIT_MAX, "heads kernel finishes at most FC_SPLIT_MAX chunks");
static_assert(FC_KCHUNK % GEMM_BK == 0, "k-chunk of whole k-tiles");

// conv0's weight gradient runs on the main stream while the other weight gradients run on
// the side stream, so its split-K partials get a region of their own
size_t max_partials0(const ba3c_handle* h, int B) {
  size_t mx = 0;
  const WgradPlan w = plan_wgrad(25 * h->cfg.channels, 32, B * 6400, 128, 32);
  mx = std::max(mx, (size_t)w.S * w.M * w.N);
  mx = std::max(mx, (size_t)WG_P0S * Conv0W<2>::M * 32);
  return mx;
}

// partial-slab floats of each layer's weight gradient (every kernel variant of that layer)
struct PartialSizes {
  size_t heads, fc1, conv3, conv2, conv1;
};
PartialSizes partial_sizes(const ba3c_handle* h, int B) {
  const int F = h->cfg.fc_neurons;
  auto sz = [](const WgradPlan& w) { return (size_t)w.S * w.M * w.N; };
  PartialSizes p;
  p.heads = sz(plan_wgrad(F + 1, h->cfg.num_actions + 1, B, 128, 32));
  const bool legacy = !h->cfg.replace_with_conv;
  p.fc1 = std::max(sz(fc1w_plan(F, B, legacy, false)), sz(fc1w_plan(F, B, legacy, true)));
  p.conv3 = std::max(sz(plan_wgrad(576, 64, B * 25, 128, 64)), (size_t)C3W_P * 576 * 64);
  p.conv2 = std::max(sz(plan_wgrad(800, 64, B * 196, 128, 64)), (size_t)W6_P2 * Lay::W2::M * Lay::W2::COUT);
  p.conv1 = std::max(sz(plan_wgrad(800, 32, B * 1296, 128, 32)), (size_t)WG_P1 * Lay::W1::M * Lay::W1::COUT);
  return p;
}

Workspace carve(const ba3c_handle* h, void* base, int B, bool train) {
  Workspace w;
  std::memset(&w, 0, sizeof(w));
  char* p = static_cast<char*>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) -> char* {
    char* r = reinterpret_cast<char*>(reinterpret_cast<uintptr_t>(p) + off);  // p may be 0: offsets
    off += align256(bytes);
    return r;
  };
  const size_t Bz = (size_t)B;
  const int F = h->cfg.fc_neurons;
  // The clip / optimizer per-chunk sum-of-squares partials come FIRST, at a batch-independent
  // offset: ba3c_clip_grads / ba3c_apply_update receive only the workspace base.
  w.sumsq = (float*)take((size_t)h->table.nchunks * 4);
  w.amax = (uint32_t*)take(((size_t)AMAX_N * (1 + h->cfg.max_batch) + TK_N) * 4);
  w.wexp = (int*)take(8 * 4);
  w.p0 = (float*)take(Bz * P0 * 4);
  w.p1 = (float*)take(Bz * P1 * 4);
  w.p2 = (float*)take(Bz * P2 * 4);
  w.a3 = (float*)take(Bz * A3 * 4);
  w.h = (float*)take(Bz * F * 4);
#ifndef BA3C_FCPART_LAST
#define BA3C_FCPART_LAST 0   // A/B: fc1's forward partials at the end of the workspace
#endif
  if (!BA3C_FCPART_LAST) w.fcpart = (float*)take((size_t)FC_SPLIT * Bz * F * 4);
  w.relu = (unsigned long long*)take(RELU_WORDS * 8);
  w.wt = (float*)take((size_t)WT_TOTAL * 4);
  w.wt6 = (uint16_t*)take((size_t)3 * WT_C0F * 2);
  if (train) {
    w.c0 = (uint8_t*)take(Bz * P0);
    w.c1 = (uint8_t*)take(Bz * P1);
    w.c2 = (uint8_t*)take(Bz * P2);
    w.dh = (float*)take(Bz * F * 4);
    w.dy3 = (float*)take(Bz * A3 * 4);
    w.dp2 = (float*)take(Bz * P2 * 4);
    w.dp1 = (float*)take(Bz * P1 * 4);
    w.dp0 = (float*)take(Bz * P0 * 4);
    w.dzv = (float*)take(Bz * MAXA * 4);
    w.terms = (float*)take(Bz * NTERMS * 4);
    const PartialSizes ps = partial_sizes(h, B);
    w.part_h = (float*)take(ps.heads * 4);
    w.part_f = (float*)take(ps.fc1 * 4);
    w.part_3 = (float*)take(ps.conv3 * 4);
    w.part_2 = (float*)take(ps.conv2 * 4);
    w.part_1 = (float*)take(ps.conv1 * 4);
    w.part0 = (float*)take(max_partials0(h, B) * 4);
  }
  if (BA3C_FCPART_LAST) w.fcpart = (float*)take((size_t)FC_SPLIT * Bz * F * 4);
  w.bytes = off;
  return w;
}

// ---- launch helpers -------------------------------------------------------------------
struct ProbeScope {
  ba3c_handle* h;
  hipStream_t s;
  bool on;
  ProbeScope(ba3c_handle* h_, hipStream_t s_, int kid) : h(h_), s(s_), on(false) {
    if (h->probe_kernel == kid && h->probe_seen++ % (unsigned)h->probe_every == 0 &&
        h->probe_used < (int)h->ev_begin.size()) {
      on = true;
      (void)hipEventRecord(h->ev_begin[h->probe_used], s);
    }
  }
  ~ProbeScope() {
    if (on) {
      (void)hipEventRecord(h->ev_end[h->probe_used], s);
      h->probe_used++;
    }
  }
};

template <int BM, int BN, int WGM, int WGN, class P, int KS = 1>
int launch_gemm(ba3c_handle* h, hipStream_t s, int kid, const P& p, int splits) {
  if (p.M <= 0 || p.N <= 0) return BA3C_OK;
  dim3 grid((p.M + BM - 1) / BM, (p.N + BN - 1) / BN, splits);
  {
    ProbeScope ps(h, s, kid);
    // fewer workgroups than CUs: each walks its K latency-bound, so keep 4 k-tiles in flight
    const bool deep = (int)(grid.x * grid.y * grid.z) < h->cus;
    if (KS == 2 && h->g6 && deep)
      hipLaunchKernelGGL((gemm6_kernel<BM, BN, WGM, WGN, P, 4, KS>), grid, dim3(GEMM_THREADS * KS), 0, s, p);
    else if (KS == 2 && h->g6)
      hipLaunchKernelGGL((gemm6_kernel<BM, BN, WGM, WGN, P, 2, KS>), grid, dim3(GEMM_THREADS * KS), 0, s, p);
    else if (h->g6 && deep)
      hipLaunchKernelGGL((gemm6_kernel<BM, BN, WGM, WGN, P, 4>), grid, dim3(GEMM_THREADS), 0, s, p);
    else if (h->g6)
      hipLaunchKernelGGL((gemm6_kernel<BM, BN, WGM, WGN, P>), grid, dim3(GEMM_THREADS), 0, s, p);
    else
      hipLaunchKernelGGL((gemm_kernel<BM, BN, WGM, WGN, P>), grid, dim3(GEMM_THREADS), 0, s, p);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int launch_reduce(ba3c_handle* h, hipStream_t s, const float* part, int S, const ReduceMap& mp) {
  if (h->defer_reduce) {
    ReduceJobs& j = h->rjobs;
    if (j.n >= MAX_RJOBS) return fail(BA3C_ERR_INVALID, "too many deferred reductions");
    j.part[j.n] = part;
    j.S[j.n] = S;
    j.mp[j.n] = mp;
    const int no = mp.kind == 0 ? (mp.M / mp.cin) * mp.cinpad * mp.N : mp.M * mp.N;
    j.vec[j.n] = reduce_vec_ok(mp) ? 1 : 0;
    j.blk0[j.n + 1] = j.blk0[j.n] + (no + (j.vec[j.n] ? 255 : 63)) / (j.vec[j.n] ? 256 : 64);
    ++j.n;
    return BA3C_OK;
  }
  const int MN = mp.M * mp.N;
  {
    ProbeScope ps(h, s, BA3C_K_WGRAD_REDUCE);
    hipLaunchKernelGGL(wgrad_reduce_kernel, dim3((MN + 63) / 64), dim3(64 * RED_G), 0, s, part, S, mp);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

#define CHECK(x)            \
  do {                      \
    int _r = (x);           \
    if (_r != BA3C_OK) return _r; \
  } while (0)

// Split operands of a band-conv launch (fp16 family): the max slots of the staged map, the
// weight job whose scale exponent applies, and the slots that receive max |out| (-1: none).
struct SplitIO {
  int amax_in, wjob, amax_out;
};

template <class L>
Band6Args band6_args(ba3c_handle* h, const BandArgs& a, const Workspace& w, int wt_off, SplitIO io) {
  return Band6Args{a.src, a.code, w.wt6 + L::NS * (size_t)wt_off, a.out, a.out_code, a.relu_count, a.batch,
                   w.am(io.amax_in, h), w.wexp + io.wjob, io.amax_out >= 0 ? w.am(io.amax_out, h) : nullptr};
}

// One launch of up to three independent jobs (ba3c_multi.h); W2: the two-workgroups-per-CU
// register budget of the band / weight-gradient kernels; T512: 512-thread jobs.
template <bool W2, class J0, class J1, class J2 = NoJob, bool T512 = false>
int launch_multi(hipStream_t s, const typename J0::Args& a0, dim3 g0, const typename J1::Args& a1, dim3 g1,
                 const typename J2::Args& a2 = typename J2::Args{}, dim3 g2 = dim3(0, 1, 1),
                 ba3c_handle* h = nullptr, int kid = -1) {
  MultiGrid g;
  const dim3 gs[3] = {g0, g1, g2};
  int end = 0;
  for (int j = 0; j < 3; ++j) {
    g.gx[j] = (int)gs[j].x;
    g.gy[j] = (int)gs[j].y;
    end += (int)(gs[j].x * gs[j].y * gs[j].z);
    g.end[j] = end;
  }
  if (end == 0) return BA3C_OK;
  // the timing probe brackets the whole launch under job 0's kernel id
  std::optional<ProbeScope> probe;
  if (h && kid >= 0) probe.emplace(h, s, kid);
  if constexpr (T512)
    hipLaunchKernelGGL((multi_kernel512<J0, J1, J2>), dim3(end), dim3(512), 0, s, a0, a1, a2, g);
  else if constexpr (W2)
    hipLaunchKernelGGL((multi_kernel_w2<J0, J1, J2>), dim3(end), dim3(256), 0, s, a0, a1, a2, g);
  else
    hipLaunchKernelGGL((multi_kernel<J0, J1, J2>), dim3(end), dim3(256), 0, s, a0, a1, a2, g);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

// A chained multi-job launch (ba3c_multi.h): jobs [0, nsig) signal, the jobs in `wmask` wait
// for them (those in `late` inside their body); `site` picks the launch site's counter words.
// Callers check chain_ok() first.
constexpr int CHAIN_PREP_CONV0 = 0, CHAIN_REDUCE_UPDATE = 1;
bool chain_ok(const ba3c_handle* h) { return h->chain_on && h->chain != nullptr; }

template <bool W2, class J0, class J1, class J2 = NoJob>
int launch_chain(hipStream_t s, int site, int nsig, int wmask, int late, const typename J0::Args& a0, dim3 g0,
                 const typename J1::Args& a1, dim3 g1, const typename J2::Args& a2 = typename J2::Args{},
                 dim3 g2 = dim3(0, 1, 1), ba3c_handle* h = nullptr, int kid = -1, bool spread = false) {
  MultiGrid g;
  const dim3 gs[3] = {g0, g1, g2};
  int end = 0;
  for (int j = 0; j < 3; ++j) {
    g.gx[j] = (int)gs[j].x;
    g.gy[j] = (int)gs[j].y;
    end += (int)(gs[j].x * gs[j].y * gs[j].z);
    g.end[j] = end;
  }
  if (end == 0) return BA3C_OK;
  int nwait = 0;
  for (int j = 0; j < 3; ++j)
    if ((wmask >> j) & 1) nwait += g.end[j] - (j ? g.end[j - 1] : 0);
  const ChainArgs c{h->chain + 4 * site, h->chain + 4 * CHAIN_SITES, nsig, wmask, nwait, late,
                    h->spread, spread ? CHAIN_SPREAD : 0};
  std::optional<ProbeScope> probe;
  if (kid >= 0) probe.emplace(h, s, kid);
  if constexpr (W2)
    hipLaunchKernelGGL((multi_chain_kernel_w2<J0, J1, J2>), dim3(end), dim3(256), 0, s, a0, a1, a2, g, c);
  else
    hipLaunchKernelGGL((multi_chain_kernel<J0, J1, J2>), dim3(end), dim3(256), 0, s, a0, a1, a2, g, c);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

// band conv on split MFMA; `ringable`: a multi-band layout that may run as the ring-walk
// persistent kernel (whole images per workgroup) at large batches
template <class L>
int launch_band6(ba3c_handle* h, hipStream_t s, int kid, const BandArgs& a, const Workspace& w,
                 int wt_off, SplitIO io, bool ringable = false) {
  const Band6Args b = band6_args<L>(h, a, w, wt_off, io);
  const int nbands = a.batch * L::G::NBANDS;
  {
    ProbeScope ps(h, s, kid);
    if constexpr (L::NPH == 1 && L::G::NBANDS > 1 && L::G::SROWS > L::G::RB) {
      // whole images per workgroup: only where they split (nearly) evenly over 2 x CUs
      const int pr = 2 * h->cus;
      if (ringable && h->ring && a.batch >= pr && (a.batch % pr == 0 || a.batch >= 8 * pr)) {
        // (the forward keeps its double-buffered A fragments and no row prefetch: the
        // no-DBUF layout with the prefetch measured 0.36 -> 0.41 ms, r02ai)
        Band6Args br = b;
        if (h->dynq && a.batch > pr)    // several images per workgroup
          br.ticket = w.ticket(kid == BA3C_K_CONV1_DGRAD ? TK_C1D : TK_C1F, h);
        hipLaunchKernelGGL(conv_band6r_kernel<L>, dim3(2 * h->cus), dim3(256), 0, s, br);
        HIP_TRY(hipGetLastError());
        return BA3C_OK;
      }
    }
    hipLaunchKernelGGL(conv_band6_kernel<L>, dim3(nbands), dim3(256), 0, s, b);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

// split weight-gradient kernel + deterministic reduction into the flat HWIO grads
template <class G>
dim3 wgrad6_grid(int pmax, int batch) {
  return dim3(std::min(pmax, batch * G::NBANDS), G::NCG * G::NOG);
}
template <class G>
int reduce_wgrad6(ba3c_handle* h, hipStream_t s, const Wg6Args& a, int P, float* dst);
template <class G>
int launch_wgrad6(ba3c_handle* h, hipStream_t s, int kid, const Wg6Args& a, int pmax, float* dst) {
  const dim3 grid = wgrad6_grid<G>(pmax, a.batch);
  {
    ProbeScope ps(h, s, kid);
    hipLaunchKernelGGL(wgrad6_kernel<G>, grid, dim3(256), 0, s, a);
  }
  HIP_TRY(hipGetLastError());
  return reduce_wgrad6<G>(h, s, a, (int)grid.x, dst);
}
template <class G>
int reduce_wgrad6(ba3c_handle* h, hipStream_t s, const Wg6Args& a, int P, float* dst) {
  ReduceMap mp{};
  mp.kind = 0;
  mp.M = G::M;
  mp.N = G::COUT;
  mp.cin = G::CIN;
  mp.cinpad = G::CIN;
  mp.dst = dst;
  return launch_reduce(h, s, a.part, P, mp);
}

// Split-path weight preparation arguments (wprep6_kernel): every job, the conv0 fragments and
// the zeroing of the ReLU counters / max slots.
// conv1's sparse input gradient at this batch (the ring-walk batches)
bool use_c1s(const ba3c_handle* h, int B) { return h->c1s && h->band && h->ring && B >= 2 * h->cus; }

WPrep6Args wprep6_args(ba3c_handle* h, const float* prm, const Workspace& w, bool train, bool c1s = false) {
  const float* W1 = prm + h->tensors[h->idx_conv[1]].offset;
  const float* W2 = prm + h->tensors[h->idx_conv[2]].offset;
  const float* W3 = prm + h->tensors[h->idx_conv[3]].offset;
  WPrep6Args pa{};
  WPrepArgs& a = pa.jobs;
  a.job[WJ_C1F] = WPrepJob{W1, w.wt + WT_C1F, 5, 5, 32, 32, 0, 800 * 32};
  a.job[WJ_C2F] = WPrepJob{W2, w.wt + WT_C2F, 5, 5, 32, 64, 0, 800 * 64};
  a.job[WJ_C3F] = WPrepJob{W3, w.wt + WT_C3F, 3, 3, 64, 64, 0, 576 * 64};
  a.job[WJ_C1D] = WPrepJob{W1, w.wt + WT_C1D, 5, 5, 32, 32, 1, 800 * 32};
  a.job[WJ_C2D] = WPrepJob{W2, w.wt + WT_C2D, 5, 5, 32, 64, 1, 1600 * 32};
  a.job[WJ_C3D] = WPrepJob{W3, w.wt + WT_C3D, 3, 3, 64, 64, 1, 576 * 64};
  a.job[WJ_C1S] = WPrepJob{W1, w.wt + WT_C1S, 5, 5, 32, 32, 2, D1S::WPLANE};
  a.njobs = train ? (c1s ? WJ_N : WJ_C1S) : WJ_FWD;
  pa.wt6 = w.wt6;
  const int offs[WJ_N] = {WT_C1F, WT_C2F, WT_C3F, WT_C1D, WT_C2D, WT_C3D, WT_C1S};
  for (int j = 0; j < WJ_N; ++j) pa.off[j] = offs[j];
  pa.w0 = prm + h->tensors[h->idx_conv[0]].offset;
  pa.wb0 = reinterpret_cast<uint4*>(w.wt + WT_C0S);
  pa.relu = train ? w.relu : nullptr;
  pa.amax = w.amax;
  pa.n_amax = AMAX_N * (1 + h->cfg.max_batch) + TK_N;   // the tickets too
  pa.wexp = w.wexp;
  return pa;
}

// Small batches (split path, C == 4): the conv0 fragments + zeroing launch alone, then the
// band-conv weight jobs run beside conv0's forward in one multi-job launch (they are only
// needed from conv1 on).  B=32: the 8 us weight-prep launch was on the critical path.
int launch_prep_conv0_multi(ba3c_handle* h, hipStream_t s, const float* prm, const uint8_t* state, int B,
                            const Workspace& w, bool train) {
  WPrep6Args first = wprep6_args(h, prm, w, train);
  WPrep6Args rest = first;
  first.jobs.njobs = 0;                 // job row 0 == njobs: conv0 fragments (+ zeroing)
  rest.w0 = nullptr;                    // rows 0..njobs-1 only, no zeroing: conv0 publishes
  rest.relu = nullptr;                  // into those counters concurrently
  rest.amax = nullptr;
  const Conv0SArgs sa{state, reinterpret_cast<const uint4*>(w.wt + WT_C0S), w.p0, train ? w.c0 : nullptr,
                      train ? w.relu : nullptr, B, w.wexp + WX_CONV0, w.am(AM_P0, h)};
  const int nconv0 = std::min(FW_P0S, B * Conv0S::NBANDS);
  if (chain_ok(h) && nconv0 <= h->cus) {
    // one launch: the zeroing workgroups signal; conv0's forward (at most one workgroup per
    // CU) splits its own weight fragments and waits for the zeroing before its first
    // publication; the band-conv weight jobs run beside it
    first.coherent = 1;
    first.w0 = nullptr;
    Conv0SArgs sc = sa;
    sc.w0 = prm + h->tensors[h->idx_conv[0]].offset;
    sc.zsig = h->chain + 4 * CHAIN_PREP_CONV0 + 1;
    sc.zneed = 64;
    sc.zerr = h->chain + 4 * CHAIN_SITES;
    return launch_chain<true, WPrep6Job, Conv0SJob, WPrep6Job>(
        s, CHAIN_PREP_CONV0, 1, 2, 2, first, dim3(64, 1), sc, dim3(nconv0), rest,
        dim3(64, rest.jobs.njobs), h, BA3C_K_CONV0_FWD);
  }
  hipLaunchKernelGGL(wprep6_kernel, dim3(64, 1), dim3(256), 0, s, first);
  HIP_TRY(hipGetLastError());
  ProbeScope ps(h, s, BA3C_K_CONV0_FWD);
  // two workgroups per CU (the register budget of conv0's plain kernel): without the bound the
  // compiler gave the fused body 216 VGPRs + 52 AGPRs, one wave per SIMD, so at B=32 the 160 conv0
  // and 192 weight-prep workgroups did not fit the 256 CUs in one round
  return launch_multi<true, Conv0SJob, WPrep6Job>(s, sa, dim3(std::min(FW_P0S, B * Conv0S::NBANDS)), rest,
                                                  dim3(64, rest.jobs.njobs));
}

// split planes of the band-conv weights for this step (forward; + rotated dgrad in training)
// and, for C == 4, conv0's MFMA B fragments: one launch
int launch_wprep(ba3c_handle* h, hipStream_t s, const float* prm, const Workspace& w, bool train, int B) {
  WPrep6Args pa = wprep6_args(h, prm, w, train, use_c1s(h, B));
  const bool c0s = h->cfg.channels == 4;
  if (!c0s) pa.w0 = nullptr;
  hipLaunchKernelGGL(wprep6_kernel, dim3(64, pa.jobs.njobs + (c0s ? 1 : 0)), dim3(256), 0, s, pa);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int launch_conv0_band(ba3c_handle* h, hipStream_t s, const BandArgs& a, const Workspace& w) {
  const Conv0SArgs sa{reinterpret_cast<const uint8_t*>(a.src), reinterpret_cast<const uint4*>(w.wt + WT_C0S),
                      a.out, a.out_code, a.relu_count, a.batch, w.wexp + WX_CONV0, w.am(AM_P0, h)};
  ProbeScope ps(h, s, BA3C_K_CONV0_FWD);
  const dim3 grid(std::min(FW_P0S, a.batch * Conv0S::NBANDS));
  HIP_TRY(launch_conv0s_fwd(grid, s, sa));   // ba3c_conv0.hip
  return BA3C_OK;
}

// conv3 forward / input gradient: persistent whole-image workgroups, two per CU (ba3c_conv3.h)
template <bool DG>
#ifndef BA3C_C3_WGPC
#define BA3C_C3_WGPC 2   // conv3's whole-image kernels: persistent workgroups per CU (r06z: 1 made
                         // the forward 19.8 -> 23.9 us and the input gradient 29.3 -> 33.8 us)
#endif
int launch_conv3(ba3c_handle* h, hipStream_t s, int kid, const Conv3Args& a) {
  if (a.batch <= 0) return BA3C_OK;
  const dim3 grid(std::min(a.batch, BA3C_C3_WGPC * h->cus));
  {
    ProbeScope ps(h, s, kid);
    hipLaunchKernelGGL(conv3_band_kernel<DG>, grid, dim3(256), 0, s, a);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

// ---- forward --------------------------------------------------------------------------
#ifndef BA3C_FC_DEPTH
#define BA3C_FC_DEPTH 2       // k-tile ring depth of fc1's forward at full grids (A/B)
#endif

// Split kernels (h->band): conv0 (C == 4) and the conv1 / conv2 band convolutions on scaled
// fp16 hi/lo MFMA (ba3c_split.h, ba3c_band6.h); C == 12's conv0, conv3 and fc1 on the bf16x6
// GEMM engine.  BA3C_GENERIC=1: every layer on the fp32-MFMA GEMM engine.
template <int CH>
int run_forward(ba3c_handle* h, hipStream_t s, const float* prm, const uint8_t* state, int B,
                const Workspace& w, bool train) {
  using LY = Lay;
  const int F = h->cfg.fc_neurons;
  const float* W0 = prm + h->tensors[h->idx_conv[0]].offset;
  const float* W1 = prm + h->tensors[h->idx_conv[1]].offset;
  const float* W2 = prm + h->tensors[h->idx_conv[2]].offset;
  const float* W3 = prm + h->tensors[h->idx_conv[3]].offset;
  unsigned long long* rc = train ? w.relu : nullptr;
  uint8_t* c0 = train ? w.c0 : nullptr;
  uint8_t* c1 = train ? w.c1 : nullptr;
  uint8_t* c2 = train ? w.c2 : nullptr;
  const SplitIO io1{AM_P0, WJ_C1F, AM_P1}, io2{AM_P1, WJ_C2F, AM_P2};
  if (!h->band) {
    ConvFwd<true, 84, 84, CH, 16, 5, 5, 32, 0> cv0{state, W0, w.p0, c0, rc, 1.0f / 255.0f, B * 6400, 32, 25 * CH, 0};
    CHECK((launch_gemm<128, 32, 4, 1>(h, s, BA3C_K_CONV0_FWD, cv0, 1)));
    ConvFwd<false, 40, 40, 32, 32, 5, 5, 32, 0> cv1{w.p0, W1, w.p1, c1, rc, 1.0f, B * 1296, 32, 800, 0};
    CHECK((launch_gemm<128, 32, 4, 1>(h, s, BA3C_K_CONV1_FWD, cv1, 1)));
    ConvFwd<false, 18, 18, 32, 32, 5, 5, 64, 0> cv2{w.p1, W2, w.p2, c2, rc, 1.0f, B * 196, 64, 800, 0};
    CHECK((launch_gemm<128, 64, 4, 1>(h, s, BA3C_K_CONV2_FWD, cv2, 1)));
  } else {
    // small batches: weight prep beside conv0's forward (one launch fewer on the critical path)
    const bool mj = h->multi && B <= OVERLAP_B && CH == 4;
    if (mj) {
      CHECK(launch_prep_conv0_multi(h, s, prm, state, B, w, train));
    } else {
      CHECK(launch_wprep(h, s, prm, w, train, B));
      if constexpr (CH == 4) {
        CHECK(launch_conv0_band(h, s, BandArgs{reinterpret_cast<const float*>(state), nullptr, nullptr, w.p0, c0,
                                               rc, B}, w));
      } else {
        ConvFwd<true, 84, 84, CH, 16, 5, 5, 32, 0> cv0{state, W0, w.p0, c0, rc, 1.0f / 255.0f,
                                                      B * 6400, 32, 25 * CH, 0, w.am(AM_P0, h)};
        CHECK((launch_gemm<128, 32, 4, 1>(h, s, BA3C_K_CONV0_FWD, cv0, 1)));
      }
    }
    CHECK((launch_band6<typename LY::C1F>(h, s, BA3C_K_CONV1_FWD, BandArgs{w.p0, nullptr, nullptr, w.p1, c1, rc, B},
                                          w, WT_C1F, io1, true)));
    const BandArgs a2{w.p1, nullptr, nullptr, w.p2, c2, rc, B};
    if (B <= SMALL_B)
      CHECK(launch_band6<typename LY::C2FS>(h, s, BA3C_K_CONV2_FWD, a2, w, WT_C2F, io2));
    else
      CHECK(launch_band6<typename LY::C2F>(h, s, BA3C_K_CONV2_FWD, a2, w, WT_C2F, io2));
  }
  if (h->band) {
    // whole-image workgroups at every batch: an image's a3 does not depend on its batch
    CHECK(launch_conv3<false>(h, s, BA3C_K_CONV3_FWD, Conv3Args{w.p2, w.wt6 + 2 * (size_t)WT_C3F, w.wexp + WJ_C3F,
                                                                  w.a3, rc, nullptr, B, nullptr}));
  } else {
    ConvFwd<false, 7, 7, 64, 64, 3, 3, 64, 2> c3{w.p2, W3, w.a3, nullptr, rc, 1.0f, B * 25, 64, 576, 0};
    // K = 576 in two halves of 9 k-tiles summed in the workgroup (KS = 2) at every batch, so
    // each output's rounding is the same whatever batch it runs in
    CHECK((launch_gemm<64, 64, 2, 2, decltype(c3), 2>(h, s, BA3C_K_CONV3_FWD, c3, 1)));
  }
  // split-K: K = 1600 in FC_SPLIT fixed chunks (a 128x64 tile over all of K is one
  // workgroup's 50 serial k-tiles: latency-bound at any batch); the chunk sums (+ legacy bias,
  // ReLU, count) are finished inside the heads kernel (run_heads), which reads them anyway
  FcFwd fc{w.a3, prm + h->tensors[h->idx_fc1].offset, w.h, rc, h->per, h->wstride,
           h->cfg.replace_with_conv ? 0 : 1, B, F, 1600, FC_KCHUNK, w.fcpart};
  {
    ProbeScope ps(h, s, BA3C_K_FC1_FWD);
    const dim3 grid((B + 127) / 128, (F + 63) / 64, FC_SPLIT);
    constexpr bool HV = BA3C_FC_HALVES;
    constexpr int KSS = HV ? 2 : 1;   // small batches: even and odd k-tiles in two groups
    if (h->g6 && B <= 64)   // 64-row tiles: same per-row K order, half the dead rows staged
      hipLaunchKernelGGL((gemm6_kernel<64, 64, 2, 2, FcFwd, 4, KSS, HV>), dim3((B + 63) / 64, grid.y, grid.z),
                         dim3(GEMM_THREADS * KSS), 0, s, fc);
    else if (h->g6 && (int)(grid.x * grid.y * grid.z) < h->cus)
      hipLaunchKernelGGL((gemm6_kernel<128, 64, 2, 2, FcFwd, 4, 1, HV>), grid, dim3(GEMM_THREADS), 0, s, fc);
#ifndef BA3C_FC1F_BIGTILE
#define BA3C_FC1F_BIGTILE 0   // full grids on 128 x 128 tiles (same K chunks: bit-identical; r06v
                              // 0.0299 -> 0.0333 ms, not used)
#endif
    else if (h->g6 && BA3C_FC1F_BIGTILE)
      hipLaunchKernelGGL((gemm6_kernel<128, 128, 2, 2, FcFwd, BA3C_FC_DEPTH, 1, HV>), dim3(grid.x, (F + 127) / 128, grid.z),
                         dim3(GEMM_THREADS), 0, s, fc);
    else if (h->g6)
      hipLaunchKernelGGL((gemm6_kernel<128, 64, 2, 2, FcFwd, BA3C_FC_DEPTH, 1, HV>), grid, dim3(GEMM_THREADS), 0, s, fc);
    else
      hipLaunchKernelGGL((gemm_kernel<128, 64, 2, 2, FcFwd>), grid, dim3(GEMM_THREADS), 0, s, fc);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

// Create the side stream + fork/join events on the first training call made outside a
// graph capture (stream creation is not a capturable operation).
int ensure_side_stream(ba3c_handle* h, hipStream_t s) {
  if (h->overlap == 0 || h->side) return BA3C_OK;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  HIP_TRY(hipStreamIsCapturing(s, &cs));
  if (cs != hipStreamCaptureStatusNone) return BA3C_OK;
  HIP_TRY(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
  for (auto& e : h->ev_fork) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  HIP_TRY(hipEventCreateWithFlags(&h->ev_join, hipEventDisableTiming));
  return BA3C_OK;
}

// phase 0: the whole backward pass.  phase 1: the heads and fc1 products and their
// reductions (those gradients are final when it returns); phase 2: conv3..conv0 and theirs.
// Phases 1 + 2 compute exactly phase 0; between them a data-parallel caller can all-reduce
// the fc1 + heads bucket (most of the parameters) while the conv layers run.
template <int CH>
int run_backward(ba3c_handle* h, hipStream_t s, const float* prm, const uint8_t* state, int B,
                 const Workspace& w, float* grads, int phase = 0) {
  using LY = Lay;
  const int F = h->cfg.fc_neurons, A = h->cfg.num_actions;
  const bool legacy = !h->cfg.replace_with_conv;
  const float* W1c = prm + h->tensors[h->idx_conv[1]].offset;
  const float* W2c = prm + h->tensors[h->idx_conv[2]].offset;
  const float* W3c = prm + h->tensors[h->idx_conv[3]].offset;
  const float* Wfc = prm + h->tensors[h->idx_fc1].offset;
  bool defer_w1 = false;   // conv1's weight gradient waits for conv0's (one paired launch)
  // The weight-gradient kernels (heads, fc1, conv3..conv1) run on the side stream `ws`,
  // each after the event that publishes its output gradient; the input-gradient chain and
  // conv0's weight gradient (own partials region) stay on `s`, which joins `ws` at the end.
  hipStream_t ws = s;
  int nfork = 0;
  auto fork = [&]() -> int {
    if (ws == s) return BA3C_OK;
    HIP_TRY(hipEventRecord(h->ev_fork[nfork], s));
    HIP_TRY(hipStreamWaitEvent(ws, h->ev_fork[nfork], 0));
    ++nfork;
    return BA3C_OK;
  };
  // small batches on the split path: each layer's input- and weight-gradient kernels as one
  // multi-job launch on `s` (no side stream, no events); otherwise the side stream joins a
  // graph capture of `s` through the fork events
  const bool mjok = h->multi && h->overlap != 1 && h->band && CH == 4;
  const bool mj = mjok && B <= OVERLAP_B;
  const bool mj_fc = mj || (mjok && (h->multi_big & 1));
  const bool mj_c2 = !mj && mjok && (h->multi_big & 2);   // large-batch conv2 pair (A/B: BA3C_MULTI_BIG=3)

  static_assert(OVERLAP_B <= SMALL_B, "multi-job conv2 input gradient is the small-batch geometry");
  if (!mj && h->side && (h->overlap == 1 || B <= OVERLAP_B)) ws = h->side;
  const bool big = B > OVERLAP_B;   // multi-job gemm jobs: 2-deep k-tile rings (full grids)
  const bool fc1big = BA3C_FC1_BIGTILE && mj_fc && big;   // fc1w_plan
  // every weight-gradient reduction is deferred into one launch at the end (RAII: an early
  // error return leaves the handle in immediate mode)
  struct DeferGuard {
    ba3c_handle* h;
    explicit DeferGuard(ba3c_handle* h_) : h(h_) {
      h->defer_reduce = true;
      h->rjobs.n = 0;
      h->rjobs.blk0[0] = 0;
    }
    ~DeferGuard() { h->defer_reduce = false; }
  } defer_guard(h);
  // join the side stream and run the deferred reductions of this phase in one launch
  auto finish = [&]() -> int {
    if (h->pend_scalars && phase != 1 && phase != 4) {   // no launch took the deferred scalar reduction
      // (phase 1 leaves it pending: conv3's input-gradient launch in phase 2 takes it)
      const ScalarsJob::Args& sa = h->scalars_args;
      ProbeScope ps(h, s, BA3C_K_SCALARS);
      hipLaunchKernelGGL(scalars_kernel, dim3(1), dim3(256), 0, s, sa.terms, sa.B, sa.beta, sa.relu, sa.out);
      HIP_TRY(hipGetLastError());
      h->pend_scalars = false;
    }
    if (ws != s) {
      HIP_TRY(hipEventRecord(h->ev_join, ws));
      HIP_TRY(hipStreamWaitEvent(s, h->ev_join, 0));
    }
    const ReduceJobs& jb = h->rjobs;
    if (jb.n > 0 && phase == 4) {
      h->held = true;          // ba3c_launch_held (or the next entry point) launches it
      h->held_stream = s;
      h->held_jobs = jb;
    } else if (jb.n > 0 && h->defer_final && phase == 0) {
      h->pend_reduce = true;   // the next fused apply runs it (flush_reduce otherwise)
      h->pend_stream = s;
      h->pend_grads = grads;
    } else if (jb.n > 0) {
      ProbeScope ps(h, s, BA3C_K_WGRAD_REDUCE);
      hipLaunchKernelGGL(wgrad_reduce_all_kernel, dim3(jb.blk0[jb.n]), dim3(64 * RED_G), 0, s, jb);
    }
    HIP_TRY(hipGetLastError());
    return BA3C_OK;
  };
  CHECK(fork());

  if (phase != 2) {
  // heads: d fc-pi/W, fc-pi/b, fc-v/W, fc-v/b  (X = h, G = [dz | dV])
  {
    WgradPlan pl = plan_wgrad(F + 1, A + 1, B, 128, 32);
    BatchWgrad g{w.h, w.dzv, w.part_h, F, MAXA, 1, pl.M, pl.N, pl.K, pl.kchunk};
    WgradPlan plf = fc1w_plan(F, B, legacy, fc1big);
    BatchWgrad gf{w.a3, w.dh, w.part_f, 1600, F, legacy ? 1 : 0, plf.M, plf.N, plf.K, plf.kchunk};
    FcDgrad d{w.dh, Wfc, w.a3, w.dy3, h->per, h->wstride, B, 1600, F, 0};
    const int dbm = fc1big ? 128 : 64, fbn = fc1big ? 128 : 64;
    const dim3 gd((d.M + dbm - 1) / dbm, (d.N + dbm - 1) / dbm, 1), gh((pl.M + 127) / 128, (pl.N + 31) / 32, pl.S),
        gff((plf.M + 127) / 128, (plf.N + fbn - 1) / fbn, plf.S);
    if (mj_fc)   // fc1 input gradient + head and fc1 weight gradients: one launch
      h->merged[BA3C_K_FC1_DGRAD] |= (1u << BA3C_K_FC1_WGRAD) | (1u << BA3C_K_HEAD_WGRAD);
    if (mj_fc && !big)
      CHECK((launch_multi<false, Gemm6Job<64, 64, 2, 2, FcDgrad, 4>, Gemm6Job<128, 32, 4, 1, BatchWgrad, 4>,
                          Gemm6Job<128, 64, 2, 2, BatchWgrad, 4>>(s, d, gd, g, gh, gf, gff, h, BA3C_K_FC1_DGRAD)));
#ifndef BA3C_FCD_DEPTH
#define BA3C_FCD_DEPTH 2      // k-tile ring depth of the large-batch fc1 backward jobs (A/B)
#endif
    else if (mj_fc && fc1big)
      CHECK((launch_multi<false, Gemm6Job<128, 128, 2, 2, FcDgrad, BA3C_FCD_DEPTH>,
                          Gemm6Job<128, 32, 4, 1, BatchWgrad, BA3C_FCD_DEPTH>,
                          Gemm6Job<128, 128, 2, 2, BatchWgrad, BA3C_FCD_DEPTH>>(s, d, gd, g, gh, gf, gff, h,
                                                                              BA3C_K_FC1_DGRAD)));
    else if (mj_fc)
      CHECK((launch_multi<false, Gemm6Job<64, 64, 2, 2, FcDgrad, BA3C_FCD_DEPTH>, Gemm6Job<128, 32, 4, 1, BatchWgrad, BA3C_FCD_DEPTH>,
                          Gemm6Job<128, 64, 2, 2, BatchWgrad, BA3C_FCD_DEPTH>>(s, d, gd, g, gh, gf, gff, h, BA3C_K_FC1_DGRAD)));
    else
      CHECK((launch_gemm<128, 32, 4, 1>(h, ws, BA3C_K_HEAD_WGRAD, g, pl.S)));
    ReduceMap mp{};
    mp.kind = 2;
    mp.M = pl.M;
    mp.N = pl.N;
    mp.A = A;
    mp.dst = grads + h->tensors[h->idx_piW].offset;
    mp.dst_pib = grads + h->tensors[h->idx_pib].offset;
    mp.dst_vW = grads + h->tensors[h->idx_vW].offset;
    mp.dst_vb = grads + h->tensors[h->idx_vb].offset;
    CHECK(launch_reduce(h, ws, w.part_h, pl.S, mp));
  }
  // fc1 weight (+ legacy bias) gradient
  {
    WgradPlan pl = fc1w_plan(F, B, legacy, fc1big);
    BatchWgrad g{w.a3, w.dh, w.part_f, 1600, F, legacy ? 1 : 0, pl.M, pl.N, pl.K, pl.kchunk};
    if (!mj_fc) CHECK((launch_gemm<128, 64, 2, 2>(h, ws, BA3C_K_FC1_WGRAD, g, pl.S)));
    ReduceMap mp{};
    mp.kind = 1;
    mp.M = pl.M;
    mp.N = pl.N;
    mp.per = h->per;
    mp.wstride = h->wstride;
    mp.dst = grads + h->tensors[h->idx_fc1].offset;
    CHECK(launch_reduce(h, ws, w.part_f, pl.S, mp));
  }
  // fc1 input gradient -> dY3 (ReluGrad of conv3 fused)
  {
    FcDgrad d{w.dh, Wfc, w.a3, w.dy3, h->per, h->wstride, B, 1600, F, 0};
    if (!mj_fc) CHECK((launch_gemm<64, 64, 2, 2>(h, s, BA3C_K_FC1_DGRAD, d, 1)));
    CHECK(fork());
  }
  }  // phase != 2
  if (phase == 1 || phase == 4) return finish();
  auto conv_reduce = [&](const WgradPlan& pl, int layer, int cin, int cinpad, const float* part) {
    ReduceMap mp{};
    mp.kind = 0;
    mp.M = pl.M;
    mp.N = pl.N;
    mp.cin = cin;
    mp.cinpad = cinpad;
    mp.dst = grads + h->tensors[h->idx_conv[layer]].offset;
    return launch_reduce(h, ws, part, pl.S, mp);
  };
  // conv3's weight gradient when it rides on conv2's launch (BA3C_C3W_RIDE)
  Conv3WArgs c3w{};
  int c3w_gx = 0;
  // conv3
  {
    WgradPlan pl = plan_wgrad(576, 64, B * 25, 128, 64);
    if (h->band) {
      // whole-image kernels (ba3c_conv3.h) at every batch: an image's dP2 rounds the same in
      // any batch.  Input gradient first: it publishes dY3's per-image maxima, the weight
      // gradient's scale (both on `s`, whatever the side-stream setting); the deferred
      // TfDictOp reduction rides on it as one extra workgroup
      const Conv3Args da{w.dy3, w.wt6 + 2 * (size_t)WT_C3D, w.wexp + WJ_C3D, w.dp2, nullptr,
                         w.am(AM_DP2, h), B, w.am(AM_DY3, h)};
      const int gx = conv3_wgrad_p(B, h->cus);
#ifndef BA3C_C3PAIR
#define BA3C_C3PAIR 1   // 0: A/B build with the small-batch conv3 gradients in two launches
#endif
      if (mj && BA3C_C3PAIR) {
        // small batches: input and weight gradient in one launch (two 256-thread workgroups per
        // weight-gradient slab; the weight gradient reduces max |dY3| itself, since the input
        // gradient publishes it only as it runs)
        const Conv3WArgs wa{w.p2, w.dy3, w.part_3, B, w.am(AM_P2, h), nullptr, 1};
        CHECK((launch_multi<true, Conv3DJob, Conv3WJob>(s, da, dim3(std::min(B, 2 * h->cus)), wa, dim3(gx, 2),
                                                         0, dim3(0, 1, 1), h, BA3C_K_CONV3_DGRAD)));
        h->merged[BA3C_K_CONV3_DGRAD] |= 1u << BA3C_K_CONV3_WGRAD;
      } else {
        if (big && h->pend_scalars) {
          CHECK((launch_multi<true, Conv3DJob, ScalarsJob>(s, da, dim3(std::min(B, BA3C_C3_WGPC * h->cus)), h->scalars_args,
                                                            dim3(1), 0, dim3(0, 1, 1), h, BA3C_K_CONV3_DGRAD)));
          h->merged[BA3C_K_CONV3_DGRAD] |= 1u << BA3C_K_SCALARS;   // the reduction rode on this launch
          h->pend_scalars = false;
        } else {
          CHECK(launch_conv3<true>(h, s, BA3C_K_CONV3_DGRAD, da));
        }
        const Conv3WArgs wa{w.p2, w.dy3, w.part_3, B, w.am(AM_P2, h), w.am(AM_DY3, h), 0};
        if (mj_c2 && h->c3ride) {
          c3w = wa;   // a job of conv2's launch below
          c3w_gx = gx;
        } else {
          ProbeScope ps(h, s, BA3C_K_CONV3_WGRAD);
          hipLaunchKernelGGL(conv3_wgrad_kernel, dim3(gx), dim3(512), 0, s, wa);
        }
        HIP_TRY(hipGetLastError());
      }
      pl.S = gx;   // one slab per workgroup
    } else {   // BA3C_GENERIC: the fp32-MFMA GEMM engine
      ConvWgrad<false, 7, 7, 64, 3, 3, 64, false> g{w.p2, w.dy3, nullptr, w.part_3, 1.0f, pl.M, pl.N, pl.K, pl.kchunk};
      ConvDgrad<7, 7, 64, 3, 3, 64, false> d{w.dy3, nullptr, W3c, w.dp2, B * 49, 64, 576, 0, nullptr};
      CHECK((launch_gemm<128, 64, 4, 1>(h, ws, BA3C_K_CONV3_WGRAD, g, pl.S)));
      CHECK((launch_gemm<64, 64, 2, 2>(h, s, BA3C_K_CONV3_DGRAD, d, 1)));
    }
    CHECK(conv_reduce(pl, 3, 64, 64, w.part_3));
    CHECK(fork());
  }
  if (phase == 2 && h->ev_mid) HIP_TRY(hipEventRecord(h->ev_mid, s));
  // conv2
  if (mj) {
    const Wg6Args wa{w.p1, w.dp2, w.c2, w.part_2, B, w.am(AM_P1, h), w.am(AM_DP2, h)};
    const dim3 wg = wgrad6_grid<typename LY::W2>(W6_P2, B);
    const Band6Args da = band6_args<typename LY::C2DS>(h, BandArgs{w.dp2, w.c2, w.wt + WT_C2D, w.dp1, nullptr, nullptr, B},
                                                      w, WT_C2D, SplitIO{AM_DP2, WJ_C2D, AM_DP1});
    CHECK((launch_multi<true, Band6Job<typename LY::C2DS>, Wg6Job<typename LY::W2>>(
        s, da, dim3(B * LY::C2DS::G::NBANDS), wa, wg)));
    h->merged[BA3C_K_CONV2_DGRAD] |= 1u << BA3C_K_CONV2_WGRAD;
    CHECK(reduce_wgrad6<typename LY::W2>(h, s, wa, (int)wg.x, grads + h->tensors[h->idx_conv[2]].offset));
  } else if (mj_c2) {
    const Wg6Args wa{w.p1, w.dp2, w.c2, w.part_2, B, w.am(AM_P1, h), w.am(AM_DP2, h)};
    const dim3 wg = wgrad6_grid<typename LY::W2>(W6_P2, B);
    const Band6Args da = band6_args<typename LY::C2D>(h, BandArgs{w.dp2, w.c2, w.wt + WT_C2D, w.dp1, nullptr, nullptr, B},
                                                     w, WT_C2D, SplitIO{AM_DP2, WJ_C2D, AM_DP1});
    const dim3 gd(B * LY::C2D::G::NBANDS), g3(c3w_gx, 2);
    if (c3w_gx && h->c3ride == 2)
      CHECK((launch_multi<true, Conv3WJob, Band6Job<typename LY::C2D>, Wg6Job<typename LY::W2>>(
          s, c3w, g3, da, gd, wa, wg, h, BA3C_K_CONV2_DGRAD)));
    else if (c3w_gx)
      CHECK((launch_multi<true, Band6Job<typename LY::C2D>, Wg6Job<typename LY::W2>, Conv3WJob>(
          s, da, gd, wa, wg, c3w, g3, h, BA3C_K_CONV2_DGRAD)));
    else
      CHECK((launch_multi<true, Band6Job<typename LY::C2D>, Wg6Job<typename LY::W2>>(
          s, da, gd, wa, wg, 0, dim3(0, 1, 1), h, BA3C_K_CONV2_DGRAD)));
    h->merged[BA3C_K_CONV2_DGRAD] |= 1u << BA3C_K_CONV2_WGRAD;
    if (c3w_gx) h->merged[BA3C_K_CONV2_DGRAD] |= 1u << BA3C_K_CONV3_WGRAD;
    CHECK(reduce_wgrad6<typename LY::W2>(h, s, wa, (int)wg.x, grads + h->tensors[h->idx_conv[2]].offset));
  } else {
    if (h->band) {
      CHECK(launch_wgrad6<typename LY::W2>(h, ws, BA3C_K_CONV2_WGRAD,
                                          Wg6Args{w.p1, w.dp2, w.c2, w.part_2, B, w.am(AM_P1, h), w.am(AM_DP2, h)},
                                          W6_P2, grads + h->tensors[h->idx_conv[2]].offset));
    } else {
      WgradPlan pl = plan_wgrad(800, 64, B * 196, 128, 64);
      ConvWgrad<false, 18, 18, 32, 5, 5, 64, true> g{w.p1, w.dp2, w.c2, w.part_2, 1.0f, pl.M, pl.N, pl.K, pl.kchunk};
      CHECK((launch_gemm<128, 64, 4, 1>(h, ws, BA3C_K_CONV2_WGRAD, g, pl.S)));
      CHECK(conv_reduce(pl, 2, 32, 32, w.part_2));
    }
    if (h->band) {
      const BandArgs ba{w.dp2, w.c2, w.wt + WT_C2D, w.dp1, nullptr, nullptr, B};
      const SplitIO io{AM_DP2, WJ_C2D, AM_DP1};
      if (B <= SMALL_B)
        CHECK(launch_band6<typename LY::C2DS>(h, s, BA3C_K_CONV2_DGRAD, ba, w, WT_C2D, io));
      else
        CHECK(launch_band6<typename LY::C2D>(h, s, BA3C_K_CONV2_DGRAD, ba, w, WT_C2D, io));
    } else {
      ConvDgrad<18, 18, 32, 5, 5, 64, true> d{w.dp2, w.c2, W2c, w.dp1, B * 324, 32, 1600, 0};
      CHECK((launch_gemm<128, 32, 4, 1>(h, s, BA3C_K_CONV2_DGRAD, d, 1)));
    }
    CHECK(fork());
  }
  // conv1
  if (mj) {
    const Wg6Args wa{w.p0, w.dp1, w.c1, w.part_1, B, w.am(AM_P0, h), w.am(AM_DP1, h)};
    const dim3 wg = wgrad6_grid<typename LY::W1>(conv1_wgrad_p(B), B);
    const Band6Args da = band6_args<typename LY::C1D>(h, BandArgs{w.dp1, w.c1, w.wt + WT_C1D, w.dp0, nullptr, nullptr, B},
                                                     w, WT_C1D, SplitIO{AM_DP1, WJ_C1D, AM_DP0});
    CHECK((launch_multi<true, Band6Job<typename LY::C1D>, Wg6Job<typename LY::W1>>(
        s, da, dim3(B * LY::C1D::G::NBANDS), wa, wg)));
    h->merged[BA3C_K_CONV1_DGRAD] |= 1u << BA3C_K_CONV1_WGRAD;
    CHECK(reduce_wgrad6<typename LY::W1>(h, s, wa, (int)wg.x, grads + h->tensors[h->idx_conv[1]].offset));
  } else {
    bool done = false, paired = false;
    {
      const bool pairgeo = h->band && h->ring && conv1_pair_geometry(B, h->cus);
      if (pairgeo && h->c1pair == 2 && CH == 4) {
        done = defer_w1 = true;                             // beside conv0's weight gradient below
      }
      // conv1 input and weight gradients in one launch, one workgroup of each per CU (each job
      // walks twice the images of its separate launch)
      if (!done && pairgeo && h->c1pair == 1) {
        using GW = typename LY::W1W;
        const Wg6Args wa{w.p0, w.dp1, w.c1, w.part_1, B, w.am(AM_P0, h), w.am(AM_DP1, h)};
        const Band6Args da = band6_args<typename LY::C1D>(h, BandArgs{w.dp1, w.c1, w.wt + WT_C1D, w.dp0, nullptr, nullptr, B},
                                                         w, WT_C1D, SplitIO{AM_DP1, WJ_C1D, AM_DP0});
        CHECK((launch_multi<true, Band6RJob<typename LY::C1D>, Wg6WJob<GW>>(
            s, da, dim3(h->cus), wa, dim3(h->cus), 0, dim3(0, 1, 1), h, BA3C_K_CONV1_DGRAD)));
        h->merged[BA3C_K_CONV1_DGRAD] |= 1u << BA3C_K_CONV1_WGRAD;
        CHECK(reduce_wgrad6<typename LY::W1>(h, s, wa, h->cus, grads + h->tensors[h->idx_conv[1]].offset));
        done = paired = true;
      }
      if (!done && h->band && B >= W6W_MIN_B) {
        using GW = typename LY::W1W;
        const Wg6Args wa{w.p0, w.dp1, w.c1, w.part_1, B, w.am(AM_P0, h), w.am(AM_DP1, h)};
        const int P = conv1_w6w_p(B, h->cus);
        {
          ProbeScope ps(h, ws, BA3C_K_CONV1_WGRAD);
          hipLaunchKernelGGL(wgrad6w_kernel<GW>, dim3(P), dim3(256), 0, ws, wa);
        }
        HIP_TRY(hipGetLastError());
        CHECK(reduce_wgrad6<typename LY::W1>(h, ws, wa, P, grads + h->tensors[h->idx_conv[1]].offset));
        done = true;
      }
    }
    if (done) {
    } else if (h->band) {
      CHECK(launch_wgrad6<typename LY::W1>(h, ws, BA3C_K_CONV1_WGRAD,
                                          Wg6Args{w.p0, w.dp1, w.c1, w.part_1, B, w.am(AM_P0, h), w.am(AM_DP1, h)},
                                          conv1_wgrad_p(B), grads + h->tensors[h->idx_conv[1]].offset));
    } else {
      WgradPlan pl = plan_wgrad(800, 32, B * 1296, 128, 32);
      ConvWgrad<false, 40, 40, 32, 5, 5, 32, true> g{w.p0, w.dp1, w.c1, w.part_1, 1.0f, pl.M, pl.N, pl.K, pl.kchunk};
      CHECK((launch_gemm<128, 32, 4, 1>(h, ws, BA3C_K_CONV1_WGRAD, g, pl.S)));
      CHECK(conv_reduce(pl, 1, 32, 32, w.part_1));
    }
    if (paired) {
      // both gradients ran in the multi-job launch above
    } else if (use_c1s(h, B)) {
      // 2:4-sparse MFMA (ba3c_dgrad1s.h): two workgroups per CU, persistent over bands
      const Band6Args b = band6_args<typename LY::C1D>(h, BandArgs{w.dp1, w.c1, nullptr, w.dp0, nullptr, nullptr, B},
                                                       w, WT_C1S, SplitIO{AM_DP1, WJ_C1S, AM_DP0});
      {
        ProbeScope ps(h, s, BA3C_K_CONV1_DGRAD);
        hipLaunchKernelGGL(dgrad1s_kernel, dim3(2 * h->cus), dim3(256), 0, s, b);
      }
      HIP_TRY(hipGetLastError());
    } else if (h->band) {
      const BandArgs ba{w.dp1, w.c1, nullptr, w.dp0, nullptr, nullptr, B};
      CHECK(launch_band6<typename LY::C1D>(h, s, BA3C_K_CONV1_DGRAD, ba, w, WT_C1D, SplitIO{AM_DP1, WJ_C1D, AM_DP0},
                                           true));
    } else {
      ConvDgrad<40, 40, 32, 5, 5, 32, true> d{w.dp1, w.c1, W1c, w.dp0, B * 1600, 32, 800, 0};
      CHECK((launch_gemm<128, 32, 4, 1>(h, s, BA3C_K_CONV1_DGRAD, d, 1)));
    }
  }
  // conv0 (no input gradient: the frames are not trainable)
  if (h->band && CH == 4) {
    // slab count: one per CU where conv1's weight gradient can share the launch (on every launch
    // path, so they all sum the same slabs), else up to WG_P0S
    const int P = conv1_pair_geometry(B, h->cus) ? h->cus : std::min(WG_P0S, B * Conv0W<2>::NBANDS);
    const Conv0WArgs a0{state, w.dp0, w.c0, w.part0, B, w.am(AM_DP0, h)};
    if (defer_w1) {
      // conv1's whole-channel weight gradient (MFMA-bound) beside conv0's (VALU-bound): one
      // workgroup of each per CU, one launch (ba3c_conv0.hip)
      const Wg6Args wa{w.p0, w.dp1, w.c1, w.part_1, B, w.am(AM_P0, h), w.am(AM_DP1, h)};
      {
        ProbeScope ps(h, s, BA3C_K_CONV0_WGRAD);
        HIP_TRY(launch_wgrad01_pair(s, wa, h->cus, a0, P));
      }
      h->merged[BA3C_K_CONV0_WGRAD] |= 1u << BA3C_K_CONV1_WGRAD;
      CHECK(reduce_wgrad6<typename LY::W1>(h, s, wa, h->cus, grads + h->tensors[h->idx_conv[1]].offset));
    } else {
      ProbeScope ps(h, s, BA3C_K_CONV0_WGRAD);
      HIP_TRY(launch_conv0s_wgrad(dim3(P), s, a0));
    }
    HIP_TRY(hipGetLastError());
    ReduceMap mp{};
    mp.kind = 0;
    mp.M = Conv0W<2>::M;
    mp.N = 32;
    mp.cin = 4;
    mp.cinpad = 16;
    mp.dst = grads + h->tensors[h->idx_conv[0]].offset;
    CHECK(launch_reduce(h, s, w.part0, P, mp));
  } else {
    WgradPlan pl = plan_wgrad(25 * CH, 32, B * 6400, 128, 32);
    ConvWgrad<true, 84, 84, CH, 5, 5, 32, true> g{state, w.dp0, w.c0, w.part0, 1.0f / 255.0f, pl.M, pl.N, pl.K, pl.kchunk};
    CHECK((launch_gemm<128, 32, 4, 1>(h, s, BA3C_K_CONV0_WGRAD, g, pl.S)));
    ReduceMap mp{};
    mp.kind = 0;
    mp.M = pl.M;
    mp.N = pl.N;
    mp.cin = CH;
    mp.cinpad = 16;
    mp.dst = grads + h->tensors[h->idx_conv[0]].offset;
    CHECK(launch_reduce(h, s, w.part0, pl.S, mp));
  }
  // all (remaining) weight-gradient reductions: one launch, every gradient element written once
  return finish();
}

int run_heads(ba3c_handle* h, hipStream_t s, const float* prm, const Workspace& w, int B,
              const int64_t* action, const float* R, float beta, float explore, bool train,
              float* probs, float* probsT, float* value, double* scalars = nullptr,
              bool defer_scalars = false) {
  HeadsArgs a{};
  a.fcpart = w.fcpart;
  a.fc_split = FC_SPLIT;
  a.per = h->per;
  a.wstride = h->wstride;
  a.fc_w1 = prm + h->tensors[h->idx_fc1].offset;
  a.relu_count = train ? w.relu : nullptr;
  a.done = w.relu + RELU_SLOTS;
  // the scalar reduction rides on the heads launch (last workgroup) for small batches only:
  // with B/4 workgroups all finishing together, B > 256 puts hundreds of same-address atomics
  // and a B-long serial reduction at the kernel's tail (r02f: heads 29 -> 75 us at B=2048)
  const bool fuse_scalars = train && scalars && B <= 256;
  a.scalars = fuse_scalars ? scalars : nullptr;
  a.h = w.h;
  a.piW = prm + h->tensors[h->idx_piW].offset;
  a.pib = prm + h->tensors[h->idx_pib].offset;
  a.vW = prm + h->tensors[h->idx_vW].offset;
  a.vb = prm + h->tensors[h->idx_vb].offset;
  a.action = action;
  a.R = R;
  a.probs = probs;
  a.probsT = probsT;
  a.value = value;
  a.dzv = w.dzv;
  a.dh = w.dh;
  a.terms = w.terms;
  a.B = B;
  a.F = h->cfg.fc_neurons;
  a.A = h->cfg.num_actions;
  a.train = train ? 1 : 0;
  a.legacy = h->cfg.replace_with_conv ? 0 : 1;
  a.beta = beta;
  a.explore = explore;
  a.invB = 1.0f / (float)B;
  {
    ProbeScope ps(h, s, BA3C_K_HEADS);
    // features per lane unrolled (heads_sample): the smallest instantiation that covers F
    const int F = a.F;
    const dim3 g((B + 3) / 4), t(256);
    // the reference's Atari action sets are mostly 4 actions: compile-time A there (heads_sample)
    if (a.A == 4 && F <= 128 && F > 64) hipLaunchKernelGGL((heads_kernel<2, FC_SPLIT, 4>), g, t, 0, s, a);
    else if (a.A == 4 && F <= 512 && F > 256) hipLaunchKernelGGL((heads_kernel<8, FC_SPLIT, 4>), g, t, 0, s, a);
    else if (F <= 64) hipLaunchKernelGGL((heads_kernel<1, FC_SPLIT>), g, t, 0, s, a);
    else if (F <= 128) hipLaunchKernelGGL((heads_kernel<2, FC_SPLIT>), g, t, 0, s, a);
    else if (F <= 256) hipLaunchKernelGGL((heads_kernel<4, FC_SPLIT>), g, t, 0, s, a);
    else if (F <= 512) hipLaunchKernelGGL((heads_kernel<8, FC_SPLIT>), g, t, 0, s, a);
    else hipLaunchKernelGGL((heads_kernel<0, FC_SPLIT>), g, t, 0, s, a);
  }
  HIP_TRY(hipGetLastError());
  if (train && scalars && !fuse_scalars && defer_scalars) {
    h->scalars_args = ScalarsJob::Args{w.terms, B, beta, w.relu, scalars};
    h->pend_scalars = true;      // launched by run_backward (conv3's input gradient or finish)
  } else if (train && scalars && !fuse_scalars) {
    ProbeScope ps(h, s, BA3C_K_SCALARS);
    hipLaunchKernelGGL(scalars_kernel, dim3(1), dim3(256), 0, s, w.terms, B, beta, w.relu, scalars);
    HIP_TRY(hipGetLastError());
  }
  return BA3C_OK;
}

bool check_ptr(const void* p) { return p != nullptr && (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

namespace {
struct Rccl {
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                             hipStream_t) = nullptr;
  ncclResult_t (*destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*abort)(ncclComm_t) = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
  bool ok = false;
};
const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* lib = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) lib = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!lib) return x;
    x.get_unique_id = reinterpret_cast<decltype(x.get_unique_id)>(dlsym(lib, "ncclGetUniqueId"));
    x.init_rank = reinterpret_cast<decltype(x.init_rank)>(dlsym(lib, "ncclCommInitRank"));
    x.all_reduce = reinterpret_cast<decltype(x.all_reduce)>(dlsym(lib, "ncclAllReduce"));
    x.destroy = reinterpret_cast<decltype(x.destroy)>(dlsym(lib, "ncclCommDestroy"));
    x.abort = reinterpret_cast<decltype(x.abort)>(dlsym(lib, "ncclCommAbort"));
    x.error_string = reinterpret_cast<decltype(x.error_string)>(dlsym(lib, "ncclGetErrorString"));
    x.ok = x.get_unique_id && x.init_rank && x.all_reduce && x.destroy && x.abort && x.error_string;
    return x;
  }();
  return r;
}
int rccl_fail(ncclResult_t e, const char* what) {
  return fail(BA3C_ERR_HIP, std::string(what) + ": " + rccl().error_string(e));
}
}  // namespace

// =========================================================================================
extern "C" {

int ba3c_version(void) { return 1; }

const char* ba3c_last_error(void) { return g_err.c_str(); }

int ba3c_create(const ba3c_config* cfg, ba3c_handle** out) {
  if (!cfg || !out) return fail(BA3C_ERR_INVALID, "null argument");
  const ba3c_config& c = *cfg;
  if (c.channels != 4 && c.channels != 12)
    return fail(BA3C_ERR_INVALID, "channels must be 4 or 12 (FRAME_HISTORY * --channels)");
  if (c.num_actions < 1 || c.num_actions >= MAXA)
    return fail(BA3C_ERR_INVALID, "num_actions must be in [1, 31]");
  if (c.max_batch < 1 || c.max_batch > kMaxBatch)
    return fail(BA3C_ERR_INVALID, "max_batch must be in [1, 16384]");
  const int splits = c.replace_with_conv ? c.fc_splits : c.ps;
  if (splits < 1 || c.fc_neurons < 4 || c.fc_neurons % splits != 0 || (c.fc_neurons / splits) % 4 != 0)
    return fail(BA3C_ERR_INVALID, "fc_neurons must be a multiple of 4*fc_splits (or 4*ps)");
  // launch-structure switches (each exercised by a GPU test; values outside the listed ones
  // are rejected rather than coerced, so an A/B run measures what it asked for)
  struct Switch {
    const char* name;
    int lo, hi;
  };
  static const Switch kSwitches[] = {{"BA3C_GENERIC", 0, 1},  {"BA3C_C1PAIR", 0, 2},   {"BA3C_SCALARS_RIDE", 0, 1},
                                     {"BA3C_OVERLAP", 0, 2},  {"BA3C_MULTI", 0, 1},    {"BA3C_MULTI_BIG", 0, 3},
                                     {"BA3C_FUSED_UPDATE", 0, 1}, {"BA3C_RING", 0, 1}, {"BA3C_CHAIN", 0, 1},
                                     {"BA3C_C1D_SPARSE", 0, 1}, {"BA3C_DYNQ", 0, 1},
                                     {"BA3C_C3W_RIDE", 0, 2}};
  constexpr int NSW = 12;
  int sw[NSW];
  const int defaults[NSW] = {0, 2, 1, 2, 1, 3, 1, 1, 1, 0, 0, 0};
  for (int i = 0; i < NSW; ++i) {
    sw[i] = defaults[i];
    const char* e = getenv(kSwitches[i].name);
    if (!e) continue;
    if (!(e[0] >= '0' && e[0] <= '9' && e[1] == 0) || e[0] - '0' < kSwitches[i].lo || e[0] - '0' > kSwitches[i].hi)
      return fail(BA3C_ERR_INVALID, std::string(kSwitches[i].name) + "=" + e + ": expected one digit in [" +
                                        std::to_string(kSwitches[i].lo) + ", " + std::to_string(kSwitches[i].hi) + "]");
    sw[i] = e[0] - '0';
  }
  ba3c_handle* h = new ba3c_handle();
  h->cfg = c;
  h->band = sw[0] == 0;
  h->c1pair = sw[1];
  h->scalars_ride = sw[2] != 0;
  h->overlap = sw[3];
  h->multi = sw[4] != 0;
  h->multi_big = sw[5];
  h->fused_update = sw[6] != 0;
  h->ring = sw[7] != 0;
  h->chain_on = sw[8] != 0;
  h->c1s = sw[9] != 0;
  h->dynq = sw[10] != 0;
  h->c3ride = sw[11];
  h->g6 = h->band;
  {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) == hipSuccess &&
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0)
      h->cus = n;
  }

  const int F = c.fc_neurons, per = F / splits;
  h->per = per;
  int64_t off = 0;
  auto add = [&](const std::string& name, std::initializer_list<int> shape) {
    TensorDesc d;
    d.name = name;
    d.offset = off;
    d.ndim = (int)shape.size();
    int64_t n = 1;
    int i = 0;
    for (int v : shape) {
      d.shape[i++] = v;
      n *= v;
    }
    for (; i < 4; ++i) d.shape[i] = 0;
    d.numel = n;
    h->tensors.push_back(d);
    off = align64(off + n);
    return (int)h->tensors.size() - 1;
  };
  h->idx_conv[0] = add("conv0/W", {5, 5, 16, 32});
  h->idx_conv[1] = add("conv1/W", {5, 5, 32, 32});
  h->idx_conv[2] = add("conv2/W", {5, 5, 32, 64});
  h->idx_conv[3] = add("conv3/W", {3, 3, 64, 64});
  h->idx_fc1 = -1;
  for (int i = 0; i < splits; ++i) {
    int t;
    if (c.replace_with_conv) {
      t = add("fc1_" + std::to_string(i) + "/W", {5, 5, 64, per});
    } else {
      t = add("fc1_" + std::to_string(i) + "/W", {1600, per});
      add("fc1_" + std::to_string(i) + "/b", {per});
    }
    if (i == 0) h->idx_fc1 = t;
  }
  h->wstride = c.replace_with_conv ? 1600 * per : (int)(1600 * per + align64(per));
  h->idx_piW = add("fc-pi/W", {F, c.num_actions});
  h->idx_pib = add("fc-pi/b", {c.num_actions});
  h->idx_vW = add("fc-v/W", {F, 1});
  h->idx_vb = add("fc-v/b", {1});
  h->flat = off;
  if ((int)h->tensors.size() > MAXT) {
    delete h;
    return fail(BA3C_ERR_INVALID, "too many tensors");
  }
  TensorTable& tt = h->table;
  std::memset(&tt, 0, sizeof(tt));
  tt.n = (int)h->tensors.size();
  int ch = 0;
  for (int i = 0; i < tt.n; ++i) {
    tt.off[i] = h->tensors[i].offset;
    tt.numel[i] = (int)h->tensors[i].numel;
    tt.chunk0[i] = ch;
    ch += (int)((h->tensors[i].numel + UPD_CHUNK - 1) / UPD_CHUNK);
  }
  tt.chunk0[tt.n] = ch;
  tt.nchunks = ch;
  // clip_update_kernel's and clip_range_kernel's tagged partials + error words (no device:
  // stay null, two-launch paths)
  const size_t ubytes = ((size_t)tt.nchunks + 1) * sizeof(unsigned long long);
  const size_t cbytes = (4 * CHAIN_SITES + 4 + CHAIN_SPREAD * CHAIN_STRIDE + 16) * sizeof(unsigned);
  if (hipMalloc(reinterpret_cast<void**>(&h->utag), 2 * ubytes + cbytes) != hipSuccess) {
    h->utag = nullptr;
    (void)hipGetLastError();
  } else if (hipMemset(h->utag, 0, 2 * ubytes + cbytes) != hipSuccess) {
    (void)hipFree(h->utag);
    h->utag = nullptr;
    (void)hipGetLastError();
  } else {
    h->ctag = h->utag + tt.nchunks + 1;
    h->chain = reinterpret_cast<unsigned*>(h->ctag + tt.nchunks + 1);
    const uintptr_t sp = reinterpret_cast<uintptr_t>(h->chain + 4 * CHAIN_SITES + 4);
    h->spread = reinterpret_cast<unsigned*>((sp + 63) & ~uintptr_t(63));
  }
  *out = h;
  return BA3C_OK;
}

int ba3c_comm_destroy(ba3c_handle* h, int32_t abort);

void ba3c_destroy(ba3c_handle* h) {
  if (!h) return;
  if (h->comm) (void)ba3c_comm_destroy(h, 0);
  for (auto e : h->ev_begin) (void)hipEventDestroy(e);
  for (auto e : h->ev_end) (void)hipEventDestroy(e);
  for (auto e : h->ev_fork)
    if (e) (void)hipEventDestroy(e);
  if (h->ev_join) (void)hipEventDestroy(h->ev_join);
  if (h->ev_pend) (void)hipEventDestroy(h->ev_pend);
  if (h->side) (void)hipStreamDestroy(h->side);
  if (h->utag) (void)hipFree(h->utag);
  delete h;
}

int ba3c_num_tensors(const ba3c_handle* h) { return h ? (int)h->tensors.size() : 0; }

int ba3c_tensor_info(const ba3c_handle* h, int32_t i, const char** name, int64_t* offset,
                     int64_t* numel, int32_t shape[4], int32_t* ndim) {
  if (!h || i < 0 || i >= (int)h->tensors.size()) return fail(BA3C_ERR_INVALID, "bad tensor index");
  const TensorDesc& d = h->tensors[i];
  if (name) *name = d.name.c_str();
  if (offset) *offset = d.offset;
  if (numel) *numel = d.numel;
  if (shape)
    for (int k = 0; k < 4; ++k) shape[k] = d.shape[k];
  if (ndim) *ndim = d.ndim;
  return BA3C_OK;
}

int64_t ba3c_flat_size(const ba3c_handle* h) { return h ? h->flat : 0; }

int ba3c_workspace_tensor(const ba3c_handle* h, int32_t batch, int32_t train, const char* name,
                          int64_t* offset_bytes, int64_t* bytes) {
  if (!h || !name || batch < 1) return fail(BA3C_ERR_INVALID, "bad argument");
  Workspace w = carve(h, nullptr, batch, train != 0);
  // carve() with a null base returns offsets as pointers from 0
  const size_t Bz = (size_t)batch;
  const int F = h->cfg.fc_neurons;
  struct Item { const char* n; const void* p; size_t b; };
  const Item items[] = {
      {"p0", w.p0, Bz * P0 * 4}, {"p1", w.p1, Bz * P1 * 4}, {"p2", w.p2, Bz * P2 * 4},
      {"a3", w.a3, Bz * A3 * 4}, {"h", w.h, Bz * F * 4},     {"c0", w.c0, Bz * P0},
      {"c1", w.c1, Bz * P1},     {"c2", w.c2, Bz * P2},     {"dh", w.dh, Bz * F * 4},
      {"dy3", w.dy3, Bz * A3 * 4}, {"dp2", w.dp2, Bz * P2 * 4}, {"dp1", w.dp1, Bz * P1 * 4},
      {"dp0", w.dp0, Bz * P0 * 4}};
  for (const Item& it : items) {
    if (std::strcmp(it.n, name) == 0) {
      if (!train && it.n[0] != 'p' && it.n[0] != 'a' && it.n[0] != 'h')
        return fail(BA3C_ERR_INVALID, "tensor only exists in the training workspace");
      if (offset_bytes) *offset_bytes = (int64_t)reinterpret_cast<uintptr_t>(it.p);
      if (bytes) *bytes = (int64_t)it.b;
      return BA3C_OK;
    }
  }
  return fail(BA3C_ERR_INVALID, std::string("unknown workspace tensor ") + name);
}

size_t ba3c_workspace_size(const ba3c_handle* h, int32_t batch, int32_t train) {
  if (!h || batch < 1) return 0;
  return carve(h, nullptr, batch, train != 0).bytes;
}

static int flush_reduce(ba3c_handle* h, hipStream_t s);
static int flush_held(ba3c_handle* h, hipStream_t s, bool order = true);

int ba3c_forward(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                 int32_t batch, float explore_factor, void* workspace, float* probs,
                 float* probsT, float* value) {
  if (!h || !check_ptr(params) || !check_ptr(state) || !check_ptr(workspace))
    return fail(BA3C_ERR_INVALID, "null or misaligned pointer");
  if (batch < 1 || batch > h->cfg.max_batch) return fail(BA3C_ERR_INVALID, "batch out of range");
  hipStream_t s = static_cast<hipStream_t>(stream);
  CHECK(flush_reduce(h, s));
  CHECK(flush_held(h, s));
  Workspace w = carve(h, workspace, batch, false);
  std::memset(h->merged, 0, sizeof(h->merged));
  int r = h->cfg.channels == 4 ? run_forward<4>(h, s, params, state, batch, w, false)
                               : run_forward<12>(h, s, params, state, batch, w, false);
  if (r != BA3C_OK) return r;
  return run_heads(h, s, params, w, batch, nullptr, nullptr, 0.f, explore_factor, false, probs,
                   probsT, value);
}

static int train_grads_impl(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                            const int64_t* action, const float* futurereward, int32_t batch,
                            float entropy_beta, void* workspace, float* grads, double* scalars,
                            int32_t phase);

// launch a reduction a phase-3 pass left pending, on the pass's stream; a call on another
// stream `s` then waits for it (an event recorded by the caller after the pass predates it)
static int flush_reduce(ba3c_handle* h, hipStream_t s) {
  if (!h || !h->pend_reduce) return BA3C_OK;
  h->pend_reduce = false;
  const ReduceJobs& jb = h->rjobs;
  {
    ProbeScope ps(h, h->pend_stream, BA3C_K_WGRAD_REDUCE);
    hipLaunchKernelGGL(wgrad_reduce_all_kernel, dim3(jb.blk0[jb.n]), dim3(64 * RED_G), 0, h->pend_stream, jb);
  }
  HIP_TRY(hipGetLastError());
  if (s != h->pend_stream) {
    if (!h->ev_pend) HIP_TRY(hipEventCreateWithFlags(&h->ev_pend, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(h->ev_pend, h->pend_stream));
    HIP_TRY(hipStreamWaitEvent(s, h->ev_pend, 0));
  }
  return BA3C_OK;
}

// launch the fc1 + heads reduction a phase-4 pass held back, on stream `s`; `order`: after
// everything enqueued on the pass's stream so far (an event, when the streams differ).
// ba3c_launch_held leaves the ordering to its caller (the N>1 step orders the exchange stream
// after the phase-2 event, i.e. after phase 1, not after the whole of phase 2)
static int flush_held(ba3c_handle* h, hipStream_t s, bool order) {
  if (!h || !h->held) return BA3C_OK;
  h->held = false;
  if (order && s != h->held_stream) {
    if (!h->ev_pend) HIP_TRY(hipEventCreateWithFlags(&h->ev_pend, hipEventDisableTiming));
    HIP_TRY(hipEventRecord(h->ev_pend, h->held_stream));
    HIP_TRY(hipStreamWaitEvent(s, h->ev_pend, 0));
  }
  const ReduceJobs& jb = h->held_jobs;
  {
    ProbeScope ps(h, s, BA3C_K_WGRAD_REDUCE);
    hipLaunchKernelGGL(wgrad_reduce_all_kernel, dim3(jb.blk0[jb.n]), dim3(64 * RED_G), 0, s, jb);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_launch_held(ba3c_handle* h, void* stream) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  return flush_held(h, static_cast<hipStream_t>(stream), false);
}

int ba3c_set_phase2_event(ba3c_handle* h, void* event) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  h->ev_mid = static_cast<hipEvent_t>(event);
  return BA3C_OK;
}

int ba3c_train_grads(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                     const int64_t* action, const float* futurereward, int32_t batch,
                     float entropy_beta, void* workspace, float* grads, double* scalars) {
  return train_grads_impl(h, stream, params, state, action, futurereward, batch, entropy_beta, workspace,
                          grads, scalars, 0);
}

int ba3c_train_grads_phase(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                           const int64_t* action, const float* futurereward, int32_t batch,
                           float entropy_beta, void* workspace, float* grads, double* scalars,
                           int32_t phase) {
  if (phase < 0 || phase > 4) return fail(BA3C_ERR_INVALID, "phase must be 0, 1, 2, 3 or 4");
  if (phase != 3)
    return train_grads_impl(h, stream, params, state, action, futurereward, batch, entropy_beta, workspace,
                            grads, scalars, phase);
  if (h) h->defer_final = true;
  const int r = train_grads_impl(h, stream, params, state, action, futurereward, batch, entropy_beta,
                                 workspace, grads, scalars, 0);
  if (h) h->defer_final = false;
  return r;
}

int ba3c_bucket_tensor(const ba3c_handle* h) { return h ? h->idx_fc1 : -1; }

int ba3c_flush_pending(ba3c_handle* h) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  CHECK(flush_reduce(h, h->pend_stream));
  return flush_held(h, h->held_stream);
}

static int train_grads_impl(ba3c_handle* h, void* stream, const float* params, const uint8_t* state,
                            const int64_t* action, const float* futurereward, int32_t batch,
                            float entropy_beta, void* workspace, float* grads, double* scalars,
                            int32_t phase) {
  if (!h || !check_ptr(params) || !check_ptr(state) || !check_ptr(workspace) || !check_ptr(grads) ||
      !action || !futurereward)
    return fail(BA3C_ERR_INVALID, "null or misaligned pointer");
  if (batch < 1 || batch > h->cfg.max_batch) return fail(BA3C_ERR_INVALID, "batch out of range");
  hipStream_t s = static_cast<hipStream_t>(stream);
  CHECK(flush_reduce(h, s));
  if (phase != 2) CHECK(flush_held(h, s));   // phase 2 runs beside the held reduction
  CHECK(ensure_side_stream(h, s));
  Workspace w = carve(h, workspace, batch, true);
  // no memset of `grads`: the backward pass's single reduction launch writes every element
  // of every tensor (incl. conv0's zero-padded channels)
  if (phase == 2)   // conv layers' backward on the workspace phase 1 left
    return h->cfg.channels == 4 ? run_backward<4>(h, s, params, state, batch, w, grads, 2)
                                : run_backward<12>(h, s, params, state, batch, w, grads, 2);
  std::memset(h->merged, 0, sizeof(h->merged));   // a new training pass
  // on the split path the weight-prep launch zeroes the ReLU counters
  if (!h->band) HIP_TRY(hipMemsetAsync(w.relu, 0, RELU_WORDS * 8, s));
  int r = h->cfg.channels == 4 ? run_forward<4>(h, s, params, state, batch, w, true)
                               : run_forward<12>(h, s, params, state, batch, w, true);
  if (r != BA3C_OK) return r;
  // heads + loss + its gradient, fc1's split-K finish and (last workgroup) the TfDictOp scalars
  h->pend_scalars = false;
  CHECK(run_heads(h, s, params, w, batch, action, futurereward, entropy_beta, 1.0f, true, nullptr,
                  nullptr, nullptr, scalars, phase != 2 && h->scalars_ride && h->g6));
  if (h->cfg.channels == 4)
    return run_backward<4>(h, s, params, state, batch, w, grads, phase);
  return run_backward<12>(h, s, params, state, batch, w, grads, phase);
}

int ba3c_clip_grads_range(ba3c_handle* h, void* stream, float* grads, void* workspace, int32_t t0,
                          int32_t t1) {
  return ba3c_clip_grads_range2(h, stream, grads, workspace, t0, t1, 0);
}

int ba3c_clip_grads_range2(ba3c_handle* h, void* stream, float* grads, void* workspace, int32_t t0,
                           int32_t t1, int32_t flags) {
  if (!h || !check_ptr(grads) || !check_ptr(workspace)) return fail(BA3C_ERR_INVALID, "null pointer");
  if (t0 < 0 || t1 > h->table.n || t0 >= t1) return fail(BA3C_ERR_INVALID, "bad tensor range");
  if (flags & ~BA3C_CLIP_NO_RESIDENCY) return fail(BA3C_ERR_INVALID, "unknown clip flags");
  hipStream_t s = static_cast<hipStream_t>(stream);
  CHECK(flush_reduce(h, s));
  if (t1 > h->idx_fc1) CHECK(flush_held(h, s));   // the range holds tensors the held reduction writes
  float* part = carve(h, workspace, 1, false).sumsq;
  const int c0 = h->table.chunk0[t0], nc = h->table.chunk0[t1] - c0;
  ProbeScope ps(h, s, BA3C_K_CLIP);
  if (h->ctag && h->fused_update && nc <= h->cus && !(flags & BA3C_CLIP_NO_RESIDENCY)) {
    // one launch (tagged partials), bit-identical to the two below
    const UpdateSync us{h->ctag, reinterpret_cast<unsigned int*>(h->ctag + h->table.nchunks)};
    hipLaunchKernelGGL(clip_range_kernel, dim3(nc), dim3(256), 0, s, grads, h->table, c0, us);
  } else {
    hipLaunchKernelGGL(sumsq_kernel, dim3(nc), dim3(256), 0, s, grads, h->table, part, c0);
    hipLaunchKernelGGL(clip_kernel, dim3(nc), dim3(256), 0, s, grads, h->table, (const float*)part, c0);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_clip_grads(ba3c_handle* h, void* stream, float* grads, void* workspace) {
  if (!h || !check_ptr(grads) || !check_ptr(workspace)) return fail(BA3C_ERR_INVALID, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  CHECK(flush_reduce(h, s));
  CHECK(flush_held(h, s));
  float* part = carve(h, workspace, 1, false).sumsq;  // batch-independent first region
  {
    ProbeScope ps(h, s, BA3C_K_CLIP);
    hipLaunchKernelGGL(sumsq_kernel, dim3(h->table.nchunks), dim3(256), 0, s, grads, h->table, part, 0);
    hipLaunchKernelGGL(clip_kernel, dim3(h->table.nchunks), dim3(256), 0, s, grads, h->table,
                       (const float*)part, 0);
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

static int apply_update_impl(ba3c_handle* h, void* stream, int32_t opt, float* params,
                             const float* grads, float* slot0, float* slot1,
                             const ba3c_opt_params* hp, float* dev_powers, float grad_scale,
                             int32_t fuse_clip, void* workspace) {
  if (!h || !hp || !check_ptr(params) || !check_ptr(grads)) return fail(BA3C_ERR_INVALID, "null pointer");
  const bool need0 = opt != BA3C_OPT_GD, need1 = opt == BA3C_OPT_ADAM || opt == BA3C_OPT_RMS || opt == BA3C_OPT_ADADELTA;
  if ((need0 && !check_ptr(slot0)) || (need1 && !check_ptr(slot1)))
    return fail(BA3C_ERR_INVALID, "missing optimizer slot");
  if (fuse_clip && !check_ptr(workspace)) return fail(BA3C_ERR_INVALID, "fuse_clip needs a workspace");
  // validated before anything is launched or the pending reduction is consumed (ADVICE r05:
  // the chained branch below clears pend_reduce, so an unknown id there would drop it)
  if (opt < BA3C_OPT_ADAM || opt > BA3C_OPT_RMS) return fail(BA3C_ERR_INVALID, "unknown optimizer id");
  hipStream_t s = static_cast<hipStream_t>(stream);
  UpdateArgs a{};
  a.p = params;
  a.g = grads;
  a.s0 = slot0;
  a.s1 = slot1;
  a.grad_scale = grad_scale;
  a.lr = hp->lr;
  // TF-1.2 float32 scalar arithmetic of ApplyAdam: alpha = lr*sqrt(1-b2^t)/(1-b1^t)
  a.alpha = dev_powers ? 0.f : adam_alpha(hp->lr, hp->beta1_power, hp->beta2_power);
  a.dev_powers = dev_powers;
  a.one_minus_b1 = 1.0f - hp->beta1;
  a.one_minus_b2 = 1.0f - hp->beta2;
  a.eps = hp->epsilon;
  a.decay_c = 1.0f - hp->decay;
  a.momentum = hp->momentum;
  a.rho = hp->rho;
  a.one_minus_rho = 1.0f - hp->rho;
  a.beta1 = hp->beta1;
  a.beta2 = hp->beta2;
  float* part = carve(h, workspace, 1, false).sumsq;  // batch-independent first region
  const bool fused = fuse_clip && h->fused_update && h->utag && h->table.nchunks <= h->cus;
  if (RED_G == 4 && fused && h->pend_reduce && h->pend_stream == s && h->pend_grads == grads && chain_ok(h)) {
    // the pending reduction and this apply as one chained launch: the reduce workgroups
    // signal, the chunks wait for them before reading their gradient
    h->pend_reduce = false;
    const ReduceJobs& jb = h->rjobs;
    ClipUpdArgs ca{a, h->table, UpdateSync{h->utag, reinterpret_cast<unsigned int*>(h->utag + h->table.nchunks)},
                   h->spread, CHAIN_SPREAD, (unsigned)jb.blk0[jb.n], h->chain + 4 * CHAIN_SITES};
    ca.a.clip_part = part;
    const dim3 gr(jb.blk0[jb.n]), gu(h->table.nchunks);
    h->merged[BA3C_K_UPDATE] |= 1u << BA3C_K_WGRAD_REDUCE;
#define BA3C_RCU(O)                                                                                     \
  launch_chain<false, ReduceJob, ClipUpdJob<O>>(s, CHAIN_REDUCE_UPDATE, 1, 2, 2, jb, gr, ca, gu, 0, dim3(0, 1, 1), h, \
                                                BA3C_K_UPDATE, true)
    switch (opt) {
      case BA3C_OPT_ADAM: return BA3C_RCU(0);
      case BA3C_OPT_GD: return BA3C_RCU(1);
      case BA3C_OPT_ADAGRAD: return BA3C_RCU(2);
      case BA3C_OPT_ADADELTA: return BA3C_RCU(3);
      case BA3C_OPT_MOMENTUM: return BA3C_RCU(4);
      case BA3C_OPT_RMS: return BA3C_RCU(5);
      default: return fail(BA3C_ERR_INVALID, "unknown optimizer id");
    }
#undef BA3C_RCU
  }
  CHECK(flush_reduce(h, s));
  CHECK(flush_held(h, s));
  if (fused) {
    a.clip_part = part;
    const dim3 grid(h->table.nchunks);
    const UpdateSync us{h->utag, reinterpret_cast<unsigned int*>(h->utag + h->table.nchunks)};
    {
      ProbeScope ps(h, s, BA3C_K_UPDATE);
      switch (opt) {
        case BA3C_OPT_ADAM: hipLaunchKernelGGL(clip_update_kernel<0>, grid, dim3(256), 0, s, a, h->table, us); break;
        case BA3C_OPT_GD: hipLaunchKernelGGL(clip_update_kernel<1>, grid, dim3(256), 0, s, a, h->table, us); break;
        case BA3C_OPT_ADAGRAD: hipLaunchKernelGGL(clip_update_kernel<2>, grid, dim3(256), 0, s, a, h->table, us); break;
        case BA3C_OPT_ADADELTA: hipLaunchKernelGGL(clip_update_kernel<3>, grid, dim3(256), 0, s, a, h->table, us); break;
        case BA3C_OPT_MOMENTUM: hipLaunchKernelGGL(clip_update_kernel<4>, grid, dim3(256), 0, s, a, h->table, us); break;
        case BA3C_OPT_RMS: hipLaunchKernelGGL(clip_update_kernel<5>, grid, dim3(256), 0, s, a, h->table, us); break;
        default: return fail(BA3C_ERR_INVALID, "unknown optimizer id");
      }
    }
    HIP_TRY(hipGetLastError());
    return BA3C_OK;   // the Adam device powers advanced inside the launch
  }
  if (fuse_clip) {
    hipLaunchKernelGGL(sumsq_kernel, dim3(h->table.nchunks), dim3(256), 0, s, grads, h->table, part, 0);
    HIP_TRY(hipGetLastError());
    a.clip_part = part;
  }
  dim3 grid(h->table.nchunks);
  {
    ProbeScope ps(h, s, BA3C_K_UPDATE);
    switch (opt) {
      case BA3C_OPT_ADAM: hipLaunchKernelGGL(update_kernel<0>, grid, dim3(256), 0, s, a, h->table); break;
      case BA3C_OPT_GD: hipLaunchKernelGGL(update_kernel<1>, grid, dim3(256), 0, s, a, h->table); break;
      case BA3C_OPT_ADAGRAD: hipLaunchKernelGGL(update_kernel<2>, grid, dim3(256), 0, s, a, h->table); break;
      case BA3C_OPT_ADADELTA: hipLaunchKernelGGL(update_kernel<3>, grid, dim3(256), 0, s, a, h->table); break;
      case BA3C_OPT_MOMENTUM: hipLaunchKernelGGL(update_kernel<4>, grid, dim3(256), 0, s, a, h->table); break;
      case BA3C_OPT_RMS: hipLaunchKernelGGL(update_kernel<5>, grid, dim3(256), 0, s, a, h->table); break;
      default: return fail(BA3C_ERR_INVALID, "unknown optimizer id");
    }
  }
  HIP_TRY(hipGetLastError());
  if (opt == BA3C_OPT_ADAM && dev_powers) {
    hipLaunchKernelGGL(adam_powers_kernel, dim3(1), dim3(64), 0, s, dev_powers, hp->beta1, hp->beta2);
    HIP_TRY(hipGetLastError());
  }
  return BA3C_OK;
}

int ba3c_apply_update(ba3c_handle* h, void* stream, int32_t opt, float* params,
                      const float* grads, float* slot0, float* slot1, const ba3c_opt_params* hp,
                      float grad_scale, int32_t fuse_clip, void* workspace) {
  return apply_update_impl(h, stream, opt, params, grads, slot0, slot1, hp, nullptr, grad_scale,
                           fuse_clip, workspace);
}

int ba3c_apply_update_dev(ba3c_handle* h, void* stream, int32_t opt, float* params,
                          const float* grads, float* slot0, float* slot1,
                          const ba3c_opt_params* hp, float* dev_powers, float grad_scale,
                          int32_t fuse_clip, void* workspace) {
  if (opt == BA3C_OPT_ADAM && !check_ptr(dev_powers) && dev_powers == nullptr)
    return fail(BA3C_ERR_INVALID, "dev_powers required");
  return apply_update_impl(h, stream, opt, params, grads, slot0, slot1, hp, dev_powers, grad_scale,
                           fuse_clip, workspace);
}

int ba3c_sample(void* stream, const float* probs, const double* u, int32_t batch,
                int32_t num_actions, int64_t* actions, int32_t* nonfinite) {
  if (!probs || !u || !actions) return fail(BA3C_ERR_INVALID, "null pointer");
  if (batch < 0 || num_actions < 1 || num_actions >= MAXA) return fail(BA3C_ERR_INVALID, "bad shape");
  if (batch == 0) return BA3C_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(sample_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, probs, u, batch,
                     num_actions, actions, nonfinite);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_greedy(void* stream, const float* probs, const double* u, const int64_t* random_actions,
                int32_t batch, int32_t num_actions, double eps, int64_t* actions) {
  if (batch < 0 || num_actions < 1) return fail(BA3C_ERR_INVALID, "bad shape");
  if (batch == 0) return BA3C_OK;
  if (!probs || !u || !random_actions || !actions) return fail(BA3C_ERR_INVALID, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipLaunchKernelGGL(greedy_kernel, dim3((batch + 255) / 256), dim3(256), 0, s, probs, u, random_actions,
                     batch, num_actions, eps, actions);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_probe_enable(ba3c_handle* h, int32_t kernel_id) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  if (kernel_id >= BA3C_NUM_KERNELS) return fail(BA3C_ERR_INVALID, "bad kernel id");
  if (h->ev_begin.empty() && kernel_id >= 0) {
    h->ev_begin.resize(4096);
    h->ev_end.resize(4096);
    // timestamps only: no system-scope fence (its L2 write-back + invalidate left a 5-6 us
    // gap around every probed launch, r06a trace)
    // (BA3C_EVENTS=torch: HIP's default events, the A/B of ba3c_amd/hipevent.py)
    const char* em = getenv("BA3C_EVENTS");
    const unsigned fl = (em && std::strcmp(em, "torch") == 0) ? hipEventDefault : hipEventDisableSystemFence;
    for (size_t i = 0; i < h->ev_begin.size(); ++i) {
      HIP_TRY(hipEventCreateWithFlags(&h->ev_begin[i], fl));
      HIP_TRY(hipEventCreateWithFlags(&h->ev_end[i], fl));
    }
  }
  h->probe_kernel = kernel_id;
  h->probe_seen = 0;
  h->probe_used = 0;
  h->probe_ms = 0.0;
  h->probe_launches = 0;
  return BA3C_OK;
}

int ba3c_nstep_returns(void* stream, const double* reward, const float* value,
                       const int32_t* start, const int32_t* length, const uint8_t* is_over,
                       int32_t n_envs, int32_t slots, double gamma, float* R, int32_t* src,
                       float* init_R, uint8_t* over, int32_t* count) {
  if (!reward || !value || !start || !length || !is_over || !R || !src || !init_R || !over || !count)
    return fail(BA3C_ERR_INVALID, "null pointer");
  if (n_envs < 0 || slots < 1) return fail(BA3C_ERR_INVALID, "bad shape");
  hipStream_t s = static_cast<hipStream_t>(stream);
  ReturnsArgs a{reward, value, start, length, is_over, n_envs, slots, gamma, R, src, init_R, over, count};
  hipLaunchKernelGGL(nstep_returns_kernel, dim3(1), dim3(1024), 0, s, a);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_gather_rows(void* stream, const void* rows, const int32_t* idx, int32_t n,
                     int64_t row_bytes, void* out) {
  if (n < 0) return fail(BA3C_ERR_INVALID, "bad count");
  if (n == 0) return BA3C_OK;
  if (!rows || !idx || !out) return fail(BA3C_ERR_INVALID, "null pointer");
  hipStream_t s = static_cast<hipStream_t>(stream);
  if (row_bytes == 8) {
    hipLaunchKernelGGL(gather_i64_kernel, dim3((n + 255) / 256), dim3(256), 0, s,
                       static_cast<const int64_t*>(rows), idx, n, static_cast<int64_t*>(out));
  } else if (row_bytes > 0 && row_bytes % 16 == 0 && check_ptr(rows) && check_ptr(out)) {
    const int words = (int)(row_bytes / 16);
    const int gx = std::min(8, (words + 255) / 256);
    hipLaunchKernelGGL(gather_rows16_kernel, dim3(gx, n), dim3(256), 0, s,
                       static_cast<const uint4*>(rows), idx, n, words, static_cast<uint4*>(out));
  } else {
    return fail(BA3C_ERR_INVALID, "row_bytes must be 8 or a multiple of 16 (16-byte aligned rows)");
  }
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_history_push(void* stream, const uint8_t* frame, uint8_t* state, const uint8_t* is_over,
                      int32_t n_envs, int32_t pixels, int32_t hist_len, int32_t channels) {
  if (!frame || !state) return fail(BA3C_ERR_INVALID, "null pointer");
  if (n_envs < 0 || pixels < 1 || hist_len < 1 || channels < 1) return fail(BA3C_ERR_INVALID, "bad shape");
  if (n_envs == 0) return BA3C_OK;
  if (hist_len * channels == 4 && channels == 1 && (!check_ptr(state) || (reinterpret_cast<uintptr_t>(frame) & 3)))
    return fail(BA3C_ERR_INVALID, "state must be 16-byte and frame 4-byte aligned");
  hipStream_t s = static_cast<hipStream_t>(stream);
  HistoryArgs a{frame, state, is_over, n_envs, pixels, hist_len, channels};
  const int groups = (pixels + 3) / 4;
  hipLaunchKernelGGL(history_push_kernel, dim3((groups + 255) / 256, n_envs), dim3(256), 0, s, a);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_kernel_split(const ba3c_handle* h, int32_t kid) {
  if (!h || kid < 0 || kid >= BA3C_NUM_KERNELS) return -1;
  const bool c4 = h->cfg.channels == 4;
  switch (kid) {
    case BA3C_K_CONV0_FWD:
    case BA3C_K_CONV0_WGRAD: return (h->band && c4) ? 2 : (h->g6 ? 6 : 1);
    case BA3C_K_CONV1_FWD:
    case BA3C_K_CONV2_FWD:
    case BA3C_K_CONV1_DGRAD:
    case BA3C_K_CONV2_DGRAD:
    case BA3C_K_CONV1_WGRAD:
    case BA3C_K_CONV2_WGRAD: return h->band ? 3 : 1;
    // conv3: whole-image fp16x3 kernels (ba3c_conv3.h)
    case BA3C_K_CONV3_FWD:
    case BA3C_K_CONV3_DGRAD:
    case BA3C_K_CONV3_WGRAD: return h->band ? 3 : (h->g6 ? 6 : 1);
    case BA3C_K_FC1_FWD:
    case BA3C_K_FC1_DGRAD:
    case BA3C_K_FC1_WGRAD:
    case BA3C_K_HEAD_WGRAD: return h->g6 ? 6 : 1;
    case BA3C_K_HEADS:
    case BA3C_K_WGRAD_REDUCE:
    case BA3C_K_CLIP:
    case BA3C_K_UPDATE: return 0;
    default: return 1;
  }
}

int ba3c_kernel_merged(const ba3c_handle* h, int32_t kid) {
  if (!h || kid < 0 || kid >= BA3C_NUM_KERNELS) return -1;
  return (int)h->merged[kid];
}

int ba3c_kernel_family(const ba3c_handle* h, int32_t kid) {
  if (!h || kid < 0 || kid >= BA3C_NUM_KERNELS) return -1;
  const int sp = ba3c_kernel_split(h, kid);
  if (sp <= 1) return sp;
  const bool band_split = kid == BA3C_K_CONV0_FWD || kid == BA3C_K_CONV0_WGRAD || kid == BA3C_K_CONV1_FWD ||
                          kid == BA3C_K_CONV2_FWD || kid == BA3C_K_CONV1_DGRAD || kid == BA3C_K_CONV2_DGRAD ||
                          kid == BA3C_K_CONV1_WGRAD || kid == BA3C_K_CONV2_WGRAD ||
                          kid == BA3C_K_CONV3_FWD || kid == BA3C_K_CONV3_DGRAD || kid == BA3C_K_CONV3_WGRAD;
  if (kid == BA3C_K_CONV0_FWD || kid == BA3C_K_CONV0_WGRAD)
    if (!(h->band && h->cfg.channels == 4)) return 3;
  return band_split ? 2 : 3;
}

int ba3c_device_errors(ba3c_handle* h, uint32_t* flags) {
  if (!h || !flags) return fail(BA3C_ERR_INVALID, "null argument");
  *flags = 0;
  CHECK(flush_reduce(h, h->pend_stream));
  CHECK(flush_held(h, h->held_stream));
  if (!h->utag) return BA3C_OK;
  // every stream, the non-blocking ones torch creates included (a null-stream copy does not
  // wait for those)
  HIP_TRY(hipDeviceSynchronize());
  uint32_t e = 0, e2 = 0, e3 = 0;
  HIP_TRY(hipMemcpy(&e, h->utag + h->table.nchunks, sizeof(e), hipMemcpyDeviceToHost));
  if (h->ctag) HIP_TRY(hipMemcpy(&e2, h->ctag + h->table.nchunks, sizeof(e2), hipMemcpyDeviceToHost));
  if (h->chain) HIP_TRY(hipMemcpy(&e3, h->chain + 4 * CHAIN_SITES, sizeof(e3), hipMemcpyDeviceToHost));
  if (e3 && h->chain_on) {
    // a chained wait gave up: a late signal may have landed after the last waiter reset the
    // site's words, so they can no longer be trusted.  Zero them from the host and stop
    // chaining on this handle (the error bit stays set)
    h->chain_on = false;
    HIP_TRY(hipMemset(h->chain, 0, 4 * CHAIN_SITES * sizeof(unsigned)));
    HIP_TRY(hipMemset(h->spread, 0, CHAIN_SPREAD * CHAIN_STRIDE * sizeof(unsigned)));
  }
  *flags = e | (e2 << 1) | (e3 << 2);
  return BA3C_OK;
}

int ba3c_occupy_cus(void* stream, int32_t n_cus, double usec) {
  if (n_cus < 0 || n_cus > 4096 || !(usec >= 0.0) || usec > 1e6)
    return fail(BA3C_ERR_INVALID, "n_cus in [0, 4096], usec in [0, 1e6]");
  if (n_cus == 0 || usec == 0.0) return BA3C_OK;
  hipLaunchKernelGGL(occupy_kernel, dim3(n_cus), dim3(64), 0, static_cast<hipStream_t>(stream),
                     (unsigned long long)(usec * 100.0));   // 100 MHz realtime clock
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

// ---- gradient exchange through the C ABI ----------
// RCCL is resolved at run time from the library already loaded in the process (torch's copy,
// or /opt/rocm's librccl.so.1 for a caller without torch): both carry the soname
// librccl.so.1, so one RCCL serves torch.distributed and these entry points.

int ba3c_comm_unique_id(void* id_out) {
  if (!id_out) return fail(BA3C_ERR_INVALID, "null argument");
  if (!rccl().ok) return fail(BA3C_ERR_HIP, "RCCL (librccl.so.1) not found");
  ncclUniqueId id;
  const ncclResult_t e = rccl().get_unique_id(&id);
  if (e != ncclSuccess) return rccl_fail(e, "ncclGetUniqueId");
  std::memcpy(id_out, &id, sizeof(id));
  return BA3C_OK;
}

int ba3c_comm_init(ba3c_handle* h, const void* id, int32_t nranks, int32_t rank) {
  if (!h || !id) return fail(BA3C_ERR_INVALID, "null argument");
  if (nranks < 1 || rank < 0 || rank >= nranks) return fail(BA3C_ERR_INVALID, "bad rank / rank count");
  if (h->comm) return fail(BA3C_ERR_INVALID, "the handle already has a communicator");
  if (!rccl().ok) return fail(BA3C_ERR_HIP, "RCCL (librccl.so.1) not found");
  ncclUniqueId uid;
  std::memcpy(&uid, id, sizeof(uid));
  const ncclResult_t e = rccl().init_rank(&h->comm, nranks, uid, rank);
  if (e != ncclSuccess) {
    h->comm = nullptr;
    return rccl_fail(e, "ncclCommInitRank");
  }
  h->comm_ranks = nranks;
  return BA3C_OK;
}

int ba3c_comm_destroy(ba3c_handle* h, int32_t abort) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  if (!h->comm) return BA3C_OK;
  const ncclResult_t e = abort ? rccl().abort(h->comm) : rccl().destroy(h->comm);
  h->comm = nullptr;
  h->comm_ranks = 0;
  if (e != ncclSuccess) return rccl_fail(e, abort ? "ncclCommAbort" : "ncclCommDestroy");
  return BA3C_OK;
}

int ba3c_allreduce_sum(ba3c_handle* h, void* stream, float* buf, int64_t count) {
  if (!h || !buf || count < 0) return fail(BA3C_ERR_INVALID, "bad argument");
  if (!h->comm) return fail(BA3C_ERR_INVALID, "no communicator (ba3c_comm_init)");
  CHECK(flush_reduce(h, static_cast<hipStream_t>(stream)));
  CHECK(flush_held(h, static_cast<hipStream_t>(stream)));
  const ncclResult_t e = rccl().all_reduce(buf, buf, (size_t)count, ncclFloat32, ncclSum, h->comm,
                                           static_cast<hipStream_t>(stream));
  if (e != ncclSuccess) return rccl_fail(e, "ncclAllReduce");
  return BA3C_OK;
}

int ba3c_allreduce_mean(ba3c_handle* h, void* stream, float* grads, int64_t count) {
  if (!check_ptr(grads)) return fail(BA3C_ERR_INVALID, "null or misaligned pointer");
  CHECK(ba3c_allreduce_sum(h, stream, grads, count));
  if (h->comm_ranks == 1 || count == 0) return BA3C_OK;   // x / 1 == x
  const float inv = 1.0f / (float)h->comm_ranks;
  hipLaunchKernelGGL(scale_kernel, dim3((unsigned)std::min<int64_t>((count + 1023) / 1024, 4096)), dim3(256), 0,
                     static_cast<hipStream_t>(stream), grads, count, inv);
  HIP_TRY(hipGetLastError());
  return BA3C_OK;
}

int ba3c_probe_every(ba3c_handle* h, int32_t n) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  if (n < 1) return fail(BA3C_ERR_INVALID, "probe interval must be >= 1");
  h->probe_every = n;
  h->probe_seen = 0;
  return BA3C_OK;
}

int ba3c_probe_read(ba3c_handle* h, double* total_ms, int32_t* launches) {
  if (!h) return fail(BA3C_ERR_INVALID, "null handle");
  for (int i = 0; i < h->probe_used; ++i) {
    HIP_TRY(hipEventSynchronize(h->ev_end[i]));
    float ms = 0.f;
    HIP_TRY(hipEventElapsedTime(&ms, h->ev_begin[i], h->ev_end[i]));
    h->probe_ms += ms;
    h->probe_launches++;
  }
  h->probe_used = 0;
  if (total_ms) *total_ms = h->probe_ms;
  if (launches) *launches = h->probe_launches;
  return BA3C_OK;
}

}  // extern "C"
