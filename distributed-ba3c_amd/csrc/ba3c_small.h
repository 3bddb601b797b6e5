// ba3c_small.h — HBM/latency-bound kernels of the BA3C step: policy/value heads + softmax +
// A3C loss + its gradient (train.py:250-327), scalar reduction, deterministic split-K
// reduction of weight gradients, tf.clip_by_average_norm (train.py:329-330), the TF-1.2
// optimizer applies (train.py:582-597) and numpy-exact action sampling (train.py:382).
#pragma once
#include "ba3c_problems.h"

namespace ba3c {

constexpr int MAXA = 32;        // dz|dv row pitch; num_actions <= 31
constexpr int NTERMS = 8;       // per-sample loss terms
constexpr int MAXT = 48;        // max tensors in the flat layout
constexpr int UPD_CHUNK = 4096; // floats per workgroup in clip / update kernels
static_assert(UPD_CHUNK % 256 == 0, "whole elements per thread");
constexpr int FC_SPLIT_MAX = 16;  // fc1 split-K chunks the heads kernel can finish

// Device-coherent (agent-scope) stores / loads for data that crosses workgroups inside one
// launch.  MI355X's 8 XCDs have non-coherent L2s: a plain store + __threadfence() pays an L2
// write-back per workgroup, these go to the coherence point directly.
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long ld_agent(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---------------------------------------------------------------------------------------
// Heads: one wave per sample.  z = h W_pi + b_pi, V = h W_v + b_v, p = softmax(z),
// pT = softmax(z * explore_factor); in training also the loss terms and
//   dL/dp_k = [adv [k==a]/(p_k+1e-6) + beta (log(p_k+1e-6) + p_k/(p_k+1e-6))] / B
//   dz_k = p_k (dL/dp_k - sum_j p_j dL/dp_j),  dV = (V - R) / B,
//   dh_f = sum_k dz_k W_pi[f][k] + dV W_v[f]  (x (h_f > 0) for the legacy ReLU FC).
// terms[n] = {log(p_a+1e-6)*adv, sum p log(p+1e-6), (V-R)^2, adv, V, max p, 0, 0}
// ---------------------------------------------------------------------------------------
struct HeadsArgs {
  float* h;
  const float* piW;
  const float* pib;
  const float* vW;
  const float* vb;
  const int64_t* action;
  const float* R;
  float* probs;
  float* probsT;
  float* value;
  float* dzv;
  float* dh;
  float* terms;
  int B, F, A, train, legacy;
  float beta, explore, invB;
  // fc1's split-K finish, fused: h = sum_z fcpart[z] in z order (+ bias, ReLU, positive count
  // for the legacy FC), written to `h` for the backward pass.  The split is fixed (FC_SPLIT
  // chunks of FC_KCHUNK), so every row's summation order — its rounding — is the same at any batch
  const float* fcpart;       // [fc_split][B][F]; null: h is already final
  int fc_split, per, wstride;
  const float* fc_w1;        // fc1 split 0 base (legacy bias rows)
  unsigned long long* relu_count;
  // training: the last workgroup to finish reduces terms into the TfDictOp scalars
  unsigned long long* done;  // completion counter (zero on entry; reset by the last workgroup)
  double* scalars;           // null: no scalars
};

// The per-sample head arithmetic runs in fp64: the softmax gradient
// p_k (g_k - sum_j p_j g_j) cancels catastrophically when the policy saturates, and fp64 here
// costs nothing measurable (F*(A+1) FMAs per sample) while keeping the fp32 stored results
// within rounding of the exact values.
__device__ __forceinline__ double wave_max_d(double v, int w = 64) { return wave_reduce_d(v, OpMax{}, w); }

// One wave per sample; after the dot products lane a < A owns action a, so the softmax /
// log / gradient run once per lane (one exp and one log per lane instead of MAXA of each,
// masked, in every lane) with wave reductions for the sums and maxima.
// FCH > 0: F <= 64 FCH, a lane's features f = lane + 64 i (i < FCH) are unrolled and EVERY
// load of the fc1 split-K finish (FCH x NZ chunk values, NZ = fc_split) is issued before the
// first sum — one global round trip per sample instead of one per 64 features (F=512: eight
// dependent HBM round trips per wave were most of the B=2048 heads launch).  The sums, their z
// order and every product are unchanged.  FCH == 0: the runtime loop over f (any F).
// AT > 0: the action count as a compile-time constant (AT == p.A).  With the runtime count the
// head-weight loads sat in `a < A` branches, each followed by a wait for every outstanding load:
// ~80 dependent global round trips per sample (r04 ISA) — the heads launch's whole time.  With
// AT every weight load of a lane's features is unconditional (features past F read feature
// F - 1 and are multiplied by zero), so they are all in flight together.
template <int FCH, int NZ, int AT>
__device__ __forceinline__ void heads_sample(const HeadsArgs& p, int n, int lane) {
  const int A = AT ? AT : p.A;
  constexpr int NA = AT ? AT : MAXA;                 // loop bound over actions
  double acc[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) acc[a] = 0.0;
  double accv = 0.0;
  float* hn = p.h + (size_t)n * p.F;
  unsigned long long pos = 0;
  const size_t MN = (size_t)p.B * p.F;
  // PRE (FCH > 0 and AT > 0): every value the sample reads besides fc1's partials — the head
  // weights of the lane's features, the biases, the legacy FC bias, R and the action — is
  // loaded together with the partials, before the first store.  The stores to h / probs / dzv
  // may alias those arrays for the compiler, which kept each later group of loads behind the
  // stores before it: three dependent global round trips per sample, one here.  Same values,
  // same arithmetic.
  constexpr bool PRE = FCH > 0 && AT > 0;
  float wpre[PRE ? FCH : 1][PRE ? AT + 1 : 1];   // [i][a < AT]: pi weights, [i][AT]: v weight
  float bpre[PRE ? AT + 1 : 1];                  // pi biases, v bias
  float blg[PRE ? FCH : 1];                      // legacy FC bias of the lane's features
  float Rpre = 0.f;
  int apre = 0;
  float hv32[FCH > 0 ? FCH : 1];
  if constexpr (PRE) {
    float pz[FCH][NZ];
    const int per = p.legacy ? p.per : 1;
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      // unconditional loads (a feature past F re-reads feature F - 1 and is discarded): a
      // branch around each load made the compiler drain the loads at every join
      const int f = min(lane + 64 * i, p.F - 1);
      const size_t e = (size_t)n * p.F + f;
      // no partials: every z re-reads h (only z = 0 is used) — a pointer select, not a branch
      const float* src = p.fcpart ? p.fcpart + e : hn + f;
      const size_t zs = p.fcpart ? MN : 0;
#pragma unroll
      for (int z = 0; z < NZ; ++z) pz[i][z] = src[z * zs];
      const int sidx = f / per;
      blg[i] = *(p.legacy ? p.fc_w1 + sidx * p.wstride + 1600 * per + (f - sidx * per) : p.pib);
#pragma unroll
      for (int a = 0; a < AT; ++a) wpre[i][a] = p.piW[(size_t)f * AT + a];
      wpre[i][AT] = p.vW[f];
    }
#pragma unroll
    for (int a = 0; a < AT; ++a) bpre[a] = p.pib[a];
    bpre[AT] = p.vb[0];
    Rpre = *(p.train ? p.R + n : p.pib);
    // the action's low word (actions are small and non-negative)
    apre = *(p.train ? reinterpret_cast<const int*>(p.action + n) : reinterpret_cast<const int*>(p.pib));
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int f = lane + 64 * i;
      float h32 = pz[i][0];
      if (p.fcpart) {
#pragma unroll
        for (int z = 1; z < NZ; ++z) h32 += pz[i][z];
        if (p.legacy && f < p.F) {
          h32 = fmaxf(h32 + blg[i], 0.f);
          pos += h32 > 0.f;
        }
        if (f < p.F) hn[f] = h32;
      }
      hv32[i] = f < p.F ? h32 : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const double hv = hv32[i];                      // 0 past F
#pragma unroll
      for (int a = 0; a < AT; ++a) acc[a] = fma(hv, (double)wpre[i][a], acc[a]);
      accv = fma(hv, (double)wpre[i][AT], accv);
    }
  } else if constexpr (FCH > 0) {
    if (p.fcpart) {
      float pz[FCH][NZ];
#pragma unroll
      for (int i = 0; i < FCH; ++i) {
        const int f = min(lane + 64 * i, p.F - 1);
        const size_t e = (size_t)n * p.F + f;
#pragma unroll
        for (int z = 0; z < NZ; ++z) pz[i][z] = p.fcpart[(size_t)z * MN + e];
      }
#pragma unroll
      for (int i = 0; i < FCH; ++i) {
        const int f = lane + 64 * i;
        float h32 = pz[i][0];
#pragma unroll
        for (int z = 1; z < NZ; ++z) h32 += pz[i][z];
        if (p.legacy && f < p.F) {
          const int sidx = f / p.per;
          h32 = fmaxf(h32 + p.fc_w1[sidx * p.wstride + 1600 * p.per + (f - sidx * p.per)], 0.f);
          pos += h32 > 0.f;
        }
        if (f < p.F) hn[f] = h32;
        hv32[i] = f < p.F ? h32 : 0.f;
      }
    } else {
#pragma unroll
      for (int i = 0; i < FCH; ++i) hv32[i] = lane + 64 * i < p.F ? hn[lane + 64 * i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int f = lane + 64 * i;
      if (f < p.F) {
        const double hv = hv32[i];
        const float* wr = p.piW + (size_t)f * A;
#pragma unroll
        for (int a = 0; a < NA; ++a)
          if (a < A) acc[a] = fma(hv, (double)wr[a], acc[a]);
        accv = fma(hv, (double)p.vW[f], accv);
      }
    }
  }
  for (int f = lane; FCH == 0 && f < p.F; f += 64) {
    float h32;
    if (p.fcpart) {
      const size_t e = (size_t)n * p.F + f;
      float pz[FC_SPLIT_MAX];                       // every chunk's load in flight, then the
#pragma unroll                                      // sum in z order
      for (int z = 0; z < FC_SPLIT_MAX; ++z) pz[z] = z < p.fc_split ? p.fcpart[(size_t)z * MN + e] : 0.f;
      h32 = pz[0];
#pragma unroll
      for (int z = 1; z < FC_SPLIT_MAX; ++z)
        if (z < p.fc_split) h32 += pz[z];
      if (p.legacy) {
        const int sidx = f / p.per;
        h32 = fmaxf(h32 + p.fc_w1[sidx * p.wstride + 1600 * p.per + (f - sidx * p.per)], 0.f);
        pos += h32 > 0.f;
      }
      hn[f] = h32;
    } else {
      h32 = hn[f];
    }
    const double hv = h32;
    const float* wr = p.piW + (size_t)f * A;
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if (AT || a < A) acc[a] = fma(hv, (double)wr[a], acc[a]);
    accv = fma(hv, (double)p.vW[f], accv);
  }
  const bool mine = lane < A;
  double z = 0.0;                                   // z[lane] for lane < A
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    if (AT || a < A) {
      const double za = wave_sum_d(acc[a]) + (double)(PRE ? bpre[a] : p.pib[a]);
      if (lane == a) z = za;
    }
  }
  if (p.fcpart && p.legacy && p.relu_count) relu_count_add(p.relu_count, pos, lane);
  const double V = wave_sum_d(accv) + (double)(PRE ? bpre[PRE ? AT : 0] : p.vb[0]);
  // softmax(z)  (tf.nn.softmax: exp(z - max) / sum)
  const double zmax = wave_max_d(mine ? z : -INFINITY, A);
  const double e = mine ? exp(z - zmax) : 0.0;
  const double pr = e / wave_sum_d(e, A);           // 0 for lane >= A
  const double pmax = wave_max_d(pr, A);
  if (p.probsT) {
    const double zt = z * (double)p.explore;
    const double ztmax = wave_max_d(mine ? zt : -INFINITY, A);
    const double et = mine ? exp(zt - ztmax) : 0.0;
    const double st = wave_sum_d(et, A);
    if (mine) p.probsT[(size_t)n * A + lane] = (float)(et / st);
  }
  if (p.probs && mine) p.probs[(size_t)n * A + lane] = (float)pr;
  if (p.value && lane == 0) p.value[n] = (float)V;
  if (!p.train) return;

  const double Rn = PRE ? (double)Rpre : (double)p.R[n];
  const int act = (int)(PRE ? apre : p.action[n]);
  const double adv = V - Rn;
  const double beta = (double)p.beta, invB = 1.0 / (double)p.B;
  const double pe = pr + 1e-6;
  const double lp = mine ? log(pe) : 0.0;
  const double xent = wave_sum_d(pr * lp, A);
  const double lpa = __shfl(lp, act, 64);
  const double gp = mine ? ((lane == act ? adv / pe : 0.0) + beta * (lp + pr / pe)) * invB : 0.0;
  const double sgp = wave_sum_d(gp * pr, A);
  const double dz = mine ? pr * (gp - sgp) : 0.0;
  const double dV = (V - Rn) * invB;
  // [dz | dV | 0...] row for the head weight-gradient product
  if (lane < MAXA) p.dzv[(size_t)n * MAXA + lane] = (float)(lane == A ? dV : dz);
  double dza[NA];
#pragma unroll
  for (int a = 0; a < NA; ++a) {
    dza[a] = 0.0;
    if (AT || a < A) {                               // uniform branch: A broadcasts only
      const unsigned long long u = __double_as_longlong(dz);
      const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, a), hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), a);
      dza[a] = __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
    }
  }
  float* dhn = p.dh + (size_t)n * p.F;
  auto dh_one = [&](int f) {
    const float* wr = p.piW + (size_t)f * A;
    double g = dV * (double)p.vW[f];
#pragma unroll
    for (int a = 0; a < NA; ++a)
      if (AT || a < A) g = fma(dza[a], (double)wr[a], g);
    if (p.legacy && !(hn[f] > 0.f)) g = 0.0;
    dhn[f] = (float)g;
  };
  if constexpr (PRE) {
    // the preloaded weights; the legacy ReLU mask from the h values this lane stored
#pragma unroll
    for (int i = 0; i < FCH; ++i) {
      const int f = lane + 64 * i;
      double g = dV * (double)wpre[i][AT];
#pragma unroll
      for (int a = 0; a < AT; ++a) g = fma(dza[a], (double)wpre[i][a], g);
      if (f < p.F) {
        if (p.legacy && !(hv32[i] > 0.f)) g = 0.0;
        dhn[f] = (float)g;
      }
    }
  } else if constexpr (FCH > 0) {
#pragma unroll
    for (int i = 0; i < FCH; ++i)
      if (lane + 64 * i < p.F) dh_one(lane + 64 * i);
  } else {
    for (int f = lane; f < p.F; f += 64) dh_one(f);
  }
  if (lane < NTERMS) {
    double t = 0.0;
    t = lane == 0 ? lpa * adv : t;
    t = lane == 1 ? xent : t;
    t = lane == 2 ? (V - Rn) * (V - Rn) : t;
    t = lane == 3 ? adv : t;
    t = lane == 4 ? V : t;
    t = lane == 5 ? pmax : t;
    st_agent(p.terms + (size_t)n * NTERMS + lane, (float)t);   // read by the last workgroup
  }
}

// Deterministic reduction of the per-sample terms into the TfDictOp scalars (one workgroup):
// per-thread strided sums, wave butterflies, then the 4 wave results in wave order.  (A
// 256-step serial loop over the ReLU-count partials by one thread was ~5 us of the B=32 step.)
__device__ __forceinline__ void scalars_block(const float* terms, int B, float beta,
                                              const unsigned long long* relu_count, double* out) {
  __shared__ double red[6][4];
  __shared__ unsigned long long rsum[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double s[5] = {0, 0, 0, 0, 0};
  double mx = 0.0;
  // U samples' loads in flight per thread, then the adds in sample order (one dependent round
  // trip per sample was 8 in a row at B = 2048: the 9 us scalars launch)
  constexpr int U = 8;
  for (int n0 = t; n0 < B; n0 += 256 * U) {
    float v[U][6];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // unconditional loads (past B: sample B - 1 again, not added): a conditional load was a
      // branch and a wait per value, 48 dependent round trips at B = 32
      const float* tn = terms + (size_t)min(n0 + 256 * u, B - 1) * NTERMS;
#pragma unroll
      for (int k = 0; k < 6; ++k) v[u][k] = ld_agent(tn + k);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (n0 + 256 * u < B) {
#pragma unroll
        for (int k = 0; k < 5; ++k) s[k] += v[u][k];
        mx = fmax(mx, (double)v[u][5]);
      }
    }
  }
  unsigned long long rc = 0;
  if (relu_count) {
    static_assert(RELU_SLOTS % 256 == 0, "whole slots per thread");
    unsigned long long r[RELU_SLOTS / 256];           // all in flight, then the (exact) sum
#pragma unroll
    for (int j = 0; j < RELU_SLOTS / 256; ++j) r[j] = ld_agent(relu_count + t + 256 * j);
#pragma unroll
    for (int j = 0; j < RELU_SLOTS / 256; ++j) rc += r[j];
  }
#pragma unroll
  for (int i = 0; i < 5; ++i) s[i] = wave_sum_d(s[i]);
  mx = wave_max_d(mx);
  rc = wave_sum_u64(rc);
  if (lane == 0) {
#pragma unroll
    for (int i = 0; i < 5; ++i) red[i][wv] = s[i];
    red[5][wv] = mx;
    rsum[wv] = rc;
  }
  __syncthreads();
  if (t == 0) {
    double r[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) r[i] = ((red[i][0] + red[i][1]) + red[i][2]) + red[i][3];
    const double pmax = fmax(fmax(red[5][0], red[5][1]), fmax(red[5][2], red[5][3]));
    const unsigned long long relu_total = rsum[0] + rsum[1] + rsum[2] + rsum[3];
    const double Bd = (double)B, b = (double)beta;
    const double pl = r[0], xe = r[1], vl = r[2] * 0.5;
    out[0] = (pl + xe * b + vl) / Bd;
    out[1] = pl * 128.0 / Bd;
    out[2] = xe * 128.0 / Bd * b;
    out[3] = vl * 128.0 / Bd;
    out[4] = r[3] / Bd;
    out[5] = r[4] / Bd;
    out[6] = pmax;
    out[7] = (double)relu_total;
  }
}

__global__ void __launch_bounds__(256) scalars_kernel(const float* terms, int B, float beta,
                                                      const unsigned long long* relu_count,
                                                      double* out) {
  scalars_block(terms, B, beta, relu_count, out);
}

// One wave per sample (heads_sample); in training with `scalars`, the last workgroup to
// finish (completion counter) runs the scalar reduction, so the step needs no separate scalars
// launch.  No early return: every wave reaches the barriers.  Hand-off protocol (no fences, the
// "every store sc1 / every load sc1" form of MI355X_MICROARCH.md §Correctness boundaries):
// every handed-off word is written with an agent-scope store (st_agent: global_store sc1, which
// leaves the XCD's L2) or a device atomic (ReLU counts); each wave drains its stores
// (s_waitcnt 0) and the workgroup barriers BEFORE thread 0 increments the counter; the last
// workgroup reads the words only with agent-scope loads (ld_agent: global_load sc1) after its
// barrier.  The counter itself is a device atomic.  No step relies on release/acquire ordering.
// (bx, nblk): the workgroup's index and the grid size (a plain launch: blockIdx.x, gridDim.x;
// a chained multi-job launch, ba3c_multi.h: the job's own)
template <int FCH, int NZ, int AT = 0>
__device__ __forceinline__ void heads_body(const HeadsArgs& p, int bx, int nblk) {
  const int lane = threadIdx.x & 63;
  const int n = bx * 4 + (threadIdx.x >> 6);
  if (n < p.B) heads_sample<FCH, NZ, AT>(p, n, lane);
  if (p.train && p.scalars) {                 // uniform over the grid
    // terms go out with st_agent and ReLU counts with device atomics; each wave waits for its
    // own stores before the workgroup's arrival is counted (no L2 write-back fence)
    __shared__ int last;
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0) last = atomicAdd(p.done, 1ull) == (unsigned long long)(nblk - 1);
    __syncthreads();
    if (last) {
      scalars_block(p.terms, p.B, p.beta, p.relu_count, p.scalars);
      if (threadIdx.x == 0) *p.done = 0ull;
    }
  }
}

template <int FCH, int NZ, int AT = 0>
__global__ void __launch_bounds__(256) heads_kernel(const HeadsArgs p) {
  heads_body<FCH, NZ, AT>(p, blockIdx.x, gridDim.x);
}

// ---------------------------------------------------------------------------------------
// Split-K weight-gradient reduction: out(m, n) = sum_z part[z][m][n] in a fixed order
// (z mod 4 lanes, then ((s0+s1)+s2)+s3), scattered into the flat gradient layout.
// ---------------------------------------------------------------------------------------
struct ReduceMap {
  int kind;          // 0 conv HWIO, 1 fc1 split, 2 heads
  int M, N;
  int cin, cinpad;   // conv: m = (kh*KW+kw)*cin + c  ->  ((kh*KW+kw)*cinpad + c)*N + n
  int per, wstride;  // fc1: split s = n / per
  int A;             // heads
  float* dst;        // conv/fc1: tensor base; heads: fc-pi/W
  float* dst_pib;
  float* dst_vW;
  float* dst_vb;
};

// a gradient element; COH: an agent-scope store (global_store sc1), for a consumer in the same
// launch on another XCD (reduce_clip_update: MI355X's L2s are not coherent)
template <bool COH = false>
__device__ __forceinline__ void grad_store(float* p, float v) {
  if constexpr (COH) st_agent_u32(reinterpret_cast<uint32_t*>(p), __float_as_uint(v));
  else *p = v;
}

template <bool COH = false>
__device__ __forceinline__ void reduce_store(const ReduceMap& mp, int m, int n, float v) {
  if (mp.kind == 0) {
    const int kk = m / mp.cin, c = m - kk * mp.cin;
    grad_store<COH>(mp.dst + ((size_t)kk * mp.cinpad + c) * mp.N + n, v);
  } else if (mp.kind == 1) {
    const int s = n / mp.per, fl = n - s * mp.per;
    grad_store<COH>(mp.dst + (size_t)s * mp.wstride + (size_t)m * mp.per + fl, v);  // m == 1600: legacy bias
  } else {
    const int F = mp.M - 1;
    if (m < F) {
      if (n < mp.A) grad_store<COH>(mp.dst + (size_t)m * mp.A + n, v);
      else if (n == mp.A) grad_store<COH>(mp.dst_vW + m, v);
    } else {
      if (n < mp.A) grad_store<COH>(mp.dst_pib + n, v);
      else if (n == mp.A) grad_store<COH>(mp.dst_vb, v);
    }
  }
}

// Slab groups of the weight-gradient reductions: RED_G groups of 64 lanes (64 RED_G threads per
// workgroup); group z sums slabs z, z + RED_G, ... in order, then the groups add in order
#ifndef BA3C_RED_GROUPS
#define BA3C_RED_GROUPS 4
#endif
constexpr int RED_G = BA3C_RED_GROUPS;
static_assert(RED_G >= 1 && RED_G <= 16, "reduction groups");

template <int NG>
__device__ __forceinline__ float red_sum(const float (*red)[64], int lane) {
  float v = red[0][lane];
#pragma unroll
  for (int z = 1; z < NG; ++z) v += red[z][lane];
  return v;
}

__global__ void __launch_bounds__(64 * RED_G) wgrad_reduce_kernel(const float* __restrict__ part, int S,
                                                                  const ReduceMap mp) {
  __shared__ float red[RED_G][64];
  const int lane = threadIdx.x & 63, zg = threadIdx.x >> 6;
  const int MN = mp.M * mp.N;
  const int o = blockIdx.x * 64 + lane;
  float s = 0.f;
  if (o < MN) {
    int z = zg;
    // 8 slab loads in flight per thread (the adds stay in slab order: deterministic)
    for (; z + 7 * RED_G < S; z += 8 * RED_G) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = part[(size_t)(z + RED_G * u) * MN + o];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += a[u];
    }
    for (; z < S; z += RED_G) s += part[(size_t)z * MN + o];
  }
  red[zg][lane] = s;
  __syncthreads();
  if (zg == 0 && o < MN) reduce_store(mp, o / mp.N, o % mp.N, red_sum<RED_G>(red, lane));
}

// All weight-gradient reductions of one backward pass in ONE launch (one job per layer, each
// with its own partial slabs).  Block b belongs to the job j with blk0[j] <= b < blk0[j+1];
// per output element the sum runs in the order of wgrad_reduce_kernel (bit-identical).  A
// conv job's output domain includes the zero-padded input channels (cin <= c < cinpad),
// written as 0, so with every job in the launch each gradient element is written exactly
// once and the flat gradient buffer needs no memset.
constexpr int MAX_RJOBS = 8;
struct ReduceJobs {
  int n;
  const float* part[MAX_RJOBS];
  int S[MAX_RJOBS];
  ReduceMap mp[MAX_RJOBS];
  int blk0[MAX_RJOBS + 1];
  int vec[MAX_RJOBS];   // 1: four consecutive outputs per lane (float4 slab loads / stores)
};

// a job can take float4 lanes when its output rows are whole float4s in the partial slabs
// and in the destination (conv HWIO / fc1 split layouts with N % 4 == 0)
__host__ __device__ inline bool reduce_vec_ok(const ReduceMap& mp) {
  return mp.kind != 2 && mp.N % 4 == 0 && (mp.kind == 0 || mp.per % 4 == 0);
}

__device__ __forceinline__ int reduce_out_size(const ReduceMap& mp) {
  return mp.kind == 0 ? (mp.M / mp.cin) * mp.cinpad * mp.N : mp.M * mp.N;
}

// workgroup b of the launch (64 NG threads); `lds`: NG x 64 float4 of scratch
template <bool COH, int NG>
__device__ __forceinline__ void wgrad_reduce_body(const ReduceJobs& jobs, int b, char* lds) {
  float4 (*red4)[64] = reinterpret_cast<float4 (*)[64]>(lds);
  float (*red)[64] = reinterpret_cast<float (*)[64]>(lds);
  int j = 0;
  while (j + 1 < jobs.n && jobs.blk0[j + 1] <= b) ++j;
  const ReduceMap& mp = jobs.mp[j];
  const float* __restrict__ part = jobs.part[j];
  const int S = jobs.S[j];
  const int lane = threadIdx.x & 63, zg = threadIdx.x >> 6;
  const int MN = mp.M * mp.N;
  if (jobs.vec[j]) {
    // 256 outputs per workgroup, 4 consecutive per lane: the per-output sums are the scalar
    // path's (z mod 4 lane groups in z order, then ((s0 + s1) + s2) + s3), bit for bit
    const int o = ((b - jobs.blk0[j]) * 64 + lane) * 4;
    const int NO = reduce_out_size(mp);
    int po = o;
    if (mp.kind == 0 && mp.cinpad != mp.cin && o < NO) {
      const int n = o % mp.N, r = o / mp.N, kk = r / mp.cinpad, c = r - kk * mp.cinpad;
      po = c < mp.cin ? (kk * mp.cin + c) * mp.N + n : -1;
    }
    float4 sv = make_float4(0.f, 0.f, 0.f, 0.f);
    if (o < NO && po >= 0) {
      const float4* __restrict__ p4 = reinterpret_cast<const float4*>(part);
      const int MN4 = MN / 4, q = po / 4;
      int z = zg;
      for (; z + 7 * NG < S; z += 8 * NG) {
        float4 a[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) a[u] = p4[(size_t)(z + NG * u) * MN4 + q];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          sv.x += a[u].x;
          sv.y += a[u].y;
          sv.z += a[u].z;
          sv.w += a[u].w;
        }
      }
      for (; z < S; z += NG) {
        const float4 a = p4[(size_t)z * MN4 + q];
        sv.x += a.x;
        sv.y += a.y;
        sv.z += a.z;
        sv.w += a.w;
      }
    }
    red4[zg][lane] = sv;
    __syncthreads();
    if (zg == 0 && o < NO) {
      float4 v = red4[0][lane];
#pragma unroll
      for (int z = 1; z < NG; ++z) {
        const float4 r = red4[z][lane];
        v.x += r.x;
        v.y += r.y;
        v.z += r.z;
        v.w += r.w;
      }
      if (po < 0) v = make_float4(0.f, 0.f, 0.f, 0.f);
      float* dst;
      if (mp.kind == 0) {
        dst = mp.dst + o;                                   // [(kk * cinpad + c) * N + n] == o
      } else {
        const int m = o / mp.N, n = o % mp.N, sidx = n / mp.per, fl = n - sidx * mp.per;
        dst = mp.dst + (size_t)sidx * mp.wstride + (size_t)m * mp.per + fl;
      }
      if constexpr (COH) {
        st_agent_u64(reinterpret_cast<unsigned long long*>(dst),
                     ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x));
        st_agent_u64(reinterpret_cast<unsigned long long*>(dst) + 1,
                     ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z));
      } else {
        *reinterpret_cast<float4*>(dst) = v;
      }
    }
    return;
  }
  const int o = (b - jobs.blk0[j]) * 64 + lane;            // output element of the job
  const int NO = reduce_out_size(mp);
  int po = o;                                               // its partial index, -1: padding
  if (mp.kind == 0 && mp.cinpad != mp.cin && o < NO) {
    const int n = o % mp.N, r = o / mp.N, kk = r / mp.cinpad, c = r - kk * mp.cinpad;
    po = c < mp.cin ? (kk * mp.cin + c) * mp.N + n : -1;
  }
  float s = 0.f;
  if (o < NO && po >= 0) {
    int z = zg;
    for (; z + 7 * NG < S; z += 8 * NG) {
      float a[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = part[(size_t)(z + NG * u) * MN + po];
#pragma unroll
      for (int u = 0; u < 8; ++u) s += a[u];
    }
    for (; z < S; z += NG) s += part[(size_t)z * MN + po];
  }
  red[zg][lane] = s;
  __syncthreads();
  if (zg == 0 && o < NO) {
    const float v = red_sum<NG>(red, lane);
    if (mp.kind == 0) grad_store<COH>(mp.dst + o, po >= 0 ? v : 0.f);   // [(kk * cinpad + c) * N + n] == o
    else reduce_store<COH>(mp, o / mp.N, o % mp.N, v);
  }
}

__global__ void __launch_bounds__(64 * RED_G) wgrad_reduce_all_kernel(const ReduceJobs jobs) {
  __shared__ float4 red4[RED_G][64];
  wgrad_reduce_body<false, RED_G>(jobs, blockIdx.x, reinterpret_cast<char*>(red4));
}

// ---------------------------------------------------------------------------------------
// Flat-buffer tensor table and the clip / optimizer kernels (one workgroup per chunk of
// UPD_CHUNK floats of one tensor).
// ---------------------------------------------------------------------------------------
struct TensorTable {
  int n;
  int nchunks;
  long long off[MAXT];
  int numel[MAXT];
  int chunk0[MAXT + 1];
};

// the tensor of chunk b: largest t with chunk0[t] <= b (binary search: ~6 dependent scalar
// loads of the kernel-argument table instead of up to n)
__device__ __forceinline__ int table_find(const TensorTable& tt, int b) {
  int lo = 0, hi = tt.n - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (tt.chunk0[mid] <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float block_sum_256(float v, float* red) {
  v = wave_sum_f(v);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) red[w] = v;
  __syncthreads();
  const float r = (red[0] + red[1]) + (red[2] + red[3]);
  __syncthreads();
  return r;
}

// cbase: first chunk of the launch (a tensor-aligned range of the table)
__global__ void __launch_bounds__(256) sumsq_kernel(const float* __restrict__ g, const TensorTable tt,
                                                    float* __restrict__ part, int cbase) {
  __shared__ float red[4];
  const int b = blockIdx.x + cbase;
  const int t = table_find(tt, b);
  const int c = b - tt.chunk0[t];
  const int beg = c * UPD_CHUNK;
  const int end = min(tt.numel[t], beg + UPD_CHUNK);
  const float* gt = g + tt.off[t];
  float s = 0.f;
  for (int i = beg + threadIdx.x; i < end; i += 256) s = fmaf(gt[i], gt[i], s);
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) part[b] = s;
}

// clip_by_average_norm multiplier of tensor t: min(rsqrt(sum g^2) * n, 1/0.1)
// Sum of the tensor's per-chunk partials: lane-strided, then a butterfly over the wave (every
// lane ends with the same, order-fixed value) — a serial loop over up to ~200 partials was a
// chain of dependent L2 round trips in every update workgroup.
__device__ __forceinline__ float clip_factor(const TensorTable& tt, int t, const float* part) {
  float ss = 0.f;
  for (int b = tt.chunk0[t] + (int)(threadIdx.x & 63); b < tt.chunk0[t + 1]; b += 64) ss += part[b];
  ss = wave_sum_f(ss);
  return fminf(rsqrtf(ss) * (float)tt.numel[t], 10.0f);
}

__global__ void __launch_bounds__(256) clip_kernel(float* __restrict__ g, const TensorTable tt,
                                                   const float* __restrict__ part, int cbase) {
  const int b = blockIdx.x + cbase;
  const int t = table_find(tt, b);
  const int c = b - tt.chunk0[t];
  const int beg = c * UPD_CHUNK;
  const int end = min(tt.numel[t], beg + UPD_CHUNK);
  const float f = clip_factor(tt, t, part);
  float* gt = g + tt.off[t];
  for (int i = beg + threadIdx.x; i < end; i += 256) gt[i] = (gt[i] * 0.1f) * f;
}

struct UpdateArgs {
  float* p;
  const float* g;
  float* s0;
  float* s1;
  const float* clip_part;   // non-null: fuse clip_by_average_norm
  float grad_scale;
  float lr, one_minus_b1, one_minus_b2, eps, alpha;   // adam
  float decay_c, momentum, rho, one_minus_rho;        // rms (decay_c = 1-decay), momentum, adadelta
  const float* dev_powers;  // non-null: Adam beta1^t, beta2^t read from the device (graph-safe)
  float beta1, beta2;       // clip_update_kernel: advances dev_powers after every block read them
};

// TF-1.2 float32 scalar arithmetic of ApplyAdam: alpha = lr*sqrt(1-b2^t)/(1-b1^t)
__host__ __device__ __forceinline__ float adam_alpha(float lr, float b1p, float b2p) {
  return (lr * sqrtf(1.0f - b2p)) / (1.0f - b1p);
}

// beta*_power.assign(beta*_power * beta*) after the apply (train.py:584 optimizer state)
__global__ void adam_powers_kernel(float* powers, float beta1, float beta2) {
  if (threadIdx.x == 0) {
    powers[0] = powers[0] * beta1;
    powers[1] = powers[1] * beta2;
  }
}

// One element of the TF-1.2 optimizer applies.  `g` (the clipped / scaled gradient) is made
// opaque first: otherwise the compiler may contract the clip product into the update's first
// subtraction in one kernel and not in another, and the launch paths would differ in the last
// bit (clip_kernel + update_kernel, update_kernel with the fused clip, clip_update_kernel).
template <int OPT>
__device__ __forceinline__ void opt_elem(float g, float& p, float& s0, float& s1, const UpdateArgs& a,
                                         float alpha) {
  asm volatile("" : "+v"(g));
  if constexpr (OPT == 0) {  // ApplyAdam
    s0 += (g - s0) * a.one_minus_b1;
    s1 += (g * g - s1) * a.one_minus_b2;
    p -= (s0 * alpha) / (sqrtf(s1) + a.eps);
  } else if constexpr (OPT == 1) {  // ApplyGradientDescent
    p -= g * a.lr;
  } else if constexpr (OPT == 2) {  // ApplyAdagrad
    s0 = s0 + g * g;
    p -= g * a.lr * rsqrtf(s0);
  } else if constexpr (OPT == 3) {  // ApplyAdadelta
    const float acc = s0 * a.rho + g * g * a.one_minus_rho;
    const float upd = sqrtf(s1 + a.eps) * rsqrtf(acc + a.eps) * g;
    p -= upd * a.lr;
    s0 = acc;
    s1 = s1 * a.rho + upd * upd * a.one_minus_rho;
  } else if constexpr (OPT == 4) {  // ApplyMomentum (use_nesterov=False)
    s0 = s0 * a.momentum + g;
    p -= s0 * a.lr;
  } else {  // ApplyRMSProp
    s0 += (g * g - s0) * a.decay_c;
    s1 = s1 * a.momentum + (g * a.lr) / sqrtf(s0 + a.eps);
    p -= s1;
  }
}

template <int OPT>
__global__ void __launch_bounds__(256) update_kernel(const UpdateArgs a, const TensorTable tt) {
  const int b = blockIdx.x;
  const int t = table_find(tt, b);
  const int c = b - tt.chunk0[t];
  const int beg = c * UPD_CHUNK;
  const int end = min(tt.numel[t], beg + UPD_CHUNK);
  const long long o = tt.off[t];
  // all loads of the thread's UPD_CHUNK / 256 elements are issued before any store: the
  // stores to p / s0 / s1 may alias later loads as far as the compiler knows, which would
  // otherwise serialise one HBM round trip per element.  Per-element arithmetic unchanged.
  constexpr int PER = UPD_CHUNK / 256;
  constexpr bool S0 = OPT != 1, S1 = OPT == 0 || OPT == 3 || OPT == 5;
  float gv[PER], pv[PER], s0v[PER], s1v[PER];
  // unconditional loads (past the chunk's end: its last element again, zeroed below): a load
  // in an `i < end` branch let only one element's loads be in flight at a time (r04 ISA)
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = beg + threadIdx.x + 256 * j;
    const long long k = o + min(i, end - 1);
    gv[j] = a.g[k];
    pv[j] = a.p[k];
    s0v[j] = S0 ? a.s0[k] : 0.f;
    s1v[j] = S1 ? a.s1[k] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (beg + (int)threadIdx.x + 256 * j >= end) gv[j] = pv[j] = s0v[j] = s1v[j] = 0.f;
  // the clip factor and Adam's powers after the element loads (their latency overlaps)
  const float f = a.clip_part ? clip_factor(tt, t, a.clip_part) : 0.f;
  const float alpha = (OPT == 0 && a.dev_powers) ? adam_alpha(a.lr, a.dev_powers[0], a.dev_powers[1])
                                                 : a.alpha;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = beg + threadIdx.x + 256 * j;
    if (i >= end) continue;
    const long long k = o + i;
    const float g = a.clip_part ? (gv[j] * 0.1f) * f : gv[j] * a.grad_scale;
    float p = pv[j], s0 = s0v[j], s1 = s1v[j];
    opt_elem<OPT>(g, p, s0, s1, a, alpha);
    if constexpr (S0) a.s0[k] = s0;
    if constexpr (S1) a.s1[k] = s1;
    a.p[k] = p;
  }
}

// ---------------------------------------------------------------------------------------
// Fused clip_by_average_norm + optimizer apply in ONE launch (one workgroup per chunk, every
// workgroup co-resident: gridDim.x = nchunks <= CUs).  Phase 1 loads the chunk's gradient,
// parameters and slots and publishes its sum of squares (sumsq_kernel's order: the same
// partials, bit for bit) as a TAGGED word {generation, Σg²}; phase 2 waits only for the
// partials of its own tensor (no grid-wide barrier, no atomics), forms the clip factor in
// clip_factor's order and applies update_kernel's arithmetic.  The generation of chunk b is
// the tag chunk b carried after the previous launch + 1: every launch runs every chunk, so
// all tags advance in lockstep from the zeros ba3c_create wrote (graph replays included).
// Cross-workgroup words go through agent-scope atomics (MI355X's 8 L2s are not coherent; a
// __threadfence per workgroup costs an L2 write-back).  With device-resident Adam powers,
// workgroup 0 advances them once every chunk has published (each reads them first).
// Waits are bounded: a broken residency assumption cannot hang the device (err flag).
// ---------------------------------------------------------------------------------------
struct UpdateSync {
  unsigned long long* tag;  // [nchunks] {generation << 32 | Σg² bits}
  unsigned int* err;        // set when a wait gave up
};

__device__ __forceinline__ unsigned long long ld_agent_u64(const unsigned long long* p) {
  return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// wave 0 of the workgroup: wait until chunks [c0, c1) carry generation `gen`; returns the sum
// of their partials in clip_factor's order (lane-strided, then the wave reduction)
__device__ __forceinline__ float wait_partials(const UpdateSync& us, int c0, int c1, unsigned gen, int lane) {
  float ss = 0.f;
  for (int j0 = c0; j0 < c1; j0 += 64) {
    const int j = j0 + lane;
    unsigned long long w = 0;
    unsigned spins = 0;
    while (true) {
      const bool ok = j >= c1 || (unsigned)((w = ld_agent_u64(us.tag + j)) >> 32) == gen;
      if (__all(ok)) break;
      __builtin_amdgcn_s_sleep(1);
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(us.err, 1u);
        break;
      }
    }
    if (j < c1) ss += __uint_as_float((unsigned)w);
  }
  return ss;
}

// Chunk b of nblk.  With `zsig` (reduce_clip_update: the gradient is being written by the
// signalling workgroups of the same launch) the chunk loads its parameters and slots, waits
// until the nctr spread counters at zsig sum to zneed, then reads its gradient with
// agent-scope loads.  `red`: 4 floats of LDS, `fsh`: 1.
template <int OPT>
__device__ __forceinline__ void clip_update_body(const UpdateArgs& a, const TensorTable& tt,
                                                 const UpdateSync& us, int b, int nblk,
                                                 const unsigned* zsig, int nctr, unsigned zneed,
                                                 unsigned* zerr, float* red, float* fsh_p) {
  float& fsh = *fsh_p;
  const int lane = threadIdx.x & 63;
  // this launch's generation (issued first: its latency hides behind the data loads)
  const unsigned gen = (unsigned)(ld_agent_u64(us.tag + b) >> 32) + 1u;
  const int t = table_find(tt, b);
  const int c = b - tt.chunk0[t];
  const int beg = c * UPD_CHUNK;
  const int end = min(tt.numel[t], beg + UPD_CHUNK);
  const long long o = tt.off[t];
  constexpr int PER = UPD_CHUNK / 256;
  constexpr bool S0 = OPT != 1, S1 = OPT == 0 || OPT == 3 || OPT == 5;
  float gv[PER], pv[PER], s0v[PER], s1v[PER];
  // unconditional loads (past the chunk's end: its last element again, zeroed below): a load
  // in an `i < end` branch let only one element's loads be in flight at a time (r04 ISA)
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = beg + threadIdx.x + 256 * j;
    const long long k = o + min(i, end - 1);
    if (!zsig) gv[j] = a.g[k];
    pv[j] = a.p[k];
    s0v[j] = S0 ? a.s0[k] : 0.f;
    s1v[j] = S1 ? a.s1[k] : 0.f;
  }
  if (zsig) {
    if (threadIdx.x < 64) chain_wait_spread(zsig, nctr, zneed, zerr);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const long long k = o + min(beg + (int)threadIdx.x + 256 * j, end - 1);
      gv[j] = __uint_as_float(__hip_atomic_load(reinterpret_cast<const unsigned*>(a.g) + k, __ATOMIC_RELAXED,
                                                __HIP_MEMORY_SCOPE_AGENT));
    }
  }
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (beg + (int)threadIdx.x + 256 * j >= end) gv[j] = pv[j] = s0v[j] = s1v[j] = 0.f;
  float alpha = (OPT == 0 && a.dev_powers) ? adam_alpha(a.lr, a.dev_powers[0], a.dev_powers[1]) : a.alpha;
  asm volatile("" : "+v"(alpha) : : "memory");   // the powers are read before this chunk publishes
  // phase 1: the chunk's sum of squares, in sumsq_kernel's order (i = beg + tid + 256 j)
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (beg + (int)threadIdx.x + 256 * j < end) ss = fmaf(gv[j], gv[j], ss);
  ss = block_sum_256(ss, red);
  if (threadIdx.x == 0)
    __hip_atomic_store(us.tag + b, ((unsigned long long)gen << 32) | __float_as_uint(ss), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // phase 2: the tensor's clip factor (clip_factor's arithmetic) once its chunks published
  if (threadIdx.x < 64) {
    const float sum = wave_sum_f(wait_partials(us, tt.chunk0[t], tt.chunk0[t + 1], gen, lane));
    if (lane == 0) fsh = fminf(rsqrtf(sum) * (float)tt.numel[t], 10.0f);
    if (OPT == 0 && a.dev_powers && b == 0) {
      (void)wait_partials(us, 0, nblk, gen, lane);   // every chunk has read the powers
      if (lane == 0) {
        float* pw = const_cast<float*>(a.dev_powers);
        pw[0] = pw[0] * a.beta1;
        pw[1] = pw[1] * a.beta2;
      }
    }
  }
  __syncthreads();
  const float f = fsh;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = beg + threadIdx.x + 256 * j;
    if (i >= end) continue;
    const long long k = o + i;
    float p = pv[j], s0 = s0v[j], s1 = s1v[j];
    opt_elem<OPT>((gv[j] * 0.1f) * f, p, s0, s1, a, alpha);
    if constexpr (S0) a.s0[k] = s0;
    if constexpr (S1) a.s1[k] = s1;
    a.p[k] = p;
  }
}

template <int OPT>
__global__ void __launch_bounds__(256) clip_update_kernel(const UpdateArgs a, const TensorTable tt,
                                                          const UpdateSync us) {
  __shared__ float red[4];
  __shared__ float fsh;
  clip_update_body<OPT>(a, tt, us, blockIdx.x, gridDim.x, nullptr, 0, 0u, nullptr, red, &fsh);
}

// ---------------------------------------------------------------------------------------
// clip_by_average_norm over a tensor-aligned chunk range [cbase, cbase + gridDim.x) in ONE
// launch (the data-parallel step clips each gradient bucket before its all-reduce): the
// sumsq_kernel + clip_kernel pair with clip_update_kernel's tagged-partials hand-off — phase 1
// publishes the chunk's sum of squares in sumsq_kernel's order, phase 2 waits for its tensor's
// chunks and scales in clip_kernel's arithmetic, bit for bit.  Its tags are a generation space
// of their own (a range launch advances only its chunks).  All chunks of the range co-resident.
// ---------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) clip_range_kernel(float* __restrict__ g, const TensorTable tt, int cbase,
                                                         const UpdateSync us) {
  __shared__ float red[4];
  __shared__ float fsh;
  const int b = blockIdx.x + cbase;
  const int lane = threadIdx.x & 63;
  const unsigned gen = (unsigned)(ld_agent_u64(us.tag + b) >> 32) + 1u;
  const int t = table_find(tt, b);
  const int c = b - tt.chunk0[t];
  const int beg = c * UPD_CHUNK;
  const int end = min(tt.numel[t], beg + UPD_CHUNK);
  float* gt = g + tt.off[t];
  constexpr int PER = UPD_CHUNK / 256;
  float gv[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = beg + threadIdx.x + 256 * j;
    const float v = gt[min(i, end - 1)];        // unconditional: every load in flight at once
    gv[j] = i < end ? v : 0.f;
  }
  float ss = 0.f;
#pragma unroll
  for (int j = 0; j < PER; ++j)
    if (beg + (int)threadIdx.x + 256 * j < end) ss = fmaf(gv[j], gv[j], ss);
  ss = block_sum_256(ss, red);
  if (threadIdx.x == 0)
    __hip_atomic_store(us.tag + b, ((unsigned long long)gen << 32) | __float_as_uint(ss), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < 64) {
    const float sum = wave_sum_f(wait_partials(us, tt.chunk0[t], tt.chunk0[t + 1], gen, lane));
    if (lane == 0) fsh = fminf(rsqrtf(sum) * (float)tt.numel[t], 10.0f);
  }
  __syncthreads();
  const float f = fsh;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int i = beg + threadIdx.x + 256 * j;
    if (i < end) gt[i] = (gv[j] * 0.1f) * f;
  }
}

// ---------------------------------------------------------------------------------------
// numpy RandomState.choice(A, p=p) given its draw u:  cdf = cumsum(double(p)); cdf /= cdf[-1];
// a = searchsorted(cdf, u, 'right').  flag bits: 1 non-finite p (train.py:381), 2 |sum-1| >
// sqrt(eps_f32) ("probabilities do not sum to 1"), 4 negative p.
// ---------------------------------------------------------------------------------------
// ba3c_allreduce_mean: the summed gradients times 1/N (grid-stride, float4 where aligned)
__global__ void __launch_bounds__(256) scale_kernel(float* __restrict__ g, int64_t n, float s) {
  const int64_t n4 = n / 4;
  float4* g4 = reinterpret_cast<float4*>(g);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 v = g4[i];
    v.x *= s; v.y *= s; v.z *= s; v.w *= s;
    g4[i] = v;
  }
  for (int64_t i = 4 * n4 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) g[i] *= s;
}

// Diagnostic (ba3c_occupy_cus): each workgroup declares the whole 160 KiB of a CU's LDS, so
// `n` workgroups hold `n` distinct CUs against every kernel that uses LDS (all the conv
// kernels) for `ticks` of the 100 MHz realtime clock — a stand-in for RCCL's channel
// workgroups sharing the chip with the persistent conv kernels during a bucket's all-reduce
// (bench.py --occupy).  No memory traffic; the spin sleeps between clock reads.
__global__ void __launch_bounds__(64) occupy_kernel(unsigned long long ticks) {
  __shared__ uint4 hold[163840 / 16];
  hold[threadIdx.x] = make_uint4(threadIdx.x, 0u, 0u, 0u);
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(32);
  __syncthreads();
  const unsigned v = hold[(threadIdx.x + 1) & 63].x;
  asm volatile("" ::"v"(v));   // keeps the LDS declaration (and so the CU) allocated
}

__global__ void __launch_bounds__(256) sample_kernel(const float* __restrict__ probs,
                                                     const double* __restrict__ u, int B, int A,
                                                     int64_t* __restrict__ actions, int* flag) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= B) return;
  const float* pn = probs + (size_t)n * A;
  double cum = 0.0;
  int bad = 0;
  for (int k = 0; k < A; ++k) {
    const float pk = pn[k];
    if (!isfinite(pk)) bad |= 1;
    if (pk < 0.f) bad |= 4;
    cum += (double)pk;
  }
  if (fabs(cum - 1.0) > 3.4526698300124393e-04) bad |= 2;
  const double tot = cum;
  const double un = u[n];
  // the cumulative sums again, in the same order (the same doubles as a stored cdf array,
  // which a runtime A put in scratch memory)
  int64_t a = 0;
  double c = 0.0;
  for (int k = 0; k < A; ++k) {
    c += (double)pn[k];
    a += (c / tot <= un) ? 1 : 0;
  }
  actions[n] = a;
  if (bad && flag) atomicOr(flag, bad);
}

// Evaluation players' action (OpenAIGym/common.py:24-33): numpy argmax of the policy (first
// maximum; a NaN counts as the maximum, first NaN wins, as np.argmax), replaced by the action
// space's random sample where the player's uniform draw is below eps.
__global__ void __launch_bounds__(256) greedy_kernel(const float* __restrict__ probs,
                                                     const double* __restrict__ u,
                                                     const int64_t* __restrict__ rand_act, int B,
                                                     int A, double eps, int64_t* __restrict__ actions) {
  const int n = blockIdx.x * 256 + threadIdx.x;
  if (n >= B) return;
  const float* pn = probs + (size_t)n * A;
  float best = pn[0];
  int arg = 0;
  for (int k = 1; k < A && !isnan(best); ++k) {
    const float v = pn[k];
    if (isnan(v) || v > best) {
      best = v;
      arg = k;
    }
  }
  actions[n] = u[n] < eps ? rand_act[n] : (int64_t)arg;
}

}  // namespace ba3c
