// ba3c_multi.h — several independent kernels in ONE launch (horizontal fusion).
//
// At small batches (configs[1]: B=32) every backward kernel is a few latency-bound
// workgroups.  The input gradient of a layer and its weight gradient read the same output
// gradient and write disjoint buffers, so they can run side by side.  A second HIP stream
// does that too, but each fork / join is an event (a barrier packet) that r02 traces show as
// 6-11 us of idle queue per layer.  A multi-job launch puts the jobs' workgroups in one grid
// instead: block b < end[0] runs job 0 with its own (x, y, z) decomposition, then job 1, then
// job 2.  No event, no second queue.  Each job's body (band6_body, wgrad6_body, gemm6_body)
// is the one its plain kernel runs, on the same inputs and with the same per-workgroup
// indices, so every output is bit-identical to the separate launches.
#pragma once
#include "ba3c_band6.h"
#include "ba3c_gemm6.h"
#include "ba3c_small.h"
#include "ba3c_wgrad6.h"

namespace ba3c {

// A job: its argument struct, its LDS bytes, and run(args, x, y, z, gx, lds, red4).
struct NoJob {
  using Args = int;
  static constexpr int LDS = 0;
  __device__ static void run(const Args&, int, int, int, int, char*, uint32_t*) {}
};

template <class L>
struct Band6Job {
  using Args = Band6Args;
  static constexpr int LDS = L::LDS_BYTES;
  __device__ static void run(const Args& a, int x, int, int, int, char* lds, uint32_t*) {
    band6_body<L>(a, x, lds);
  }
};

// ring-walk band kernel as a job: x = first image group, gx = the job's own grid size
template <class L>
struct Band6RJob {
  using Args = Band6Args;
  static constexpr int LDS = L::LDS_BYTES;
  __device__ static void run(const Args& a, int x, int, int, int gx, char* lds, uint32_t* red4) {
    int* tslot = reinterpret_cast<int*>(red4);   // the ticket slot (dynamic queue only)
    if constexpr (L::G::SRC == 1 && L::NS == 2) band6r_up_body<L>(a, x, gx, lds, tslot);
    else band6r_body<L>(a, x, gx, lds, tslot);
  }
};

// whole-channel weight gradient as a job
template <class G>
struct Wg6WJob {
  using Args = Wg6Args;
  static constexpr int LDS = wgrad6w_lds_bytes<G>();
  __device__ static void run(const Args& a, int x, int, int, int gx, char* lds, uint32_t* red4) {
    wgrad6w_body<G>(a, x, gx, lds, red4);
  }
};

template <class G>
struct Wg6Job {
  using Args = Wg6Args;
  static constexpr int LDS = G::X_BYTES + G::Y_BYTES;
  __device__ static void run(const Args& a, int x, int y, int, int gx, char* lds, uint32_t* red4) {
    wgrad6_body<G>(a, x, y, gx, lds, red4);
  }
};

template <int BM, int BN, int WGM, int WGN, class P, int D, int KS = 1>
struct Gemm6Job {
  using Args = P;
  static constexpr int LDS = KS * Gemm6Lds<BM, BN, P>::BYTES;
  __device__ static void run(const Args& p, int x, int y, int z, int, char* lds, uint32_t*) {
    gemm6_body<BM, BN, WGM, WGN, P, D, KS>(p, x, y, z, lds);
  }
};

struct Conv0SJob {
  using Args = Conv0SArgs;
  static constexpr int LDS = conv0s_fwd_lds_bytes();
  __device__ static void run(const Args& a, int x, int, int, int gx, char* lds, uint32_t*) {
    conv0s_fwd_body(a, x, gx, lds);
  }
};

struct WPrep6Job {
  using Args = WPrep6Args;
  static constexpr int LDS = 0;
  __device__ static void run(const Args& a, int x, int y, int, int gx, char*, uint32_t* red4) {
    wprep6_body(a, x, y, gx, reinterpret_cast<float*>(red4));
  }
};

// the pass's weight-gradient reductions, stored for a consumer in the same launch (a chained
// reduce_clip_update's signalling job; 256 threads: the host chains it only when RED_G == 4, so
// its sums are the plain launch's)
struct ReduceJob {
  using Args = ReduceJobs;
  static constexpr int LDS = 4 * 64 * 16;
  __device__ static void run(const Args& a, int x, int, int, int, char* lds, uint32_t*) {
    wgrad_reduce_body<true, 4>(a, x, lds);
  }
};

// the fused clip + optimizer apply as a waiting job: each chunk loads its parameters and
// slots, then waits for the reduction (zsig: the chain's signal count) before its gradient
struct ClipUpdArgs {
  UpdateArgs a;
  TensorTable tt;
  UpdateSync us;
  const unsigned* zsig;   // the chain's spread counters
  int nctr;
  unsigned zneed;
  unsigned* zerr;
};

template <int OPT>
struct ClipUpdJob {
  using Args = ClipUpdArgs;
  static constexpr int LDS = 32;
  __device__ static void run(const Args& a, int x, int, int, int gx, char* lds, uint32_t*) {
    float* f = reinterpret_cast<float*>(lds);
    clip_update_body<OPT>(a.a, a.tt, a.us, x, gx, a.zsig, a.nctr, a.zneed, a.zerr, f, f + 4);
  }
};

// Per job: grid (gx, gy, gz) and the exclusive end of its block range in the launch.
struct MultiGrid {
  int gx[3], gy[3], end[3];
};

constexpr int cmax(int a, int b) { return a > b ? a : b; }

template <class J0, class J1, class J2>
__device__ __forceinline__ void multi_body(const typename J0::Args& a0, const typename J1::Args& a1,
                                           const typename J2::Args& a2, const MultiGrid& g, char* lds,
                                           uint32_t* red4) {
  // the job index is uniform per workgroup, so every barrier inside a body is reached by all
  // of its waves
  const int b = blockIdx.x;
  if (b < g.end[0]) {
    const int r = b, xy = g.gx[0] * g.gy[0];
    J0::run(a0, r % g.gx[0], (r % xy) / g.gx[0], r / xy, g.gx[0], lds, red4);
  } else if (b < g.end[1]) {
    const int r = b - g.end[0], xy = g.gx[1] * g.gy[1];
    J1::run(a1, r % g.gx[1], (r % xy) / g.gx[1], r / xy, g.gx[1], lds, red4);
  } else if (b < g.end[2]) {
    const int r = b - g.end[1], xy = g.gx[2] * g.gy[2];
    J2::run(a2, r % g.gx[2], (r % xy) / g.gx[2], r / xy, g.gx[2], lds, red4);
  }
}

// ---------------------------------------------------------------------------------------
// Chained multi-job launch: an in-launch dependency instead of a kernel boundary (configs[1],
// B=32: the zeroing of the step's ReLU counters / max slots -> conv0's forward, which splits
// its own weight fragments and waits only before its first publication into those words).
// Jobs [0, nsig) signal when a workgroup is done; the jobs in `wmask` wait until every
// signalling workgroup has — before their body, or inside it (`late`: the body polls the
// count itself).  Nothing assumes a dispatch order: signalling workgroups never wait, and the
// host chains a launch only when its waiting workgroups fit one per CU, so they cannot keep a
// signalling workgroup from being scheduled.  Hand-off without fences (MI355X_MICROARCH.md
// §Correctness boundaries, the sc1 form): every handed-off word is stored with an agent-scope
// store (global_store sc1: it leaves the XCD's non-coherent L2) and used only by device-scope
// atomics or agent-scope loads; each storing wave drains (s_waitcnt 0), the workgroup
// barriers, then thread 0 bumps the signal count.  Measured and not kept (r05k-n): a
// per-workgroup release / acquire (an L2 write-back each: +18 us per B=32 step), a ticket
// counter drawn by every workgroup (+40 us: same-address returning atomics serialise), fc1's
// split-K forward chained with the heads over sc1 partials (14.3 -> 16.9 us), conv0 reading
// the prep's fragments with sc1 loads (21.2 -> 26.4 us).  The last waiting workgroup resets
// the words (every signal was counted before any waiter passed), so each launch starts from
// zeros (ba3c_create zeroes them; graph replays included).  Waits are bounded: a broken
// assumption sets the error word instead of hanging the device.
struct ChainArgs {
  unsigned* w;      // [4]: ticket, signals, finished
  unsigned* err;    // bit 0: a wait gave up (ba3c_device_errors bit 2)
  int nsig, wmask, nwait;   // nwait: workgroups of the waiting jobs
  int late;                 // waiting jobs that wait inside their body (not before it)
  // > 0: signalling workgroup b counts into spread counter b % spread (ctr + CHAIN_STRIDE *
  // that: one 64-byte line each) instead of w[1], so over a thousand signals do not queue on
  // one address (r05aa: reduce -> clip + update with one counter, +25 us at B=32)
  unsigned* ctr;
  int spread;
};

__device__ __forceinline__ unsigned chain_ld(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <class J0, class J1, class J2>
__device__ __forceinline__ void multi_chain_body(const typename J0::Args& a0, const typename J1::Args& a1,
                                                 const typename J2::Args& a2, const MultiGrid& g,
                                                 const ChainArgs& c, char* lds, uint32_t* red4) {
  const int b = blockIdx.x;
  const int job = b < g.end[0] ? 0 : (b < g.end[1] ? 1 : 2);
  const bool waits = (c.wmask >> job) & 1;
  if (waits && !((c.late >> job) & 1)) {
    if (c.spread) {
      if (threadIdx.x < 64) chain_wait_spread(c.ctr, c.spread, (unsigned)g.end[c.nsig - 1], c.err);
    } else if (threadIdx.x == 0) {
      const unsigned need = (unsigned)g.end[c.nsig - 1];
      unsigned spins = 0;
      while (chain_ld(c.w + 1) < need) {
        __builtin_amdgcn_s_sleep(2);
        if (++spins > (1u << 22)) {
          atomicOr(c.err, 1u);
          break;
        }
      }
    }
    __syncthreads();
  }
  if (job == 0) {
    const int r = b, xy = g.gx[0] * g.gy[0];
    J0::run(a0, r % g.gx[0], (r % xy) / g.gx[0], r / xy, g.gx[0], lds, red4);
  } else if (job == 1) {
    const int r = b - g.end[0], xy = g.gx[1] * g.gy[1];
    J1::run(a1, r % g.gx[1], (r % xy) / g.gx[1], r / xy, g.gx[1], lds, red4);
  } else if (b < g.end[2]) {
    const int r = b - g.end[1], xy = g.gx[2] * g.gy[2];
    J2::run(a2, r % g.gx[2], (r % xy) / g.gx[2], r / xy, g.gx[2], lds, red4);
  }
  if (job < c.nsig) {
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_fetch_add(c.spread ? c.ctr + CHAIN_STRIDE * (b % c.spread) : c.w + 1, 1u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  } else if (waits && threadIdx.x == 0) {
    // the last waiter resets the words (every signal was counted before any waiter passed)
    if (__hip_atomic_fetch_add(c.w + 2, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(c.nwait - 1)) {
      __hip_atomic_store(c.w + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(c.w + 2, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      for (int k = 0; k < c.spread; ++k)
        __hip_atomic_store(c.ctr + CHAIN_STRIDE * k, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <class J0, class J1, class J2>
struct MultiLds {
  static constexpr int BYTES = cmax(cmax(J0::LDS, J1::LDS), cmax(J2::LDS, 16));
};

template <class J0, class J1, class J2>
__global__ void __launch_bounds__(256) multi_kernel(const typename J0::Args a0, const typename J1::Args a1,
                                                    const typename J2::Args a2, const MultiGrid g) {
  __shared__ uint4 lds4[MultiLds<J0, J1, J2>::BYTES / 16];
  __shared__ uint32_t red4[4];
  multi_body<J0, J1, J2>(a0, a1, a2, g, reinterpret_cast<char*>(lds4), red4);
}

// 512-thread jobs (gemm6 bodies with KS = 2)
template <class J0, class J1, class J2>
__global__ void __launch_bounds__(512) multi_kernel512(const typename J0::Args a0, const typename J1::Args a1,
                                                       const typename J2::Args a2, const MultiGrid g) {
  __shared__ uint4 lds4[MultiLds<J0, J1, J2>::BYTES / 16];
  __shared__ uint32_t red4[4];
  multi_body<J0, J1, J2>(a0, a1, a2, g, reinterpret_cast<char*>(lds4), red4);
}

// the band / weight-gradient bodies are tuned for two workgroups per CU (their plain kernels
// carry the same attribute)
template <class J0, class J1, class J2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
multi_kernel_w2(const typename J0::Args a0, const typename J1::Args a1, const typename J2::Args a2,
                const MultiGrid g) {
  __shared__ uint4 lds4[MultiLds<J0, J1, J2>::BYTES / 16];
  __shared__ uint32_t red4[4];
  multi_body<J0, J1, J2>(a0, a1, a2, g, reinterpret_cast<char*>(lds4), red4);
}

template <class J0, class J1, class J2>
__global__ void __launch_bounds__(256) multi_chain_kernel(const typename J0::Args a0, const typename J1::Args a1,
                                                          const typename J2::Args a2, const MultiGrid g,
                                                          const ChainArgs c) {
  __shared__ uint4 lds4[MultiLds<J0, J1, J2>::BYTES / 16];
  __shared__ uint32_t red4[4];
  multi_chain_body<J0, J1, J2>(a0, a1, a2, g, c, reinterpret_cast<char*>(lds4), red4);
}

template <class J0, class J1, class J2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2)))
multi_chain_kernel_w2(const typename J0::Args a0, const typename J1::Args a1, const typename J2::Args a2,
                      const MultiGrid g, const ChainArgs c) {
  __shared__ uint4 lds4[MultiLds<J0, J1, J2>::BYTES / 16];
  __shared__ uint32_t red4[4];
  multi_chain_body<J0, J1, J2>(a0, a1, a2, g, c, reinterpret_cast<char*>(lds4), red4);
}

}  // namespace ba3c
