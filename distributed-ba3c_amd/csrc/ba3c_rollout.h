// ba3c_rollout.h — the data formats on either side of the learner/predictor path, on the GPU
// (SURVEY.md §8f ranks 1 and 3):
//
//  * n-step returns + batch assembly: MySimulatorMaster._on_datapoint / _on_episode_over /
//    _parse_memory (OpenAIGym/train.py:394-437) for every simulator at once, and the
//    BatchData / EnqueueThread hand-off (dataflow/common.py:64-99, train/trainer.py:116-155)
//    as a gather of the datapoints' states and actions into the learner's batch tensors;
//  * frame history: HistoryFramePlayer (RL/history.py:12-55) — the stacked state is itself
//    the history: push = drop the oldest frame's channels, append the new frame's; an
//    episode start clears it to zeros + the new frame (history.clear(); append(s)).
//
// All three are latency / HBM-bound byte work: coalesced 16-byte accesses, no MFMA.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace ba3c {

// ---------------------------------------------------------------------------------------
// n-step discounted returns.  Env e keeps its memory in a ring of T slots (slot of the i-th
// transition = (start[e] + i) % T); length[e] transitions are in it, the reward of each
// known.  Like _parse_memory:
//   not over:  the last transition only bootstraps, R = value of it, and stays in memory;
//   over:      R = 0 and every transition is emitted.
//   for the emitted transitions in REVERSE time order: R = clip(r, -1, 1) + gamma * R
// in float64 (Python float / np.float64 arithmetic), emitted as float32 (the TF feed cast of
// the float64 batch, dataflow/common.py:86-92).  Datapoints are written env by env in the
// order _parse_memory puts them on its queue; src[i] = e * T + slot locates the state /
// action of datapoint i.  One workgroup of 1024 threads: a block scan assigns offsets.
// ---------------------------------------------------------------------------------------
struct ReturnsArgs {
  const double* reward;     // [E][T] ring slots
  const float* value;       // [E][T] predictor value of each transition ('pred_value')
  const int32_t* start;     // [E] ring slot of the oldest transition
  const int32_t* length;    // [E] transitions in memory (0..T)
  const uint8_t* is_over;   // [E] 1: the episode ended with the last transition
  int E, T;
  double gamma;
  float* R;                 // [E*T] futurereward per datapoint
  int32_t* src;             // [E*T] e*T + ring slot of the datapoint's transition
  float* init_R;            // [E*T] the segment's bootstrap value (0 when over)
  uint8_t* over;            // [E*T] the segment's isOver
  int32_t* count;           // [1] datapoints written
};

__global__ void __launch_bounds__(1024) nstep_returns_kernel(const ReturnsArgs a) {
  __shared__ int32_t scan[1024];
  const int tid = threadIdx.x;
  int carry = 0;
  for (int base = 0; base < a.E; base += 1024) {
    const int e = base + tid;
    int len = 0, n = 0;
    bool over = false;
    if (e < a.E) {
      len = a.length[e];
      over = a.is_over[e] != 0;
      n = over ? len : (len > 0 ? len - 1 : 0);
    }
    // inclusive Hillis-Steele scan of n over the block
    scan[tid] = n;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
      const int v = tid >= d ? scan[tid - d] : 0;
      __syncthreads();
      scan[tid] += v;
      __syncthreads();
    }
    const int off = carry + scan[tid] - n;
    const int total = scan[1023];
    __syncthreads();
    if (n > 0) {
      const int s0 = a.start[e];
      const size_t row = (size_t)e * a.T;
      const float boot = over ? 0.f : a.value[row + (s0 + len - 1) % a.T];
      double R = (double)boot;
      for (int k = 0; k < n; ++k) {            // k-th emitted = transition n-1-k
        const int slot = (s0 + n - 1 - k) % a.T;
        const double r = a.reward[row + slot];
        R = fmin(fmax(r, -1.0), 1.0) + a.gamma * R;
        a.R[off + k] = (float)R;
        a.src[off + k] = (int32_t)(row + slot);
        a.init_R[off + k] = boot;
        a.over[off + k] = over ? 1 : 0;
      }
    }
    carry += total;
  }
  if (tid == 0) *a.count = carry;
}

// dst[i] = src[idx[i]] for rows of `row_words` 16-byte words (states: 84*84*C bytes).
__global__ void __launch_bounds__(256) gather_rows16_kernel(const uint4* __restrict__ src,
                                                            const int32_t* __restrict__ idx,
                                                            int n, int row_words,
                                                            uint4* __restrict__ dst) {
  const int i = blockIdx.y;
  if (i >= n) return;
  const uint4* s = src + (size_t)idx[i] * row_words;
  uint4* d = dst + (size_t)i * row_words;
  for (int w = blockIdx.x * 256 + threadIdx.x; w < row_words; w += gridDim.x * 256) d[w] = s[w];
}

// dst[i] = src[idx[i]] for 8-byte elements (actions)
__global__ void __launch_bounds__(256) gather_i64_kernel(const int64_t* __restrict__ src,
                                                         const int32_t* __restrict__ idx, int n,
                                                         int64_t* __restrict__ dst) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) dst[i] = src[idx[i]];
}

// ---------------------------------------------------------------------------------------
// Frame history (HistoryFramePlayer, hist_len H): state[e] is [84*84][H*c] bytes, channel
// block h = the h-th oldest frame.  push: state = concat(state[..., c:], frame); on an
// episode start (is_over[e], the frame is the new episode's first): zeros + frame.
// One thread per 4 pixels (16 bytes of state when H*c == 4).
// ---------------------------------------------------------------------------------------
struct HistoryArgs {
  const uint8_t* frame;     // [E][P][c] newest frame per env (P = 84*84 pixels)
  uint8_t* state;           // [E][P][H*c] stacked history, updated in place
  const uint8_t* is_over;   // [E] (may be null)
  int E, P, H, c;
};

__global__ void __launch_bounds__(256) history_push_kernel(const HistoryArgs a) {
  const int e = blockIdx.y;
  const int q = blockIdx.x * 256 + threadIdx.x;     // 4-pixel group
  if (q * 4 >= a.P) return;
  const bool reset = a.is_over && a.is_over[e];
  const int S = a.H * a.c;
  if (S == 4 && a.c == 1 && a.P % 4 == 0) {
    // fast path (84x84x4 grayscale): one dword per pixel, little-endian channel order
    uint4* st = reinterpret_cast<uint4*>(a.state + (size_t)e * a.P * 4) + q;
    const uint32_t f4 = *reinterpret_cast<const uint32_t*>(a.frame + (size_t)e * a.P + 4 * q);
    uint4 v = reset ? make_uint4(0, 0, 0, 0) : *st;
    v.x = (v.x >> 8) | ((f4 & 0xFFu) << 24);
    v.y = (v.y >> 8) | (((f4 >> 8) & 0xFFu) << 24);
    v.z = (v.z >> 8) | (((f4 >> 16) & 0xFFu) << 24);
    v.w = (v.w >> 8) | ((f4 >> 24) << 24);
    *st = v;
    return;
  }
  for (int p = 4 * q; p < 4 * q + 4 && p < a.P; ++p) {
    uint8_t* st = a.state + ((size_t)e * a.P + p) * S;
    const uint8_t* fr = a.frame + ((size_t)e * a.P + p) * a.c;
    for (int k = 0; k < S - a.c; ++k) st[k] = reset ? 0 : st[k + a.c];
    for (int k = 0; k < a.c; ++k) st[S - a.c + k] = fr[k];
  }
}

}  // namespace ba3c
