// Probe of gfx950's v_smfmac_f32_32x32x32_f16 (2:4 structured-sparse A, 32 x 32 logical K, B
// 32 x 32): which lane layouts reproduce a host reference, and its issue rate against
// v_smfmac_f32_16x16x64_f16 (the same bytes of operands per lane, twice the products).  Test
// infrastructure for the sparse conv1 weight gradient (not linked into libba3c).
// Build: hipcc --offload-arch=gfx950 -O3 smfmac32_probe.hip -o smfmac32_probe
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void one(const f16x8* a, const f16x16* b, const int* idx, f32x16* c) {
  const int l = threadIdx.x;
  f32x16 acc = {};
  acc = __builtin_amdgcn_smfmac_f32_32x32x32_f16(a[l], b[l], acc, idx[l], 0, 0);
  c[l] = acc;
}

template <bool BIG>
__global__ void rate(const f16x8* a, const f16x16* b, const int* idx, float* c, int iters) {
  const int l = threadIdx.x & 63;
  f16x8 av = a[l];
  f16x16 bv = b[l];
  const int ix = idx[l];
  float s = 0.f;
  if constexpr (BIG) {
    f32x16 acc[4] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_smfmac_f32_32x32x32_f16(av, bv, acc[j], ix, 0, 0);
    }
    for (int j = 0; j < 4; ++j)
      for (int i = 0; i < 16; ++i) s += acc[j][i];
  } else {
    f32x4 acc[8] = {};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, acc[j], ix, 0, 0);
    }
    for (int j = 0; j < 8; ++j)
      for (int i = 0; i < 4; ++i) s += acc[j][i];
  }
  c[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// logical K of lane l's logical element e (0..15): hyp 0 contiguous halves, hyp 1 interleaved
static int kK(int hyp, int l, int e) {
  const int g = l >> 5;
  return hyp == 0 ? 16 * g + e : (e < 8 ? 8 * g + e : 16 + 8 * g + (e - 8));
}
// C element i of lane l: hyp 0 = the dense 32x32 layout (column l & 31, row 8 (i / 4) + 4 (l / 32)
// + i % 4)
static void cRC(int l, int i, int& r, int& n) {
  n = l & 31;
  r = 8 * (i >> 2) + 4 * (l >> 5) + (i & 3);
}

int main() {
  srand(11);
  float A[32][32], B[32][32], C[32][32];
  for (int r = 0; r < 32; ++r)
    for (int q = 0; q < 8; ++q) {
      int i0 = rand() % 4, i1 = rand() % 4;
      while (i1 == i0) i1 = rand() % 4;
      for (int j = 0; j < 4; ++j) A[r][4 * q + j] = 0.f;
      A[r][4 * q + i0] = (float)(rand() % 9 - 4);
      A[r][4 * q + i1] = (float)(rand() % 9 - 4);
    }
  for (int k = 0; k < 32; ++k)
    for (int n = 0; n < 32; ++n) B[k][n] = (float)(rand() % 7 - 3);
  for (int r = 0; r < 32; ++r)
    for (int n = 0; n < 32; ++n) {
      float s = 0;
      for (int k = 0; k < 32; ++k) s += A[r][k] * B[k][n];
      C[r][n] = s;
    }
  f16x8* da; f16x16* db; int* di; f32x16* dc; float* dr;
  (void)hipMalloc(&da, 64 * sizeof(f16x8));
  (void)hipMalloc(&db, 64 * sizeof(f16x16));
  (void)hipMalloc(&di, 64 * 4);
  (void)hipMalloc(&dc, 64 * sizeof(f32x16));
  (void)hipMalloc(&dr, sizeof(float) * 2048 * 256);
  for (int ha = 0; ha < 2; ++ha)
    for (int hb = 0; hb < 2; ++hb)
      for (int hi = 0; hi < 2; ++hi) {
        std::vector<f16x8> a(64);
        std::vector<f16x16> b(64);
        std::vector<int> ix(64, 0);
        for (int l = 0; l < 64; ++l) {
          const int r = l & 31;
          int bits = 0;
          for (int q = 0; q < 4; ++q) {
            const int k0 = kK(ha, l, 4 * q);
            int pos[2], np = 0;
            for (int j = 0; j < 4 && np < 2; ++j)
              if (A[r][k0 + j] != 0.f) pos[np++] = j;
            a[l][2 * q] = (_Float16)A[r][k0 + pos[0]];
            a[l][2 * q + 1] = (_Float16)A[r][k0 + pos[1]];
            const int nib = hi == 0 ? (pos[0] | (pos[1] << 2)) : (pos[1] | (pos[0] << 2));
            bits |= nib << (4 * q);
          }
          ix[l] = bits;
          const int n = l & 31;
          for (int e = 0; e < 16; ++e) b[l][e] = (_Float16)B[kK(hb, l, e)][n];
        }
        (void)hipMemcpy(da, a.data(), 64 * sizeof(f16x8), hipMemcpyHostToDevice);
        (void)hipMemcpy(db, b.data(), 64 * sizeof(f16x16), hipMemcpyHostToDevice);
        (void)hipMemcpy(di, ix.data(), 64 * 4, hipMemcpyHostToDevice);
        one<<<1, 64>>>(da, db, di, dc);
        std::vector<f32x16> c(64);
        (void)hipMemcpy(c.data(), dc, 64 * sizeof(f32x16), hipMemcpyDeviceToHost);
        int bad = 0, badT = 0;
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 16; ++i) {
            int r, n;
            cRC(l, i, r, n);
            bad += fabsf(c[l][i] - C[r][n]) > 1e-3f;
            badT += fabsf(c[l][i] - C[n][r]) > 1e-3f;
          }
        printf("32x32x32: A-layout %d B-layout %d index %d: mismatches %d (transposed C: %d)\n", ha, hb, hi, bad,
               badT);
      }
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 2048;
  for (int rep = 0; rep < 2; ++rep) {
    float ms32 = 0, ms16 = 0;
    (void)hipEventRecord(e0);
    rate<true><<<2048, 256>>>(da, db, di, dr, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms32, e0, e1);
    (void)hipEventRecord(e0);
    rate<false><<<2048, 256>>>(da, db, di, dr, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms16, e0, e1);
    // wave-instructions per SIMD: 2048 x 4 waves x iters x {4, 8} over 1024 SIMDs
    const double n32 = 2048.0 * 4 * iters * 4 / 1024, n16 = 2048.0 * 4 * iters * 8 / 1024;
    printf("rate: 32x32x32 %.2f ns / instr / SIMD (%.1f logical TF/s), 16x16x64 %.2f ns (%.1f TF/s)\n",
           ms32 * 1e6 / n32, 2048.0 * 4 * iters * 4 * 32768 * 2 / (ms32 * 1e-3) / 1e12, ms16 * 1e6 / n16,
           2048.0 * 4 * iters * 8 * 16384 * 2 / (ms16 * 1e-3) / 1e12);
  }
  return 0;
}
