// Probe of gfx950's v_smfmac_f32_16x16x64_f16 (2:4 structured-sparse A): which lane layout
// and index encoding reproduce a host reference, and its issue rate against the dense
// v_mfma_f32_16x16x32_f16.  Test infrastructure for the sparse weight-gradient design (not
// linked into libba3c).  Build: hipcc --offload-arch=gfx950 -O3 smfmac_probe.hip -o smfmac_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

__global__ void one(const f16x8* a, const f16x16* b, const int* idx, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a[l], b[l], acc, idx[l], 0, 0);
  c[l] = acc;
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
__global__ void one32(const f16x4* a, const f16x8* b, const int* idx, f32x4* c) {
  const int l = threadIdx.x;
  f32x4 acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_smfmac_f32_16x16x32_f16(a[l], b[l], acc, idx[l], 0, 0);
  c[l] = acc;
}
__global__ void rate32(const f16x8* a, const f16x16* b, const int* idx, f32x4* c, int iters) {
  const int l = threadIdx.x & 63;
  f16x8 a8 = a[l];
  f16x4 av = {a8[0], a8[1], a8[2], a8[3]};
  f16x16 bv = b[l];
  f16x8 bl = {bv[0], bv[1], bv[2], bv[3], bv[4], bv[5], bv[6], bv[7]};
  const int ix = idx[l];
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = __builtin_amdgcn_smfmac_f32_16x16x32_f16(av, bl, acc[j], ix, 0, 0);
  }
  f32x4 s = acc[0];
  for (int j = 1; j < 8; ++j) s += acc[j];
  c[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <bool SPARSE>
__global__ void rate(const f16x8* a, const f16x16* b, const int* idx, f32x4* c, int iters) {
  const int l = threadIdx.x & 63;
  f16x8 av = a[l];
  f16x16 bv = b[l];
  f16x8 bl = {bv[0], bv[1], bv[2], bv[3], bv[4], bv[5], bv[6], bv[7]};
  const int ix = idx[l];
  f32x4 acc[8];
  for (int j = 0; j < 8; ++j) acc[j] = f32x4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      if (SPARSE) acc[j] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, acc[j], ix, 0, 0);
      else acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(av, bl, acc[j], 0, 0, 0);
    }
  }
  f32x4 s = acc[0];
  for (int j = 1; j < 8; ++j) s += acc[j];
  c[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// dependent chains: NACC accumulators round-robin (NACC = 1: every smfmac waits for the
// previous one's result)
template <int NACC>
__global__ void chain(const f16x8* a, const f16x16* b, const int* idx, f32x4* c, int iters) {
  const int l = threadIdx.x & 63;
  f16x8 av = a[l];
  f16x16 bv = b[l];
  const int ix = idx[l];
  f32x4 acc[NACC];
  for (int j = 0; j < NACC; ++j) acc[j] = f32x4{0, 0, 0, 0};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k % NACC] = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, acc[k % NACC], ix, 0, 0);
  }
  f32x4 s = acc[0];
  for (int j = 1; j < NACC; ++j) s += acc[j];
  c[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

static int kA(int hyp, int lane, int e) {  // logical K of lane's logical A element e (0..15)
  const int g = lane >> 4;
  return hyp == 0 ? 16 * g + e : (e < 8 ? 8 * g + e : 32 + 8 * g + (e - 8));
}

int main() {
  srand(7);
  // dense-with-2:4 A [16][64], B [64][16]
  float A[16][64], B[64][16], C[16][16];
  for (int r = 0; r < 16; ++r)
    for (int q = 0; q < 16; ++q) {
      int i0 = rand() % 4, i1 = rand() % 4;
      while (i1 == i0) i1 = rand() % 4;
      for (int j = 0; j < 4; ++j) A[r][4 * q + j] = 0.f;
      A[r][4 * q + i0] = (float)(rand() % 9 - 4);
      A[r][4 * q + i1] = (float)(rand() % 9 - 4);
    }
  for (int k = 0; k < 64; ++k)
    for (int n = 0; n < 16; ++n) B[k][n] = (float)(rand() % 7 - 3);
  for (int r = 0; r < 16; ++r)
    for (int n = 0; n < 16; ++n) {
      float s = 0;
      for (int k = 0; k < 64; ++k) s += A[r][k] * B[k][n];
      C[r][n] = s;
    }
  f16x8* da; f16x16* db; int* di; f32x4* dc;
  hipMalloc(&da, 64 * sizeof(f16x8)); hipMalloc(&db, 64 * sizeof(f16x16));
  hipMalloc(&di, 64 * 4); hipMalloc(&dc, sizeof(f32x4) * 2048 * 256);
  for (int ha = 0; ha < 2; ++ha)
    for (int hb = 0; hb < 2; ++hb)
      for (int hi = 0; hi < 2; ++hi) {
        std::vector<f16x8> a(64); std::vector<f16x16> b(64); std::vector<int> ix(64, 0);
        for (int l = 0; l < 64; ++l) {
          const int r = l & 15;
          // the lane's 16 logical A elements = 4 quads of consecutive logical K (quad-aligned
          // in both hypotheses); compress each quad to its 2 non-zeros (ascending positions)
          int bits = 0;
          for (int q = 0; q < 4; ++q) {
            const int k0 = kA(ha, l, 4 * q);
            int pos[2], np = 0;
            for (int j = 0; j < 4 && np < 2; ++j) if (A[r][k0 + j] != 0.f) pos[np++] = j;
            while (np < 2) { pos[np] = (np == 0 ? 0 : (pos[0] == 3 ? 2 : 3)); if (np == 1 && pos[1] < pos[0]) { int t = pos[0]; pos[0] = pos[1]; pos[1] = t; } ++np; }
            a[l][2 * q] = (_Float16)A[r][k0 + pos[0]];
            a[l][2 * q + 1] = (_Float16)A[r][k0 + pos[1]];
            const int nib = hi == 0 ? (pos[0] | (pos[1] << 2)) : (pos[1] | (pos[0] << 2));
            bits |= nib << (4 * q);
          }
          ix[l] = bits;
          const int n = l & 15;
          for (int e = 0; e < 16; ++e) b[l][e] = (_Float16)B[kA(hb, l, e)][n];
        }
        hipMemcpy(da, a.data(), 64 * sizeof(f16x8), hipMemcpyHostToDevice);
        hipMemcpy(db, b.data(), 64 * sizeof(f16x16), hipMemcpyHostToDevice);
        hipMemcpy(di, ix.data(), 64 * 4, hipMemcpyHostToDevice);
        one<<<1, 64>>>(da, db, di, dc);
        std::vector<f32x4> c(64);
        hipMemcpy(c.data(), dc, 64 * sizeof(f32x4), hipMemcpyDeviceToHost);
        int bad = 0, badT = 0;
        for (int l = 0; l < 64; ++l)
          for (int i = 0; i < 4; ++i) {
            const int n = l & 15, r = 4 * (l >> 4) + i;
            bad += fabsf(c[l][i] - C[r][n]) > 1e-3f;
            badT += fabsf(c[l][i] - C[n][r]) > 1e-3f;
          }
        printf("A-layout %d B-layout %d index %d: mismatches %d (transposed C: %d)\n", ha, hb, hi, bad, badT);
      }
  // v_smfmac_f32_16x16x32_f16 (A 16 x 32 logical, 4 stored halves per lane; B 32 x 16): lane
  // layouts 0 / 1 for the A and B halves of K (16 lanes per K block of 8), nibble order 0 / 1
  for (int hb = 0; hb < 2; ++hb)
    for (int hi = 0; hi < 2; ++hi) {
      std::vector<_Float16> a(64 * 4); std::vector<_Float16> b(64 * 8); std::vector<int> ix(64, 0);
      for (int l = 0; l < 64; ++l) {
        const int r = l & 15, g = l >> 4;
        int bits = 0;
        for (int q = 0; q < 2; ++q) {
          const int k0 = 8 * g + 4 * q;
          int pos[2], np = 0;
          for (int j = 0; j < 4 && np < 2; ++j) if (A[r][k0 + j] != 0.f) pos[np++] = j;
          while (np < 2) { pos[np] = (np == 0 ? 0 : (pos[0] == 3 ? 2 : 3)); if (np == 1 && pos[1] < pos[0]) { int t = pos[0]; pos[0] = pos[1]; pos[1] = t; } ++np; }
          a[4 * l + 2 * q] = (_Float16)A[r][k0 + pos[0]];
          a[4 * l + 2 * q + 1] = (_Float16)A[r][k0 + pos[1]];
          const int nib = hi == 0 ? (pos[0] | (pos[1] << 2)) : (pos[1] | (pos[0] << 2));
          bits |= nib << (4 * q);
        }
        ix[l] = bits;
        const int n = l & 15;
        for (int e = 0; e < 8; ++e) {
          const int k = hb == 0 ? 8 * g + e : (e < 4 ? 4 * g + e : 16 + 4 * g + (e - 4));
          b[8 * l + e] = (_Float16)B[k][n];
        }
      }
      // reference over K 0..31 only
      float C32[16][16];
      for (int r = 0; r < 16; ++r)
        for (int n = 0; n < 16; ++n) {
          float s = 0;
          for (int k = 0; k < 32; ++k) s += A[r][k] * B[k][n];
          C32[r][n] = s;
        }
      hipMemcpy(da, a.data(), 64 * 8, hipMemcpyHostToDevice);
      hipMemcpy(db, b.data(), 64 * 16, hipMemcpyHostToDevice);
      hipMemcpy(di, ix.data(), 64 * 4, hipMemcpyHostToDevice);
      one32<<<1, 64>>>(reinterpret_cast<const f16x4*>(da), reinterpret_cast<const f16x8*>(db), di, dc);
      std::vector<f32x4> c(64);
      hipMemcpy(c.data(), dc, 64 * sizeof(f32x4), hipMemcpyDeviceToHost);
      int bad = 0;
      for (int l = 0; l < 64; ++l)
        for (int i = 0; i < 4; ++i) bad += fabsf(c[l][i] - C32[4 * (l >> 4) + i][l & 15]) > 1e-3f;
      printf("16x16x32: B-layout %d index %d: mismatches %d\n", hb, hi, bad);
    }
  // issue rate: 2048 workgroups x 256 threads, 8 independent accumulators per wave
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  const int iters = 4096;
  for (int rep = 0; rep < 2; ++rep)
    for (int sp = 0; sp < 2; ++sp) {
      hipEventRecord(e0);
      if (sp) rate<true><<<2048, 256>>>(da, db, di, dc, iters);
      else rate<false><<<2048, 256>>>(da, db, di, dc, iters);
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double n = 2048.0 * 4 * iters * 8;   // wave-instructions
      const double flop = n * (sp ? 16.0 * 16 * 64 * 2 : 16.0 * 16 * 32 * 2);
      printf("%s: %.3f ms, %.1f logical TFLOP/s, %.2f ns per wave-instruction per SIMD\n",
             sp ? "smfmac_16x16x64_f16" : "mfma_16x16x32_f16", ms, flop / ms / 1e9,
             ms * 1e6 / (n / 1024.0));
    }
  for (int rep = 0; rep < 2; ++rep) {
    hipEventRecord(e0);
    rate32<<<2048, 256>>>(da, db, di, dc, iters);
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    const double n = 2048.0 * 4 * iters * 8;
    printf("smfmac_16x16x32_f16: %.3f ms, %.1f logical TFLOP/s, %.2f ns per wave-instruction per SIMD\n", ms,
           n * 16.0 * 16 * 32 * 2 / ms / 1e9, ms * 1e6 / (n / 1024.0));
  }
  // dependent-chain rate: one wave per SIMD (256 workgroups x 256 threads) and 2 per SIMD
  for (int wps = 1; wps <= 2; ++wps)
    for (int nacc : {1, 2, 3, 4, 8}) {
      hipEventRecord(e0);
      const int nb = 256 * wps;
      switch (nacc) {
        case 1: chain<1><<<nb, 256>>>(da, db, di, dc, iters); break;
        case 2: chain<2><<<nb, 256>>>(da, db, di, dc, iters); break;
        case 3: chain<3><<<nb, 256>>>(da, db, di, dc, iters); break;
        case 4: chain<4><<<nb, 256>>>(da, db, di, dc, iters); break;
        default: chain<8><<<nb, 256>>>(da, db, di, dc, iters); break;
      }
      hipEventRecord(e1); hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1);
      const double n = (double)nb * 4 * iters * 8;   // wave-instructions
      printf("smfmac_16x16x64 chain: %d waves/SIMD, %d accumulators: %.2f ns per wave-instruction per SIMD\n",
             wps, nacc, ms * 1e6 / (n / 1024.0));
    }
  return 0;
}
